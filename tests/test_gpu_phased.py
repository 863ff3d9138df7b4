"""External events inside a captured HIP graph — the mechanism the DP step's exchange ordering rests on
(step.FusedTrainStep._run_phased: the gradient all-reduce of a backward phase waits, outside the graph,
on an event the graph records when that phase is done).

A graph whose first part is ~ms of work ends by writing a per-replay counter value into ``x`` and
recording an external event, then runs more work.  After each replay another stream waits on the
event and copies ``x``: the copy must see THIS replay's value (never the previous one's)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_external_event_in_graph_orders_outside_stream(gpu):
    from tspm_amd import _lib as L
    dev = torch.device("cuda", 0)
    z = torch.ones(1 << 22, device=dev)
    cnt = torch.zeros(1, device=dev)
    x = torch.zeros(1, device=dev)
    ev = L.ExternalEvent()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        for _ in range(300):  # a few ms before the event
            z.mul_(1.0000001)
        cnt.add_(1.0)
        x.copy_(cnt)
        ev.record()
        for _ in range(300):  # and after it
            z.mul_(0.9999999)
    seen = []
    y = torch.zeros(1, device=dev)
    for _ in range(6):
        g.replay()
        ev.wait(s)
        with torch.cuda.stream(s):
            y.copy_(x)
            seen.append(y.clone())
        torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    assert [float(v) for v in seen] == [1.0, 2.0, 3.0, 4.0, 5.0, 6.0]

