"""Step flags across a captured HIP graph's boundary — the mechanism the DP step's exchange ordering
rests on (step.FusedTrainStep._run_phased: the gradient all-reduce of a backward phase waits, outside
the graph, for a per-step count the graph publishes to pinned host memory when that phase is done;
ROCm 7 refuses graph-external event records, the CUDA idiom for this).

A graph whose first part is ~ms of work ends by writing a per-replay counter value into ``x`` and
bumping a ``DeviceFlag``, then runs more work.  After each replay the host waits for the flag, then
enqueues a copy of ``x`` on another stream: the copy must see THIS replay's value (never the previous
one's) — and the host must have seen the flag before the graph's tail finished (checked on timing)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_flag_in_graph_orders_outside_stream(gpu):
    from tspm_amd import _lib as L
    dev = torch.device("cuda", 0)
    z = torch.ones(1 << 22, device=dev)
    cnt = torch.zeros(1, device=dev)
    x = torch.zeros(1, device=dev)
    flag = L.DeviceFlag()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        for _ in range(300):  # a few ms before the flag
            z.mul_(1.0000001)
        cnt.add_(1.0)
        x.copy_(cnt)
        flag.bump()
        for _ in range(300):  # and after it
            z.mul_(0.9999999)
    seen, early = [], []
    y = torch.zeros(1, device=dev)
    main = torch.cuda.current_stream()
    for k in range(6):
        g.replay()
        flag.host_wait(k + 1)
        early.append(not main.query())  # the graph's tail (~ms) is still running when the host sees the flag
        with torch.cuda.stream(s):
            y.copy_(x)
            seen.append(y.clone())
        torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    assert [float(v) for v in seen] == [1.0, 2.0, 3.0, 4.0, 5.0, 6.0]
    assert sum(early) >= 5, early
