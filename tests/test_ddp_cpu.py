"""Data-parallel exchange logic on CPU: world-size-2 gloo process group (the GPU path uses the same
code over RCCL).  Checks the bucketed all-reduce of a flat gradient buffer, last-bucket-first
order, the 1/world fold, and parameter broadcast."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import tspm_amd
from tspm_amd import ddp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    try:
        r, w, _ = ddp.init_from_env("gloo")
        assert (r, w) == (rank, world)
        n = 1_000_003
        g = torch.arange(n, dtype=torch.float32) * (rank + 1)
        ar = ddp.GradAllReduce([g], bucket_mb=1.0)
        assert len(ar.buckets) == -(-n // (1 << 18))
        assert ar.buckets[0].data_ptr() > ar.buckets[-1].data_ptr()  # last bucket first
        ar()
        exp = torch.arange(n, dtype=torch.float32) * sum(range(1, world + 1))
        ok_sum = bool(torch.equal(g, exp))
        m = torch.nn.Linear(4, 3)
        torch.manual_seed(100 + rank)
        with torch.no_grad():
            m.weight.normal_()
        ddp.broadcast_parameters(m, src=0)
        wsum = torch.tensor([m.weight.sum().item()])
        gathered = [torch.zeros(1) for _ in range(world)]
        dist.all_gather(gathered, wsum)
        ok_bcast = all(torch.equal(t, gathered[0]) for t in gathered)
        q.put((rank, ok_sum, ok_bcast))
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover - surfaced by the parent
        q.put((rank, repr(e), None))


def test_gloo_world2_bucketed_allreduce_and_broadcast():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for rank, ok_sum, ok_bcast in res:
        assert ok_sum is True, (rank, ok_sum)
        assert ok_bcast is True, (rank, ok_bcast)


def _phased_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    try:
        ddp.init_from_env("gloo")
        # a flat buffer of 5 "parameters" (slots padded to 4 floats), phases interleaved
        numels = [10, 3, 7, 1, 12]
        offsets, off = [], 0
        for n in numels:
            offsets.append(off)
            off += -(-n // 4) * 4
        flat = torch.arange(off, dtype=torch.float32) * (rank + 1)
        sel1 = [False, True, True, False, True]
        r1 = ddp.flat_ranges(offsets, numels, off, sel1)
        r2 = ddp.flat_ranges(offsets, numels, off, [not s for s in sel1])
        ok_ranges = r1 == [(12, 24), (28, 40)] and r2 == [(0, 12), (24, 28)]
        ar = ddp.PhasedGradAllReduce([[flat[a:b] for a, b in r1], [flat[a:b] for a, b in r2]], bucket_mb=1e-5)
        w1 = ar.launch(0)
        w2 = ar.launch(1)
        ar.wait(w1 + w2)
        ok_sum = bool(torch.equal(flat, torch.arange(off, dtype=torch.float32) * sum(range(1, world + 1))))
        q.put((rank, ok_ranges, ok_sum))
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover - surfaced by the parent
        q.put((rank, repr(e), None))


def test_gloo_world2_phased_allreduce_ranges():
    """flat_ranges merges adjacent selected slots (padding included) and the two phases together
    cover the buffer; PhasedGradAllReduce sums every range across ranks (small buckets)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_phased_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for rank, ok_ranges, ok_sum in res:
        assert ok_ranges is True, (rank, ok_ranges)
        assert ok_sum is True, (rank, ok_sum)


def test_single_process_allreduce_is_noop():
    g = torch.ones(10)
    ddp.GradAllReduce([g])()
    assert torch.equal(g, torch.ones(10))
    assert ddp.init_from_env() == (0, 1, 0) or not dist.is_initialized()
