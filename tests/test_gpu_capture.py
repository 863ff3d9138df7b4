"""Graph capture beside torch.distributed's NCCL watchdog.

The round-4 abort in destroy_process_group and the round-5 abort of ``bench.py --phased``
(gpurun_out/r5a_phased.err: "Process group watchdog thread terminated with exception: HIP error: operation
not permitted when stream is capturing", thrown from WorkNCCL::finishedGPUExecutionInternal's hipEventQuery)
have one cause: a step graph captured in torch's default GLOBAL capture mode while a collective of an earlier
eager step was still in the watchdog's list — the watchdog thread's event query during the capture is illegal
in that mode, it throws and the process terminates.  Every step of this package now captures in thread-local
mode (``_lib.graph_capture``).  This test holds a capture open for several watchdog periods with an
un-waited all-reduce outstanding; under the old mode it takes the process down."""
import os
import socket
import time

import pytest
import torch

import tspm_amd
from tspm_amd import _lib as L

pytestmark = pytest.mark.gpu


def test_capture_survives_watchdog_with_pending_collective(gpu):
    import torch.distributed as dist
    s_ = socket.socket()
    s_.bind(("127.0.0.1", 0))
    port = s_.getsockname()[1]
    s_.close()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    created = False
    if not dist.is_initialized():
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=gpu)
        created = True
    try:
        x = torch.ones(1 << 20, device=gpu)
        y = torch.zeros(1 << 20, device=gpu)
        for _ in range(3):
            work = dist.all_reduce(x, async_op=True)  # left to the watchdog (no wait before the capture)
            del work
            g = torch.cuda.CUDAGraph()
            with L.graph_capture(g):
                y.add_(1.0)
                time.sleep(0.5)  # five watchdog periods with the capture open
            g.replay()
        torch.cuda.synchronize()
        assert float(y[0]) == 3.0
        # a real step captured right behind an eager phased step's collectives (the bench's --phased order)
        torch.manual_seed(3)
        m = tspm_amd.AVMNIST(tspm_amd.ResNet18(1, 64), tspm_amd.ResNet34(1, 128), 128, dropout=0.5).to(gpu)
        opt = tspm_amd.FusedAdam(m.parameters(), lr=5e-4, weight_decay=1e-4)
        st = tspm_amd.FusedTrainStep(m, opt, None, 32)
        st.allreduce = st.phased_allreduce(force=True)
        from oracle import avmnist_ref as orc
        a, i, lab, _ = orc.synthetic_batch(32, seed=5)
        a, i, lab = a.to(gpu), i.to(gpu), lab.to(gpu)
        st.step(a, i, lab)          # eager: all-reduces launched
        st.step(a, i, lab)          # capture with those works outstanding
        st.allreduce, st.graph = None, None
        st.step(a, i, lab)          # the local step re-captured behind the phased step's works
        st.step(a, i, lab)
        torch.cuda.synchronize()
        assert torch.isfinite(st.loss).all()
        st.close()
    finally:
        if created:
            dist.destroy_process_group()
