"""Graph-timed BN backward per layer shape: single-launch (in-launch barrier) vs two-launch path.

    python scripts/bn_bench.py
"""
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.dirname(HERE), HERE]
from tspm_amd import _lib as L  # noqa: E402
from tune_convs import graph_time  # noqa: E402

SHAPES = [(96256, 64), (24576, 64), (6144, 128), (1536, 256), (384, 512), (25088, 64), (6272, 64), (2048, 128),
          (512, 256), (128, 512)]


def main():
    dev = torch.device("cuda", 0)
    lib = L.lib()
    g = torch.Generator().manual_seed(0)
    for m, c in SHAPES:
        y = torch.randn(m, c, generator=g).to(dev)
        out = torch.randn(m, c, generator=g).relu().to(dev)
        gg = torch.randn(m, c, generator=g).to(dev)
        mean, inv = y.mean(0).contiguous(), torch.ones(c, device=dev)
        gamma = torch.ones(c, device=dev)
        wsb = lib.tspm_bn_bwd_workspace(m, c)
        ws = torch.zeros(wsb, dtype=torch.uint8, device=dev)
        dy, gw, gb = torch.empty(m, c, device=dev), torch.empty(c, device=dev), torch.empty(c, device=dev)
        res = {}
        for fused in ("1", "0"):
            os.environ["TSPM_BN_BWD_FUSED"] = fused

            def make():
                def f():
                    return lib.tspm_bn_bwd(m, c, gg.data_ptr(), out.data_ptr(), y.data_ptr(), mean.data_ptr(),
                                           inv.data_ptr(), gamma.data_ptr(), gw.data_ptr(), gb.data_ptr(), dy.data_ptr(),
                                           None, None, None, None, None, None, None, None, None, None, 0,
                                           ws.data_ptr(), wsb, L.stream_handle())
                return f
            res[fused] = graph_time(make, 20, 5)
        print(f"m={m:6d} c={c:4d}  fused {res['1']:7.2f} us   two-launch {res['0']:7.2f} us   "
              f"bytes {m * c * 16 / 1e6:6.2f} MB", flush=True)
    print("timeouts", lib.tspm_debug_barrier_timeouts())


if __name__ == "__main__":
    main()
