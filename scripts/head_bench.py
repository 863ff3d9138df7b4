"""Graph-timed tspm_head_train_step (both launches) at batch 128 / 1024, and its two kernels' device
durations from torch.profiler: the fusion head's cost in isolation.

    python scripts/head_bench.py            # timing
    python scripts/head_bench.py --stamps   # + phase stamps of k_head_rows (needs `make stamps`)
"""
import ctypes
import os
import sys

import numpy as np
import torch

STAMPS = "--stamps" in sys.argv
if STAMPS:
    os.environ["TSPM_LIB"] = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                          "task-specific-pretraining-multimodal_amd", "libtspm_stamps.so")

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import tspm_amd  # noqa: E402,F401
from tspm_amd import _lib as L  # noqa: E402
from test_gpu_head import _buffers  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    for n in (128, 1024):
        ws, out = _buffers(n, 192, 128, 64, 10, dev, seed=1)
        keep = torch.ones(n, 128, dtype=torch.uint8, device=dev)
        ctr = torch.zeros(1, dtype=torch.int64, device=dev)
        d = L.HeadDesc(n=n, in_=192, hidden=128, hidden2=64, classes=10, ldx=192, lddx=192, gen_keep=1, p=0.5,
                       loss_weight=1.0, seed=7, counter=ctr.data_ptr(), keep=keep.data_ptr(),
                       labels=ws["labels"].data_ptr(),
                       **{k: ws[k].data_ptr() for k in ("x", "w0", "b0", "w3", "b3", "w5", "b5")},
                       **{k: v.data_ptr() for k, v in out.items()})
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            for _ in range(5):
                L.check(L.lib().tspm_head_train_step(ctypes.byref(d), s.cuda_stream), "head")
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            R = 50
            with torch.cuda.graph(g, stream=s):
                for _ in range(R):
                    L.check(L.lib().tspm_head_train_step(ctypes.byref(d), torch.cuda.current_stream().cuda_stream),
                            "head")
            g.replay()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                g.replay()
            e1.record()
            torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / (5 * R)
        from tspm_amd.roofline import device_kernels
        ks = device_kernels(lambda: g.replay(), 2)
        per = {}
        for k in ks:
            nm = "rows" if "k_head_rows" in k["name"] else "wgrad" if "k_head_wgrad" in k["name"] else k["name"][:30]
            per[nm] = per.get(nm, 0.0) + k["dur"] / (2 * R)
        print(f"n={n}: graph-timed {us:.2f} us per head step; device us per launch {per}", flush=True)
        if STAMPS:
            lib = L.lib()
            lib.tspm_debug_stamps_misc.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
            assert lib.tspm_debug_stamps_misc_clear() == 0
            torch.cuda.synchronize()
            L.check(lib.tspm_head_train_step(ctypes.byref(d), torch.cuda.current_stream().cuda_stream), "head")
            torch.cuda.synchronize()
            buf = np.zeros((1 << 18) * 12, dtype=np.uint64)
            assert lib.tspm_debug_stamps_misc(buf.ctypes.data, buf.nbytes) == 0
            st = buf.reshape(-1, 12).astype(np.int64)
            st = st[st[:, 0] > 0]
            rel = (st[:, :6] - st[:, 0].min()) * 0.01
            names = ["entry", "staged", "fc0", "fc3+fc5", "CE", "bwd (dz3, dz0, dx)"]
            print(f"   {len(st)} waves; entry spread p50 {np.percentile(rel[:, 0], 50):.2f} max {rel[:, 0].max():.2f} us; "
                  f"last stamp max {rel.max():.2f} us", flush=True)
            for i in range(1, 6):
                dd = (st[:, i] - st[:, i - 1]) * 0.01
                print(f"   {names[i]:20s} p50 {np.percentile(dd, 50):6.2f}  p90 {np.percentile(dd, 90):6.2f}  "
                      f"max {dd.max():6.2f} us", flush=True)
            clk = (st[:, 7] - st[:, 6]) / ((st[:, 5] - st[:, 0]) * 0.01)
            print(f"   in-kernel clock p50 {np.percentile(clk, 50):.0f} MHz", flush=True)


if __name__ == "__main__":
    main()
