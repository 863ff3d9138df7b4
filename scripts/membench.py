"""Dependent-load latency on the GPU by working set and stride (diagnostic; not the product).

    python scripts/membench.py          # builds build/membench.so with hipcc if missing
"""
import ctypes
import os
import subprocess
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(os.path.dirname(HERE), "build", "membench.so")


def build():
    os.makedirs(os.path.dirname(SO), exist_ok=True)
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "--offload-arch=gfx950", "-shared", "-fPIC",
                    os.path.join(HERE, "membench.hip"), "-o", SO], check=True)


def main():
    if not os.path.exists(SO) or (len(sys.argv) > 1 and sys.argv[1] == "build"):
        build()
        if len(sys.argv) > 1:
            return
    lib = ctypes.CDLL(SO)
    lib.mb_chase.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_int]
    dev = torch.device("cuda", 0)
    out = torch.zeros(2, dtype=torch.int64, device=dev)
    rng = np.random.default_rng(0)
    lib.mb_shape.argtypes = [ctypes.c_void_p, ctypes.c_longlong, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                             ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
    big = torch.randn(1 << 20, device=dev)  # 4 MB
    fo = torch.zeros(4, device=dev)
    for row_bytes in (256, 1024):
        for blocks, threads in ((256, 64), (256, 256), (1024, 256), (2048, 512)):
            for pattern in (0, 1):
                iters = 64
                for _ in range(2):
                    lib.mb_shape(big.data_ptr(), big.numel(), row_bytes, iters, pattern, fo.data_ptr(), blocks, threads)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(5):
                    lib.mb_shape(big.data_ptr(), big.numel(), row_bytes, iters, pattern, fo.data_ptr(), blocks, threads)
                e1.record()
                torch.cuda.synchronize()
                us = e0.elapsed_time(e1) * 1000 / 5
                nbytes = blocks * threads * iters * 8 * 16
                print(f"shape row {row_bytes:5d} B grid {blocks:5d}x{threads:4d} pattern {pattern}: {us:8.1f} us "
                      f"{nbytes / us / 1e6:7.2f} TB/s", flush=True)
    for ws_bytes, stride in [(16 << 10, 64), (64 << 10, 128), (256 << 10, 128), (1 << 20, 128), (2 << 20, 1024),
                             (2 << 20, 4096), (16 << 20, 4096), (64 << 20, 4096), (1 << 30, 4096)]:
        n = ws_bytes // 4
        step = stride // 4
        slots = np.arange(0, n, step, dtype=np.int64)
        perm = rng.permutation(len(slots))
        nxt = np.zeros(n, dtype=np.uint32)
        order = slots[perm]
        nxt[order] = np.roll(order, -1).astype(np.uint32)
        buf = torch.from_numpy(nxt).to(dev)
        hops = min(len(slots), 2000)
        res = []
        for cold in (1, 1, 0):
            torch.cuda.synchronize()
            assert lib.mb_chase(buf.data_ptr(), hops, int(order[0]), out.data_ptr(), cold) == 0
            torch.cuda.synchronize()
            res.append(out[0].item() * 10.0 / hops)
        print(f"working set {ws_bytes / 1024:10.0f} KiB stride {stride:8d} B  hops {hops:5d}: "
              f"cold {res[0]:7.1f}  next-kernel {res[1]:7.1f}  in-kernel warm {res[2]:7.1f} ns/hop", flush=True)
        del buf


if __name__ == "__main__":
    main()
