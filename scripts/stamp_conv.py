"""Phase timing of single conv launches from in-kernel s_memrealtime stamps (diagnostic build).

    make -C task-specific-pretraining-multimodal_amd/csrc stamps
    python scripts/stamp_conv.py --only "dgrad:2,2,256,256,3,1;fwd:8,24,64,64,3,1"

Stamps (lane 0 of every wave, 100 MHz chip clock): 0 entry, 1 main loop done, 2 split-K combine
done, 3 epilogue stores done, 4 (fwd) in-launch BN tail done.  Prints, per launch, the spread of
wave start times and percentiles of each phase, in microseconds.
"""
from __future__ import annotations

import argparse
import ctypes
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
os.environ.setdefault("TSPM_LIB", os.path.join(REPO, "task-specific-pretraining-multimodal_amd", "libtspm_stamps.so"))
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from tspm_amd import _lib as L  # noqa: E402
from conv_bench import step_ops  # noqa: E402
from tune_convs import Bufs, launcher  # noqa: E402

SLOTS = 12  # TSPM_STAMP_SLOTS (common.h)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", required=True)
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--algo", default=None, help="override tm,tn,wn,wk,splits for every listed shape")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    lib = L.lib()
    lib.tspm_debug_stamps.restype = ctypes.c_int
    lib.tspm_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    lib.tspm_debug_stamps_clear.restype = ctypes.c_int
    lib.tspm_debug_stamps_lds.restype = ctypes.c_int
    lib.tspm_debug_stamps_lds.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    lib.tspm_debug_stamps_lds_clear.restype = ctypes.c_int
    want = set()
    for f in args.only.split(";"):
        k, v = f.split(":")
        want.add((k,) + tuple(int(t) for t in v.split(",")))
    for key, (s, xs, stem, count, algo) in sorted(step_ops(args.batch, dev).items(), key=lambda kv: str(kv[0])):
        kind = key[0]
        if (kind, s.h, s.w, s.c, s.k, s.r, s.stride) not in want:
            continue
        algos = [tuple(int(t) for t in a.split(",")) for a in args.algo.split("/")] if args.algo else [algo]
        b = Bufs(s, stem, dev)
        for algo in algos:
            report(lib, kind, key, s, xs, b, algo)
        del b


def report(lib, kind, key, s, xs, b, algo):
    if True:
        f, _ = launcher(kind, s, xs, b, algo)
        for _ in range(5):
            assert f() == 0
        torch.cuda.synchronize()
        buf = np.zeros((1 << 18) * SLOTS, dtype=np.uint64)
        lds_variant = len(algo) > 5 and algo[5] in (1, 2)
        assert (lib.tspm_debug_stamps_lds_clear if lds_variant else lib.tspm_debug_stamps_clear)() == 0
        torch.cuda.synchronize()
        assert f() == 0
        torch.cuda.synchronize()
        assert (lib.tspm_debug_stamps_lds if lds_variant else lib.tspm_debug_stamps)(buf.ctypes.data, buf.nbytes) == 0
        st = buf.reshape(-1, SLOTS).astype(np.int64)
        used = st[:, 0] > 0
        nw = int(used.sum())
        if nw == 0:
            print(f"{kind:6s} {tuple(key[1:])} algo {algo}: no stamps (kernel not instrumented)", flush=True)
            return
        st = st[used]
        t0 = st[:, 0].min()
        rel = (st - t0) * 0.01  # us
        print(f"{kind:6s} {tuple(key[1:])} algo {algo}: {nw} waves", flush=True)
        print(f"   start spread: p50 {np.percentile(rel[:, 0], 50):.2f} p90 {np.percentile(rel[:, 0], 90):.2f} "
              f"max {rel[:, 0].max():.2f} us;  last stamp max {rel.max():.2f} us")
        if lds_variant:
            pairs = [(1, 0, "1st data"), (2, 1, "loop rest"), (3, 2, "combine"), (6, 3, "slab+tkt"),
                     (4, 6, "slab rd"), (4, 3, "split-K"), (5, 4, "epilogue"), (5, 0, "total")]
        else:
            pairs = [(5, 0, "1st data"), (1, 5, "loop rest"), (2, 1, "combine"), (3, 2, "epilogue"), (4, 3, "bn tail")]
        if lds_variant and (st[:, 7] > 0).any():
            ok = (st[:, 7] > 0) & (st[:, 6] > 0)
            clk = (st[ok, 7] - st[ok, 6]) / ((st[ok, 5] - st[ok, 0]) * 0.01)  # cycles per us = MHz
            print(f"   in-kernel clock: p10 {np.percentile(clk, 10):.0f}  p50 {np.percentile(clk, 50):.0f}  "
                  f"p90 {np.percentile(clk, 90):.0f} MHz")
        lc = st[:, 11] > 0  # compute waves of the LDS kernels: per-stage shader cycles (conv_lds.hip LoopClock)
        if lds_variant and lc.any():
            n = st[lc, 11].astype(np.float64)
            per = {nm: st[lc, k] / n for k, nm in ((8, "barrier"), (9, "frag rd"), (10, "mfma"))}
            tot = per["barrier"] + per["frag rd"] + per["mfma"]
            print(f"   loop, cycles/stage (compute waves, {int(lc.sum())}; stages p50 {np.percentile(n, 50):.0f}): " +
                  "  ".join(f"{k} p50 {np.percentile(v, 50):.0f}" for k, v in per.items()) +
                  f"  -> mfma share p50 {np.percentile(per['mfma'] / tot, 50):.2f}")
        for i, j, nm in pairs:
            d = st[:, i] - st[:, j]
            ok = (st[:, i] > 0) & (st[:, j] > 0)
            if ok.sum() == 0:
                continue
            d = d[ok] * 0.01
            print(f"   {nm:9s}: p10 {np.percentile(d, 10):6.2f}  p50 {np.percentile(d, 50):6.2f}  "
                  f"p90 {np.percentile(d, 90):6.2f}  max {d.max():6.2f} us")


if __name__ == "__main__":
    main()
