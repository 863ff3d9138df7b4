"""Graph-timed cost of every distinct conv launch of the bench step (batch 128 by default).

    python scripts/conv_bench.py [--batch 128] [--algo-file tuned.json] [--reps 20]

Each (kind, shape) is captured as `reps` back-to-back launches on one stream in a HIP graph and
replayed, so the per-launch figure is device time + the dependent-launch boundary — what the step
pays for that launch (host launch overhead, which dominates a Python launch loop for kernels below
~10 us, is excluded).  Prints per-launch us, valid-tap TFLOP/s, the count per step and the step
total; also the boundary floor (a chain of trivial launches).
"""
from __future__ import annotations

import argparse
import collections
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import tspm_amd  # noqa: E402
from tspm_amd import _lib as L  # noqa: E402
from tspm_amd.engine import EncoderEngine, prepare_encoder_layout  # noqa: E402
from tspm_amd.roofline import conv_macs  # noqa: E402
from tune_convs import Bufs, graph_time, launcher  # noqa: E402


def step_ops(batch, dev, encoders=("audio", "image")):
    """(kind, key) -> [ConvShape, strides, is_stem, count per step, tuned algo]."""
    out = {}
    encs = [(tspm_amd.ResNet18(1, 64), 32, 94, True)] if "audio" in encoders else []
    encs += [(tspm_amd.ResNet34(1, 128), 28, 28, False)] if "image" in encoders else []
    for enc, h, w, three_d in encs:
        enc = enc.to(dev)
        prepare_encoder_layout(enc)
        eng = EncoderEngine(enc, batch, h, w, dev)
        for op in eng.all_convs():
            s = op.shape
            key = (s.n, s.h, s.w, s.c, s.k, s.r, s.s, s.stride, s.pad)
            if op is eng.stem:
                # (sn, sh, sw, sc) of the reference NCHW input, as EncoderEngine.input_strides: [N,H,W] audio, [N,1,H,W] image
                xs = L.Strides4(h * w, w, 1, 0) if three_d else L.Strides4(h * w, w, 1, h * w)
                kinds = (("fwd", op.algo_fwd), ("wgrad", op.algo_wgrad))
            else:
                xs = L.hwnc_strides(s.n, s.h, s.w, s.c)
                kinds = (("fwd", op.algo_fwd), ("dgrad", op.algo_dgrad), ("wgrad", op.algo_wgrad))
            for kind, algo in kinds:
                e = out.setdefault((kind,) + key, [s, xs, op is eng.stem, 0,
                                                   (algo.tm, algo.tn, algo.wn, algo.wk, algo.splits, algo.variant)])
                e[3] += 1
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--json", default=None, help="write results here")
    ap.add_argument("--only", default=None, help="comma-separated kind:h,w,c,k,r,stride filters (e.g. dgrad:2,2,256,256,3,1)")
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    lib = L.lib()
    # boundary floor: a chain of trivial launches
    tiny = torch.zeros(64, device=dev)
    floor = graph_time(lambda: (lambda: lib.tspm_reduce_slabs(4, 1, 0, tiny.data_ptr(), tiny[32:].data_ptr(),
                                                              L.stream_handle())), args.reps)
    print(f"trivial-launch chain: {floor:.2f} us per launch", flush=True)
    rows = []
    tot = collections.defaultdict(float)
    only = None
    if args.only:
        only = set()
        for f in args.only.split(";"):
            k, v = f.split(":")
            h, w, c, kk, r, st = (int(t) for t in v.split(","))
            only.add((k, h, w, c, kk, r, st))
    for key, (s, xs, stem, count, algo) in sorted(step_ops(args.batch, dev).items(), key=lambda kv: str(kv[0])):
        kind = key[0]
        if only is not None and (kind, s.h, s.w, s.c, s.k, s.r, s.stride) not in only:
            continue
        b = Bufs(s, stem, dev)
        us = graph_time(lambda: launcher(kind, s, xs, b, algo)[0], args.reps, args.iters)
        _, valid = conv_macs(s.n, s.h, s.w, s.c, s.k, s.r, s.s, s.stride, s.pad)
        tf = 2 * valid / (us * 1e-6) / 1e12
        tot[kind] += us * count
        rows.append({"kind": kind, "shape": list(key[1:]), "algo": list(algo), "count": count, "us": round(us, 2),
                     "valid_tflops": round(tf, 2)})
        print(f"{kind:6s} {str(tuple(key[1:])):44s} x{count:2d} {us:8.2f} us  {tf:6.2f} TF/s  algo {algo}", flush=True)
        del b
    print("per-step totals (us):", {k: round(v, 1) for k, v in tot.items()}, "all", round(sum(tot.values()), 1))
    if args.json:
        with open(args.json, "w") as fh:
            json.dump({"floor_us": floor, "rows": rows, "totals": tot}, fh, indent=1)


if __name__ == "__main__":
    main()
