"""Do two conv launches on two streams overlap?  For selected (kind, shape) and algos: per-launch
time of 2R back-to-back launches on one stream vs R launches on each of two streams (HIP graph).

    python scripts/concurrency_probe.py --only "dgrad:2,2,256,256,3,1" --algo 1,1,2,2,4,1/1,1,2,2,1,1
"""
from __future__ import annotations

import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from conv_bench import step_ops  # noqa: E402
from tune_convs import Bufs, launcher  # noqa: E402


def time_graph(body, iters=20):
    body()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        body()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000.0 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", required=True)
    ap.add_argument("--algo", default=None)
    ap.add_argument("--reps", type=int, default=10)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    want = set()
    for f in args.only.split(";"):
        k, v = f.split(":")
        want.add((k,) + tuple(int(t) for t in v.split(",")))
    side = torch.cuda.Stream()
    R = args.reps
    for key, (s, xs, stem, count, algo0) in sorted(step_ops(128, dev).items(), key=lambda kv: str(kv[0])):
        kind = key[0]
        if (kind, s.h, s.w, s.c, s.k, s.r, s.stride) not in want:
            continue
        algos = [tuple(int(t) for t in a.split(",")) for a in args.algo.split("/")] if args.algo else [algo0]
        ba, bb = Bufs(s, stem, dev), Bufs(s, stem, dev)
        for algo in algos:
            launcher(kind, s, xs, ba, algo)[0]()
            launcher(kind, s, xs, bb, algo)[0]()
            torch.cuda.synchronize()

            def one_stream():
                fa = launcher(kind, s, xs, ba, algo)[0]
                fb = launcher(kind, s, xs, bb, algo)[0]
                for _ in range(R):
                    fa()
                    fb()

            def two_streams():
                main = torch.cuda.current_stream()
                side.wait_stream(main)
                fa = launcher(kind, s, xs, ba, algo)[0]
                for _ in range(R):
                    fa()
                with torch.cuda.stream(side):
                    fb = launcher(kind, s, xs, bb, algo)[0]
                    for _ in range(R):
                        fb()
                main.wait_stream(side)

            t1 = time_graph(one_stream) / (2 * R)
            t2 = time_graph(two_streams) / (2 * R)
            print(f"{kind:6s} {tuple(key[1:])} algo {algo}: serial {t1:6.2f} us/launch  two streams {t2:6.2f} "
                  f"us/launch  overlap gain {t1 / t2:4.2f}x", flush=True)


if __name__ == "__main__":
    main()
