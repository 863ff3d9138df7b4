"""Variant 1 vs variant 4 (the same tiles with every fp32 product formed from exact bf16 pieces on the bf16 MFMA)
on every distinct conv launch of the bench step, graph-timed as scripts/tune_convs.py times its candidates.

    python scripts/split_ab.py [--batch 128] [--json out.json]

For each launch: the tuned algo (variant 1) and its variant-4 twin (same tm, tn, wn, wk, splits; wk == 4 entries
also try wk = 2 with twice the wm), both checked against the tuned output (|diff| <= 1e-5 max|y|), per-launch us and
the per-step sums weighted by launch count.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from conv_bench import step_ops  # noqa: E402
from tune_convs import Bufs, graph_time, launcher  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--iters", type=int, default=8)
    ap.add_argument("--json", default=None)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    ops = step_ops(args.batch, dev)
    rows, t1, t4 = [], 0.0, 0.0
    for key, (s, xs, stem, count, base) in sorted(ops.items(), key=lambda kv: str(kv[0])):
        kind = key[0]
        if stem or len(base) < 6 or base[5] not in (1, 2):
            continue
        b = Bufs(s, stem, dev)
        f, out = launcher(kind, s, xs, b, base)
        if f() != 0:
            continue
        torch.cuda.synchronize()
        ref = out.clone()
        scale = float(ref.abs().max()) + 1e-30
        tb = graph_time(lambda: launcher(kind, s, xs, b, base)[0], args.reps, args.iters)
        twins = []
        tm, tn, wn, wk, sp = base[:5]
        if wk <= 2:
            twins.append((tm, tn, wn, wk, sp, 4))
        else:
            twins.append((tm, tn, wn, 2, sp, 4))
            twins.append((tm, tn, wn, 1, sp, 4))
        best = None
        for a in twins:
            f, out = launcher(kind, s, xs, b, a)
            out.fill_(float("nan"))
            if f() != 0:
                continue
            torch.cuda.synchronize()
            err = float((out - ref).abs().max())
            if not err <= 1e-5 * scale:
                print(f"  MISMATCH {kind} {key[1:]} {a} err={err:.3e} scale={scale:.3e}", flush=True)
                continue
            t = graph_time(lambda: launcher(kind, s, xs, b, a)[0], args.reps, args.iters)
            if t is not None and (best is None or t < best[0]):
                best = (t, a, err / scale)
        del b
        if best is None:
            continue
        t1 += tb * count
        t4 += min(best[0], tb) * count
        rows.append({"kind": kind, "shape": list(key[1:]), "count": count, "v1_algo": list(base), "v1_us": round(tb, 2),
                     "v4_algo": list(best[1]), "v4_us": round(best[0], 2), "rel_diff": best[2]})
        print(f"{kind:5s} {str(tuple(key[1:])):42s} x{count:2d} v1 {tb:7.2f} us {base}  v4 {best[0]:7.2f} us {best[1]}"
              f"  ({best[0] / tb:.2f}x)", flush=True)
    print(f"per-step sum: tuned {t1:.0f} us, with the faster variant-4 twins {t4:.0f} us", flush=True)
    if args.json:
        with open(args.json, "w") as fh:
            json.dump({"batch": args.batch, "rows": rows, "sum_v1_us": t1, "sum_best_us": t4}, fh, indent=1)


if __name__ == "__main__":
    main()
