"""Sweep the register-direct (variant 0) configurations of the two 7x7 stems (Cin = 1: the LDS-staged
kernels need 32-channel chunks, so scripts/tune_convs.py has no candidates for them): forward (with the
BN-statistics epilogue, as the engine launches it) and weight gradient (split-K over up to 256 slabs,
reduced by tspm's slab pass).  Each candidate is checked against the current configuration's output
(max |diff| <= 1e-5 x max |y|) and graph-timed (tune_convs.graph_time).  Prints the best per launch
and writes them as tuned-table entries.

    python scripts/tune_stem.py --batch 128 --out gpurun_out/stem_tuning_b128.json
"""
from __future__ import annotations

import argparse
import itertools
import json
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.dirname(HERE), HERE]
from tspm_amd.engine import tuned_table  # noqa: E402
from tune_convs import Bufs, distinct_ops, graph_time, launcher  # noqa: E402


def candidates(kind):
    for tm, tn, wn, wk in itertools.product((1, 2), (1, 2), (1, 2, 4), (1, 2, 4, 8, 16)):
        if wn * wk > 16:
            continue
        for sp in ((1, 2, 4, 8, 16, 32, 64, 128, 256) if kind == "wgrad" else (1,)):
            yield (tm, tn, wn, wk, sp, 0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    table = tuned_table()
    entries = []
    for key, (s, xs, stem) in distinct_ops(a.batch, dev).items():
        if not stem:
            continue
        kind = key[0]
        b = Bufs(s, True, dev)
        base = tuple(table.get(key[:9], (0, 0, 0, 0, 0, 0)))
        f, out = launcher(kind, s, xs, b, base)
        assert f() == 0
        torch.cuda.synchronize()
        ref = out.clone()
        scale = ref.abs().max().item() or 1.0
        base_us = graph_time(lambda: launcher(kind, s, xs, b, base)[0], a.reps)
        res = []
        for c in candidates(kind):
            t = graph_time(lambda: launcher(kind, s, xs, b, c)[0], a.reps)
            if t is None:
                continue
            if (out - ref).abs().max().item() > 1e-5 * scale:
                print("  mismatch", c, flush=True)
                continue
            res.append((t, c))
        res.sort()
        print(f"{key}: base {base} {base_us:.2f} us; best " +
              ", ".join(f"{c} {t:.2f}" for t, c in res[:5]), flush=True)
        if res and res[0][0] < base_us:
            entries.append({"kind": kind, "shape": list(key[1:]), "algo": list(res[0][1]), "us": round(res[0][0], 2),
                            "base_us": round(base_us, 2), "base_algo": list(base), "count": 1,
                            "candidates": len(res)})
    if a.out:
        os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
        with open(a.out, "w") as fh:
            json.dump({"batch": a.batch, "timing": "hip-graph replay", "entries": entries}, fh, indent=1)


if __name__ == "__main__":
    main()
