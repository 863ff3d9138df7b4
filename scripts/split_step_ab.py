"""Whole-step A/B of variant 4 (bf16-piece products): the current tuned table against the same table with every
launch whose variant-4 twin was faster in isolation (scripts/split_ab.py --json) switched to that twin.  Fused
dgrad + wgrad entries switch when both twins exist and their sum is faster.  Paired FusedTrainStep replays, fresh
builds in alternating order (scripts/tune_in_step.py's compare).

    TUNE_BATCH=128 python scripts/split_step_ab.py gpurun_out/r6s1_split_ab.json --out gpurun_out/t4.json
"""
from __future__ import annotations

import argparse
import gc
import json
import os
import statistics
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.dirname(HERE), HERE]
from tspm_amd import engine as E  # noqa: E402
import tune_in_step as T  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("ab_json", nargs="?", default=None)
    ap.add_argument("--table", default=None, help="instead of twins: a tuned table (tune_convs --out) whose entries "
                                                  "for this batch replace the current ones")
    ap.add_argument("--threshold", type=float, default=0.97, help="switch when v4_us <= threshold * v1_us")
    ap.add_argument("--out", required=True)
    ap.add_argument("--pairs", type=int, default=3)
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--steps", type=int, default=30)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    base = dict(E.tuned_table())
    new = dict(base)
    n = 0
    twin = {}
    if a.table:
        for e in json.load(open(a.table))["entries"]:
            k = (e["kind"],) + tuple(e["shape"][:8])
            if k[1] == T.B and base.get(k) != tuple(e["algo"]):
                new[k] = tuple(e["algo"])
                n += 1
    else:
        ab = json.load(open(a.ab_json))
        twin = {(r["kind"],) + tuple(r["shape"][:8]): (r["v1_us"], r["v4_us"], tuple(r["v4_algo"])) for r in ab["rows"]}
    for k, v in (base.items() if twin else ()):
        if k[0] in ("fwd", "dgrad", "wgrad") and k in twin:
            t1, t4, alg = twin[k]
            if t4 <= a.threshold * t1:
                new[k] = alg
                n += 1
        elif k[0] == "bwd":
            kd, kw = ("dgrad",) + k[1:], ("wgrad",) + k[1:]
            if kd in twin and kw in twin:
                (d1, d4, ad), (w1, w4, aw) = twin[kd], twin[kw]
                if d4 + w4 <= a.threshold * (d1 + w1):
                    new[k] = ad + aw
                    n += 1
    print(f"{n} of {len(base)} entries changed", flush=True)
    res = []
    for i in range(a.pairs):
        T.n_pair = [i]
        first, second = (base, new) if i % 2 == 0 else (new, base)
        x = T.build(first, dev)
        y = T.build(second, dev)
        sb, sn = (x, y) if i % 2 == 0 else (y, x)
        med, d = T.paired(sb, sn, a.rounds, a.steps)
        ub = statistics.median(T.time_steps(sb, a.steps) for _ in range(3))
        un = statistics.median(T.time_steps(sn, a.steps) for _ in range(3))
        print(f"pair {i}: new - base median {med:+.2f} us/step  ({sum(x < 0 for x in d)}/{len(d)} faster); "
              f"base {ub:.1f} us, new {un:.1f} us", flush=True)
        res.append({"median_diff_us": med, "rounds": d, "base_us": ub, "new_us": un})
        del x, y, sb, sn
        gc.collect()
        torch.cuda.empty_cache()
    doc = {"batch": T.B, "threshold": a.threshold, "switched": n, "source": a.table or a.ab_json, "pairs": res,
           "changed": [{"kind": k[0], "shape": list(k[1:]), "algo": list(v)} for k, v in new.items() if base.get(k) != v],
           "entries": [{"kind": k[0], "shape": list(k[1:]), "algo": list(v)} for k, v in sorted(new.items())]}
    json.dump(doc, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
