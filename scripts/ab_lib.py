"""A/B of two builds of libtspm.so on the same box: alternating bench.py processes (fresh process per run, so
each loads its own library via TSPM_LIB), same arguments, medians reported.  Library A/B is how kernel build
switches (launch bounds, loop structure) are measured in the captured step; results stay bitwise comparable
only where the switch does not change the arithmetic (checked by the caller's tests).

    python scripts/ab_lib.py --rounds 3 -- --batch-per-rank 128 --steps 100
    (A = task-specific-pretraining-multimodal_amd/libtspm.so, B = .../libtspm_alt.so)
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
PKG = os.path.join(REPO, "task-specific-pretraining-multimodal_amd")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--a", default=os.path.join(PKG, "libtspm.so"))
    ap.add_argument("--b", default=os.path.join(PKG, "libtspm_alt.so"))
    ap.add_argument("--env-b", default="", help="extra KEY=VAL,... for the B runs")
    ap.add_argument("rest", nargs=argparse.REMAINDER)
    a = ap.parse_args()
    rest = a.rest[1:] if a.rest and a.rest[0] == "--" else a.rest
    base = ["--no-cpu-baseline", "--pcie-steps", "0", "--exchange-steps", "0"]
    res = {"A": [], "B": []}
    lines = {"A": None, "B": None}
    for r in range(a.rounds):
        for side in (("A", "B") if r % 2 == 0 else ("B", "A")):
            env = dict(os.environ, TSPM_LIB=a.a if side == "A" else a.b)
            if side == "B" and a.env_b:
                env.update(kv.split("=", 1) for kv in a.env_b.split(","))
            p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + base + rest, env=env,
                               capture_output=True, text=True, timeout=400)
            if p.returncode != 0:
                print(p.stderr[-3000:], file=sys.stderr)
                raise SystemExit(f"{side} run failed ({p.returncode})")
            d = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
            res[side].append(d["ms_per_step"])
            lines[side] = d
            print(f"round {r} {side}: {d['ms_per_step']:.4f} ms/step, conv frac {d['roofline'].get('frac')}", file=sys.stderr,
                  flush=True)
    out = {"args": rest, "a": a.a, "b": a.b, "env_b": a.env_b,
           "ms_per_step": {k: {"median": sorted(v)[len(v) // 2], "all": v} for k, v in res.items()},
           "conv": {k: {f: lines[k]["roofline"].get(f) for f in ("frac", "conv_ms_per_step", "kernel_ms_per_step_by_family")}
                    for k in lines},
           "r34_3x3": {k: (lines[k]["roofline"].get("r34_3x3") or {}).get("frac") for k in lines}}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
