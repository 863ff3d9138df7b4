"""Summarise bench lines written by scripts/gpu_r3_abn.sh: python scripts/ab_summary.py gpurun_out/<tag>"""
import glob
import json
import sys
from collections import defaultdict

rows = defaultdict(list)
for f in sorted(glob.glob(sys.argv[1] + "_*_[0-9].json")):
    name = f[len(sys.argv[1]) + 1:].rsplit("_", 1)[0]
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception as e:  # noqa: BLE001
        print(f, "unreadable", e)
        continue
    r = d["roofline"]
    rows[name].append((d["ms_per_step"], r["frac"], r["r34_3x3"]["frac"], r["kernel_ms_per_step_by_family"]["conv"],
                       r["kernel_ms_per_step_by_family"]["bn"]))
for n, v in rows.items():
    print(f"{n:10s} ms/step {[x[0] for x in v]}  conv-frac {[x[1] for x in v]}  r34 {[x[2] for x in v]}  "
          f"conv-ms {[x[3] for x in v]}  bn-ms {[x[4] for x in v]}")
