"""L2 hit rate per kernel family and step from one rocprofv3 pass `--pmc TCC_HIT_sum TCC_MISS_sum` over
a short bench run (same step cut as scripts/pmc_traffic.py: dispatches between consecutive k_adam
launches, median over complete steps).  Supports DESIGN §0 item 4 (where the conv family's re-reads go).

  python scripts/pmc_l2.py gpurun_out/r3_l2 > profiles/r3_l2_hit.json
"""
import csv
import json
import os
import statistics
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_traffic import family, steps  # noqa: E402


def load(d: str, counter: str):
    rows = []
    with open(os.path.join(d, "run_counter_collection.csv")) as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] == counter:
                rows.append((int(r["Dispatch_Id"]), r["Kernel_Name"], float(r["Counter_Value"])))
    rows.sort()
    return rows


def main(d: str) -> None:
    out = {"method": "rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum (one pass) over `bench.py --steps 3 --warmup 2 "
                     "--no-cpu-baseline --profile-steps 0 --pcie-steps 0`; per step = dispatches between consecutive "
                     "k_adam launches; median over complete steps; requests, not bytes", "per_step": {}}
    per = {}
    for c in ("TCC_HIT_sum", "TCC_MISS_sum"):
        res = []
        for st in steps(load(d, c)):
            fam = defaultdict(float)
            for name, v in st:
                fam[family(name)] += v
            res.append(fam)
        per[c] = res
    fams = sorted({f for s in per["TCC_HIT_sum"] for f in s})
    for f in fams:
        h = statistics.median([s.get(f, 0.0) for s in per["TCC_HIT_sum"]])
        m = statistics.median([s.get(f, 0.0) for s in per["TCC_MISS_sum"]])
        out["per_step"][f] = {"hits": h, "misses": m, "hit_rate": round(h / (h + m), 4) if h + m else None}
    out["steps"] = len(per["TCC_HIT_sum"])
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
