"""Where the `__amd_rocclr_copyBuffer` kernels of a bench run sit.

Reads a rocprofv3 kernel trace (csv or csv.gz) of `bench.py`, orders it by start time, cuts it into
steps at the optimizer's `k_adam` launch and prints how many copy kernels fall before the first step
(setup: weight init, corpus upload, graph capture) and inside each step interval.

  python scripts/copy_audit.py profiles/r2_v9_kernel_trace.csv.gz [--json out.json]
"""
from __future__ import annotations

import bisect
import csv
import gzip
import json
import sys


def main() -> None:
    path = sys.argv[1]
    out = sys.argv[sys.argv.index("--json") + 1] if "--json" in sys.argv else None
    fh = gzip.open(path, "rt") if path.endswith(".gz") else open(path)
    rows = sorted(csv.DictReader(fh), key=lambda r: int(r["Start_Timestamp"]))
    adam = [i for i, r in enumerate(rows) if "k_adam(" in r["Kernel_Name"]]
    copies = [i for i, r in enumerate(rows) if "copyBuffer" in r["Kernel_Name"]]
    per = [0] * (len(adam) + 1)
    for i in copies:
        per[bisect.bisect(adam, i)] += 1
    steps_with = [k for k in range(1, len(adam)) if per[k]]
    doc = {"trace": path, "kernels": len(rows), "steps": len(adam), "copy_kernels": len(copies),
           "before_first_step": per[0],
           "inside_step_intervals": {str(k): per[k] for k in steps_with},
           "after_last_step": per[-1],
           "note": "interval k = kernels after the k-th k_adam and up to the (k+1)-th"}
    print(json.dumps(doc, indent=1))
    if out:
        with open(out, "w") as f:
            json.dump(doc, f, indent=1)


if __name__ == "__main__":
    main()
