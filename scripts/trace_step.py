"""Print one step of a rocprofv3 kernel trace (the dispatches from one input gather, k_avmnist_gather, to the next;
between k_adam_begin launches when the trace has no gather) as
index / start offset / duration / kernel / grid, plus per-kernel-name totals.
    python scripts/trace_step.py gpurun_out/<tag>_serial/run_kernel_trace.csv [step index, default -2]"""
import csv
import re
import sys
from collections import defaultdict


def main(path, k=-2):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    # a step starts at the bench's input gather (one per step); the optimizer launches k_adam once per flat-buffer
    # range (several per step, on two streams), so k_adam does not mark step ends
    mark = "k_avmnist_gather" if any("k_avmnist_gather" in r["Kernel_Name"] for r in rows) else "k_adam_begin"
    steps, cur = [], []
    for r in rows:
        if mark in r["Kernel_Name"] and cur:
            steps.append(cur)
            cur = []
        cur.append(r)
    st = steps[k]
    t0 = int(st[0]["Start_Timestamp"])
    tot = defaultdict(lambda: [0, 0.0])
    for i, r in enumerate(st):
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        m = re.search(r"(k_\w+)", r["Kernel_Name"])
        nm = m.group(1) if m else r["Kernel_Name"][:30]
        tot[nm][0] += 1
        tot[nm][1] += (e - s) / 1e3
        print(f"{i:3d} {(s - t0) / 1e3:8.1f} {(e - s) / 1e3:6.1f} {nm:24s} g={r['Grid_Size_X']}/{r['Workgroup_Size_X']}")
    print("kernels", len(st), "sum_us", round(sum(v[1] for v in tot.values()), 1),
          "span_us", (int(st[-1]["End_Timestamp"]) - t0) / 1e3)
    for nm, (n, us) in sorted(tot.items(), key=lambda kv: -kv[1][1]):
        print(f"  {nm:24s} {n:4d} {us:8.1f}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else -2)
