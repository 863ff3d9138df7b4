"""Summarise one graph-replayed train step from a rocprofv3 kernel trace.

    python scripts/trace_summary.py gpurun_out/prof/run_kernel_trace.csv|run_results.db [--step -3]

A step is delimited by consecutive `k_adam<...>` launches (Adam ends every step).  Prints the step's
wall time, summed kernel time, busy time (union of kernel intervals, i.e. with concurrency folded),
per-queue busy time, and the top kernels by summed duration inside that step.
"""
from __future__ import annotations

import argparse
import collections
import csv


def short(name: str) -> str:
    name = name.replace("(anonymous namespace)::", "").replace("void ", "")
    return name.split("(")[0][:70]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--step", type=int, default=-3, help="which step (index into the list of Adam-delimited steps)")
    ap.add_argument("--top", type=int, default=25)
    args = ap.parse_args()
    if args.trace.endswith(".db"):  # rocprofv3 rocpd SQLite output (the default format)
        import sqlite3
        con = sqlite3.connect(args.trace)
        ks = sorted((int(s), int(e), n, str(q)) for s, e, n, q in con.execute("select start, end, name, queue_id from kernels"))
    else:
        rows = list(csv.DictReader(open(args.trace)))
        ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r["Queue_Id"]) for r in rows))
    adam = [i for i, k in enumerate(ks) if "k_adam<" in k[2] or "k_adam(" in k[2] or k[2].startswith("void k_adam")
            and "begin" not in k[2]]
    if len(adam) < 2:
        adam = [i for i, k in enumerate(ks) if "adam" in k[2] and "begin" not in k[2]]
    lo, hi = adam[args.step - 1], adam[args.step]
    step = ks[lo + 1:hi + 1]
    t0, t1 = step[0][0], step[-1][1]
    wall = (t1 - t0) / 1e3
    ksum = sum(e - s for s, e, _, _ in step) / 1e3
    busy = 0
    cur_s, cur_e = None, None
    for s, e, _, _ in step:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    print(f"step kernels {len(step)}  wall {wall:.1f} us  kernel-sum {ksum:.1f} us  busy(union) {busy / 1e3:.1f} us  "
          f"concurrency {ksum / max(busy / 1e3, 1e-9):.2f}")
    q = collections.defaultdict(float)
    for s, e, _, qid in step:
        q[qid] += (e - s) / 1e3
    print("per-queue kernel time:", {k: round(v, 1) for k, v in sorted(q.items())})
    agg = collections.defaultdict(lambda: [0.0, 0])
    for s, e, n, _ in step:
        a = agg[short(n)]
        a[0] += (e - s) / 1e3
        a[1] += 1
    for n, (t, c) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:args.top]:
        print(f"{t:8.1f} us  x{c:3d}  avg {t / c:6.1f}  {n}")


if __name__ == "__main__":
    main()
