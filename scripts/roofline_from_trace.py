"""Recompute bench.py's conv-family roofline from a rocprofv3 kernel trace of the bench command.

    python scripts/roofline_from_trace.py gpurun_out/<tag>_prof/run_kernel_trace.csv [valid_tap_flop_per_step]

A step = the dispatches from one input gather (k_avmnist_gather, one per bench step) to the next; traces without
gathers split at the step-count increment (k_adam_begin) or at k_adam.  Steps whose
kernel count equals the modal count are the graph-replayed training steps; for those it prints the
summed conv-kernel duration per step, the busy time (union of the conv kernels' intervals) and the
resulting fractions of the fp32 MFMA peak, plus the per-family kernel time — the same quantities
bench.py measures in-process with torch.profiler.
"""
import csv
import re
import statistics
import sys
from collections import Counter, defaultdict

CONV = re.compile(r"\bk_(fwd_lds|fwd_pair_lds|bwd_lds|bwd_quad_lds|dgrad_lds|wgrad_lds|fwd_x9|fwd_pair_x9|bwd_x9|bwd_quad_x9|dgrad_x9|wgrad_x9|conv_fwd_vec|conv_fwd_gather|conv_dgrad|conv_wgrad|"
                  r"conv_wgrad_t|reduce_slabs|reduce_slabs_wide)\b")
PEAK = 157.3
FLOPS = 82030559232  # valid-tap FLOPs of the conv launches of one batch-128 step (bench.py line)


def family(name):
    if CONV.search(name):
        return "conv"
    if "k_bn_" in name:
        return "bn"
    if "k_adam" in name:
        return "adam"
    if "pool" in name:
        return "pool"
    return "other"


def union(iv):
    tot, end = 0, None
    for a, b in sorted(iv):
        if end is None or a >= end:
            tot += b - a
            end = b
        elif b > end:
            tot += b - end
            end = b
    return tot


def main(path, flops=FLOPS):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    steps, cur = [], []
    if any("k_avmnist_gather" in n for _, _, n in rows):  # bench steps start at the input gather (round 5: the Adam
        for a, b, n in rows:                               # step count is advanced inside the head's launch)
            if "k_avmnist_gather" in n and cur:
                steps.append(cur)
                cur = []
            cur.append((a, b, n))
    else:
        mark = "k_adam_begin(" if any("k_adam_begin(" in n for _, _, n in rows) else "k_adam("
        for a, b, n in rows:
            cur.append((a, b, n))
            if mark in n:
                steps.append(cur)
                cur = []
    mode = Counter(len(s) for s in steps).most_common(1)[0][0]
    good = [s for s in steps if len(s) == mode]
    conv_sum = [sum(b - a for a, b, n in s if CONV.search(n)) / 1e6 for s in good]
    conv_busy = [union([(a, b) for a, b, n in s if CONV.search(n)]) / 1e6 for s in good]
    fam = defaultdict(list)
    for s in good:
        d = defaultdict(float)
        for a, b, n in s:
            d[family(n)] += (b - a) / 1e6
        for k, v in d.items():
            fam[k].append(v)
    cs, cb = statistics.median(conv_sum), statistics.median(conv_busy)
    print(f"steps {len(steps)} ({len(good)} with the modal {mode} kernels)")
    print(f"conv kernel time per step (sum) {cs:.4f} ms -> {flops / (cs * 1e-3) / 1e12:.2f} TF/s, "
          f"frac {flops / (cs * 1e-3) / 1e12 / PEAK:.4f}")
    print(f"conv busy time per step (union) {cb:.4f} ms -> frac {flops / (cb * 1e-3) / 1e12 / PEAK:.4f}")
    print("per-family kernel ms/step (median):", {k: round(statistics.median(v), 4) for k, v in fam.items()})


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else FLOPS)
