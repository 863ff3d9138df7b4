"""Per-kernel statistics (the rocprofv3 --stats kernel table) from a rocprofv3 rocpd SQLite file.

    python scripts/rocpd_stats.py gpurun_out/prof/run_results.db > profiles/<name>_kernel_stats.csv
"""
import csv
import sqlite3
import statistics
import sys
from collections import defaultdict


def main(path: str) -> None:
    con = sqlite3.connect(path)
    d = defaultdict(list)
    for name, dur in con.execute("select name, duration from kernels"):
        d[name].append(int(dur))
    total = sum(sum(v) for v in d.values())
    w = csv.writer(sys.stdout, quoting=csv.QUOTE_NONNUMERIC)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev"])
    for name, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
        s = sum(v)
        w.writerow([name, len(v), s, s / len(v), round(100.0 * s / total, 4), min(v), max(v),
                    statistics.pstdev(v) if len(v) > 1 else 0.0])


if __name__ == "__main__":
    main(sys.argv[1])
