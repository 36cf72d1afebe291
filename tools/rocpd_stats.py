#!/usr/bin/env python3
"""Per-kernel summary of a rocprofv3 --kernel-trace database (rocpd sqlite: *_results.db), in the column layout of
rocprofv3's kernel_stats.csv (Name, Calls, TotalDurationNs, AverageNs, Percentage, MinNs, MaxNs).

    python tools/rocpd_stats.py gpurun_out/<run>/<dir>/<name>_results.db > profiles/<tag>_kernel_stats.csv"""
import csv
import sqlite3
import sys
from collections import defaultdict


def main(path: str) -> None:
    c = sqlite3.connect(path)
    names = {kid: name for kid, name in c.execute("select id, kernel_name from rocpd_info_kernel_symbol")}
    d = defaultdict(list)
    for kid, start, end in c.execute("select kernel_id, start, end from rocpd_kernel_dispatch"):
        d[names.get(kid, str(kid))].append(end - start)
    total = sum(sum(v) for v in d.values()) or 1
    w = csv.writer(sys.stdout)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
    for name, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
        w.writerow([name, len(v), sum(v), round(sum(v) / len(v), 3), round(100.0 * sum(v) / total, 4), min(v), max(v)])


if __name__ == "__main__":
    main(sys.argv[1])
