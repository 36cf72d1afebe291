"""Average rocprofv3 counter values per kernel: python profiles/pmc_summary.py <dir>..."""
import collections
import csv
import glob
import sys

for d in sys.argv[1:]:
    agg = collections.defaultdict(list)
    for f in glob.glob(f"{d}/**/run_counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Kernel_Name"].startswith("k_"):
                agg[(r["Kernel_Name"].split("<")[0][:18], r["Counter_Name"])].append(float(r["Counter_Value"]))
    for (k, c), v in sorted(agg.items()):
        print(f"{d:28s} {k:18s} {c:24s} n={len(v):3d} mean={sum(v) / len(v):.4g}")
