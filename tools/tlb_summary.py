#!/usr/bin/env python3
"""Summarise the UTCL1 (address translation) PMC passes of probes/run_r05zv.sh: per plane size and extraction kernel,
the counters summed over the pass's dispatches, the miss rate, and misses per dispatch. Host-side, reads CSVs only.

    python tools/tlb_summary.py gpurun_out/r05zv > profiles/r05zv_tlb.json
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def summarise(root):
    out = {}
    for d in sorted(glob.glob(os.path.join(root, "pmc_*"))):
        if not os.path.isdir(d):
            continue
        rows = os.path.basename(d)[4:]
        files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
        if not files:
            continue
        sums = defaultdict(lambda: defaultdict(float))
        disp = defaultdict(set)
        for f in files:
            with open(f, newline="") as fh:
                for rec in csv.DictReader(fh):
                    k = rec["Kernel_Name"]
                    if "stft_power" not in k and "peak_pick" not in k and "landmark" not in k:
                        continue
                    k = k.split("(")[0].split("<")[0].replace("void ", "").strip()
                    sums[k][rec["Counter_Name"]] += float(rec["Counter_Value"])
                    disp[k].add(rec["Dispatch_Id"])
        per = {}
        for k, c in sums.items():
            req = c.get("TCP_UTCL1_REQUEST_sum", 0.0)
            hit = c.get("TCP_UTCL1_TRANSLATION_HIT_sum", 0.0)
            miss = c.get("TCP_UTCL1_TRANSLATION_MISS_sum", 0.0)
            n = len(disp[k])
            per[k] = {"dispatches": n, "requests": req, "hits": hit, "misses": miss,
                      "miss_rate": round(miss / (hit + miss), 5) if hit + miss else None,
                      "misses_per_request": round(miss / req, 5) if req else None}
        out["plane_rows_" + rows] = per
    return out


if __name__ == "__main__":
    print(json.dumps(summarise(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/r05zv"), indent=1))
