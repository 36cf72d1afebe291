#!/usr/bin/env python3
"""Summarise PMC passes of k1_shape_probe.py runs by K1 -> K2 plane bound (probes/run_r05zy.sh): every counter summed
over a kernel's dispatches and divided by the probe's extraction calls (its timed launches + 1 warm-up call, read from
the pass's stdout), so bounds that split a call into different numbers of groups compare per call. Host-side only.

    python tools/pmc_by_plane.py gpurun_out/r05zy > profiles/r05zy_plane_pmc.json
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
        tag = os.path.basename(d)[4:]
        with open(d + ".out") as fh:
            calls = sum(json.loads(l)["launches"] + 1 for l in fh if l.startswith("{"))
        sums = defaultdict(lambda: defaultdict(float))
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f, newline="") as fh:
                for rec in csv.DictReader(fh):
                    k = rec["Kernel_Name"].split("(")[0].split("<")[0].replace("void ", "").strip()
                    if k.split("::")[-1] not in ("k_stft_power", "k_peak_pick"):
                        continue
                    sums[k][rec["Counter_Name"]] += float(rec["Counter_Value"])
        out[tag] = {"calls": calls, "per_call": {k: {n: round(v / calls, 1) for n, v in c.items()}
                                                  for k, c in sums.items()}}
    return out


if __name__ == "__main__":
    print(json.dumps(summarise(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/r05zy"), indent=1))
