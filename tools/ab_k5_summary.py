"""Summarise a probes/run_ab_k5.sh output file: per build and round, clips/s, K5 ms and K5 frac of the auto path."""
import json
import sys

cur = None
for line in open(sys.argv[1]):
    if line.startswith("=="):
        cur = line.strip("= \n")
        continue
    try:
        d = json.loads(line)
    except ValueError:
        continue
    if "tracks" in d and "auto" in d:
        v = d["auto"]
        print(f"{cur:12s} {v['clips_per_s']:>10} clips/s  K5 {v['k5_ms']} ms  frac {v['k5_frac']}  {v['s']}")
