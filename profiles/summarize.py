"""Summarise a rocprofv3 round: kernel_stats (trace pass) + FETCH_SIZE/WRITE_SIZE (separate PMC
passes) -> profiles/pmc_<tag>.json with HBM bytes per launch per kernel.

usage: python profiles/summarize.py <tag> <prof_dir>   (prof_dir = gpurun_out/prof_<tag>)

gfx950 correction (MI355X_MICROARCH.md, HBM section): FETCH_SIZE reports half the bytes
of a wide coalesced streaming read, so hbm_read = 2 x FETCH_SIZE x 1 KiB; WRITE_SIZE
(KiB) is exact for 16-B/lane stores. Both raw values are kept next to the corrected sum.
"""
import csv
import collections
import json
import sys
from pathlib import Path

NAMES = {"k_stft_power": "stft_power", "k_peak_pick": "peak_pick", "k_landmarks": "landmarks",
         "k_vote_hist": "vote_hist", "k_vote_final": "vote_final", "k_synth": "synth",
         "k_index_count": "index_count", "k_index_scatter": "index_scatter", "k_downmix": "downmix"}


def short(name):
    base = name.split("<")[0].split("(")[0].strip()
    return NAMES.get(base, base)


def counters(path, counter):
    agg = collections.defaultdict(list)
    for f in Path(path).glob("**/run_counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter:
                agg[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in agg.items()}


def main():
    tag, d = sys.argv[1], Path(sys.argv[2])
    stats = {}
    for f in (d / "trace").glob("**/run_kernel_stats.csv"):
        for r in csv.DictReader(open(f)):
            stats[short(r["Name"])] = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]),
                                       "pct": float(r["Percentage"])}
    fetch = counters(d / "fetch", "FETCH_SIZE")
    write = counters(d / "write", "WRITE_SIZE")
    out = {"tag": tag, "source": str(d), "correction": "hbm_bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950)",
           "kernels": {}}
    for k in sorted(set(stats) | set(fetch) | set(write)):
        e = dict(stats.get(k, {}))
        if k in fetch:
            e["fetch_kib_raw"] = fetch[k]
        if k in write:
            e["write_kib_raw"] = write[k]
        if k in fetch and k in write:
            e["hbm_bytes_per_launch"] = (2 * fetch[k] + write[k]) * 1024
        out["kernels"][k] = e
    Path(f"profiles/pmc_{tag}.json").write_text(json.dumps(out, indent=1))
    ks = d / "trace"
    for f in ks.glob("**/run_kernel_stats.csv"):
        Path(f"profiles/{tag}_kernel_stats.csv").write_text(f.read_text())
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
