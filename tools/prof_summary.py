"""Summarise one round's rocprofv3 passes (profiles/run_rocprof.sh TAG, profiles/run_sq.sh TAG) into the committed
files bench.py reads:

    python tools/prof_summary.py TAG
      gpurun_out/prof_TAG/trace/run_kernel_stats.csv  -> profiles/TAG_kernel_stats.csv (copied)
      gpurun_out/prof_TAG/{fetch,write}/run_counter_collection.csv
                                                      -> profiles/pmc_TAG.json (per kernel: calls and avg_ns from the
                                                         trace, mean FETCH_SIZE / WRITE_SIZE per dispatch in KiB, and
                                                         hbm_bytes_per_launch = (2 FETCH_SIZE + WRITE_SIZE) x 1024,
                                                         the gfx950 correction of MI355X_MICROARCH.md)
      gpurun_out/sq_TAG/p*/run_counter_collection.csv -> profiles/sq_TAG.txt (mean of each SQ counter per dispatch)
"""
import csv
import json
import shutil
import sys
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def short(name: str) -> str:
    """'void aid::k_stft_power<false, 4>(...)' -> 'stft_power'; library kernels keep their names."""
    n = name.split("(")[0].split("<")[0].split()[-1]
    n = n.split("::")[-1]
    return n[2:] if n.startswith("k_") else n


def counter_means(path: Path) -> dict:
    acc = defaultdict(lambda: defaultdict(list))
    with open(path, newline="") as f:
        for row in csv.DictReader(f):
            acc[short(row["Kernel_Name"])][row["Counter_Name"]].append(float(row["Counter_Value"]))
    return {k: {c: (sum(v) / len(v), len(v)) for c, v in cs.items()} for k, cs in acc.items()}


def main():
    tag = sys.argv[1]
    prof = ROOT / "gpurun_out" / f"prof_{tag}"
    stats = prof / "trace" / "run_kernel_stats.csv"
    trace = {}
    if stats.exists():
        shutil.copy(stats, ROOT / "profiles" / f"{tag}_kernel_stats.csv")
        with open(stats, newline="") as f:
            for row in csv.DictReader(f):
                trace[short(row["Name"])] = (int(row["Calls"]), float(row["AverageNs"]), float(row["Percentage"]))
    fetch = counter_means(prof / "fetch" / "run_counter_collection.csv")
    write = counter_means(prof / "write" / "run_counter_collection.csv")
    kernels = {}
    for k in sorted(set(fetch) | set(write)):
        fk = fetch.get(k, {}).get("FETCH_SIZE", (0.0, 0))[0]
        wk = write.get(k, {}).get("WRITE_SIZE", (0.0, 0))[0]
        calls, avg, pct = trace.get(k, (0, None, None))
        kernels[k] = {"calls": calls, "avg_ns": avg, "pct": pct, "fetch_kib_raw": fk, "write_kib_raw": wk,
                      "hbm_bytes_per_launch": (2 * fk + wk) * 1024}
    out = {"tag": tag, "source": f"gpurun_out/prof_{tag}",
           "correction": "hbm_bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950)", "kernels": kernels}
    (ROOT / "profiles" / f"pmc_{tag}.json").write_text(json.dumps(out, indent=1) + "\n")
    lines = []
    for p in sorted((ROOT / "gpurun_out" / f"sq_{tag}").glob("p*/run_counter_collection.csv")):
        d = p.parent.relative_to(ROOT)
        for k, cs in sorted(counter_means(p).items()):
            if not k.startswith("__amd"):
                for c, (m, n) in sorted(cs.items()):
                    lines.append(f"{str(d):28s} k_{k:16s} {c:24s} n={n:3d} mean={m:.4g}")
    if lines:
        (ROOT / "profiles" / f"sq_{tag}.txt").write_text("\n".join(lines) + "\n")
    print(json.dumps({k: round(v["hbm_bytes_per_launch"] / 1e6, 1) for k, v in kernels.items()}))


if __name__ == "__main__":
    main()
