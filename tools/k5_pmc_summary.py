"""Summarise the config-4 match kernels (K5) from one rocprofv3 run of bench.py's catalog leg into the committed file
bench.py reads (load_pmc_k5):

    python tools/k5_pmc_summary.py TAG RUNDIR
      RUNDIR/trace/run_kernel_trace.csv, RUNDIR/trace/run_kernel_stats.csv  (rocprofv3 --kernel-trace --stats)
      RUNDIR/fetch/run_counter_collection.csv                              (--pmc FETCH_SIZE)
      RUNDIR/write/run_counter_collection.csv                              (--pmc WRITE_SIZE)
    -> profiles/pmc_TAG_k5.json, profiles/TAG_k5_kernel_stats.csv

Only the full exact-lane calls are summarised: the dispatches whose grid is the largest one seen for k_match_lds
(4096 clips x 3 sub-windows = 12288 workgroups, one per query). Per call: each K5 kernel's mean duration (trace)
and its FETCH_SIZE / WRITE_SIZE bytes (raw counter values x 1 KiB; FETCH_SIZE counts the L2's fabric-side read
requests, Infinity-Cache hits included, so it bounds the HBM reads from above). `fetch_factor` converts FETCH_SIZE to
bytes for the kernel's access width: 2 for 16-B-per-lane streaming reads (MI355X_MICROARCH.md, HBM), and the value
the probes/fetch_calib.hip calibration measured (RUNDIR/calib.json, else profiles/fetch_calib_r05b.json: 2 for 4-,
8- and 16-B-per-lane reads).
"""
import csv
import json
import shutil
import sys
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
K5 = ("k_query_votes", "k_match_lds", "k_vote_hist", "k_hot_scan", "k_vote_final", "k_exact_consensus")


def short(name: str) -> str:
    return name.split("(")[0].split("<")[0].split()[-1].split("::")[-1]


def main() -> None:
    tag, run = sys.argv[1], Path(sys.argv[2])
    trace = list(csv.DictReader(open(run / "trace" / "run_kernel_trace.csv", newline="")))
    lds = [(int(r["Grid_Size_X"]), int(r["Workgroup_Size_X"])) for r in trace if short(r["Kernel_Name"]) == "k_match_lds"]
    if not lds:
        raise SystemExit("no k_match_lds dispatch in the trace")
    g_lds, wg = max(lds)
    queries = g_lds // wg  # one workgroup per query
    # the other kernels of a full lane call, by their grid for that many queries
    full_grid = {"k_match_lds": g_lds, "k_query_votes": queries * 256, "k_exact_consensus": None}
    dur = defaultdict(list)
    for r in trace:
        k = short(r["Kernel_Name"])
        if k in full_grid and (full_grid[k] is None or int(r["Grid_Size_X"]) == full_grid[k]):
            dur[k].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    # k_exact_consensus of the full calls: the largest grid seen
    cons = [int(r["Grid_Size_X"]) for r in trace if short(r["Kernel_Name"]) == "k_exact_consensus"]
    if cons:
        g = max(cons)
        dur["k_exact_consensus"] = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in trace
                                    if short(r["Kernel_Name"]) == "k_exact_consensus" and int(r["Grid_Size_X"]) == g]
        full_grid["k_exact_consensus"] = g
    ctr = defaultdict(list)
    for pas, cname in (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE")):
        for r in csv.DictReader(open(run / pas / "run_counter_collection.csv", newline="")):
            k = short(r["Kernel_Name"])
            if k in full_grid and int(r["Grid_Size"]) == full_grid[k] and r["Counter_Name"] == cname:
                ctr[(k, cname)].append(float(r["Counter_Value"]) * 1024.0)
    calib = None
    for c in (run / "calib.json", ROOT / "profiles" / "fetch_calib_r05b.json"):
        if c.exists():
            calib = json.loads(c.read_text())
            break
    f8 = float(calib["fetch_factor_8B"]) if calib else None
    kernels = {}
    for k in full_grid:
        if not dur.get(k):
            continue
        fe = ctr.get((k, "FETCH_SIZE"), [])
        wr = ctr.get((k, "WRITE_SIZE"), [])
        kernels[k] = {"calls": len(dur[k]), "avg_ns": sum(dur[k]) / len(dur[k]),
                      "fetch_bytes_raw": sum(fe) / len(fe) if fe else None,
                      "write_bytes": sum(wr) / len(wr) if wr else None}
    fetch_raw = sum(v["fetch_bytes_raw"] or 0.0 for v in kernels.values())
    write = sum(v["write_bytes"] or 0.0 for v in kernels.values())
    ms = sum(v["avg_ns"] for v in kernels.values()) * 1e-6
    k5 = {"queries_per_call": queries, "kernels": kernels, "k5_ms_per_call": ms,
          "fetch_bytes_raw_per_call": fetch_raw, "write_bytes_per_call": write,
          "fetch_factor_8B": f8, "calibration": calib,
          "hbm_bytes_per_call": (f8 * fetch_raw + write) if f8 else None,
          "note": "per full 4096-clip exact-lane call (12288 sub-window queries); FETCH_SIZE counts L2 fabric-side "
                  "read requests (Infinity-Cache hits included); hbm_bytes_per_call = fetch_factor_8B x FETCH + "
                  "WRITE, with the factor calibrated for K5's 8-B-per-lane posting reads (probes/fetch_calib.hip)"}
    out = {"tag": tag, "source": str(run.relative_to(ROOT)) if run.is_absolute() else str(run), "k5": k5}
    (ROOT / "profiles" / f"pmc_{tag}_k5.json").write_text(json.dumps(out, indent=1) + "\n")
    stats = run / "trace" / "run_kernel_stats.csv"
    if stats.exists():
        shutil.copy(stats, ROOT / "profiles" / f"{tag}_k5_kernel_stats.csv")
    print(json.dumps(k5, indent=1))


if __name__ == "__main__":
    main()
