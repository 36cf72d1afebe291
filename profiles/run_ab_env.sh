#!/bin/bash
# Interleaved same-box A/B over environment settings of the in-tree lib, bench.py --no-cpu each.
# usage: bash profiles/run_ab_env.sh R "VAR=a" "VAR=b" ...   ("-" = no extra env)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/abenv
R=$1; shift
for r in $(seq 1 $R); do
  i=0
  for v in "$@"; do
    i=$((i+1))
    if [ "$v" = "-" ]; then timeout -k 10 120 python3 bench.py --steps 30 --warmup 3 --no-cpu > gpurun_out/abenv/${i}_$r.log 2>&1 || exit 1
    else env $v timeout -k 10 120 python3 bench.py --steps 30 --warmup 3 --no-cpu > gpurun_out/abenv/${i}_$r.log 2>&1 || exit 1; fi
  done
done
python3 - "$R" "$@" <<'PY'
import json, sys
R = int(sys.argv[1])
for i, v in enumerate(sys.argv[2:], 1):
    rows = []
    for r in range(1, R + 1):
        d = json.loads(open(f"gpurun_out/abenv/{i}_{r}.log").read().strip().splitlines()[-1])
        k = d["kernels"]
        rows.append("%.0f step %.4f K1 %.4fx%d K2 %.4fx%d" % (d["value"], d["ms_per_step"], k["stft_power"]["ms_per_launch"],
                    k["stft_power"]["launches"], k["peak_pick"]["ms_per_launch"], k["peak_pick"]["launches"]))
    print(v, " | ".join(rows))
PY
