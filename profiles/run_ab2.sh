#!/bin/bash
# Interleaved same-box A/B: R rounds over the variant list (main = in-tree lib), bench.py --no-cpu each.
# usage: bash profiles/run_ab2.sh R v1 v2 ...
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/ab
R=$1; shift
for r in $(seq 1 $R); do
  for v in "$@"; do
    LIBP=audio-ident_amd/aidfp/libaidfp.so; [ "$v" != main ] && LIBP=audio-ident_amd/build/$v/libaidfp.so
    AIDFP_LIB=$PWD/$LIBP timeout -k 10 120 python3 bench.py --steps 30 --warmup 3 --no-cpu --no-catalog > gpurun_out/ab/${v}_$r.log 2>&1 || exit 1
  done
done
python3 - "$R" "$@" <<'PY'
import json, sys
R = int(sys.argv[1])
for v in sys.argv[2:]:
    rows = []
    for r in range(1, R + 1):
        d = json.loads(open(f"gpurun_out/ab/{v}_{r}.log").read().strip().splitlines()[-1])
        fb = (d.get("fullband") or {}).get("kernels", {})
        rows.append((d["value"], *(d["kernels"][k]["ms_per_launch"] for k in ("stft_power", "peak_pick", "landmark_write")),
                     fb.get("peak_pick", 0.0)))
    print(v, " | ".join("%.0f K1 %.4f K2 %.4f K3 %.4f fbK2 %.4f" % x for x in rows))
PY
