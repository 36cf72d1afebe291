#!/bin/bash
# K5a A/B: the seen-filter LDS atomic only on lanes whose vote belongs to the workgroup's key partition (exec-masked)
# instead of an atomicOr with mask 0 on the others. Exact lane (config 4) timed by bench.py's exact-lane leg.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03ak
mkdir -p $O
for r in 1 2 3; do
  for v in main k5or; do
    LIBP=audio-ident_amd/aidfp/libaidfp.so; [ "$v" != main ] && LIBP=audio-ident_amd/build/$v/libaidfp.so
    AIDFP_LIB=$PWD/$LIBP timeout -k 10 200 python3 bench.py --no-cpu --no-fullband --steps 5 --exact-clips 16384 > $O/${v}_$r.json 2> $O/${v}_$r.err
  done
done
python3 - <<'PY'
import json
for v in ("main", "k5or"):
    rows = []
    for r in (1, 2, 3):
        d = json.loads(open(f"gpurun_out/r03ak/{v}_{r}.json").read().strip().splitlines()[-1])
        e = d["catalog"]["exact_lane"]
        rows.append("%.0f clips/s (%.4f s, top1 %.4f, fpr %.4f)" % (e["value"], e["gpu_s_max_over_ranks"], e["rank0"]["top1"], e["rank0"]["false_positive_rate"]))
    print(v, " | ".join(rows))
PY
echo done
