#!/bin/bash
# Interleaved same-box A/B of two libaidfp builds on the config-4 exact lane (probes/k5_path_probe.py, auto path):
# bash probes/run_ab_k5.sh OUT VARIANT ROUNDS  (VARIANT = audio-ident_amd/build/<VARIANT>/libaidfp.so)
set -o pipefail
OUT=$1; V=$2; N=${3:-2}
mkdir -p $(dirname $OUT)
cd $GRAFT_REPO_ROOT
for i in $(seq $N); do
  for lib in product $V; do
    if [ $lib = product ]; then L=""; else L="AIDFP_LIB=$GRAFT_REPO_ROOT/audio-ident_amd/build/$lib/libaidfp.so"; fi
    echo "== $lib $i" >> $OUT
    env $L timeout -k 10 300 python3 probes/k5_path_probe.py --paths auto --reps 3 >> $OUT 2>/dev/null || exit 3
  done
done
echo ok
