#!/bin/bash
# Interleaved same-box A/B of two libaidfp builds on the extraction batch (probes/fullband_probe.py, adaptive strips):
# bash probes/run_ab_lib.sh OUT VARIANT ROUNDS  (VARIANT = audio-ident_amd/build/<VARIANT>/libaidfp.so)
set -o pipefail
OUT=$1; V=$2; N=${3:-3}
mkdir -p $(dirname $OUT)
cd $GRAFT_REPO_ROOT
for i in $(seq $N); do
  for lib in product $V; do
    if [ $lib = product ]; then L=""; else L="AIDFP_LIB=$GRAFT_REPO_ROOT/audio-ident_amd/build/$lib/libaidfp.so"; fi
    echo "== $lib $i" >> $OUT
    env $L timeout -k 10 200 python3 probes/fullband_probe.py 0 >> $OUT 2>/dev/null || exit 3
  done
done
echo ok
