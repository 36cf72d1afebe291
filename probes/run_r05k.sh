#!/bin/bash
# r05k: K1/K2 overlap probe (VERDICT r4 next #5 option (a)): one engine on one stream vs two engines on two streams,
# with the product K1 (16 waves, all the LDS) and the 12-wave K1 build (room for one K2 workgroup beside it).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05k
mkdir -p $O
for i in 1 2; do
for lib in product k1w12; do
  if [ $lib = product ]; then L=""; else L="AIDFP_LIB=$GRAFT_REPO_ROOT/audio-ident_amd/build/$lib/libaidfp.so"; fi
  echo "== $lib $i" >> $O/dual.txt
  env $L timeout -k 10 200 python3 probes/dual_stream_probe.py >> $O/dual.txt 2>> $O/dual.err || exit 4
done
done
echo done
