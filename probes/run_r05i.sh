#!/bin/bash
# r05i: combinations of the r05h K5 winners (interleaved same-box A/B, probes/k5_path_probe.py): product, maxv4,
# c1 = 8-posting chunks + LDS path up to 2^18 votes, c2 = c1 on four 512-thread workgroups per CU (2^15 counters,
# 1024-entry table), c3 = c2 with 3 windows, c4 = four workgroups with 4-posting chunks.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05i
mkdir -p $O
for i in 1 2; do
for lib in product maxv4 c1 c2 c3 c4; do
  if [ $lib = product ]; then L=""; else L="AIDFP_LIB=$GRAFT_REPO_ROOT/audio-ident_amd/build/$lib/libaidfp.so"; fi
  echo "== $lib $i" >> $O/k5_ab.txt
  env $L timeout -k 10 300 python3 probes/k5_path_probe.py --paths auto --reps 3 >> $O/k5_ab.txt 2>/dev/null || exit 4
done
done
echo done
