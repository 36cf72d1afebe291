#!/bin/bash
# K1 waves of one SIMD started a fraction of a frame apart (s_sleep 16 / 45 x 64 cycles per step of wave >> 2), so the
# LDS-heavy and VALU-heavy phases of the 4 waves overlap; ABBA bench A/B against the current build (bench.py checks
# the hashes against the oracle).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03u
mkdir -p $O
for v in cur k1st16 k1st45 k1st45 k1st16 cur; do
  n=$(ls $O | grep -c "ab_${v}_" || true)
  if [ $v = cur ]; then
    timeout -k 10 120 python3 bench.py --no-cpu --no-catalog --steps 50 > $O/ab_${v}_$((n+1)).json 2>/dev/null
  else
    AIDFP_LIB=audio-ident_amd/build/$v/libaidfp.so timeout -k 10 120 python3 bench.py --no-cpu --no-catalog --steps 50 > $O/ab_${v}_$((n+1)).json 2>/dev/null
  fi
done
echo done
