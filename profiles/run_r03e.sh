#!/bin/bash
# K1 DPP-split store experiment: same-box A/B of the new K1 with non-temporal stores (base), plain stores (k1nt0),
# no power stores (k1nost, timing only) and the previous K1 (k1old).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03e
mkdir -p $O
B=audio-ident_amd/build
for r in 1 2; do
  timeout -k 10 120 python3 bench.py --no-cpu --no-catalog --steps 50 > $O/ab_base_$r.json 2>/dev/null
  AIDFP_LIB=$B/k1nt0/libaidfp.so timeout -k 10 120 python3 bench.py --no-cpu --no-catalog --steps 50 > $O/ab_k1nt0_$r.json 2>/dev/null
  AIDFP_LIB=$B/k1nost/libaidfp.so timeout -k 10 120 python3 bench.py --no-cpu --no-catalog --no-fullband --steps 50 > $O/ab_k1nost_$r.json 2>/dev/null || true
  AIDFP_LIB=$B/k1old/libaidfp.so timeout -k 10 120 python3 bench.py --no-cpu --no-catalog --steps 50 > $O/ab_k1old_$r.json 2>/dev/null
done
echo done
