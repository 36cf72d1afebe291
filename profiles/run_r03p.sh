#!/bin/bash
# LLVM scheduler strategies (-mllvm -amdgpu-sched-strategy=...) for stft.hip (K1) or peaks.hip (K2) alone,
# same-box A/B against the product build, order reversed in the second round. bench.py checks every clip's
# hashes against the C oracle bit for bit (parity field).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03p
mkdir -p $O
V="cur k1_max-ilp k1_max-memory-clause k1_iterative-ilp k2_max-ilp k2_iterative-ilp"
R=$(echo $V | tr ' ' '\n' | tac | tr '\n' ' ')
for r in 1 2; do
  L=$V; [ $r = 2 ] && L=$R
  for v in $L; do
    if [ $v = cur ]; then
      timeout -k 10 120 python3 bench.py --no-cpu --no-catalog --steps 50 > $O/ab_${v}_$r.json 2>/dev/null
    else
      AIDFP_LIB=audio-ident_amd/build/$v/libaidfp.so timeout -k 10 120 python3 bench.py --no-cpu --no-catalog --steps 50 > $O/ab_${v}_$r.json 2>/dev/null
    fi
  done
done
echo done
