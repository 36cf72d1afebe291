#!/bin/bash
# K1 phase ablations (timing-only builds, wrong results): bench K1 time per variant.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/ablate
for v in 0 6 7 8 9 10 11; do
  LIBP=audio-ident_amd/aidfp/libaidfp.so; [ $v != 0 ] && LIBP=audio-ident_amd/build/diag$v/libaidfp.so
  AIDFP_LIB=$PWD/$LIBP timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/ablate/b$v.log 2>&1 || exit 1
done
