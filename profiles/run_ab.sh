#!/bin/bash
# A/B timing of diagnostic builds: bench.py per library variant (arg list: variant names; "main" = in-tree lib)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/ab
for v in "$@"; do
  LIBP=audio-ident_amd/aidfp/libaidfp.so; [ "$v" != main ] && LIBP=audio-ident_amd/build/$v/libaidfp.so
  AIDFP_LIB=$PWD/$LIBP timeout -k 10 200 python3 bench.py --steps 30 --warmup 3 --no-cpu > gpurun_out/ab/$v.log 2>&1 || exit 1
done
