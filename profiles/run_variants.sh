#!/bin/bash
# Screen diagnostic builds: smoke (hashes bit-exact vs the oracle) with each variant's library, then an
# interleaved same-box A/B (run_ab2.sh). usage: bash profiles/run_variants.sh R v1 v2 ... (main = in-tree lib)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/ab
R=$1; shift
for v in "$@"; do
  LIBP=audio-ident_amd/aidfp/libaidfp.so; [ "$v" != main ] && LIBP=audio-ident_amd/build/$v/libaidfp.so
  AIDFP_LIB=$PWD/$LIBP timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/ab/smoke_$v.log 2>&1 \
    || { echo "variant $v: smoke FAILED"; tail -5 gpurun_out/ab/smoke_$v.log; exit 1; }
  echo "variant $v: $(grep 'smoke ok' gpurun_out/ab/smoke_$v.log)"
done
bash profiles/run_ab2.sh "$R" "$@"
