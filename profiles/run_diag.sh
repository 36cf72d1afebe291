#!/bin/bash
# LDS-conflict attribution for K1 diagnostic variants (timing-only builds). usage: bash profiles/run_diag.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/diag
for v in 0 1 2 3 4 5; do
  LIBP=audio-ident_amd/aidfp/libaidfp.so; [ $v != 0 ] && LIBP=audio-ident_amd/build/diag$v/libaidfp.so
  AIDFP_LIB=$PWD/$LIBP timeout -k 10 200 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS -T -d gpurun_out/diag/v$v -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/diag/v$v.log 2>&1 || exit 1
  AIDFP_LIB=$PWD/$LIBP timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/diag/b$v.log 2>&1 || exit 1
done
