#!/bin/bash
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/${K2VAR:-k2diag}
export AIDFP_LIB=$PWD/audio-ident_amd/build/${K2VAR:-k2diag}/libaidfp.so
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS -T -d gpurun_out/${K2VAR:-k2diag}/p -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --settle 0 --no-cpu > gpurun_out/${K2VAR:-k2diag}/p.log 2>&1
