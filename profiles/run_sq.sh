#!/bin/bash
# SQ counter passes (occupancy / issue / LDS) for the extraction kernels. usage: bash profiles/run_sq.sh <tag>
set -e
TAG=${1:-sq}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/sq_$TAG
mkdir -p $OUT
rocprofv3 -L > $OUT/counters.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS -T -d $OUT/p1 -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --settle 0 --no-cpu --no-fullband --no-catalog --no-service --no-stream > $OUT/p1.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU -T -d $OUT/p2 -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --settle 0 --no-cpu --no-fullband --no-catalog --no-service --no-stream > $OUT/p2.log 2>&1
