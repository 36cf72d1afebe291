#!/bin/bash
# r05v: SQ counters of the exact-lane kernels (k_match_lds, K1-K3 of the lane) on the catalog leg, two passes.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05v
mkdir -p $O
B="python3 bench.py --steps 3 --warmup 1 --settle 0 --no-cpu --no-fullband --no-service --no-stream"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS -T -d $O/p1 -o run --output-format csv -- $B > $O/p1.log 2>&1 || exit 4
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU -T -d $O/p2 -o run --output-format csv -- $B > $O/p2.log 2>&1 || exit 5
echo done
