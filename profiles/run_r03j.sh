#!/bin/bash
# K4: SQ counters per dispatch over the A/B probe (two PMC passes), to see why the first radix scatter pass takes
# ~10 ms against ~6 for the others.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03j
mkdir -p $O
timeout -s KILL 400 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS -d $O/p1 -o run --output-format csv -- python3 probes/k4_probe.py --reps 1 > $O/p1.json 2> $O/p1.err
timeout -s KILL 400 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU -d $O/p2 -o run --output-format csv -- python3 probes/k4_probe.py --reps 1 > $O/p2.json 2> $O/p2.err
echo done
