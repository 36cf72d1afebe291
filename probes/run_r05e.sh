#!/bin/bash
# r05e: where K5's LDS path spends its time -- timing-only ablations (k5diag1: phase 1 without LDS atomics, k5diag2:
# no phase 3, k5diag3: both), SQ and FETCH/WRITE counters of k_match_lds, then the bench line (stream outlier trace).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05e
mkdir -p $O
for lib in product k5diag1 k5diag2 k5diag3; do
  if [ $lib = product ]; then L=""; else L="AIDFP_LIB=$GRAFT_REPO_ROOT/audio-ident_amd/build/$lib/libaidfp.so"; fi
  echo "== $lib" >> $O/k5_diag.txt
  env $L timeout -k 10 300 python3 probes/k5_path_probe.py --paths auto --reps 3 >> $O/k5_diag.txt 2>/dev/null || exit 3
done
P="python3 probes/k5_path_probe.py --paths auto --reps 1"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS -T -d $O/sq1 -o run --output-format csv -- $P > $O/sq1.log 2>&1 || exit 4
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU -T -d $O/sq2 -o run --output-format csv -- $P > $O/sq2.log 2>&1 || exit 5
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -T -d $O/fetch -o run --output-format csv -- $P > $O/fetch.log 2>&1 || exit 6
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $O/trace -o run --output-format csv -- $P > $O/trace.log 2>&1 || exit 7
timeout -k 10 400 python bench.py --no-cpu > $O/bench.json 2> $O/bench.err || { echo bench rc=$?; tail -5 $O/bench.err; exit 8; }
echo done
