#!/bin/bash
# r05g: K5 insert pass queues hot votes in LDS (product) vs loading their postings inside the walk (nohotq), the
# same-box A/B on the config-4 lane: product / sig1_r05d (one signature per lane) / prev_r05a (8-B postings) /
# k5diag2 (product without the insert pass, timing only); then the bench line.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05g
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_match.py tests/test_gpu_match_load.py tests/test_gpu_exact.py tests/test_gpu_lane_parity.py tests/test_gpu_adapter.py -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { echo tests failed; tail -40 $O/gpu_tests.txt; exit 3; }
tail -3 $O/gpu_tests.txt
for i in 1 2; do
for lib in product nohotq prev_r05a k5diag2; do
  if [ $lib = product ]; then L=""; else L="AIDFP_LIB=$GRAFT_REPO_ROOT/audio-ident_amd/build/$lib/libaidfp.so"; fi
  echo "== $lib $i" >> $O/k5_ab.txt
  env $L timeout -k 10 300 python3 probes/k5_path_probe.py --paths auto --reps 3 >> $O/k5_ab.txt 2>/dev/null || exit 4
done
done
timeout -k 10 400 python bench.py --no-cpu > $O/bench.json 2> $O/bench.err || { echo bench rc=$?; tail -5 $O/bench.err; exit 5; }
echo done
