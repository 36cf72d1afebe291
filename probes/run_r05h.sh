#!/bin/bash
# r05h: K5 LDS path variants on the config-4 lane (interleaved same-box A/B, probes/k5_path_probe.py):
# product (4-posting chunks, U=4 windows, records loaded once for both passes), reuse0 (records reloaded for the
# insert pass), cw8u4 / cw8u3 (8-posting chunks), cw4u3 (3 windows), maxv4 (LDS path up to 2^18 votes per query),
# wg4 (four 512-thread workgroups per CU: 2^15 counters, 1024-entry table).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05h
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_match.py tests/test_gpu_match_load.py tests/test_gpu_exact.py tests/test_gpu_lane_parity.py -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { echo tests failed; tail -40 $O/gpu_tests.txt; exit 3; }
tail -3 $O/gpu_tests.txt
for i in 1 2; do
for lib in product reuse0 cw8u4 cw8u3 cw4u3 maxv4 wg4; do
  if [ $lib = product ]; then L=""; else L="AIDFP_LIB=$GRAFT_REPO_ROOT/audio-ident_amd/build/$lib/libaidfp.so"; fi
  echo "== $lib $i" >> $O/k5_ab.txt
  env $L timeout -k 10 300 python3 probes/k5_path_probe.py --paths auto --reps 3 >> $O/k5_ab.txt 2>/dev/null || exit 4
done
done
echo done
