#!/bin/bash
# r05zn: the LDS match path launched with the vote counts for batches of any size (one host round trip less per
# query call): K5 / lane / stream / service GPU tests, then the headline + service + stream legs against the
# previous build, alternated on one box.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05zn
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_match.py tests/test_gpu_match_load.py tests/test_gpu_lane_parity.py tests/test_gpu_stream.py tests/test_gpu_adapter.py tests/test_gpu_concurrency.py tests/test_gpu_exact.py -x -v --timeout 200 --timeout-method thread > $O/tests.txt 2>&1 || exit 4
B=probes/ab/libaidfp_head.so
for i in 1 2; do
  AIDFP_LIB=$B timeout -k 10 300 python bench.py --no-cpu --no-fullband --no-catalog > $O/base_$i.json 2>>$O/err.txt || exit 5
  timeout -k 10 300 python bench.py --no-cpu --no-fullband --no-catalog > $O/tree_$i.json 2>>$O/err.txt || exit 6
done
echo done
