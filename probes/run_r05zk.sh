#!/bin/bash
# r05zk: K3 with coalesced mask loads (16 lanes per frame): extraction parity tests, then a same-box A/B against the
# round's previous library: kernel times by shape (k1_shape_probe) and the headline-only bench line, alternated.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05zk
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_extract.py tests/test_gpu_lane_parity.py -x -v --timeout 200 --timeout-method thread > $O/tests.txt 2>&1 || exit 4
B=probes/ab/libaidfp_r05base.so
for i in 1 2; do
  AIDFP_LIB=$B timeout -k 10 120 python -u probes/k1_shape_probe.py --rounds 1 --seconds 1 --shapes 256x10,1024x30 > $O/shape_base_$i.jsonl 2>>$O/err.txt || exit 5
  timeout -k 10 120 python -u probes/k1_shape_probe.py --rounds 1 --seconds 1 --shapes 256x10,1024x30 > $O/shape_tree_$i.jsonl 2>>$O/err.txt || exit 6
done
for i in 1 2 3; do
  AIDFP_LIB=$B timeout -k 10 200 python bench.py --no-cpu --no-fullband --no-catalog --no-service --no-stream > $O/head_base_$i.json 2>>$O/err.txt || exit 7
  timeout -k 10 200 python bench.py --no-cpu --no-fullband --no-catalog --no-service --no-stream > $O/head_tree_$i.json 2>>$O/err.txt || exit 8
done
echo done
