#!/bin/bash
# r05zl: K3 coalesced mask loads, second form (8 frames of loads in flight per 16-lane group): extraction parity,
# then kernel times by shape against the round's previous library, alternated.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05zl
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_extract.py -x -v --timeout 200 --timeout-method thread > $O/tests.txt 2>&1 || exit 4
B=probes/ab/libaidfp_r05base.so
for i in 1 2; do
  AIDFP_LIB=$B timeout -k 10 120 python -u probes/k1_shape_probe.py --rounds 1 --seconds 1 --shapes 256x10,1024x30 > $O/shape_base_$i.jsonl 2>>$O/err.txt || exit 5
  timeout -k 10 120 python -u probes/k1_shape_probe.py --rounds 1 --seconds 1 --shapes 256x10,1024x30 > $O/shape_tree_$i.jsonl 2>>$O/err.txt || exit 6
done
echo done
