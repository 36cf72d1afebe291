#!/bin/bash
# r05zs: K1 -> K2 per clip group (bounded power planes): extraction / lane / match / stream GPU tests, then same-box
# A/B against the previous build: the catalog loop at 1,024-track calls (2.6 M rows: four groups) and the config-4
# lane legs (4096-clip calls, ~3.7 M rows: five groups).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05zs
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_extract.py tests/test_gpu_exact.py tests/test_gpu_lane_parity.py tests/test_gpu_match.py tests/test_gpu_stream.py -x -v --timeout 200 --timeout-method thread > $O/tests.txt 2>&1 || exit 4
B=probes/ab/libaidfp_head.so
for i in 1 2; do
  AIDFP_LIB=$B timeout -k 10 150 python -u probes/catalog_async_ab.py --sr 44100 --reps 1 --batch 1024 >> $O/catalog.jsonl 2>>$O/err.txt || exit 5
  timeout -k 10 150 python -u probes/catalog_async_ab.py --sr 44100 --reps 1 --batch 1024 >> $O/catalog.jsonl 2>>$O/err.txt || exit 6
done
for i in 1 2; do
  AIDFP_LIB=$B timeout -k 10 300 python bench.py --no-cpu --no-fullband --no-service --no-stream --steps 3 --warmup 1 > $O/lane_base_$i.json 2>>$O/err.txt || exit 7
  timeout -k 10 300 python bench.py --no-cpu --no-fullband --no-service --no-stream --steps 3 --warmup 1 > $O/lane_tree_$i.json 2>>$O/err.txt || exit 8
done
echo done
