#!/bin/bash
# r05zh: asynchronous posting append + asynchronous generation: match/index GPU tests, then a same-box A/B of
# the catalog ingest (baseline library, synchronous generation / this tree, both / this tree, async append only).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05zh
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_match.py tests/test_gpu_comm.py -x -v --timeout 200 --timeout-method thread > $O/tests.txt 2>&1 || exit 4
for i in 1 2; do
  AIDFP_LIB=probes/ab/libaidfp_r05base.so timeout -k 10 150 python -u probes/catalog_async_ab.py --wait-synth >> $O/ab.jsonl 2>>$O/ab.err || exit 5
  timeout -k 10 150 python -u probes/catalog_async_ab.py >> $O/ab.jsonl 2>>$O/ab.err || exit 6
  timeout -k 10 150 python -u probes/catalog_async_ab.py --wait-synth >> $O/ab.jsonl 2>>$O/ab.err || exit 7
done
echo done
