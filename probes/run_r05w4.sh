#!/bin/bash
# r05w2 (r05w3: + the threaded host batch copy from 4 MiB; r05w4: from 16 MiB): service leg with the coalescer resolving asyncio requests once per loop and batch (olaf_query), against the
# per-request wrap_future path of r05zz / r05zf; adapter and concurrency GPU tests first. Two service runs.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05w4
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_adapter.py tests/test_gpu_concurrency.py tests/test_gpu_exact.py -x -q --timeout 200 --timeout-method thread > $O/tests.txt 2>&1 || exit 4
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu --no-fullband --no-catalog --no-stream > $O/svc_$i.json 2> $O/svc_$i.err || exit 5
done
echo done
