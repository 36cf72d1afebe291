#!/bin/bash
# r05t2: the K4 / CSR tests incl. the tile-edge cases.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05t2
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_match.py -x -v --timeout 200 --timeout-method thread > $O/tests.txt 2>&1 || exit 4
echo done
