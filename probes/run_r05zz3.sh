#!/bin/bash
# r05zz3: the library relinked without the offload-bundle intermediates: whole GPU suite, smoke, default bench line.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05zz3
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.txt 2>&1 || exit 4
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit 5
timeout -k 10 500 python bench.py > $O/bench.json 2> $O/bench.err || exit 6
echo done
