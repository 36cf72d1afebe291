#!/bin/bash
# r05zj: the whole GPU suite and smoke on the asynchronous-append build, then extraction time per audio-second by
# batch shape (headline 256 x 10 s vs catalog 1,024 x 30 s).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05zj
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/tests.txt 2>&1 || exit 4
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit 5
timeout -k 10 200 python -u probes/k1_shape_probe.py > $O/shape.jsonl 2>$O/shape.err || exit 6
echo done
