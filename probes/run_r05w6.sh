#!/bin/bash
# r05w6: host-side profile of StreamBank pushes (probes/stream_host_profile.py).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05w6
mkdir -p $O
timeout -k 10 300 python3 probes/stream_host_profile.py > $O/prof.txt 2> $O/prof.err || exit 4
echo done
