#!/bin/bash
# r05l: decoupled look-back price for K4 (probes/lookback_probe.hip): copy-only vs look-back (1 or 8 predecessors
# per step) at two and one workgroups per CU.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05l
mkdir -p $O
timeout -k 10 150 probes/lookback_probe 141553 3 60 > $O/lb60.json 2> $O/lb.err || exit 4
timeout -k 10 150 probes/lookback_probe 141553 3 100 > $O/lb100.json 2>> $O/lb.err || exit 5
echo done
