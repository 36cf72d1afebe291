#!/bin/bash
# r05w5: same-box interleaved A/B of the threaded host batch copy on the service leg (probes/service_copy_ab.py):
# single-threaded copy, threads from 1 M floats (4 MiB), threads from 4 M floats (16 MiB); 3 rounds.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05w5
mkdir -p $O
for i in 1 2 3; do
  for m in 1099511627776 1048576 4194304; do
    timeout -k 10 300 python probes/service_copy_ab.py $m > $O/svc_${m}_$i.json 2> $O/svc_${m}_$i.err || exit 5
  done
done
echo done
