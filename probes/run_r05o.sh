#!/bin/bash
# r05o: K4 with the one-atomic in-wave rank: the CSR layout and sort-build tests, then the build timed (radix with the
# default rank, radix with ballot ranks, rocPRIM) under a kernel trace.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05o
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_match.py -k "csr_layout or sort_build" -x -v --timeout 200 --timeout-method thread > $O/tests.txt 2>&1 || exit 4
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $O/trace -o run --output-format csv -- python3 probes/k4_probe.py --modes radix,radix_ballot,rocprim,radix_again --reps 3 > $O/k4.json 2> $O/k4.err || exit 5
echo done
