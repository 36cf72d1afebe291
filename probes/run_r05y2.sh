#!/bin/bash
# r05y2: kernel trace of the service leg (olaf_query through the coalescer at 1/16/64 clients). The first try added
# --memory-copy-trace: the bench finished and printed its line, then rocprofv3 faulted in its exit-time finalisation
# (profiles/r05y2_memcopy_trace_exit_sigsegv.txt, the r04y signature) and wrote no trace.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05y2
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $O/trace -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-fullband --no-catalog --no-stream > $O/bench.json 2> $O/bench.err || exit 4
echo done
