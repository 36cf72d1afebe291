#!/bin/bash
# r05a: K5 (config 4 exact lane) kernel trace + FETCH/WRITE PMC passes through bench.py's catalog leg, then the
# r04y exit-time SIGSEGV command once more under rocprofv3 with the process maps dumped (last: it may dump core).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05a
mkdir -p $O
B="python3 bench.py --steps 3 --warmup 1 --no-cpu --no-fullband --no-service"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $O/trace -o run --output-format csv -- $B > $O/trace.json 2> $O/trace.err || exit 3
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -T -d $O/fetch -o run --output-format csv -- $B > $O/fetch.json 2> $O/fetch.err || exit 4
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -T -d $O/write -o run --output-format csv -- $B > $O/write.json 2> $O/write.err || exit 5
AIDFP_DUMP_MAPS=$O/svc_maps.txt timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $O/svc -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-fullband --no-catalog --service-tracks 1000 --service-requests 256 > $O/svc.json 2> $O/svc.err
echo "svc rc=$?"
echo done
