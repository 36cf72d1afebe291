#!/bin/bash
# r05m: where the K4 scatter's time goes (timing-only AID_K4_DIAG builds): product vs in-place sequential writes (2),
# no global writes (3), unstable one-atomic rank (4), each under a kernel trace of probes/k4_probe.py.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05m
mkdir -p $O
for lib in product k4diag2 k4diag3 k4diag4; do
  if [ $lib = product ]; then unset AIDFP_LIB; else export AIDFP_LIB=$GRAFT_REPO_ROOT/audio-ident_amd/build/$lib/libaidfp.so; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -T -d $O/$lib -o run --output-format csv -- python3 probes/k4_probe.py --modes radix --reps 3 > $O/$lib.json 2> $O/$lib.err || exit 4
done
unset AIDFP_LIB
echo done
