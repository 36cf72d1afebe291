#!/bin/bash
# Timing-only probes: K2 without its two workgroup barriers per 4-row step (AID_K2_DIAG_NOBAR: wrong results, the
# bench's parity check fails by design) against the product build, ABBA order: what barrier removal could buy.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03r
mkdir -p $O
V=audio-ident_amd/build/k2nobar/libaidfp.so
timeout -k 10 120 python3 bench.py --no-cpu --no-catalog --steps 50 > $O/ab_cur_1.json 2>/dev/null || exit 1
AIDFP_LIB=$V timeout -k 10 120 python3 bench.py --no-cpu --no-catalog --steps 50 > $O/ab_nobar_1.json 2>/dev/null
[ $? -le 1 ] || exit 1
AIDFP_LIB=$V timeout -k 10 120 python3 bench.py --no-cpu --no-catalog --steps 50 > $O/ab_nobar_2.json 2>/dev/null
[ $? -le 1 ] || exit 1
timeout -k 10 120 python3 bench.py --no-cpu --no-catalog --steps 50 > $O/ab_cur_2.json 2>/dev/null || exit 1
# K2 with every row load out of range (zeros; same instructions and waits, no memory latency): timing only
V2=audio-ident_amd/build/k2noload/libaidfp.so
AIDFP_LIB=$V2 timeout -k 10 120 python3 bench.py --no-cpu --no-catalog --steps 50 > $O/ab_noload_1.json 2>/dev/null
[ $? -le 1 ] || exit 1
timeout -k 10 120 python3 bench.py --no-cpu --no-catalog --steps 50 > $O/ab_cur_3.json 2>/dev/null || exit 1
echo done
