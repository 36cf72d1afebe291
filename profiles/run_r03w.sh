#!/bin/bash
# Timing-only probe: K2 without its horizontal pass (no LDS row, no barriers; the vertical ring, decisions and mask
# stores as in K2), the K2 half of the DESIGN 9 split, ABBA against the product build (parity fails by design).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03w
mkdir -p $O
V=audio-ident_amd/build/k2vonly/libaidfp.so
timeout -k 10 120 python3 bench.py --no-cpu --no-catalog --steps 50 > $O/ab_cur_1.json 2>/dev/null || exit 1
AIDFP_LIB=$V timeout -k 10 120 python3 bench.py --no-cpu --no-catalog --steps 50 > $O/ab_vonly_1.json 2>/dev/null; [ $? -le 1 ] || exit 1
AIDFP_LIB=$V timeout -k 10 120 python3 bench.py --no-cpu --no-catalog --steps 50 > $O/ab_vonly_2.json 2>/dev/null; [ $? -le 1 ] || exit 1
timeout -k 10 120 python3 bench.py --no-cpu --no-catalog --steps 50 > $O/ab_cur_2.json 2>/dev/null || exit 1
echo done
