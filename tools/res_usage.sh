#!/bin/bash
# Per-kernel resource usage (VGPRs, scratch, occupancy, LDS) of one HIP source under extra flags.
# usage: tools/res_usage.sh <src.hip> [flags ...]
SRC=$(readlink -f "$1"); shift
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-fast-math"
case "$SRC" in *stft.hip) FLAGS="$FLAGS -fno-slp-vectorize";; esac
T=$(mktemp -d)
/opt/rocm/bin/hipcc $FLAGS "$@" -c "$SRC" -o $T/k.o -Rpass-analysis=kernel-resource-usage 2>&1 | python3 -c '
import re, sys
cur = None
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)[:60]}; continue
    m = re.search(r"remark:\s+(VGPRs|AGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (\d+)", line)
    if m and cur is not None:
        cur[m.group(1).split()[0]] = int(m.group(2))
        if m.group(1).startswith("LDS"):
            print("%-62s vgpr %3d agpr %3d scratch %3d occ %d lds %d" % (cur["name"], cur.get("VGPRs", -1), cur.get("AGPRs", 0), cur.get("ScratchSize", -1), cur.get("Occupancy", -1), cur["LDS"]))
            cur = None
'
rm -rf $T
