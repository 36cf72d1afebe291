#!/bin/bash
# ISA statistics of one kernel of a HIP source under extra -D defines (static instruction counts of
# the kernel body as hipcc emits it, plus the resource remark). usage:
#   tools/isa_stats.sh <src.hip> <kernel-symbol-regex> [-Dxxx ...]
set -e
SRC=$(readlink -f "$1"); KRE=$2; shift 2
T=$(mktemp -d); cd "$T"
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-fast-math"
case "$SRC" in *stft.hip) FLAGS="$FLAGS -fno-slp-vectorize";; esac
/opt/rocm/bin/hipcc $FLAGS "$@" -c "$SRC" -o k.o --save-temps -Rpass-analysis=kernel-resource-usage > remarks.txt 2>&1
S=$(ls *-gfx950.s)
SYM=$(grep -oE "^$KRE[A-Za-z0-9_]*:" "$S" | head -1 | tr -d :)
awk -v s="$SYM:" '$1==s{on=1} on{print} on&&/s_endpgm/{exit}' "$S" > k.s
grep -A12 "Function Name: $SYM" remarks.txt | grep -E "VGPRs:|TotalSGPRs|Occupancy|LDS Size|ScratchSize" | sed 's/.*remark: [^ ]* //'
printf "%s\n" "$SYM"
echo "instr $(grep -cE '^\s+[a-z]' k.s) valu $(grep -cE '^\s+v_' k.s) salu $(grep -cE '^\s+s_' k.s) ds $(grep -cE '^\s+ds_' k.s) ds_write $(grep -cE '^\s+ds_write' k.s) dpp $(grep -c _dpp k.s) permlane $(grep -c permlane k.s) s_nop $(grep -c s_nop k.s) global $(grep -cE '^\s+global_' k.s) waitcnt $(grep -c s_waitcnt k.s)"
cp k.s /tmp/isa_last.s
rm -rf "$T"
