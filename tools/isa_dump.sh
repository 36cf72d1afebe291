#!/bin/bash
# Device assembly of every csrc/*.hip (same flags as build_ext.py) into $1, for
# comparing two source trees kernel for kernel: tools/isa_dump.sh /tmp/a; ...; diff -r /tmp/a /tmp/b
set -eo pipefail
OUT=${1:?usage: isa_dump.sh OUTDIR [CSRC]}
CSRC=${2:-$(dirname "$0")/../audio-ident_amd/csrc}
mkdir -p "$OUT"
for f in "$CSRC"/*.hip; do
  b=$(basename "$f" .hip)
  extra=""
  [ "$b" = stft ] && extra="-fno-slp-vectorize"
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math $extra \
    --cuda-device-only -S "$f" -o - 2>/dev/null \
    | grep -v '^\s*\.\(file\|loc\|ident\)\|^\s*;\|\.debug\|Ltmp\|amdhsa.version\|\.amdgcn_target' > "$OUT/$b.s" &
done
wait
