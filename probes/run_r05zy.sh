#!/bin/bash
# r05zy: the memory side of the K1 plane-bound knee: TCC -> EA write requests and their stalls, and DRAM
# read-credit stalls, per extraction call of the catalog shape (1024 x 30 s) at 3 GiB, 6 GiB and the whole plane.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05zy
mkdir -p $O
for rows in 786432 1572864 4194304; do
  timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum GRBM_GUI_ACTIVE -d $O/pmc_$rows -o run --output-format csv -- python3 probes/k1_shape_probe.py --rounds 1 --seconds 0.3 --shapes 1024x30 --plane-rows $rows > $O/pmc_$rows.out 2> $O/pmc_$rows.err || exit 5
done
echo done
