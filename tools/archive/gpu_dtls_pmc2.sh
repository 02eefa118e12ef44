#!/bin/bash
# PMC passes of the DTLS 1.4 KiB AES-128-GCM batch (64 K connections x 16 datagrams,
# the 4-lane wave-pass GCM kernel since r02) -> gpurun_out/dtlspmc2/
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
cd /tmp
O=$R/gpurun_out/dtlspmc2; mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/stats -o run --output-format csv \
  -- python3 $R/tools/bench_dtls.py --steps 3 > $O/stats.json 2> $O/stats.err || { echo "stats failed"; exit 1; }
pass() { local n=$1; shift; timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace -d $O/$n -o run --output-format csv \
  -- python3 $R/tools/bench_dtls.py --steps 1 > $O/$n.json 2> $O/$n.err || { echo "pass $n failed"; return 1; }; }
pass pmc_sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT && \
pass pmc_sq2 SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE && \
pass pmc_sq3 SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE && \
pass pmc_fetch FETCH_SIZE && pass pmc_write WRITE_SIZE && echo pmc done
