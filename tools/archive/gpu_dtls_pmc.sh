#!/bin/bash
# c4 kernel breakdown + PMC passes of the DTLS 1.4 KiB AES-128-GCM receive (wave-pass GCM kernel)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/c4prof -o run --output-format csv \
  -- python3 $R/bench.py --config c4 --no-cpu --no-e2e --steps 5 > $R/gpurun_out/c4prof.json 2>&1 || exit 1
O=$R/gpurun_out/dtlspmc; mkdir -p $O
pass() { local n=$1; shift; timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace -d $O/$n -o run --output-format csv \
  -- python3 $R/tools/bench_dtls.py --steps 1 > $O/$n.json 2> $O/$n.err || { echo "pass $n failed"; return 1; }; }
pass sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT && \
pass sq2 SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE && \
pass sq3 SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE && \
pass fetch FETCH_SIZE && pass write WRITE_SIZE
echo pmc done
