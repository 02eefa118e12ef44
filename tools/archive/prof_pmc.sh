#!/bin/bash
# PMC passes (one counter group per rocprofv3 run) over a bench config:
#   tools/prof_pmc.sh <tag> <bench args...>
# -> gpurun_out/pmc_<tag>/<pass>/...
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
ARGS=(--no-cpu --no-e2e --steps 2 --warmup 1 "$@")
run() {
  local name=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" --kernel-trace -d "$OUT/$name" -o run --output-format csv \
    -- python3 "$R/bench.py" "${ARGS[@]}" > "$OUT/$name.json" 2> "$OUT/$name.err" || { echo "pass $name failed"; return 1; }
}
run sq SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU && \
run ic SQC_ICACHE_MISSES SQC_ICACHE_HITS SQC_ICACHE_REQ SQ_IFETCH && \
run vm SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_LEVEL_VMEM SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS && \
run ld SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH
echo "pmc done $TAG"
