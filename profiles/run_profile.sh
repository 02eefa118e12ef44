#!/bin/bash
# Profile the bench workload on a GPU box (run from the repo root via gpurun).
#   profiles/run_profile.sh <tag> [bench args...]
# 1) rocprofv3 --kernel-trace --stats on the default bench command
# 2) separate --pmc passes (SQ instruction mix / LDS, FETCH_SIZE, WRITE_SIZE)
#    on a 256K-record run of the same config.
# Output: gpurun_out/prof_<tag>/...  (copy the summaries into profiles/)
set -euo pipefail
TAG=${1:-r01}; shift || true
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/stats" -o run --output-format csv \
    -- python3 "$R/bench.py" --no-cpu --no-e2e "$@" > "$OUT/bench.json" 2> "$OUT/bench.err"
PMC_ARGS=(--no-cpu --no-e2e --steps 2 --warmup 1 --records ${PMC_RECORDS:-262144} "$@")
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT \
    --kernel-trace -d "$OUT/pmc_sq1" -o run --output-format csv \
    -- python3 "$R/bench.py" "${PMC_ARGS[@]}" > "$OUT/pmc_sq1.json" 2> "$OUT/pmc_sq1.err"
timeout -k 10 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE \
    --kernel-trace -d "$OUT/pmc_sq2" -o run --output-format csv \
    -- python3 "$R/bench.py" "${PMC_ARGS[@]}" > "$OUT/pmc_sq2.json" 2> "$OUT/pmc_sq2.err"
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE \
    --kernel-trace -d "$OUT/pmc_sq3" -o run --output-format csv \
    -- python3 "$R/bench.py" "${PMC_ARGS[@]}" > "$OUT/pmc_sq3.json" 2> "$OUT/pmc_sq3.err"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/pmc_fetch" -o run --output-format csv \
    -- python3 "$R/bench.py" "${PMC_ARGS[@]}" > "$OUT/pmc_fetch.json" 2> "$OUT/pmc_fetch.err"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$OUT/pmc_write" -o run --output-format csv \
    -- python3 "$R/bench.py" "${PMC_ARGS[@]}" > "$OUT/pmc_write.json" 2> "$OUT/pmc_write.err"
echo "profile done: $OUT"
