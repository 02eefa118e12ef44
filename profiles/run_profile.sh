#!/bin/bash
# Profile a workload on a GPU box (run from the repo root via gpurun).
#   profiles/run_profile.sh <tag> [bench args...]
#   profiles/run_profile.sh <tag> --cmd <python script> [args...]   (any workload, e.g. tools/bench_dtls.py)
# 1) rocprofv3 --kernel-trace --stats on the workload
# 2) separate --pmc passes (SQ instruction mix / LDS, FETCH_SIZE, WRITE_SIZE,
#    and the L2->fabric read requests by size, TCC_EA0_RDREQ_{32B,64B,128B};
#    PROFILE_CACHE=1 adds vector-L1 / UTCL1 and L2 hit passes)
#    on a PMC_RECORDS-record run of the same bench config (default 262144;
#    multi-key configs pass their full record count so the launch path is the
#    same), or on the same --cmd workload.
# Output: gpurun_out/prof_<tag>/...  (copy the summaries into profiles/)
set -euo pipefail
TAG=${1:-r01}; shift || true
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
if [ "${1:-}" = "--cmd" ]; then
  shift
  SCRIPT=$R/$1; shift
  STATS_CMD=(python3 "$SCRIPT" "$@")
  PMC_CMD=(python3 "$SCRIPT" "$@")
else
  STATS_CMD=(python3 "$R/bench.py" --no-cpu --no-e2e "$@")
  PMC_CMD=(python3 "$R/bench.py" --no-cpu --no-e2e --steps 2 --warmup 1 --records ${PMC_RECORDS:-262144} "$@")
fi
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/stats" -o run --output-format csv \
    -- "${STATS_CMD[@]}" > "$OUT/bench.json" 2> "$OUT/bench.err"
pass() {   # name, counters...
  local name=$1; shift
  timeout -s KILL 300 rocprofv3 --pmc "$@" --kernel-trace -d "$OUT/$name" -o run --output-format csv \
      -- "${PMC_CMD[@]}" > "$OUT/$name.json" 2> "$OUT/$name.err"
}
pass pmc_sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT
pass pmc_sq2 SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE
pass pmc_sq3 SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE
pass pmc_fetch FETCH_SIZE
pass pmc_write WRITE_SIZE
if [ "${PROFILE_RDREQ:-1}" = 1 ]; then
  pass pmc_rdreq TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum
fi
if [ "${PROFILE_CACHE:-0}" = 1 ]; then
  pass pmc_tcp TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum
  pass pmc_tcc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_DRAM_sum
fi
echo "profile done: $OUT"
