set -euo pipefail
R=$(pwd); OUT=$R/gpurun_out/prof_c3; mkdir -p $OUT; export TMPDIR=/tmp
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR \
    --kernel-trace -d "$OUT/pmc1" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu --config c3 --steps 2 --warmup 1 > /dev/null 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_INSTS_VALU_INT32 \
    --kernel-trace -d "$OUT/pmc2" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu --config c3 --steps 2 --warmup 1 > /dev/null 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_MFMA_MOPS_I8 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SMEM \
    --kernel-trace -d "$OUT/pmc3" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu --config c3 --steps 2 --warmup 1 > /dev/null 2>&1 || true
echo done
