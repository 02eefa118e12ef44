set -euo pipefail
R=$(pwd); OUT=$R/gpurun_out/wr; mkdir -p $OUT; export TMPDIR=/tmp; cd /tmp
for A in 16 128 256; do
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$OUT/w$A" -o run --output-format csv \
    -- python3 "$R/bench.py" --no-cpu --steps 2 --warmup 1 --records 262144 --align $A > "$OUT/w$A.json" 2> "$OUT/w$A.err"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/f$A" -o run --output-format csv \
    -- python3 "$R/bench.py" --no-cpu --steps 2 --warmup 1 --records 262144 --align $A > "$OUT/f$A.json" 2> "$OUT/f$A.err"
done
