set -euo pipefail
R=$(pwd); OUT=$R/gpurun_out/prof_c4; mkdir -p $OUT; export TMPDIR=/tmp; cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/stats" -o run --output-format csv \
    -- python3 "$R/bench.py" --no-cpu --config c4 --steps 3 --warmup 1 > "$OUT/bench.json" 2> "$OUT/bench.err"
