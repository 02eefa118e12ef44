set -euo pipefail
R=$(pwd); OUT=$R/gpurun_out/prof_stream; mkdir -p $OUT; export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT" -o run --output-format csv -- python3 "$R/tools/bench_stream.py" --conns 65536 --recs 4 --steps 2 > $OUT/out.json 2> $OUT/err.txt
echo done
