set -euo pipefail
R=$(pwd); OUT=$R/gpurun_out/prof_stream; mkdir -p $OUT; export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/cp" -o run --output-format csv -- python3 "$R/tools/bench_stream.py" --conns 262144 --recs 4 --content 1400 --cipher 3 --steps 3 > $OUT/cp.json 2> $OUT/cp.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/gcm" -o run --output-format csv -- python3 "$R/tools/bench_stream.py" --conns 65536 --recs 4 --steps 3 > $OUT/gcm.json 2> $OUT/gcm.err
echo done
