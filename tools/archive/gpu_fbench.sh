# 8(f) row benches (one box); JSON lines under gpurun_out/
set -o pipefail
mkdir -p gpurun_out
for c in ccm ccm8 gcm192; do
  timeout -k 10 300 python bench.py --config $c --no-cpu > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.err || exit 1
done
timeout -k 10 300 python tools/bench_stream.py > gpurun_out/bench_stream.json 2> gpurun_out/bench_stream.err &&
timeout -k 10 300 python tools/bench_stream.py --conns 262144 --recs 4 --content 1400 --cipher 3 >> gpurun_out/bench_stream.json 2>> gpurun_out/bench_stream.err
echo rc=$?
