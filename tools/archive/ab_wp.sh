# A/B of the wave-pass GCM variant (TLSREC_GCM_WP) on one box; JSON lines under gpurun_out/
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "wave_pass or many_keys or mixed_keys" > gpurun_out/wp_tests.log 2>&1 || exit 1
o=gpurun_out/ab_wp.jsonl; : > $o
for wp in 0 1; do
  for args in "--conns 65536 --recs 16" "--conns 262144 --recs 4 --content 1400" "--conns 262144 --recs 4 --content 4096" "--conns 65536 --recs 4 --content 16384"; do
    echo "wp=$wp $args" >> $o
    TLSREC_GCM_WP=$wp timeout -k 10 200 python tools/bench_stream.py $args >> $o 2>> gpurun_out/ab_wp.err || exit 1
  done
  echo "wp=$wp c4" >> $o
  TLSREC_GCM_WP=$wp timeout -k 10 300 python bench.py --config c4 --no-cpu >> $o 2>> gpurun_out/ab_wp.err || exit 1
done
echo "c2" >> $o
timeout -k 10 300 python bench.py --config c2 --no-cpu >> $o 2>> gpurun_out/ab_wp.err || exit 1
echo rc=$?
