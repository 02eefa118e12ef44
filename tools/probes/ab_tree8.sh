set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_dtls_gpu.py tests/test_stream_gpu.py tests/test_gpu_parity_edges.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t8.txt 2>&1 || { tail -20 gpurun_out/t8.txt; exit 1; }
tail -1 gpurun_out/t8.txt
tools/probes/ab_lib.sh abso/libtlsrec_prev.so c4s k4
for lib in new old old new; do
  if [ $lib = old ]; then L=abso/libtlsrec_prev.so; else L=mbedtls_amd/libtlsrec.so; fi
  echo "dtls_small $lib $(TLSREC_LIBRARY=$L timeout -k 10 200 python3 tools/bench_dtls.py | tail -2 | python3 -c 'import sys,json; print([json.loads(l)["value"] for l in sys.stdin])')"
  echo "stream16x1.4K $lib $(TLSREC_LIBRARY=$L timeout -k 10 200 python3 tools/bench_stream.py --conns 65536 --recs 16 --content 1400 | tail -2 | python3 -c 'import sys,json; print([json.loads(l)["value"] for l in sys.stdin])')"
done
