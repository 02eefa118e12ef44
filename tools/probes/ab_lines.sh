#!/bin/bash
# same-box A/B of line-grouped loads in the small-record paired passes, + traffic of both builds
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_stream_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/tl.txt 2>&1 || { tail -20 gpurun_out/tl.txt; exit 1; }
tail -1 gpurun_out/tl.txt
tools/probes/ab_lib.sh abso/libtlsrec_prev.so c4s || exit 1
for lib in new old old new; do
  if [ $lib = old ]; then L=abso/libtlsrec_prev.so; else L=mbedtls_amd/libtlsrec.so; fi
  echo "stream16Kx64x1.4K $lib $(TLSREC_LIBRARY=$L timeout -k 10 200 python3 tools/bench_stream.py --conns 16384 --recs 64 --content 1400 | tail -2 | python3 -c 'import sys,json; print([json.loads(l)["value"] for l in sys.stdin])')"
done
mkdir -p gpurun_out/tr_lines; export TMPDIR=/tmp
for lib in new old; do
  if [ $lib = old ]; then L=$PWD/abso/libtlsrec_prev.so; else L=$PWD/mbedtls_amd/libtlsrec.so; fi
  for c in FETCH_SIZE WRITE_SIZE; do
    (cd /tmp && TLSREC_LIBRARY=$L timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/tr_lines/${lib}_$c -o run --output-format csv \
      -- python3 $GRAFT_REPO_ROOT/bench.py --config c4s --no-cpu --no-e2e --steps 2 --warmup 1 > /dev/null 2>&1) || exit 1
  done
  python3 -c "
import sys; sys.path.insert(0,'profiles'); from summarize_pmc import summarize
f=summarize('gpurun_out/tr_lines/${lib}_FETCH_SIZE','tlsrec_gcm_kernel'); w=summarize('gpurun_out/tr_lines/${lib}_WRITE_SIZE','tlsrec_gcm_kernel')
n=2097152; print('$lib gcm read/rec', round(f['hbm_read_bytes_corrected']/n), 'write/rec', round(w['hbm_write_bytes']/n))"
done
