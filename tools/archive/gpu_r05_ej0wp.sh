#!/bin/bash
# r05: E_K(J0) once per lane in the 8-wave wave passes too -- parity, then
# same-box A/B on the shapes that take them (under 4 records per key of
# 16 KiB, under 12 per key of 1.4 KiB)
set -o pipefail
O=gpurun_out/ej0wp; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_evp_parity_gpu.py tests/test_dtls_gpu.py tests/test_stream_gpu.py tests/test_gpu_parity.py tests/test_gpu_parity_edges.py > $O/gpu_tests.txt 2>&1 || { tail -30 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
for shape in "k4 65536" "k4 131072" "c2s 262144" "c2s 524288"; do
  set -- $shape
  for lib in ablib/libtlsrec_ej0.so ablib/libtlsrec_ej0wp.so ablib/libtlsrec_ej0wp.so ablib/libtlsrec_ej0.so; do
    f=$O/$1_$2.$(basename $lib .so).json
    TLSREC_LIBRARY=$lib timeout -k 10 300 python3 bench.py --config $1 --keys 65536 --records $2 --no-cpu --no-e2e --verify 16 > $f 2> $f.err || { echo "FAIL $shape $lib"; tail -3 $f.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], d['value'], d['check']['bad_records'])" $f "$shape" $(basename $lib .so)
  done
done
