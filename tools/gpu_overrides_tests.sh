set -o pipefail
mkdir -p gpurun_out/ov
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu "tests/test_evp_parity_gpu.py::test_engine_overrides_vs_openssl_evp" "tests/test_stream_gpu.py::test_send_copy_path_matches_oracle" > gpurun_out/ov/tests.txt 2>&1
rc=$?; tail -20 gpurun_out/ov/tests.txt; exit $rc
