#!/bin/bash
# r04: key setup H^1..H^64 over four lanes per power -- key-schedule / GCM parity, then the key-schedule row
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/${TAG:-r04s}
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider \
  tests/test_keysched_gpu.py tests/test_server_gpu.py tests/test_evp_parity_gpu.py tests/test_gpu_parity.py > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
  timeout -k 10 300 python3 tools/bench_keysched.py > $O/keysched_$rep.json 2> $O/keysched_$rep.err || { echo "keysched failed"; tail -3 $O/keysched_$rep.err; exit 1; }
  cut -c1-200 $O/keysched_$rep.json
done
