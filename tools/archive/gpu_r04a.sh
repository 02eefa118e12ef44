#!/bin/bash
# r04 GPU pass: the new/changed GPU tests first (verbose), then the whole -m gpu
# suite (all failures listed), smoke, the c2 line
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/${TAG:-r04a}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -v -x --timeout 300 --timeout-method thread -p no:cacheprovider \
    tests/test_engine_hygiene_gpu.py tests/test_fail_closed_gpu.py tests/test_lane_ops_gpu.py tests/test_scan_gpu.py \
    > $O/new_tests.txt 2>&1 || { echo "new tests failed"; tail -40 $O/new_tests.txt; exit 1; }
tail -3 $O/new_tests.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > $O/gpu_tests.txt 2>&1
rc=$?
tail -15 $O/gpu_tests.txt
case $rc in 0|1) ;; *) echo "pytest rc $rc: stopping"; exit $rc;; esac
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { echo "smoke failed"; tail -5 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 300 python bench.py > $O/bench_c2.json 2> $O/bench_c2.err || { echo "bench failed"; tail -5 $O/bench_c2.err; exit 1; }
cut -c1-400 $O/bench_c2.json
tools/probes/run_fetch_calib.sh ${TAG:-r04a} > $O/calib.log 2>&1 || { echo "calib failed"; tail -5 $O/calib.log; exit 1; }
grep -E '"(calib_|fetch_factor|write_factor)' $O/calib.log | tr -d ' \n' | cut -c1-1500; echo
timeout -k 10 300 python tools/bench_mixed.py --label r04_yield > $O/mixed_yield.json 2> $O/mixed_yield.err || { echo "mixed failed"; tail -5 $O/mixed_yield.err; exit 1; }
cat $O/mixed_yield.json
TLSREC_SERVER_YIELD=0 TLSREC_SERVER_IDLE_MS=20 timeout -k 10 300 python tools/bench_mixed.py --label r03_behaviour > $O/mixed_r03.json 2> $O/mixed_r03.err || { echo "mixed r03 failed"; tail -5 $O/mixed_r03.err; exit 1; }
cat $O/mixed_r03.json
exit $rc
