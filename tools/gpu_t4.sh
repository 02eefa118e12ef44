#!/bin/bash
# Same-box A/B of the four-table AES GCM kernel (TLSREC_GCM_T4=1, default)
# against the two-table kernel (=0): GPU tests first, then bench rows.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out/t4
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t4/gpu_tests.txt 2>&1 || { echo "gpu tests failed"; tail -20 gpurun_out/t4/gpu_tests.txt; exit 1; }
tail -1 gpurun_out/t4/gpu_tests.txt
for cfg in ${CFGS:-c2 c4 c4s gcm192 k4}; do
  for i in 1 2; do
    for t in 0 1; do
      TLSREC_GCM_T4=$t timeout -k 10 300 python bench.py --config $cfg --no-cpu --no-e2e --steps ${STEPS:-10} > gpurun_out/t4/${cfg}_t${t}_$i.json 2> gpurun_out/t4/${cfg}_t${t}_$i.err || { echo "bench $cfg t=$t failed"; tail -5 gpurun_out/t4/${cfg}_t${t}_$i.err; exit 1; }
      python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['roofline']['frac'], d['check'])" gpurun_out/t4/${cfg}_t${t}_$i.json "$cfg t4=$t run $i"
    done
  done
done
