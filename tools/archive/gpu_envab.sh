#!/bin/bash
# Same-box A/B of an engine environment switch: the -m gpu suite (switch at
# its default), then $CFGS with $VAR set to each of $VALS (default 0 1), alternating, $REPS times.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out/envab
if [ -z "$NOTEST" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/envab/gpu_tests.txt 2>&1 || { echo "gpu tests failed"; tail -20 gpurun_out/envab/gpu_tests.txt; exit 1; }
tail -1 gpurun_out/envab/gpu_tests.txt
fi
for cfg in $CFGS; do
  for i in $(seq 1 ${REPS:-2}); do
    for v in ${VALS:-0 1}; do
      env $VAR=$v timeout -k 10 300 python bench.py --config $cfg --no-cpu --no-e2e --steps ${STEPS:-10} $EXTRA > gpurun_out/envab/${cfg}_${v}_$i.json 2> gpurun_out/envab/${cfg}_${v}_$i.err || { echo "bench $cfg $VAR=$v failed"; tail -5 gpurun_out/envab/${cfg}_${v}_$i.err; exit 1; }
      python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['roofline']['frac'], d['roofline'].get('kernel_ms_avg'), d['check'])" gpurun_out/envab/${cfg}_${v}_$i.json "$cfg $VAR=$v run $i"
    done
  done
done
