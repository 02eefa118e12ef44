#!/bin/bash
# Same-box A/B/n: the -m gpu suite on the current build, then each config of
# $CFGS with every library of $LIBS (in-tree .so paths; "cur" = the current
# build), alternating, $REPS times.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out/abn
if [ -z "$NOTEST" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/abn/gpu_tests.txt 2>&1 || { echo "gpu tests failed"; tail -20 gpurun_out/abn/gpu_tests.txt; exit 1; }
tail -1 gpurun_out/abn/gpu_tests.txt
fi
for cfg in $CFGS; do
  for i in $(seq 1 ${REPS:-2}); do
    for lib in $LIBS; do
      tag=$(basename $lib .so)
      if [ "$lib" = cur ]; then unset TLSREC_LIBRARY; else export TLSREC_LIBRARY=$R/$lib; fi
      timeout -k 10 300 python bench.py --config $cfg --no-cpu --no-e2e --steps ${STEPS:-10} $EXTRA > gpurun_out/abn/${cfg}_${tag}_$i.json 2> gpurun_out/abn/${cfg}_${tag}_$i.err || { echo "bench $cfg $tag failed"; tail -5 gpurun_out/abn/${cfg}_${tag}_$i.err; exit 1; }
      python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['roofline']['frac'], d['roofline'].get('kernel_ms_avg'), d['check'])" gpurun_out/abn/${cfg}_${tag}_$i.json "$cfg $tag run $i"
    done
  done
done
unset TLSREC_LIBRARY
