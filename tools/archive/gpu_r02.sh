#!/bin/bash
# Round-2 GPU pass: full -m gpu suite, default bench (c2, with CPU legs and the
# end-to-end leg), C-host latency table, then the c2 profile incl. LDS counters.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
STEP=${1:-all}
if [ "$STEP" = all ] || [ "$STEP" = tests ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
      > gpurun_out/gputests.log 2>&1 || { tail -30 gpurun_out/gputests.log; exit 1; }
  tail -3 gpurun_out/gputests.log
fi
if [ "$STEP" = all ] || [ "$STEP" = bench ]; then
  timeout -k 10 400 python bench.py > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err || { tail gpurun_out/bench_c2.err; exit 1; }
  cat gpurun_out/bench_c2.json
  : > gpurun_out/latency.jsonl
  for a in "2 1.3 16383" "2 1.3 1400" "3 1.3 1400" "1 1.2 1400" "5 1.3 1400" "2 1.3 100"; do
    timeout -k 10 120 ./tests/c/abi_host latency $a 2000 >> gpurun_out/latency.jsonl || exit 1
  done
  timeout -k 10 120 ./tests/c/abi_host threads 16 400 >> gpurun_out/latency.jsonl || exit 1
  cat gpurun_out/latency.jsonl
fi
if [ "$STEP" = all ] || [ "$STEP" = prof ]; then
  timeout -k 10 1000 bash profiles/run_profile.sh r02a_c2 && \
  python3 profiles/summarize_pmc.py gpurun_out/prof_r02a_c2/pmc_sq3 gcm_kernel
fi
