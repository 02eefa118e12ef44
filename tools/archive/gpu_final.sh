#!/bin/bash
# End-of-round measurement on one box, in two gpurun calls (each under the
# 20-minute limit):
#   tools/gpu_final.sh rows   -- -m gpu suite, smoke, every DESIGN row (tools/gpu_rows.sh)
#   tools/gpu_final.sh prof   -- bench.py through the process-group path at WORLD_SIZE=1,
#                                c2 / c3 rocprofv3 kernel stats + PMC passes
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${TAG:-r03}
if [ "$1" = rows ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.txt 2>&1 || { echo "gpu tests failed"; tail -20 gpurun_out/gpu_tests.txt; exit 1; }
  tail -1 gpurun_out/gpu_tests.txt
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.txt 2>&1 || { echo "smoke failed"; tail -5 gpurun_out/smoke.txt; exit 1; }
  tail -1 gpurun_out/smoke.txt
  tools/gpu_rows.sh > gpurun_out/rows.log 2>&1 || { echo "rows failed"; tail -5 gpurun_out/rows.log; exit 1; }
  cat gpurun_out/rows.log
elif [ "$1" = prof ]; then
  timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
      --master-port 29533 bench.py --dist --steps 5 --no-cpu --no-e2e > gpurun_out/dist1.json 2> gpurun_out/dist1.err \
      || { echo "dist rehearsal failed"; tail -5 gpurun_out/dist1.err; exit 1; }
  cat gpurun_out/dist1.json
  profiles/run_profile.sh ${TAG}_c2 > gpurun_out/prof_c2.log 2>&1 || { echo "c2 profile failed"; tail -5 gpurun_out/prof_c2.log; exit 1; }
  profiles/run_profile.sh ${TAG}_c3 --config c3 > gpurun_out/prof_c3.log 2>&1 || { echo "c3 profile failed"; tail -5 gpurun_out/prof_c3.log; exit 1; }
  echo prof done
else
  echo "usage: tools/gpu_final.sh rows|prof"; exit 2
fi
