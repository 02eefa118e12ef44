#!/bin/bash
# End-of-round measurement on one box: every DESIGN row, the RCCL-path
# rehearsal of bench.py at WORLD_SIZE=1, and the c2 / c3 profiles.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
tools/gpu_rows.sh > gpurun_out/rows.log 2>&1 || { echo "rows failed"; tail -5 gpurun_out/rows.log; exit 1; }
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --dist --steps 5 --no-cpu --no-e2e > gpurun_out/dist1.json 2> gpurun_out/dist1.err \
    || { echo "dist rehearsal failed"; tail -5 gpurun_out/dist1.err; exit 1; }
profiles/run_profile.sh r02g_c2 > gpurun_out/prof_c2.log 2>&1 || { echo "c2 profile failed"; exit 1; }
profiles/run_profile.sh r02g_c3 --config c3 > gpurun_out/prof_c3.log 2>&1 || { echo "c3 profile failed"; exit 1; }
echo final done
