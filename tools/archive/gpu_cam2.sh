# golden GPU parity (now incl. Camellia vectors), camellia128 bench with CPU baseline, rocprof stats
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/cam2
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/cam2/parity.txt 2>&1 || exit 1
timeout -k 10 300 python bench.py --config camellia128 > gpurun_out/cam2/bench_camellia128.json 2>gpurun_out/cam2/bench.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/cam2/prof -o cam -- python3 bench.py --no-cpu --config camellia128 --steps 5 > gpurun_out/cam2/prof_bench.json 2>gpurun_out/cam2/prof.err || exit 1
