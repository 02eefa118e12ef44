#!/bin/bash
# r04: key setup at 8 waves/SIMD -- full -m gpu suite + key-schedule row
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/${TAG:-r04x2}
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.txt 2>&1 || { echo "gpu tests failed"; tail -30 $O/gpu_tests.txt; exit 1; }
tail -1 $O/gpu_tests.txt
timeout -k 10 300 python3 tools/bench_keysched.py > $O/keysched.json 2> $O/keysched.err || { echo "keysched failed"; exit 1; }
cut -c1-200 $O/keysched.json
