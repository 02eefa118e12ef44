#!/bin/bash
# the whole -m gpu suite and smoke() on the in-tree build, output under gpurun_out/<tag>/
set -o pipefail
O=gpurun_out/${1:-tests}; mkdir -p $O
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/ > $O/gpu_tests.txt 2>&1 || { tail -40 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 && cat $O/smoke.txt
