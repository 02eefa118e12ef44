#!/bin/bash
# r04: ChaCha20 first-column-round cache -- parity, then same-box A/B vs the previous build
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/${TAG:-r04l}
mkdir -p $O
: timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_evp_parity_gpu.py tests/test_gpu_parity.py tests/test_server_gpu.py > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
: tail -2
bash tools/gpu_ab_lib.sh ${TAG:-r04l}/ab abso/libtlsrec_base.so abso/libtlsrec_cc.so c3 c3d c4 chacha16k
