#!/bin/bash
# r04: ChaCha20 first-column-round cache in registers (2 waves/SIMD, and forced 3 with small spills) vs base
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
T=${TAG:-r04m}
bash tools/gpu_ab_lib.sh $T/reg abso/libtlsrec_base.so abso/libtlsrec_ccreg.so c3 chacha16k || exit 1
bash tools/gpu_ab_lib.sh $T/w3 abso/libtlsrec_base.so abso/libtlsrec_ccw3.so c3 c3d chacha16k c4
