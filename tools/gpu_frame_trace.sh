#!/bin/bash
# Round-6 profiling probes (one box per call; each GPU step under its own
# timeout, chained).
#   tools/gpu_pcs.sh frame   -- kernel trace of the 1 M-record receive calls (stream / DTLS, ChaCha and AES)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
T=${TAG:-r06pcs}
O=$R/gpurun_out/$T
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
case "$1" in
frame)
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stream_cp -o run --output-format csv -- python3 $R/tools/bench_stream.py --conns 262144 --recs 4 --content 1400 --cipher 3 --no-cpu --steps 3 > $O/stream_cp.json 2>&1 &&
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/dtls_cp -o run --output-format csv -- python3 $R/tools/bench_dtls.py --cipher 3 --no-cpu --steps 3 > $O/dtls_cp.json 2>&1 &&
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/dtls_small -o run --output-format csv -- python3 $R/tools/bench_dtls.py --no-cpu --steps 3 > $O/dtls_small.json 2>&1 &&
  echo frame done
  ;;
esac
