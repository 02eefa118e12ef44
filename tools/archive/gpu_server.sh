#!/bin/bash
# Record server (server.hip): parity tests, then single-record latency and
# threaded round trips through the C ABI.  -> gpurun_out/srv/
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/srv
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_server_gpu.py -x -v --timeout 120 --timeout-method thread \
    > $O/tests.txt 2>&1 || { echo "server tests failed"; tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
: > $O/latency.jsonl
for a in "2 1.3 16383" "2 1.3 1400" "3 1.3 1400" "1 1.2 1400" "2 1.3 100"; do
  TLSREC_SERVER_DEBUG=${SRV_DEBUG:-} timeout -k 10 120 ./tests/c/abi_host latency $a 2000 >> $O/latency.jsonl 2>> $O/stderr.txt || { echo "latency $a failed"; exit 1; }
done
for t in 1 16 32; do
  timeout -k 10 120 ./tests/c/abi_host threads $t 2000 gcm_chacha >> $O/latency.jsonl || { echo "threads $t failed"; exit 1; }
done
timeout -k 10 120 ./tests/c/abi_host threads 16 2000 mix >> $O/latency.jsonl || { echo "threads mix failed"; exit 1; }
cat $O/latency.jsonl
timeout -k 10 300 python -u -m pytest tests/test_coalesce_gpu.py tests/test_c_host.py -x -q --timeout 120 --timeout-method thread \
    > $O/tests2.txt 2>&1 || { echo "coalesce/c_host tests failed"; tail -30 $O/tests2.txt; exit 1; }
tail -2 $O/tests2.txt
