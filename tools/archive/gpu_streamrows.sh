#!/bin/bash
# stream / DTLS rows (tools/bench_stream.py, tools/bench_dtls.py) -> gpurun_out/streamrows.txt
set -o pipefail
O=gpurun_out/streamrows.txt
: > $O
run() { echo "== $*" >> $O; timeout -k 10 200 "$@" 2>/dev/null | grep '^{' >> $O || exit 1; }
run python3 tools/bench_dtls.py
run python3 tools/bench_dtls.py --cipher 3
run python3 tools/bench_dtls.py --content 16384 --recs 4 --cipher 2
run python3 tools/bench_stream.py --conns 65536 --recs 16
run python3 tools/bench_stream.py --conns 65536 --recs 4
run python3 tools/bench_stream.py --conns 262144 --recs 4 --content 1400 --cipher 3
run python3 tools/bench_stream.py --conns 65536 --recs 16 --content 1400 --cipher 2
