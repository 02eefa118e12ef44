#!/bin/bash
# r05: per-kernel times of the ChaCha20-Poly1305 stream / DTLS send and receive rows
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/sendprof; mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stream_cp -o run --output-format csv -- python3 $R/tools/bench_stream.py --conns 262144 --recs 4 --content 1400 --cipher 3 > $O/stream_cp.json 2> $O/stream_cp.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/dtls_cp -o run --output-format csv -- python3 $R/tools/bench_dtls.py --cipher 3 > $O/dtls_cp.json 2> $O/dtls_cp.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stream16s -o run --output-format csv -- python3 $R/tools/bench_stream.py --conns 65536 --recs 16 --content 1400 > $O/stream16s.json 2> $O/stream16s.err &&
for d in stream_cp dtls_cp stream16s; do echo "== $d"; cat $O/$d.json; f=$(find $O/$d -name '*kernel_stats.csv' | head -1); cut -d, -f1-5 "$f" | head -14; done
