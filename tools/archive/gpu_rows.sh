#!/bin/bash
# Every measured row of DESIGN.md section 5 on one box: bench configs (device
# resident), stream layer, key schedule, C-host single-record latency.
# -> gpurun_out/rows/*.json ; prints a one-line summary per row.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/rows
mkdir -p $O
row() {   # name, timeout, command...
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $O/$name.json 2> $O/$name.err || { echo "FAIL $name"; tail -3 $O/$name.err; return 1; }
}
summ() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d.get('value'), d.get('roofline',{}).get('kernel_ms_avg'), d.get('roofline',{}).get('frac'), d.get('check'))" $O/$1.json $1; }
row c2 400 python3 bench.py && summ c2 &&
for c in c3 c4 c1 ccm ccm8 gcm192 aria256 camellia128 chacha16k k4 c4s c2s c3d; do
  row $c 400 python3 bench.py --config $c --no-e2e && summ $c || exit 1
done &&
row stream16 300 python3 tools/bench_stream.py --conns 65536 --recs 16 && cat $O/stream16.json &&
row stream4 300 python3 tools/bench_stream.py --conns 65536 --recs 4 && cat $O/stream4.json &&
row stream_cp 300 python3 tools/bench_stream.py --conns 262144 --recs 4 --content 1400 --cipher 3 && cat $O/stream_cp.json &&
row dtls_small 300 python3 tools/bench_dtls.py && cat $O/dtls_small.json &&
row dtls_cp 300 python3 tools/bench_dtls.py --cipher 3 && cat $O/dtls_cp.json &&
row dtls16k 300 python3 tools/bench_dtls.py --content 16384 --recs 4 --cipher 2 && cat $O/dtls16k.json &&
row keysched 300 python3 tools/bench_keysched.py && cat $O/keysched.json &&
: > $O/latency.jsonl &&
for a in "2 1.3 16383" "2 1.3 1400" "3 1.3 1400" "1 1.2 1400" "2 1.3 100"; do
  timeout -k 10 120 ./tests/c/abi_host latency $a 2000 >> $O/latency.jsonl || exit 1
done && for t in 1 16 32; do timeout -k 10 120 ./tests/c/abi_host threads $t 2000 gcm_chacha >> $O/latency.jsonl || exit 1; done &&
cat $O/latency.jsonl
