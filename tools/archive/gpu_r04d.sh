#!/bin/bash
# r04: server fallback debug, then the lane-power A/B and crossover
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/${TAG:-r04d}
mkdir -p $O
TLSREC_SERVER_DEBUG=1 timeout -k 10 300 python -u -m pytest tests/test_server_gpu.py -q -x --timeout 120 --timeout-method thread \
    -p no:cacheprovider -k "match_oracle" > $O/server_alone.txt 2> $O/server_alone.err
echo "server alone rc $?"; tail -3 $O/server_alone.txt
grep -c "grid ended" $O/server_alone.err; grep "grid ended\|launch failed" $O/server_alone.err | head -5
timeout -k 10 400 python -u -m pytest tests/test_coalesce_gpu.py tests/test_dist.py tests/test_dtls_gpu.py tests/test_engine_hygiene_gpu.py tests/test_server_gpu.py -q --timeout 120 --timeout-method thread \
    -p no:cacheprovider > $O/server_seq.txt 2>&1
echo "server seq rc $?"; tail -3 $O/server_seq.txt
b() {  # name, env, args
  local name=$1 envs=$2; shift 2
  env $envs timeout -k 10 300 python3 bench.py --no-cpu --no-e2e "$@" > $O/$name.json 2> $O/$name.err || { echo "FAIL $name"; tail -3 $O/$name.err; return 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['roofline']['kernel_ms_avg'], d['check'])" $O/$name.json $name
}
for rep in 1 2; do
  for c in k4 c4s; do
    b ${c}_tm7_$rep TLSREC_GCM_TREEMUL=7 --config $c || exit 1
    b ${c}_lp_$rep X=1 --config $c || exit 1
  done
done
b c4s_contig X=1 --config c4s --key-order contiguous || exit 1
for rep in 1 2; do
  env TLSREC_GCM_TREEMUL=7 timeout -k 10 300 python3 tools/bench_dtls.py > $O/dtls_tm7_$rep.json 2>&1 || exit 1
  timeout -k 10 300 python3 tools/bench_dtls.py > $O/dtls_lp_$rep.json 2>&1 || exit 1
  env TLSREC_GCM_TREEMUL=7 timeout -k 10 300 python3 tools/bench_stream.py --conns 65536 --recs 4 > $O/stream4_tm7_$rep.json 2>&1 || exit 1
  timeout -k 10 300 python3 tools/bench_stream.py --conns 65536 --recs 4 > $O/stream4_lp_$rep.json 2>&1 || exit 1
done
for f in $O/dtls_*.json $O/stream4_*.json; do echo "$f $(grep -o '"GiBps": [0-9.]*\|"value": [0-9.]*' $f | tr '\n' ' ')"; done
timeout -k 10 400 python3 tools/bench_crossover.py > $O/crossover.jsonl 2> $O/crossover.err || { echo "crossover failed"; tail -3 $O/crossover.err; exit 1; }
tail -1 $O/crossover.jsonl
