#!/bin/bash
# r04: GPU suite on the lane-power build, then same-box A/B of lane powers
# (TLSREC_GCM_TREEMUL=7 = r03's table-free tree) on the paired-pass rows,
# and the per-record crossover measurement
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/${TAG:-r04c}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider \
    > $O/gpu_tests.txt 2>&1 || { echo "gpu tests failed"; tail -30 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
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
for rep in 1 2; do
  env TLSREC_GCM_TREEMUL=7 timeout -k 10 300 python3 tools/bench_dtls.py > $O/dtls_tm7_$rep.json 2>&1 || exit 1
  timeout -k 10 300 python3 tools/bench_dtls.py > $O/dtls_lp_$rep.json 2>&1 || exit 1
  env TLSREC_GCM_TREEMUL=7 timeout -k 10 300 python3 tools/bench_stream.py --conns 65536 --recs 4 > $O/stream4_tm7_$rep.json 2>&1 || exit 1
  timeout -k 10 300 python3 tools/bench_stream.py --conns 65536 --recs 4 > $O/stream4_lp_$rep.json 2>&1 || exit 1
done
grep -h GiB $O/dtls_*.json $O/stream4_*.json | cut -c1-300
timeout -k 10 400 python3 tools/bench_crossover.py > $O/crossover.jsonl 2> $O/crossover.err || { echo "crossover failed"; tail -3 $O/crossover.err; exit 1; }
tail -1 $O/crossover.jsonl
