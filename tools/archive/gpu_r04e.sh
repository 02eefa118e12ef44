#!/bin/bash
# r04: GPU suite on the aligned lane-power build, A/B vs TREEMUL=7, then
# k4 / c4s profiles of the new build
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
T=${TAG:-r04e}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > $O/gpu_tests.txt 2>&1
rc=$?
tail -4 $O/gpu_tests.txt
case $rc in 0|1) ;; *) echo "pytest rc $rc: stopping"; exit $rc;; esac
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
  env TLSREC_GCM_TREEMUL=7 timeout -k 10 300 python3 tools/bench_stream.py --conns 65536 --recs 16 --content 1400 > $O/stream16s_tm7_$rep.json 2>&1 || exit 1
  timeout -k 10 300 python3 tools/bench_stream.py --conns 65536 --recs 16 --content 1400 > $O/stream16s_lp_$rep.json 2>&1 || exit 1
  timeout -k 10 300 python3 tools/bench_dtls.py > $O/dtls_lp_$rep.json 2>&1 || exit 1
done
for f in $O/stream16s_*.json $O/dtls_*.json; do echo "$f $(grep -o '"value": [0-9.]*' $f | tr '\n' ' ')"; done
export PROFILE_RDREQ=1
PMC_RECORDS=262144 profiles/run_profile.sh ${T}_k4 --config k4 > $O/prof_k4.log 2>&1 || { echo "profile k4 failed"; tail -5 $O/prof_k4.log; exit 1; }
PMC_RECORDS=4194304 profiles/run_profile.sh ${T}_c4s --config c4s > $O/prof_c4s.log 2>&1 || { echo "profile c4s failed"; tail -5 $O/prof_c4s.log; exit 1; }
echo profiled
exit $rc
