#!/bin/bash
# r04: GPU suite on the word-nonce build (no scratch nonce bytes), same-box A/B
# against the previous build (abso/libtlsrec_lp.so), k4 / c4s profiles
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
T=${TAG:-r04f}
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
  for c in c2 c3 k4 c4s; do
    b ${c}_prev_$rep TLSREC_LIBRARY=$R/abso/libtlsrec_lp.so --config $c || exit 1
    b ${c}_new_$rep X=1 --config $c || exit 1
  done
done
export PROFILE_RDREQ=1
PMC_RECORDS=262144 profiles/run_profile.sh ${T}_k4 --config k4 > $O/prof_k4.log 2>&1 || { echo "profile k4 failed"; tail -5 $O/prof_k4.log; exit 1; }
PMC_RECORDS=4194304 profiles/run_profile.sh ${T}_c4s --config c4s > $O/prof_c4s.log 2>&1 || { echo "profile c4s failed"; tail -5 $O/prof_c4s.log; exit 1; }
echo profiled
exit $rc
