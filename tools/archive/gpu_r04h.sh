#!/bin/bash
# r04: GPU suite (server withdrawal-streak fix), then same-box A/B on one build:
# lane powers in the key-pass kernels (TREEMUL=7 turns them off) and the
# key-ordered descriptor copy (TLSREC_GCM_SRECS=0 turns it off)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
T=${TAG:-r04h}
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
  for c in c2 c2s; do
    b ${c}_tm7_$rep TLSREC_GCM_TREEMUL=7 --config $c || exit 1
    b ${c}_new_$rep X=1 --config $c || exit 1
  done
  b c4_tm7_$rep TLSREC_GCM_TREEMUL=7 --config c4 || exit 1
  b c4_nosrecs_$rep TLSREC_GCM_SRECS=0 --config c4 || exit 1
  b c4_new_$rep X=1 --config c4 || exit 1
  for c in k4 c4s; do
    b ${c}_nosrecs_$rep TLSREC_GCM_SRECS=0 --config $c || exit 1
    b ${c}_new_$rep X=1 --config $c || exit 1
  done
done
exit $rc
