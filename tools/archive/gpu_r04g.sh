#!/bin/bash
# r04: the full GPU suite with the record server's debug lines (the failing
# test's captured stderr shows them), then the lane-power A/B on the key-pass
# kernels (c2, c2s, c4) against abso/libtlsrec_wn.so
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
T=${TAG:-r04g}
O=gpurun_out/$T
mkdir -p $O
TLSREC_SERVER_DEBUG=1 timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider \
    > $O/gpu_tests.txt 2> $O/gpu_tests.err
rc=$?
tail -4 $O/gpu_tests.txt
grep -c "grid ended" $O/gpu_tests.txt
grep "grid ended" $O/gpu_tests.txt | head -5
case $rc in 0|1) ;; *) echo "pytest rc $rc: stopping"; exit $rc;; esac
b() {  # name, env, args
  local name=$1 envs=$2; shift 2
  env $envs timeout -k 10 300 python3 bench.py --no-cpu --no-e2e "$@" > $O/$name.json 2> $O/$name.err || { echo "FAIL $name"; tail -3 $O/$name.err; return 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['roofline']['kernel_ms_avg'], d['check'])" $O/$name.json $name
}
for rep in 1 2; do
  for c in c2 c2s c4 c1; do
    b ${c}_prev_$rep TLSREC_LIBRARY=$R/abso/libtlsrec_wn.so --config $c || exit 1
    b ${c}_new_$rep X=1 --config $c || exit 1
  done
done
exit $rc
