#!/bin/bash
# r04: mixed batches' ChaCha20-Poly1305 kernel on a second queue (TLSREC_OVERLAP) -- GPU suite, then same-box A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/${TAG:-r04ov}
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.txt 2>&1 || { echo "gpu tests failed"; tail -30 $O/gpu_tests.txt; exit 1; }
tail -1 $O/gpu_tests.txt
b() {  # name, env, args
  local name=$1 envs=$2; shift 2
  env $envs timeout -k 10 300 python3 bench.py --no-cpu --no-e2e --verify 64 "$@" > $O/$name.json 2> $O/$name.err || { echo "FAIL $name"; tail -3 $O/$name.err; return 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['roofline']['kernel_ms_avg'], d['check'])" $O/$name.json $name
}
for rep in 1 2 3; do
  for c in c4s c4; do
    b ${c}_ov0_$rep TLSREC_OVERLAP=0 --config $c || exit 1
    b ${c}_ov1_$rep TLSREC_OVERLAP=1 --config $c || exit 1
  done
done
