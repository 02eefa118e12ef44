#!/bin/bash
# r04: key-pass tree mode (TLSREC_GCM_TREEMUL 1 = HEAD default vs 9 = lane powers) x lanes per record (auto 8 vs 4)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/${TAG:-r04q}
mkdir -p $O
b() {  # name, env, args
  local name=$1 envs=$2; shift 2
  env $envs timeout -k 10 300 python3 bench.py --no-cpu --no-e2e --verify 16 "$@" > $O/$name.json 2> $O/$name.err || { echo "FAIL $name"; tail -3 $O/$name.err; return 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['roofline']['kernel_ms_avg'], d['check']['bad_records'])" $O/$name.json $name
}
for rep in 1 2; do
  b c2_r04a_$rep TLSREC_LIBRARY=$R/ablib/libtlsrec_r04a.so --config c2 || exit 1
  for c in c2 c2s c4; do
    b ${c}_tm1_$rep X=1 --config $c || exit 1
    b ${c}_tm9_$rep TLSREC_GCM_TREEMUL=9 --config $c || exit 1
    b ${c}_L4tm1_$rep TLSREC_GCM_LANES=4 --config $c || exit 1
    b ${c}_L4tm9_$rep "TLSREC_GCM_LANES=4 TLSREC_GCM_TREEMUL=9" --config $c || exit 1
  done
done
