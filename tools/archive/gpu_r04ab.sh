#!/bin/bash
# r04: lanes per record, env / flag A/B on the final build: c2 8 vs 16, gcm192 8 vs 4, c3 2 vs 4
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/${TAG:-r04ab}
mkdir -p $O
b() {  # name, env, args
  local name=$1 envs=$2; shift 2
  env $envs timeout -k 10 300 python3 bench.py --no-cpu --no-e2e --verify 16 "$@" > $O/$name.json 2> $O/$name.err || { echo "FAIL $name"; tail -3 $O/$name.err; return 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['roofline']['kernel_ms_avg'], d['check']['bad_records'])" $O/$name.json $name
}
for rep in 1 2; do
  b c2_auto_$rep X=1 --config c2 || exit 1
  b c2_L16_$rep TLSREC_GCM_LANES=16 --config c2 || exit 1
  b gcm192_auto_$rep X=1 --config gcm192 || exit 1
  b gcm192_L4_$rep TLSREC_GCM_LANES=4 --config gcm192 || exit 1
  b c3_auto_$rep X=1 --config c3 || exit 1
  b c3_L4_$rep X=1 --config c3 --lanes 4 || exit 1
done
