#!/bin/bash
# r04: c2s (1 M x 1.4 KiB AES-256-GCM, one key) -- lanes per record 4 / 8 (auto) / 16
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/${TAG:-r04n}
mkdir -p $O
b() {  # name, env, args
  local name=$1 envs=$2; shift 2
  env $envs timeout -k 10 300 python3 bench.py --no-cpu --no-e2e --verify 16 "$@" > $O/$name.json 2> $O/$name.err || { echo "FAIL $name"; tail -3 $O/$name.err; return 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['roofline']['kernel_ms_avg'], d['check'])" $O/$name.json $name
}
for rep in 1 2; do
  b c2s_auto_$rep X=1 --config c2s || exit 1
  b c2s_L4_$rep TLSREC_GCM_LANES=4 --config c2s || exit 1
  b c2s_L16_$rep TLSREC_GCM_LANES=16 --config c2s || exit 1
  b c2s_L4tm7_$rep "TLSREC_GCM_LANES=4 TLSREC_GCM_TREEMUL=7" --config c2s || exit 1
done
