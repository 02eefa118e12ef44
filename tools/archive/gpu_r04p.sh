#!/bin/bash
# r04: c2 regression bisect, same box: r04a-era (3ad90bd), lane powers (e5b95fb), nonce words (3bd8e47), HEAD
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/${TAG:-r04p}
mkdir -p $O
b() {  # name, env, args
  local name=$1 envs=$2; shift 2
  env $envs timeout -k 10 300 python3 bench.py --no-cpu --no-e2e --verify 16 "$@" > $O/$name.json 2> $O/$name.err || { echo "FAIL $name"; tail -3 $O/$name.err; return 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['roofline']['kernel_ms_avg'], d['check']['bad_records'])" $O/$name.json $name
}
for rep in 1 2; do
  for v in r04a e5 3b head; do
    b c2_${v}_$rep TLSREC_LIBRARY=$R/ablib/libtlsrec_$v.so --config c2 || exit 1
  done
done
