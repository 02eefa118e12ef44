#!/bin/bash
# ad-hoc same-box environment-variable A/B of bench rows:
#   tools/gpu_envab.sh "<config> [bench args]" "VAR=a" "VAR=b"   (runs a, b, b, a)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
row=$1; A=$2; B=$3
for v in "$A" "$B" "$B" "$A"; do
  env $v timeout -k 10 300 python3 bench.py --config $row --no-cpu --no-e2e --verify 16 > gpurun_out/envab.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/envab.json').read().strip().splitlines()[-1]); print('$row', '$v', d['value'], d['check']['bad_records'])"
done
