#!/bin/bash
# bench.py rows on one box: tools/gpu_bench_rows.sh <outdir> <config>...
# (c2 with its CPU and end-to-end legs; the others with their CPU legs)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/$1; shift
mkdir -p $O
for c in "$@"; do
  extra=""
  [ "$c" = c2 ] || extra="--no-e2e"
  timeout -k 10 400 python3 bench.py --config $c $extra > $O/$c.json 2> $O/$c.err || { echo "FAIL $c"; tail -3 $O/$c.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); c=d.get('cpu_baseline') or {}; print(sys.argv[2], d['value'], d['roofline']['kernel_ms_avg'], d['roofline']['frac'], d['check'], [(l['leg'], l['value']) for l in c.get('legs', [])])" $O/$c.json $c
done
