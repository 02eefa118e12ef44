#!/bin/bash
# r04: c4s paired-pass lanes per record vs the L1 TLB (2 = default, 4, 8)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
T=${TAG:-r04j}
O=gpurun_out/$T
mkdir -p $O
b() {  # name, env, args
  local name=$1 envs=$2; shift 2
  env $envs timeout -k 10 300 python3 bench.py --no-cpu --no-e2e "$@" > $O/$name.json 2> $O/$name.err || { echo "FAIL $name"; tail -3 $O/$name.err; return 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['roofline']['kernel_ms_avg'], d['check'])" $O/$name.json $name
}
for rep in 1 2; do
  for l in 2 4 8; do
    b c4s_L${l}_$rep TLSREC_GCM_PAIR_L=$l --config c4s || exit 1
  done
done
export TMPDIR=/tmp
for l in 4 8; do
  (cd /tmp && TLSREC_GCM_PAIR_L=$l timeout -s KILL 300 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TOTAL_CACHE_ACCESSES_sum \
     --kernel-trace -d $R/$O/tlb_L$l -o run --output-format csv -- python3 $R/bench.py --no-cpu --no-e2e --config c4s --steps 2 --warmup 1 \
     > $R/$O/tlb_L$l.json 2> $R/$O/tlb_L$l.err) || { echo "tlb pass failed"; exit 1; }
done
echo done
