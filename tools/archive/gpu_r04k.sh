#!/bin/bash
# r04: arena allocation vs the c4s GCM kernel's L1 TLB misses
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/${TAG:-r04k}
mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do
  for al in default contiguous; do
    timeout -k 10 300 python3 tools/probes/tlb_probe.py --alloc $al > $O/tlb_${al}_$rep.json 2> $O/tlb_${al}_$rep.err || { echo "probe $al failed"; tail -5 $O/tlb_${al}_$rep.err; exit 1; }
    cat $O/tlb_${al}_$rep.json
  done
done
for al in default contiguous; do
  (cd /tmp && timeout -s KILL 300 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TOTAL_CACHE_ACCESSES_sum \
     --kernel-trace -d $R/$O/pmc_$al -o run --output-format csv -- python3 $R/tools/probes/tlb_probe.py --alloc $al --steps 2 \
     > $R/$O/pmc_$al.json 2> $R/$O/pmc_$al.err) || { echo "pmc $al failed"; exit 1; }
done
echo done
