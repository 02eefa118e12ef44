#!/bin/bash
# r04: c4s GCM read amplification diagnosis -- L2 hit/miss, L1->L2 read
# requests and L1 TLB misses, round-robin vs contiguous key order; plus the
# new optional-path GPU tests
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
T=${TAG:-r04i}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_evp_parity_gpu.py -q -k "key_ordered or key_pass_lane_powers" --timeout 300 \
    --timeout-method thread -p no:cacheprovider > $O/new_tests.txt 2>&1 || { echo "new tests failed"; tail -20 $O/new_tests.txt; exit 1; }
tail -1 $O/new_tests.txt
export TMPDIR=/tmp
for order in round-robin contiguous; do
  for pass in "TCC_HIT_sum TCC_MISS_sum TCC_READ_sum TCC_EA0_RDREQ_DRAM_sum" "TCP_TCC_READ_REQ_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TOTAL_CACHE_ACCESSES_sum"; do
    name=$(echo $pass | cut -c1-8)_$order
    (cd /tmp && timeout -s KILL 300 rocprofv3 --pmc $pass --kernel-trace -d $R/$O/$name -o run --output-format csv \
      -- python3 $R/bench.py --no-cpu --no-e2e --config c4s --steps 2 --warmup 1 --key-order $order > $R/$O/$name.json 2> $R/$O/$name.err) \
      || { echo "pass $name failed"; tail -3 $O/$name.err; exit 1; }
    echo "done $name"
  done
done
