#!/bin/bash
# r04: lane powers back to compile-time (wave passes) + single-key L = 4: parity, then same-box A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/${TAG:-r04r}
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider \
  tests/test_evp_parity_gpu.py tests/test_gpu_parity.py tests/test_gpu_parity_edges.py > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
b() {  # name, env, args
  local name=$1 envs=$2; shift 2
  env $envs timeout -k 10 300 python3 bench.py --no-cpu --no-e2e --verify 16 "$@" > $O/$name.json 2> $O/$name.err || { echo "FAIL $name"; tail -3 $O/$name.err; return 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['roofline']['kernel_ms_avg'], d['check']['bad_records'])" $O/$name.json $name
}
for rep in 1 2; do
  b c2_r04a_$rep TLSREC_LIBRARY=$R/ablib/libtlsrec_r04a.so --config c2 || exit 1
  b c2_fixL8_$rep "TLSREC_LIBRARY=$R/ablib/libtlsrec_fix.so TLSREC_GCM_LANES=8" --config c2 || exit 1
  b c2_fix_$rep TLSREC_LIBRARY=$R/ablib/libtlsrec_fix.so --config c2 || exit 1
  for c in c2s c2se gcm192 k4 c4s c4; do
    b ${c}_head_$rep TLSREC_LIBRARY=$R/ablib/libtlsrec_head.so --config $c || exit 1
    b ${c}_fix_$rep TLSREC_LIBRARY=$R/ablib/libtlsrec_fix.so --config $c || exit 1
  done
done
