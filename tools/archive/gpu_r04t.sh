#!/bin/bash
# r04: key-schedule row, same box: round-3 build, HEAD before the ladder, the H-power ladder; parity first
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/${TAG:-r04t}
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider tests/test_keysched_gpu.py tests/test_server_gpu.py tests/test_evp_parity_gpu.py > $O.pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O.pytest.log; exit 1; }
tail -1 $O.pytest.log
mkdir -p $O
export TMPDIR=/tmp
for v in r03 prev lad r03 prev lad; do
  TLSREC_LIBRARY=$R/ablib/libtlsrec_$v.so timeout -k 10 300 python3 tools/bench_keysched.py > $O/ks_$v.json 2> $O/ks_$v.err || { echo "keysched $v failed"; tail -3 $O/ks_$v.err; exit 1; }
  echo $v $(cut -c1-160 $O/ks_$v.json)
done
for v in lad; do
  (cd /tmp && TLSREC_LIBRARY=$R/ablib/libtlsrec_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof_$v -o run --output-format csv -- python3 $R/tools/bench_keysched.py > $R/$O/prof_$v.json 2> $R/$O/prof_$v.err) || { echo "prof $v failed"; exit 1; }
  cut -d, -f1-4 $O/prof_$v/run_kernel_stats.csv | head -6
done
# c4's GCM half: lanes per record 16 (auto, 64 records per key) vs 8
b() {  # name, env, args
  local name=$1 envs=$2; shift 2
  env $envs timeout -k 10 300 python3 bench.py --no-cpu --no-e2e --verify 16 "$@" > $O/$name.json 2> $O/$name.err || { echo "FAIL $name"; tail -3 $O/$name.err; return 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['roofline']['kernel_ms_avg'], d['check']['bad_records'])" $O/$name.json $name
}
for rep in 1 2; do
  b c4_auto_$rep X=1 --config c4 || exit 1
  b c4_L8_$rep TLSREC_GCM_LANES=8 --config c4 || exit 1
done
