#!/bin/bash
# r04: bucket count kernel, 4 / 16 records per thread vs 1 -- GPU suite on RPT 4, then same-box A/B + the kernel's time
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/${TAG:-r04bc}
mkdir -p $O
export TMPDIR=/tmp
TLSREC_LIBRARY=$R/ablib/libtlsrec_rpt4.so timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.txt 2>&1 || { echo "gpu tests failed"; tail -30 $O/gpu_tests.txt; exit 1; }
tail -1 $O/gpu_tests.txt
for rep in 1 2; do
  for v in base rpt4 rpt16; do
    TLSREC_LIBRARY=$R/ablib/libtlsrec_$v.so timeout -k 10 300 python3 bench.py --config c4s --no-cpu --no-e2e --verify 64 > $O/c4s_${v}_$rep.json 2> $O/c4s_${v}_$rep.err || { echo "FAIL $v"; tail -3 $O/c4s_${v}_$rep.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['roofline']['kernel_ms_avg'], d['check'])" $O/c4s_${v}_$rep.json c4s_${v}_$rep
  done
done
for v in base rpt4 rpt16; do
  (cd /tmp && TLSREC_LIBRARY=$R/ablib/libtlsrec_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof_$v -o run --output-format csv -- python3 $R/bench.py --config c4s --no-cpu --no-e2e --verify 16 > $R/$O/prof_$v.json 2> $R/$O/prof_$v.err) || { echo "prof $v failed"; exit 1; }
  echo $v $(grep bucket_count $O/prof_$v/run_kernel_stats.csv | awk -F'",' '{print $2}' | cut -d, -f1-3)
done
