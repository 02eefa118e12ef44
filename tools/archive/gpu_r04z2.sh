#!/bin/bash
# r04: bucket counters swizzled within each class -- GPU suite, then same-box A/B (c4s, c4, k4) and the count kernel's time
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/${TAG:-r04z2}
mkdir -p $O
export TMPDIR=/tmp
TLSREC_LIBRARY=$R/ablib/libtlsrec_swz.so timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.txt 2>&1 || { echo "gpu tests failed"; tail -30 $O/gpu_tests.txt; exit 1; }
tail -1 $O/gpu_tests.txt
bash tools/gpu_ab_lib.sh ${TAG:-r04z2}/ab ablib/libtlsrec_base.so ablib/libtlsrec_swz.so c4s k4 c4 || exit 1
for v in base swz; do
  (cd /tmp && TLSREC_LIBRARY=$R/ablib/libtlsrec_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof_$v -o run --output-format csv -- python3 $R/bench.py --config c4s --no-cpu --no-e2e --verify 16 > $R/$O/prof_$v.json 2> $R/$O/prof_$v.err) || { echo "prof $v failed"; exit 1; }
  echo $v $(grep bucket_count $O/prof_$v/run_kernel_stats.csv | awk -F'",' '{print $2}' | cut -d, -f1-3)
done
