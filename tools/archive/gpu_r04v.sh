#!/bin/bash
# r04: key-schedule row bisect, same box: r03, r04a (3ad90bd), lane powers (e5b95fb), HEAD (ladder); keysetup kernel time each
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/${TAG:-r04v}
mkdir -p $O
export TMPDIR=/tmp
for v in r03 lad w6 w8 lad w6 w8; do
  TLSREC_LIBRARY=$R/ablib/libtlsrec_$v.so timeout -k 10 300 python3 tools/bench_keysched.py > $O/ks_$v.json 2> $O/ks_$v.err || { echo "keysched $v failed"; tail -3 $O/ks_$v.err; exit 1; }
  (cd /tmp && TLSREC_LIBRARY=$R/ablib/libtlsrec_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof_$v -o run --output-format csv -- python3 $R/tools/bench_keysched.py > $R/$O/prof_$v.json 2> $R/$O/prof_$v.err) || { echo "prof $v failed"; exit 1; }
  echo $v $(python3 -c "import json,sys; print(json.loads(open(sys.argv[1]).read())['value'])" $O/ks_$v.json) $(grep keysetup $O/prof_$v/run_kernel_stats.csv | awk -F'",' '{print $2}' | cut -d, -f1-3)
done
