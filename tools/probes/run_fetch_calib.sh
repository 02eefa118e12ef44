#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration passes over tools/probes/fetch_calib (one
# counter group per pass, each under its own time limit); output under
# gpurun_out/<tag>/calib/
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-calib}/calib
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -k 10 60 $R/tools/probes/fetch_calib > $O/expected.json || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/fetch -o run --output-format csv \
    -- $R/tools/probes/fetch_calib > /dev/null || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/write -o run --output-format csv \
    -- $R/tools/probes/fetch_calib > /dev/null || exit 1
timeout -s KILL 60 rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum \
    --kernel-trace -d $O/rdreq -o run --output-format csv -- $R/tools/probes/fetch_calib > /dev/null || exit 1
timeout -s KILL 60 rocprofv3 -L > $O/counters_avail.txt 2>&1 || true
grep -o "TCC_EA0_[A-Z0-9_]*" $O/counters_avail.txt | sort -u > $O/tcc_ea_counters.txt || true
python3 $R/tools/probes/fetch_calib.py $O/expected.json $O/fetch $O/write $O/rdreq > $O/calib.json || exit 1
cat $O/calib.json
