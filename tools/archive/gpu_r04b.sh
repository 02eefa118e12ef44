#!/bin/bash
# r04 profiling pass 1: calibration with the sized read-request counters, then
# kernel stats + PMC passes of c2, c3, c4s, k4 (build of this commit)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
T=${TAG:-r04b}
O=gpurun_out/$T
mkdir -p $O
tools/probes/run_fetch_calib.sh $T > $O/calib.log 2>&1 && RDQ=1 || { RDQ=0; echo "calib (sized counters) failed"; tail -3 $O/calib.log; }
python3 -c "
import json; d=json.load(open('$O/calib/calib.json'))
print({k: (v.get('fetch_factor'), v.get('rdreq_sized_factor')) for k, v in d.items()})" 2>/dev/null || true
export PROFILE_RDREQ=$RDQ
for c in c2 c3 c4s k4; do
  case $c in c4s) export PMC_RECORDS=4194304;; *) export PMC_RECORDS=262144;; esac
  profiles/run_profile.sh ${T}_$c --config $c > $O/prof_$c.log 2>&1 || { echo "profile $c failed"; tail -5 $O/prof_$c.log; exit 1; }
  echo "profiled $c"
done
