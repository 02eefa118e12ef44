#!/bin/bash
# Record server thread-scaling probe: the box's CPU share, then the wait
# modes (TLSREC_SERVER_SPIN_US -1 spin, -2 yield past the CPU count; r06 also
# measured -3, spin tokens + naps, since removed) at 16 and 32 threads,
# interleaved, each under its own limit.
set -o pipefail
O=gpurun_out/${TAG:-srvp}
mkdir -p $O
{ nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null || echo "no cpu.max"; python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)))"; } > $O/cpu.txt
cat $O/cpu.txt
: > $O/probe.jsonl
for rep in 1 2 3; do for mode in ${MODES:--1 -2}; do for t in 16 32; do
  TLSREC_SERVER_SPIN_US=$mode timeout -k 10 120 ./tests/c/abi_host threads $t ${RECS:-4000} gcm_chacha > $O/t.json || exit 1
  python3 -c "import json; d=json.loads(open('$O/t.json').read()); d['mode']=$mode; d['rep']=$rep; print(json.dumps(d))" >> $O/probe.jsonl
done; done; done
python3 -c "
import json
for l in open('$O/probe.jsonl'):
    d=json.loads(l); print(d['rep'], 'mode', d['mode'], 'threads', d['threads'], d['round_trips_per_s'], 'launches', d['server_launches'], 'fallback', d['server_fallback'])"
