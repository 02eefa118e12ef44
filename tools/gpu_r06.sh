#!/bin/bash
# Round-6 GPU steps (one box per call; every GPU step under its own timeout,
# chained so the first failure ends the call).
#   tools/gpu_r06.sh base    -- c2 / c4s / c2s lines + stream / DTLS 1.4 KiB rows (HEAD baseline)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
T=${TAG:-r06}
O=gpurun_out/$T
mkdir -p $O
row() {   # name, timeout, command...
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $O/$name.json 2> $O/$name.err || { echo "FAIL $name"; tail -3 $O/$name.err; return 1; }
}
summ() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d.get('roofline') or {}; print(sys.argv[2], d.get('value'), r.get('kernel_ms_avg'), r.get('frac'), r.get('traffic'), (d.get('cpu_baseline') or {}).get('value'), d.get('check'))" $O/$1.json $1; }
case "$1" in
base)
  row c2 300 python3 bench.py --no-cpu --no-e2e && summ c2 &&
  for c in c4s c2s; do row $c 300 python3 bench.py --config $c --no-cpu --no-e2e && summ $c || exit 1; done &&
  row stream16s 300 python3 tools/bench_stream.py --conns 65536 --recs 16 --content 1400 && cat $O/stream16s.json &&
  row dtls_small 300 python3 tools/bench_dtls.py && cat $O/dtls_small.json
  ;;
srv)   # record server: GPU tests, then threads 1/16/32, spin-only (old) vs spin-then-yield (new), ABAB
  timeout -k 10 300 python -u -m pytest tests/test_server_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/srv_tests.txt 2>&1 \
      || { echo "server tests failed"; tail -20 $O/srv_tests.txt; exit 1; }
  tail -1 $O/srv_tests.txt
  : > $O/threads.jsonl
  for rep in 1 2; do for spin in -1 2 20; do for t in 16 32; do
    TLSREC_SERVER_SPIN_US=$spin timeout -k 10 120 ./tests/c/abi_host threads $t 2000 gcm_chacha > $O/t.json || exit 1
    python3 -c "import json,sys; d=json.loads(open('$O/t.json').read()); d['spin_us']=$spin; d['rep']=$rep; print(json.dumps(d))" >> $O/threads.jsonl
  done; done; done
  cat $O/threads.jsonl
  ;;
*) echo "usage: tools/gpu_r06.sh base|srv"; exit 2;;
esac
