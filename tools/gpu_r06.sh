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
  for rep in 1 2 3; do for spin in -1 20; do for t in 16 32; do
    TLSREC_SERVER_SPIN_US=$spin timeout -k 10 120 ./tests/c/abi_host threads $t 2000 gcm_chacha > $O/t.json || exit 1
    python3 -c "import json,sys; d=json.loads(open('$O/t.json').read()); d['spin_us']=$spin; d['rep']=$rep; print(json.dumps(d))" >> $O/threads.jsonl
  done; done; done
  cat $O/threads.jsonl
  ;;
frame)   # fused receive framing: stream GPU tests, A/B of the framing paths, kernel trace
  timeout -k 10 400 python -u -m pytest tests/test_stream_gpu.py tests/test_dtls_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/stream_tests.txt 2>&1 \
      || { echo "stream tests failed"; tail -30 $O/stream_tests.txt; exit 1; }
  tail -1 $O/stream_tests.txt
  : > $O/frame_ab.jsonl
  for rep in 1 2; do for f in 0 1; do
    TLSREC_RX_GROUPWALK=$f TLSREC_GROUPED=$f timeout -k 10 200 python3 tools/bench_stream.py --conns 262144 --recs 4 --content 1400 --cipher 3 --no-cpu > $O/t.json || exit 1
    python3 -c "import json; [print(json.dumps(dict(json.loads(l), fused=$f, rep=$rep, row='stream_cp'))) for l in open('$O/t.json')]" >> $O/frame_ab.jsonl
    TLSREC_RX_GROUPWALK=$f TLSREC_GROUPED=$f timeout -k 10 200 python3 tools/bench_stream.py --conns 65536 --recs 16 --content 1400 --no-cpu > $O/t.json || exit 1
    python3 -c "import json; [print(json.dumps(dict(json.loads(l), fused=$f, rep=$rep, row='stream16s'))) for l in open('$O/t.json')]" >> $O/frame_ab.jsonl
    TLSREC_RX_GROUPWALK=$f TLSREC_GROUPED=$f timeout -k 10 200 python3 tools/bench_dtls.py --cipher 3 --no-cpu > $O/t.json || exit 1
    python3 -c "import json; [print(json.dumps(dict(json.loads(l), fused=$f, rep=$rep, row='dtls_cp'))) for l in open('$O/t.json')]" >> $O/frame_ab.jsonl
    TLSREC_RX_GROUPWALK=$f TLSREC_GROUPED=$f timeout -k 10 200 python3 tools/bench_dtls.py --no-cpu > $O/t.json || exit 1
    python3 -c "import json; [print(json.dumps(dict(json.loads(l), fused=$f, rep=$rep, row='dtls_small'))) for l in open('$O/t.json')]" >> $O/frame_ab.jsonl
  done; done
  python3 -c "
import json
for l in open('$O/frame_ab.jsonl'):
    d=json.loads(l); print(d['row'], d['metric'].split()[2], 'fused', d['fused'], d['value'], d['ms_per_call'], (d.get('roofline') or {}).get('kernel_ms_avg'))"
  cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof_frame -o run --output-format csv -- python3 $R/tools/bench_stream.py --conns 262144 --recs 4 --content 1400 --cipher 3 --no-cpu --steps 3 > $R/$O/prof_frame.json 2>&1 && \
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof_frame_dtls -o run --output-format csv -- python3 $R/tools/bench_dtls.py --cipher 3 --no-cpu --steps 3 > $R/$O/prof_frame_dtls.json 2>&1 && cd $R
  ;;
libab)   # same-box A/B of two libraries on bench.py configs: LIBA LIBB CONFIGS (env)
  : > $O/libab.txt
  for c in $CONFIGS; do for lib in $LIBA $LIBB $LIBB $LIBA; do
    tag=$(basename $lib .so)
    TLSREC_LIBRARY=$R/$lib timeout -k 10 300 python3 bench.py --config $c --no-cpu --no-e2e --verify 16 > $O/t.json 2> $O/t.err || { echo "FAIL $c $tag"; tail -3 $O/t.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], d['value'], d['roofline']['kernel_ms_avg'], d['check']['bad_records'])" $O/t.json $c $tag | tee -a $O/libab.txt
  done; done
  ;;
rowab)   # same-box A/B of libraries on the stream / DTLS rows: LIBS (env, space separated)
  : > $O/rowab.jsonl
  for rep in 1 2; do for lib in $LIBS; do
    tag=$(basename $lib .so)
    for row in "stream16s tools/bench_stream.py --conns 65536 --recs 16 --content 1400" "dtls_small tools/bench_dtls.py"; do
      set -- $row; name=$1; shift
      TLSREC_LIBRARY=$R/$lib timeout -k 10 200 python3 "$@" --no-cpu > $O/t.json 2> $O/t.err || { echo "FAIL $name $tag"; tail -3 $O/t.err; exit 1; }
      python3 -c "import json; [print(json.dumps(dict(json.loads(l), lib='$tag', rep=$rep, row='$name'))) for l in open('$O/t.json')]" >> $O/rowab.jsonl
    done
  done; done
  python3 -c "
import json
for l in open('$O/rowab.jsonl'):
    d=json.loads(l); print(d['row'], d['metric'].split()[-7] if 0 else d['metric'][:40], d['lib'], d['value'], d['ms_per_call'], (d.get('roofline') or {}).get('kernel_ms_avg'), d['check'])"
  ;;
rxab)   # receive / send rows under the framing toggles: GROUPWALK x GROUPED
  timeout -k 10 400 python -u -m pytest tests/test_stream_gpu.py tests/test_dtls_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/stream_tests.txt 2>&1 \
      || { echo "stream tests failed"; tail -30 $O/stream_tests.txt; exit 1; }
  tail -1 $O/stream_tests.txt
  : > $O/rxab.jsonl
  for rep in 1 2; do for gw in 0 1; do for gr in 0 1; do
    for row in "stream_cp tools/bench_stream.py --conns 262144 --recs 4 --content 1400 --cipher 3" "stream16s tools/bench_stream.py --conns 65536 --recs 16 --content 1400" "dtls_cp tools/bench_dtls.py --cipher 3" "dtls_small tools/bench_dtls.py"; do
      set -- $row; name=$1; shift
      TLSREC_RX_GROUPWALK=$gw TLSREC_GROUPED=$gr timeout -k 10 200 python3 "$@" --no-cpu > $O/t.json 2> $O/t.err || { echo "FAIL $name"; tail -3 $O/t.err; exit 1; }
      python3 -c "import json; [print(json.dumps(dict(json.loads(l), gw=$gw, gr=$gr, rep=$rep, row='$name'))) for l in open('$O/t.json')]" >> $O/rxab.jsonl
    done
  done; done; done
  python3 -c "
import json
for l in open('$O/rxab.jsonl'):
    d=json.loads(l); print(d['row'], d['metric'][:40], 'gw', d['gw'], 'gr', d['gr'], d['value'], d['ms_per_call'], (d.get('roofline') or {}).get('kernel_ms_avg'))"
  cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof_rx_stream -o run --output-format csv -- python3 $R/tools/bench_stream.py --conns 262144 --recs 4 --content 1400 --cipher 3 --no-cpu --steps 3 > $R/$O/prof_rx_stream.json 2>&1 && \
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof_rx_dtls -o run --output-format csv -- python3 $R/tools/bench_dtls.py --no-cpu --steps 3 > $R/$O/prof_rx_dtls.json 2>&1 && cd $R
  ;;
*) echo "usage: tools/gpu_r06.sh base|srv|frame|libab|rowab|rxab"; exit 2;;
esac
