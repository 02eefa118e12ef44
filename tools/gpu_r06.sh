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
tests)   # the stream / DTLS / server GPU tests
  timeout -k 10 500 python -u -m pytest tests/test_stream_gpu.py tests/test_dtls_gpu.py tests/test_server_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/sds_tests.txt 2>&1 \
      || { echo "tests failed"; tail -30 $O/sds_tests.txt; exit 1; }
  tail -1 $O/sds_tests.txt
  ;;
suite)   # the whole -m gpu suite
  timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.txt 2>&1 \
      || { echo "gpu tests failed"; tail -30 $O/gpu_tests.txt; exit 1; }
  tail -1 $O/gpu_tests.txt
  ;;
srv)   # record server: GPU tests, then threads 1/16/32, spin-only (old) vs spin-then-yield (new), ABAB
  timeout -k 10 300 python -u -m pytest tests/test_server_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/srv_tests.txt 2>&1 \
      || { echo "server tests failed"; tail -20 $O/srv_tests.txt; exit 1; }
  tail -1 $O/srv_tests.txt
  : > $O/threads.jsonl
  for rep in 1 2 3; do for spin in ${SPINS:--1 20}; do for t in 16 32; do
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
multiab)   # same-box A/B of several libraries (LIBS) on bench configs (CONFIGS) and rows (ROWS: stream16s dtls_small stream_cp dtls_cp), alternating, REPS reps
  : > $O/multiab.jsonl
  for rep in $(seq ${REPS:-2}); do for ent in $LIBS; do
    lib=${ent%%:*}; envs=""; [ "$ent" != "$lib" ] && envs=$(echo "${ent#*:}" | tr ',' ' ')
    tag=$(basename $lib .so)${envs:+:$envs}
    for c in $CONFIGS; do
      env $envs TLSREC_LIBRARY=$R/$lib timeout -k 10 300 python3 bench.py --config $c --no-cpu --no-e2e --verify 16 > $O/t.json 2> $O/t.err || { echo "FAIL $c $tag"; tail -3 $O/t.err; exit 1; }
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(json.dumps(dict(row=sys.argv[2], lib=sys.argv[3], rep=$rep, value=d['value'], kernel_ms=d['roofline']['kernel_ms_avg'], bad=d['check']['bad_records'])))" $O/t.json $c $tag >> $O/multiab.jsonl
    done
    for name in $ROWS; do
      case $name in
        stream16s) set -- tools/bench_stream.py --conns 65536 --recs 16 --content 1400;;
        stream_cp) set -- tools/bench_stream.py --conns 262144 --recs 4 --content 1400 --cipher 3;;
        dtls_small) set -- tools/bench_dtls.py;;
        dtls_cp) set -- tools/bench_dtls.py --cipher 3;;
      esac
      env $envs TLSREC_LIBRARY=$R/$lib timeout -k 10 200 python3 "$@" --no-cpu > $O/t.json 2> $O/t.err || { echo "FAIL $name $tag"; tail -3 $O/t.err; exit 1; }
      python3 -c "import json; [print(json.dumps(dict(row='$name'+('_enc' if 'encrypt' in d['metric'] else '_dec'), lib='$tag', rep=$rep, value=d['value'], kernel_ms=(d.get('roofline') or {}).get('kernel_ms_avg'), check=d.get('check')))) for d in map(json.loads, open('$O/t.json'))]" >> $O/multiab.jsonl
    done
  done; done
  python3 tools/ab_summary.py $O/multiab.jsonl
  ;;
fusedab)   # one-pass receive framing: stream / DTLS GPU tests, A/B (TLSREC_RX_FUSED 0 / 1) on the receive rows, kernel trace
  timeout -k 10 500 python -u -m pytest tests/test_stream_gpu.py tests/test_dtls_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/stream_tests.txt 2>&1 \
      || { echo "stream tests failed"; tail -30 $O/stream_tests.txt; exit 1; }
  tail -1 $O/stream_tests.txt
  : > $O/fusedab.jsonl
  for rep in 1 2; do for f in 0 1; do
    for row in "stream_cp tools/bench_stream.py --conns 262144 --recs 4 --content 1400 --cipher 3" "stream16s tools/bench_stream.py --conns 65536 --recs 16 --content 1400" "dtls_cp tools/bench_dtls.py --cipher 3" "dtls_small tools/bench_dtls.py"; do
      set -- $row; name=$1; shift
      TLSREC_RX_FUSED=$f timeout -k 10 200 python3 "$@" --no-cpu > $O/t.json 2> $O/t.err || { echo "FAIL $name"; tail -3 $O/t.err; exit 1; }
      python3 -c "import json; [print(json.dumps(dict(row='$name'+('_enc' if 'encrypt' in d['metric'] else '_dec'), lib='fused$f', rep=$rep, value=d['value'], kernel_ms=(d.get('roofline') or {}).get('kernel_ms_avg'), check=d.get('check')))) for d in map(json.loads, open('$O/t.json'))]" >> $O/fusedab.jsonl
    done
  done; done
  python3 tools/ab_summary.py $O/fusedab.jsonl
  cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof_stream_cp -o run --output-format csv -- python3 $R/tools/bench_stream.py --conns 262144 --recs 4 --content 1400 --cipher 3 --no-cpu --steps 3 > $R/$O/prof_stream_cp.json 2>&1 && \
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof_dtls_cp -o run --output-format csv -- python3 $R/tools/bench_dtls.py --cipher 3 --no-cpu --steps 3 > $R/$O/prof_dtls_cp.json 2>&1 && cd $R && echo prof done
  ;;
rowab)   # same-box A/B of libraries on the stream / DTLS rows: LIBS (env, space separated)
  : > $O/rowab.jsonl
  for rep in 1 2; do for lib in $LIBS; do
    tag=$(basename $lib .so)
    for row in "stream16s tools/bench_stream.py --conns 65536 --recs 16 --content 1400" "dtls_small tools/bench_dtls.py" "stream_cp tools/bench_stream.py --conns 262144 --recs 4 --content 1400 --cipher 3" "dtls_cp tools/bench_dtls.py --cipher 3"; do
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
rows)   # the round's one full sweep on the final build: -m gpu suite, smoke, every bench row
  timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.txt 2>&1 \
      || { echo "gpu tests failed"; tail -20 $O/gpu_tests.txt; exit 1; }
  tail -1 $O/gpu_tests.txt
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { echo "smoke failed"; tail -5 $O/smoke.txt; exit 1; }
  tail -1 $O/smoke.txt
  row c2 400 python3 bench.py && summ c2 &&
  for c in c3 c4 c4s k4 c1 c2s c3d chacha16k gcm192 ccm ccm8 aria256 camellia128; do
    row $c 400 python3 bench.py --config $c --no-e2e && summ $c || exit 1
  done
  [ "${ROWS_SPLIT:-0}" = 1 ] && { echo "rows part 1 done"; exit 0; }
  ;&
rows2)   # the second half of rows (ROWS_SPLIT=1 rows, then rows2: each call under gpurun's 20-minute limit)
  row count_gpus 60 python3 -c "import bench, json; print(json.dumps({'count_gpus': bench.count_gpus()}))" && cat $O/count_gpus.json &&
  row dist1 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --dist && summ dist1 &&
  row stream16 300 python3 tools/bench_stream.py --conns 65536 --recs 16 &&
  row stream4 300 python3 tools/bench_stream.py --conns 65536 --recs 4 &&
  row stream16s 300 python3 tools/bench_stream.py --conns 65536 --recs 16 --content 1400 &&
  row stream_cp 300 python3 tools/bench_stream.py --conns 262144 --recs 4 --content 1400 --cipher 3 &&
  row dtls_small 300 python3 tools/bench_dtls.py &&
  row dtls_cp 300 python3 tools/bench_dtls.py --cipher 3 &&
  row dtls16k 300 python3 tools/bench_dtls.py --content 16384 --recs 4 --cipher 2 &&
  row keysched 300 python3 tools/bench_keysched.py &&
  make -s -C tests/c abi_host &&
  : > $O/latency.jsonl &&
  for a in "2 1.3 16383" "2 1.3 1400" "3 1.3 1400" "1 1.2 1400" "2 1.3 100"; do
    timeout -k 10 120 ./tests/c/abi_host latency $a 2000 >> $O/latency.jsonl || exit 1
  done && for t in 1 16 32; do timeout -k 10 120 ./tests/c/abi_host threads $t 2000 gcm_chacha >> $O/latency.jsonl || exit 1; done &&
  python3 profiles/rows_table.py $O
  ;;
prof)   # rocprofv3 kernel stats + PMC passes on the final build
  export PROFILE_RDREQ=1
  PMC_RECORDS=262144 profiles/run_profile.sh ${T}_c2 > $O/prof_c2.log 2>&1 || { echo "c2 failed"; tail -5 $O/prof_c2.log; exit 1; }
  PMC_RECORDS=262144 profiles/run_profile.sh ${T}_c2s --config c2s > $O/prof_c2s.log 2>&1 || { echo "c2s failed"; tail -5 $O/prof_c2s.log; exit 1; }
  PMC_RECORDS=4194304 profiles/run_profile.sh ${T}_c4s --config c4s > $O/prof_c4s.log 2>&1 || { echo "c4s failed"; tail -5 $O/prof_c4s.log; exit 1; }
  profiles/run_profile.sh ${T}_dtls_small --cmd tools/bench_dtls.py --steps 3 --no-cpu > $O/prof_dtls.log 2>&1 || { echo "dtls failed"; tail -5 $O/prof_dtls.log; exit 1; }
  profiles/run_profile.sh ${T}_stream16s --cmd tools/bench_stream.py --conns 65536 --recs 16 --content 1400 --steps 3 --no-cpu > $O/prof_stream.log 2>&1 || { echo "stream failed"; tail -5 $O/prof_stream.log; exit 1; }
  echo prof done
  ;;
profa)   # final-build profiles, part 1: c2 (headline), c2s, c4s (kernel stats + PMC passes, cache passes for c4s)
  export PROFILE_RDREQ=1
  PMC_RECORDS=262144 profiles/run_profile.sh ${T}_c2 > $O/prof_c2.log 2>&1 || { echo "c2 failed"; tail -5 $O/prof_c2.log; exit 1; }
  PMC_RECORDS=262144 profiles/run_profile.sh ${T}_c2s --config c2s > $O/prof_c2s.log 2>&1 || { echo "c2s failed"; tail -5 $O/prof_c2s.log; exit 1; }
  PROFILE_CACHE=1 PMC_RECORDS=4194304 profiles/run_profile.sh ${T}_c4s --config c4s > $O/prof_c4s.log 2>&1 || { echo "c4s failed"; tail -5 $O/prof_c4s.log; exit 1; }
  echo profa done
  ;;
profb)   # final-build profiles, part 2: DTLS and stream 16 x 1.4 KiB AES rows (+ cache passes)
  export PROFILE_RDREQ=1 PROFILE_CACHE=1
  profiles/run_profile.sh ${T}_dtls_small --cmd tools/bench_dtls.py --steps 3 --no-cpu > $O/prof_dtls.log 2>&1 || { echo "dtls failed"; tail -5 $O/prof_dtls.log; exit 1; }
  profiles/run_profile.sh ${T}_stream16s --cmd tools/bench_stream.py --conns 65536 --recs 16 --content 1400 --steps 3 --no-cpu > $O/prof_stream.log 2>&1 || { echo "stream failed"; tail -5 $O/prof_stream.log; exit 1; }
  echo profb done
  ;;
profsmall)   # the paired-pass rows only: c4s, DTLS and stream 16 x 1.4 KiB (+ cache / UTCL1 passes)
  export PROFILE_RDREQ=1 PROFILE_CACHE=1
  PMC_RECORDS=4194304 profiles/run_profile.sh ${T}_c4s --config c4s > $O/prof_c4s.log 2>&1 || { echo "c4s failed"; tail -5 $O/prof_c4s.log; exit 1; }
  profiles/run_profile.sh ${T}_dtls_small --cmd tools/bench_dtls.py --steps 3 --no-cpu > $O/prof_dtls.log 2>&1 || { echo "dtls failed"; tail -5 $O/prof_dtls.log; exit 1; }
  profiles/run_profile.sh ${T}_stream16s --cmd tools/bench_stream.py --conns 65536 --recs 16 --content 1400 --steps 3 --no-cpu > $O/prof_stream.log 2>&1 || { echo "stream failed"; tail -5 $O/prof_stream.log; exit 1; }
  echo profsmall done
  ;;
*) echo "usage: tools/gpu_r06.sh base|suite|srv|profsmall|frame|libab|rowab|rxab|tests|rows|prof"; exit 2;;
esac
