#!/bin/bash
# End-of-round measurement on one box (each part under the 20-minute limit):
#   tools/gpu_final.sh rows    -- -m gpu suite, smoke, every DESIGN row
#   tools/gpu_final.sh prof1   -- rocprofv3 stats + PMC (incl. sized reads): c2 c3 c4s k4
#   tools/gpu_final.sh prof1b  -- prof1 for c4s and k4 only
#   tools/gpu_final.sh prof2   -- the same for c4, c2s, DTLS 1.4 KiB AES-128-GCM, stream 1.4 KiB
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
T=${TAG:-r05}
O=gpurun_out/$T
mkdir -p $O
row() {   # name, timeout, command...
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $O/$name.json 2> $O/$name.err || { echo "FAIL $name"; tail -3 $O/$name.err; return 1; }
}
summ() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d.get('roofline',{}); print(sys.argv[2], d.get('value'), r.get('kernel_ms_avg'), r.get('frac'), r.get('traffic'), (d.get('cpu_baseline') or {}).get('value'), d.get('check'))" $O/$1.json $1; }
export PROFILE_RDREQ=1
case "$1" in
rows)
  timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.txt 2>&1 \
      || { echo "gpu tests failed"; tail -20 $O/gpu_tests.txt; exit 1; }
  tail -1 $O/gpu_tests.txt
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { echo "smoke failed"; tail -5 $O/smoke.txt; exit 1; }
  tail -1 $O/smoke.txt
  row c2 400 python3 bench.py && summ c2 &&
  for c in c3 c4 c4s k4 c1 c2s c3d chacha16k gcm192 ccm ccm8 aria256 camellia128; do
    row $c 400 python3 bench.py --config $c --no-e2e && summ $c || exit 1
  done &&
  row stream16 300 python3 tools/bench_stream.py --conns 65536 --recs 16 && cat $O/stream16.json &&
  row count_gpus 60 python3 -c "import bench, json; print(json.dumps({'count_gpus': bench.count_gpus()}))" && cat $O/count_gpus.json &&
  row dist1 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --dist --no-cpu --no-e2e && summ dist1 &&
  row stream4 300 python3 tools/bench_stream.py --conns 65536 --recs 4 && cat $O/stream4.json &&
  row stream16s 300 python3 tools/bench_stream.py --conns 65536 --recs 16 --content 1400 && cat $O/stream16s.json &&
  row stream_cp 300 python3 tools/bench_stream.py --conns 262144 --recs 4 --content 1400 --cipher 3 && cat $O/stream_cp.json &&
  row dtls_small 300 python3 tools/bench_dtls.py && cat $O/dtls_small.json &&
  row dtls_cp 300 python3 tools/bench_dtls.py --cipher 3 && cat $O/dtls_cp.json &&
  row dtls16k 300 python3 tools/bench_dtls.py --content 16384 --recs 4 --cipher 2 && cat $O/dtls16k.json &&
  row keysched 300 python3 tools/bench_keysched.py && cat $O/keysched.json &&
  make -s -C tests/c abi_host &&
  : > $O/latency.jsonl &&
  for a in "2 1.3 16383" "2 1.3 1400" "3 1.3 1400" "1 1.2 1400" "2 1.3 100"; do
    timeout -k 10 120 ./tests/c/abi_host latency $a 2000 >> $O/latency.jsonl || exit 1
  done && for t in 1 16 32; do timeout -k 10 120 ./tests/c/abi_host threads $t 2000 gcm_chacha >> $O/latency.jsonl || exit 1; done &&
  cat $O/latency.jsonl
  ;;
prof1)
  PMC_RECORDS=262144 profiles/run_profile.sh ${T}_c2 > $O/prof_c2.log 2>&1 || { echo "c2 failed"; tail -5 $O/prof_c2.log; exit 1; }
  PMC_RECORDS=262144 profiles/run_profile.sh ${T}_c3 --config c3 > $O/prof_c3.log 2>&1 || { echo "c3 failed"; tail -5 $O/prof_c3.log; exit 1; }
  PMC_RECORDS=4194304 profiles/run_profile.sh ${T}_c4s --config c4s > $O/prof_c4s.log 2>&1 || { echo "c4s failed"; tail -5 $O/prof_c4s.log; exit 1; }
  PMC_RECORDS=262144 profiles/run_profile.sh ${T}_k4 --config k4 > $O/prof_k4.log 2>&1 || { echo "k4 failed"; tail -5 $O/prof_k4.log; exit 1; }
  echo prof1 done
  ;;
prof1b)   # prof1 without c2 / c3 (their kernels unchanged since the last prof1)
  PMC_RECORDS=4194304 profiles/run_profile.sh ${T}_c4s --config c4s > $O/prof_c4s.log 2>&1 || { echo "c4s failed"; tail -5 $O/prof_c4s.log; exit 1; }
  PMC_RECORDS=262144 profiles/run_profile.sh ${T}_k4 --config k4 > $O/prof_k4.log 2>&1 || { echo "k4 failed"; tail -5 $O/prof_k4.log; exit 1; }
  echo prof1b done
  ;;
prof2)
  PMC_RECORDS=4194304 profiles/run_profile.sh ${T}_c4 --config c4 > $O/prof_c4.log 2>&1 || { echo "c4 failed"; tail -5 $O/prof_c4.log; exit 1; }
  PMC_RECORDS=262144 profiles/run_profile.sh ${T}_c2s --config c2s > $O/prof_c2s.log 2>&1 || { echo "c2s failed"; tail -5 $O/prof_c2s.log; exit 1; }
  profiles/run_profile.sh ${T}_dtls_small --cmd tools/bench_dtls.py --steps 3 > $O/prof_dtls.log 2>&1 || { echo "dtls failed"; tail -5 $O/prof_dtls.log; exit 1; }
  profiles/run_profile.sh ${T}_stream16s --cmd tools/bench_stream.py --conns 65536 --recs 16 --content 1400 --steps 3 > $O/prof_stream.log 2>&1 || { echo "stream failed"; tail -5 $O/prof_stream.log; exit 1; }
  profiles/run_profile.sh ${T}_stream16 --cmd tools/bench_stream.py --conns 65536 --recs 16 --steps 3 > $O/prof_stream16.log 2>&1 || { echo "stream16 failed"; tail -5 $O/prof_stream16.log; exit 1; }
  echo prof2 done
  ;;
*) echo "usage: tools/gpu_final.sh rows|prof1|prof1b|prof2"; exit 2;;
esac
