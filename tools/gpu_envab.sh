#!/bin/bash
# Same-box environment-variable A/B (runs a, b, b, a):
#   tools/gpu_envab.sh <outdir> "VAR=a" "VAR=b" <row>...
# row = a bench.py config (c4s, k4, ...) or one of dtls_small, stream16s,
# stream4, stream16, stream_cp, dtls_cp, dtls16k (tools/bench_dtls.py /
# bench_stream.py shapes of DESIGN 5.0).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/$1; A=$2; B=$3; shift 3
mkdir -p $O
for row in "$@"; do
  case $row in
    dtls_small) cmd=(python3 tools/bench_dtls.py) ;;
    stream16s) cmd=(python3 tools/bench_stream.py --conns 65536 --recs 16 --content 1400) ;;
    stream4) cmd=(python3 tools/bench_stream.py --conns 65536 --recs 4) ;;
    stream16) cmd=(python3 tools/bench_stream.py --conns 65536 --recs 16) ;;
    stream_cp) cmd=(python3 tools/bench_stream.py --conns 262144 --recs 4 --content 1400 --cipher 3) ;;
    dtls_cp) cmd=(python3 tools/bench_dtls.py --cipher 3) ;;
    dtls16k) cmd=(python3 tools/bench_dtls.py --content 16384 --recs 4 --cipher 2) ;;
    *) cmd=(python3 bench.py --config $row --no-cpu --no-e2e --verify 16) ;;
  esac
  k=0
  for v in "$A" "$B" "$B" "$A"; do
    k=$((k + 1))
    f=$O/$row.$k.${v//[^A-Za-z0-9_]/_}.json
    env $v timeout -k 10 300 "${cmd[@]}" > $f 2> $f.err || { echo "FAIL $row $v"; tail -3 $f.err; exit 1; }
    python3 - "$f" "$row" "$v" <<'PY'
import json, sys
vals = []
for ln in open(sys.argv[1]).read().splitlines():
    if ln.startswith("{"):
        d = json.loads(ln)
        vals.append("%s=%s" % (d.get("metric", "?").split(" throughput")[0].split()[-1], d.get("value")))
        if isinstance(d.get("check"), dict) and d["check"].get("bad_records"):
            vals.append("BAD=%s" % d["check"]["bad_records"])
print(sys.argv[2], sys.argv[3], " ".join(vals))
PY
  done
done
