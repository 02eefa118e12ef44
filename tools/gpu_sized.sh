set -o pipefail
mkdir -p gpurun_out/sz
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/sz/tests.txt 2>&1 || { tail -20 gpurun_out/sz/tests.txt; exit 1; }
tail -1 gpurun_out/sz/tests.txt
for c in c4s c4 k4 c2 c3; do
  timeout -k 10 300 python bench.py --config $c --no-cpu --no-e2e > gpurun_out/sz/$c.json 2> gpurun_out/sz/$c.err || { tail -5 gpurun_out/sz/$c.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['roofline']['frac'], d['check'])" gpurun_out/sz/$c.json $c
done
