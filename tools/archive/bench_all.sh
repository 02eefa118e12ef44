# every bench config once on one box; JSON lines into gpurun_out/bench_<cfg>.json
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err &&
timeout -k 10 300 python bench.py --config c3 > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err &&
timeout -k 10 400 python bench.py --config c4 --no-cpu > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err
