set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05a; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_server_gpu.py tests/test_coalesce_gpu.py tests/test_engine_hygiene_gpu.py tests/test_bench_launcher.py > $O/tests1.txt 2>&1 || { tail -30 $O/tests1.txt; exit 1; }
tail -2 $O/tests1.txt
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_evp_parity_gpu.py -k full_size > $O/tests2.txt 2>&1 || { tail -30 $O/tests2.txt; exit 1; }
tail -2 $O/tests2.txt
timeout -k 10 300 python bench.py > $O/c2.json 2> $O/c2.err || { tail -5 $O/c2.err; exit 1; }
cat $O/c2.json
