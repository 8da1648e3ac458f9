# After the look-ahead fallback change: e2e + multirank + train-layer tests, bench.
set -x
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests/test_gpu_e2e.py tests/test_gpu_multirank.py tests/test_gpu_relation.py -x -q --timeout 150 --timeout-method thread > gpurun_out/pytest_l.log 2>&1 ; rc=$?; tail -4 gpurun_out/pytest_l.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py > gpurun_out/bench_l.log 2>&1 || { tail -20 gpurun_out/bench_l.log; exit 1; }
grep -h metric gpurun_out/bench_l.log | cut -c1-200
