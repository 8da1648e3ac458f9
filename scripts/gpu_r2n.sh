# Batched input copies: e2e + multirank tests, bench x3.
set -x
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests/test_gpu_e2e.py tests/test_gpu_multirank.py -x -q --timeout 150 --timeout-method thread > gpurun_out/pytest_n.log 2>&1 ; rc=$?; tail -3 gpurun_out/pytest_n.log; [ $rc -eq 0 ] || exit 1
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 300 --warmup 30 > gpurun_out/bench_n.log 2>&1 || { tail -20 gpurun_out/bench_n.log; exit 1; }
  grep -h metric gpurun_out/bench_n.log | cut -c100-190
done
timeout -k 10 300 python bench.py --cfg configs/cifar100/dot/res32x4_res8x4.yaml --steps 300 --warmup 30 > gpurun_out/bench_n.log 2>&1 || { tail -20 gpurun_out/bench_n.log; exit 1; }
grep -h metric gpurun_out/bench_n.log | cut -c100-190
