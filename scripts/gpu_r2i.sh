# Look-ahead under DOT's dual replay + multi-rank: tests, then DOT / flagship numbers.
set -x
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_e2e.py tests/test_gpu_multirank.py -x -q --timeout 150 --timeout-method thread -k "lookahead or graph_matches or native_bf16_graph or multirank or replicas" > gpurun_out/pytest_i.log 2>&1 ; rc=$?; tail -5 gpurun_out/pytest_i.log; [ $rc -eq 0 ] || exit 1
for c in configs/cifar100/dot/res32x4_res8x4.yaml configs/cifar100/dkd/res32x4_res8x4.yaml; do
  timeout -k 10 300 python bench.py --cfg $c --steps 300 --warmup 30 > gpurun_out/bench_i.log 2>&1 || { tail -20 gpurun_out/bench_i.log; exit 1; }
  echo $c; grep -h metric gpurun_out/bench_i.log | cut -c60-200
done
timeout -k 10 300 python bench.py --cfg configs/cifar100/dot/res32x4_res8x4.yaml --steps 300 --warmup 30 RUNTIME.TEACHER_LOOKAHEAD off > gpurun_out/bench_i.log 2>&1 || { tail -20 gpurun_out/bench_i.log; exit 1; }
echo dot-off; grep -h metric gpurun_out/bench_i.log | cut -c60-200
