# Weight-gradient side stream in the captured backward: numerics, then A/B on the flagship,
# DOT, and the ImageNet / depthwise configs.
set -x
mkdir -p gpurun_out
[ -n "$SKIP_TESTS" ] || timeout -k 10 600 python -u -m pytest tests/test_gpu_e2e.py tests/test_gpu_multirank.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_g.log 2>&1 ; rc=$?; tail -5 gpurun_out/pytest_g.log; [ $rc -eq 0 ] || exit 1
for o in "RUNTIME.WGRAD_STREAM auto" "RUNTIME.WGRAD_STREAM on" "RUNTIME.WGRAD_STREAM auto"; do
  timeout -k 10 300 python bench.py --steps 300 --warmup 30 $o > gpurun_out/bench_g.log 2>&1 || { tail -20 gpurun_out/bench_g.log; exit 1; }
  echo "$o"; grep -h metric gpurun_out/bench_g.log | cut -c100-190
done
timeout -k 10 300 python bench.py --cfg configs/cifar100/dot/res32x4_res8x4.yaml --steps 200 --warmup 30 > gpurun_out/bench_g.log 2>&1 || { tail -20 gpurun_out/bench_g.log; exit 1; }
echo dot; grep -h metric gpurun_out/bench_g.log | cut -c100-190
timeout -k 10 900 python -u benchmarks/throughput.py --configs reviewkd_imagenet_r34_r18,dkd_imagenet_r50_mv1,dkd_cifar_vgg13_mv2,dkd_cifar_wrn40_2_wrn16_2,crd_cifar_res32x4_res8x4 --steps 60 --warmup 15 --out gpurun_out/tp_g.jsonl > gpurun_out/tp_g.log 2>&1 || { tail -30 gpurun_out/tp_g.log; exit 1; }
cut -c1-140 gpurun_out/tp_g.jsonl
