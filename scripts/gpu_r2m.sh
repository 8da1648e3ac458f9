# Deferred multi-layer wgrad reductions: graph==eager tests, then A/B.
set -x
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests/test_gpu_e2e.py tests/test_gpu_multirank.py tests/test_gpu_conv.py -x -q --timeout 150 --timeout-method thread > gpurun_out/pytest_m.log 2>&1 ; rc=$?; tail -4 gpurun_out/pytest_m.log; [ $rc -eq 0 ] || exit 1
for o in "RUNTIME.WGRAD_DEFER True" "RUNTIME.WGRAD_DEFER False" "RUNTIME.WGRAD_DEFER True" "RUNTIME.WGRAD_DEFER False"; do
  timeout -k 10 300 python bench.py --steps 300 --warmup 30 $o > gpurun_out/bench_m.log 2>&1 || { tail -20 gpurun_out/bench_m.log; exit 1; }
  echo "$o"; grep -h metric gpurun_out/bench_m.log | cut -c100-190
done
for o in "RUNTIME.WGRAD_DEFER True" "RUNTIME.WGRAD_DEFER False"; do
  timeout -k 10 300 python bench.py --cfg configs/cifar100/dot/res32x4_res8x4.yaml --steps 300 --warmup 30 $o > gpurun_out/bench_m.log 2>&1 || { tail -20 gpurun_out/bench_m.log; exit 1; }
  echo "dot $o"; grep -h metric gpurun_out/bench_m.log | cut -c100-190
done
timeout -k 10 600 python -u benchmarks/throughput.py --configs dkd_cifar_vgg13_mv2,dkd_cifar_wrn40_2_wrn16_2,dkd_imagenet_r50_mv1 --steps 60 --warmup 15 --out gpurun_out/tp_m.jsonl > gpurun_out/tp_m.log 2>&1 || { tail -30 gpurun_out/tp_m.log; exit 1; }
cut -c1-120 gpurun_out/tp_m.jsonl
