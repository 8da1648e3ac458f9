# Teacher look-ahead: equivalence tests, then A/B on the flagship and other configs.
set -x
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_e2e.py -x -q --timeout 120 --timeout-method thread -k "lookahead or graph_matches or native_bf16_graph or trainer_epoch or validation" > gpurun_out/pytest_h.log 2>&1 ; rc=$?; tail -5 gpurun_out/pytest_h.log; [ $rc -eq 0 ] || exit 1
for o in "RUNTIME.TEACHER_LOOKAHEAD auto" "RUNTIME.TEACHER_LOOKAHEAD off" "RUNTIME.TEACHER_LOOKAHEAD auto"; do
  timeout -k 10 300 python bench.py --steps 300 --warmup 30 $o > gpurun_out/bench_h.log 2>&1 || { tail -20 gpurun_out/bench_h.log; exit 1; }
  echo "$o"; grep -h metric gpurun_out/bench_h.log | cut -c60-200
done
timeout -k 10 900 python -u benchmarks/throughput.py --configs kd_cifar_res32x4_res8x4,fitnet_cifar_res32x4_res8x4,reviewkd_cifar_res32x4_res8x4,crd_cifar_res32x4_res8x4,ofd_cifar_res32x4_res8x4,dkd_cifar_vgg13_mv2,reviewkd_imagenet_r34_r18,dkd_imagenet_r50_mv1 --steps 60 --warmup 15 --out gpurun_out/tp_h.jsonl > gpurun_out/tp_h.log 2>&1 || { tail -30 gpurun_out/tp_h.log; exit 1; }
cut -c1-140 gpurun_out/tp_h.jsonl
