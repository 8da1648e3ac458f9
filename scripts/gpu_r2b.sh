# Round-2 (session 2) check: dw/BN kernel numerics, flagship bench, MV2 + ImageNet
# kernel profiles with per-grid times of the dw / BN kernels.
set -x
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_dwconv.py tests/test_gpu_train_layers.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_dw_bn.log 2>&1 ; rc=$?; tail -5 gpurun_out/pytest_dw_bn.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --steps 200 --warmup 30 > gpurun_out/bench_200.log 2>&1 || { tail -20 gpurun_out/bench_200.log; exit 1; }
grep -h metric gpurun_out/bench_200.log | cut -c1-200
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for cfg in configs/cifar100/dkd/vgg13_mv2.yaml; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_mv2 -o run -- python bench.py --cfg $cfg --steps 20 --warmup 10 > gpurun_out/prof_mv2.log 2>&1 || { tail -20 gpurun_out/prof_mv2.log; exit 1; }
  grep -h metric gpurun_out/prof_mv2.log | cut -c1-160
  python scripts/prof_summary.py gpurun_out/prof_mv2/run_results.db --skip 12 --top 40 --md gpurun_out/prof_mv2_summary.md | cut -c1-160 | head -30
  python scripts/kernel_times.py gpurun_out/prof_mv2/run_results.db "dw_" > gpurun_out/prof_mv2_dw.txt
  python scripts/kernel_times.py gpurun_out/prof_mv2/run_results.db "bn_" > gpurun_out/prof_mv2_bn.txt
  rm -f gpurun_out/prof_mv2/run_results.db
done
cat gpurun_out/prof_mv2_dw.txt
