# dw kernels (hoisted loads) + depthwise rows in the multi-layer pack: numerics, then
# throughput of the depthwise configs and the flagship, and dw kernel times on MV2.
set -x
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_dwconv.py tests/test_gpu_train_layers.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_dw2.log 2>&1 ; rc=$?; tail -5 gpurun_out/pytest_dw2.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 600 python -u benchmarks/throughput.py --configs dkd_cifar_res32x4_res8x4,dkd_cifar_vgg13_mv2,dkd_cifar_res32x4_shuv1,dkd_imagenet_r50_mv1 --steps 60 --warmup 15 --out gpurun_out/tp_dw.jsonl > gpurun_out/tp_dw.log 2>&1 || { tail -30 gpurun_out/tp_dw.log; exit 1; }
cut -c1-200 gpurun_out/tp_dw.jsonl
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_mv2b -o run -- python bench.py --cfg configs/cifar100/dkd/vgg13_mv2.yaml --steps 20 --warmup 10 > gpurun_out/prof_mv2b.log 2>&1 || { tail -20 gpurun_out/prof_mv2b.log; exit 1; }
python scripts/prof_summary.py gpurun_out/prof_mv2b/run_results.db --skip 12 --top 40 --md gpurun_out/prof_mv2b_summary.md | cut -c1-160 | head -24
python scripts/kernel_times.py gpurun_out/prof_mv2b/run_results.db "dw_" > gpurun_out/prof_mv2b_dw.txt
rm -f gpurun_out/prof_mv2b/run_results.db
