# PyTorch-path param grads batched in captured backwards: tests, then A/B on configs with torch layers.
set -x
mkdir -p gpurun_out
MDA_BATCH_TORCH_GRADS=1 timeout -k 10 800 python -u -m pytest tests/test_gpu_e2e.py tests/test_gpu_multirank.py -x -q --timeout 150 --timeout-method thread > gpurun_out/pytest_o.log 2>&1 ; rc=$?; tail -3 gpurun_out/pytest_o.log; [ $rc -eq 0 ] || exit 1
for o in on off; do
[ $o = on ] && export MDA_BATCH_TORCH_GRADS=1 || export MDA_BATCH_TORCH_GRADS=0
timeout -k 10 900 python -u benchmarks/throughput.py --configs dkd_cifar_res32x4_res8x4,dkd_cifar_res32x4_shuv1,dkd_cifar_vgg13_mv2,fitnet_cifar_res32x4_res8x4,crd_cifar_res32x4_res8x4,vid_cifar_res32x4_res8x4,ofd_cifar_res32x4_res8x4 --steps 60 --warmup 15 --out gpurun_out/tp_o.jsonl > gpurun_out/tp_o.log 2>&1 || { tail -30 gpurun_out/tp_o.log; exit 1; }
echo "batch torch grads: $o"; cut -c1-120 gpurun_out/tp_o.jsonl; rm -f gpurun_out/tp_o.jsonl
done
