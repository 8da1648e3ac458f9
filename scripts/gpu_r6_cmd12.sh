# halo-narrow default + conv / BN tests after the halo2 deletion + R50->MV1 BN apply width
export PYTHONPATH=$PWD TMPDIR=/tmp
TESTS="tests/test_gpu_conv.py tests/test_gpu_bn_dgrad_sums.py" ARMS=" ;MDA_HALO_NARROW=1" ROUNDS=2 bash scripts/gpu_r6_ab.sh || exit 1
ARMS=" ;MDA_HALO_NARROW=1" ROUNDS=1 BENCH_ARGS="--cfg configs/cifar100/vanilla.yaml DISTILLER.STUDENT resnet8x4" bash scripts/gpu_r6_ab.sh || exit 1
ARMS=" ;MDA_HALO_NARROW=1" ROUNDS=1 BENCH_ARGS="--cfg configs/cifar100/dot/res32x4_res8x4.yaml" bash scripts/gpu_r6_ab.sh || exit 1
for v in 0 4; do
  MDA_BN_APPLY_V=$v timeout -k 10 300 python benchmarks/throughput.py --configs dkd_imagenet_r50_mv1 --steps 20 --warmup 8 2>/dev/null | grep "^{" | cut -c1-200 || exit 1
done
