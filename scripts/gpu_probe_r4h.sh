set -o pipefail
mkdir -p gpurun_out; export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_bn_dgrad_sums.py tests/test_gpu_dwconv.py tests/test_gpu_conv1x1_stream.py tests/test_gpu_train_layers.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_mv2.log 2>&1; rc=$?; echo "tests rc=$rc"
grep -E "FAILED|passed|failed|Error" gpurun_out/t_mv2.log | head -12
[ $rc -ne 0 ] && exit 1
timeout -k 10 300 python scripts/conv_microbench.py --set mv1 --graph --iters 30 --ops fwd,mio --json gpurun_out/cmb_mv1b.json > gpurun_out/cmb_mv1b.log 2>&1 || exit 1
head -2 gpurun_out/cmb_mv1b.log | cut -c1-200
timeout -k 10 900 python benchmarks/throughput.py --configs dkd_imagenet_r50_mv1,dkd_cifar_vgg13_mv2,dkd_cifar_res32x4_shuv1,dot_cifar_res32x4_shuv2,dot_tiny_r18_mv2,dot_tiny_r18_shuv2 --steps 30 --warmup 10 | cut -c1-160
