set -o pipefail
mkdir -p gpurun_out; export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_bn_dgrad_sums.py tests/test_gpu_dwconv.py tests/test_gpu_conv1x1_stream.py tests/test_gpu_train_layers.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_mv.log 2>&1; rc=$?; echo "tests rc=$rc"
grep -E "FAILED|passed|failed|Error" gpurun_out/t_mv.log | head -12
[ $rc -ne 0 ] && exit 1
timeout -k 10 600 python benchmarks/throughput.py --configs dkd_imagenet_r50_mv1,dkd_cifar_vgg13_mv2,dot_tiny_r18_mv2 --steps 30 --warmup 10 || exit 1
BYDISP=1 PROF="configs/imagenet/r50_mv1/dkd.yaml:r4_r50_mv1_b" bash scripts/gpu_run.sh
