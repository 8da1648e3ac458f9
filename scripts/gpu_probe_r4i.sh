set -o pipefail
mkdir -p gpurun_out; export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_dwconv.py tests/test_gpu_bn_dgrad_sums.py tests/test_gpu_train_layers.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_dwt.log 2>&1; rc=$?; echo "tests rc=$rc"
grep -E "FAILED|passed|failed|Error|assert" gpurun_out/t_dwt.log | head -12
[ $rc -ne 0 ] && exit 1
C=dkd_imagenet_r50_mv1,dkd_cifar_vgg13_mv2
for combo in "1 40" "1 64" "1 24" "0 40"; do
  set -- $combo
  echo "TILE=$1 KB=$2"
  MDA_DW_TILE=$1 MDA_DW_TILE_KB=$2 timeout -k 10 300 python benchmarks/throughput.py --configs $C --steps 30 --warmup 10 | cut -c1-110 || exit 1
done
