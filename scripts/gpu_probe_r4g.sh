set -o pipefail
mkdir -p gpurun_out; export PYTHONPATH=$PWD TMPDIR=/tmp
C=dkd_imagenet_r50_mv1,dkd_cifar_vgg13_mv2
for combo in "0 0 8" "1 0 8" "0 1 8" "1 1 8" "0 0 4" "1 1 4"; do
  set -- $combo
  echo "VIN=$1 BNB=$2 VMAX=$3"
  MDA_DW_VIN=$1 MDA_DW_BNB=$2 MDA_DW_VMAX=$3 timeout -k 10 300 python benchmarks/throughput.py --configs $C --steps 30 --warmup 10 | cut -c1-120 || exit 1
done
