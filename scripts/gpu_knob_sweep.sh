set -o pipefail
mkdir -p gpurun_out; export PYTHONPATH=$PWD TMPDIR=/tmp
run() {  # label env... -- configs
  local label=$1; shift
  echo "== $label"
  env "$@" timeout -k 10 300 python benchmarks/throughput.py --configs $CFGS --steps 100 --warmup 20 | cut -c1-100 || exit 1
}
CFGS=dkd_cifar_res32x4_res8x4,dot_cifar_res32x4_res8x4
run base MDA_X=0
run target384 MDA_CONV_TARGET=384
run target512 MDA_CONV_TARGET=512
run bnper2 MDA_BN_BWD_PER=2
run bnper8 MDA_BN_BWD_PER=8
run noparity MDA_DGRAD_PARITY=0
run xcd0 MDA_CONV_XCD=0
CFGS=kdsvd_cifar_res32x4_res8x4
run eig256 MDA_EIG_THREADS=256
run eig128 MDA_EIG_THREADS=128
run eig64 MDA_EIG_THREADS=64
