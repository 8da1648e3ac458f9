set -o pipefail
mkdir -p gpurun_out; export PYTHONPATH=$PWD TMPDIR=/tmp
BYDISP=1 TOP=40 PROF="configs/cifar100/dkd/res32x4_res8x4.yaml:r4_flagship_final" bash scripts/gpu_run.sh
