set -o pipefail
mkdir -p gpurun_out; export PYTHONPATH=$PWD TMPDIR=/tmp
TOP=30 PROF="configs/cifar100/dkd/res32x4_shuv1.yaml:r4_shuv1;configs/cifar100/dkd/vgg13_mv2.yaml:r4_vgg13_mv2;configs/cifar100/dot/res32x4_res8x4.yaml:r4_dot_final" bash scripts/gpu_run.sh
