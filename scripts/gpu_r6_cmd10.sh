export PYTHONPATH=$PWD TMPDIR=/tmp
ARMS=" ;MDA_CONV_HALO2=0;MDA_CONV_HALO1=0;MDA_CONV_HALO2=0 MDA_CONV_HALO1=0" ROUNDS=3 bash scripts/gpu_r6_ab.sh || exit 1
ARMS=" ;MDA_CONV_HALO2=0" ROUNDS=2 BENCH_ARGS="--cfg configs/cifar100/vanilla.yaml DISTILLER.STUDENT resnet8x4" bash scripts/gpu_r6_ab.sh
