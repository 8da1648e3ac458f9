export PYTHONPATH=$PWD TMPDIR=/tmp
TESTS="tests/test_gpu_kernels_losses_optim.py tests/test_gpu_vid_nst.py" bash scripts/gpu_run.sh && \
BENCH="--steps 500 --warmup 30;--steps 500 --warmup 30 EXPERIMENT.DETERMINISTIC True;--steps 500 --warmup 30 --batch 8;--cfg configs/cifar100/vanilla.yaml --steps 500 --warmup 30" bash scripts/gpu_run.sh && \
PROF="configs/cifar100/dkd/res32x4_res8x4.yaml:flag_r5b;configs/cifar100/vanilla.yaml:van_r5b" TOP=60 bash scripts/gpu_run.sh
