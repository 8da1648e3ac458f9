export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1; rc=$?; tail -2 gpurun_out/smoke.log; [ $rc -ne 0 ] && exit $rc
BENCH="--steps 20 --warmup 5;--steps 500 --warmup 30;--cfg configs/cifar100/vanilla.yaml --steps 500 --warmup 30;--steps 500 --warmup 30 --batch 8" bash scripts/gpu_run.sh && \
PROF="configs/cifar100/dkd/res32x4_res8x4.yaml:flag_r5d;configs/cifar100/vanilla.yaml:van_r5d" TOP=60 bash scripts/gpu_run.sh
