set -o pipefail
mkdir -p gpurun_out; export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 200 python -u scripts/launch_floor_probe.py > gpurun_out/floor.log 2>&1 || { cat gpurun_out/floor.log; exit 1; }
cat gpurun_out/floor.log
timeout -k 10 300 python bench.py --steps 300 > gpurun_out/b300.log 2>&1 || { tail -5 gpurun_out/b300.log; exit 1; }
tail -1 gpurun_out/b300.log | cut -c1-250
PROF="configs/cifar100/dkd/res32x4_res8x4.yaml:flag;configs/cifar100/vanilla.yaml:van" bash scripts/gpu_run.sh
