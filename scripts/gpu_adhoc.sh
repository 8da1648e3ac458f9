set -o pipefail
mkdir -p gpurun_out; export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/full_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/full_gpu.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" gpurun_out/full_gpu.log | head -20; exit $rc; }
timeout -k 10 200 python bench.py --steps 300 --warmup 20 > gpurun_out/flag300.log 2>&1 || exit 1
tail -1 gpurun_out/flag300.log | cut -c1-200
timeout -k 10 900 python benchmarks/throughput.py --configs all --steps 60 --warmup 15 --out gpurun_out/r3_tp_all.jsonl > gpurun_out/tp_all.log 2>&1 || exit 1
PROF="configs/cifar100/dkd/res32x4_res8x4.yaml:r3_flagship;configs/imagenet/r50_mv1/dkd.yaml:r3_r50_mv1;configs/cifar100/dkd/vgg13_mv2.yaml:r3_vgg13_mv2;configs/cifar100/dkd/res32x4_shuv1.yaml:r3_shuv1" bash scripts/gpu_run.sh
