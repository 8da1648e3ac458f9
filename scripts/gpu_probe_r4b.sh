set -o pipefail
mkdir -p gpurun_out; export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_vid_nst.py -q --timeout 200 --timeout-method thread > gpurun_out/t_nst.log 2>&1; echo "tests rc=$?"
grep -E "FAILED|passed|failed" gpurun_out/t_nst.log | head -8
timeout -k 10 300 python -u scripts/debug/kdsvd_nan_probe.py > gpurun_out/kdsvd_probe.log 2>&1; echo "probe rc=$?"
timeout -k 10 300 python benchmarks/throughput.py --configs nst_cifar_res32x4_res8x4 --steps 30 --warmup 10 || exit 1
PROF="configs/imagenet/r50_mv1/dkd.yaml:r4_r50_mv1;configs/imagenet/r34_r18/reviewkd.yaml:r4_r34_r18:--batch 32" bash scripts/gpu_run.sh
