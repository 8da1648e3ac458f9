set -o pipefail
mkdir -p gpurun_out; export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kdsvd.py -q --timeout 200 --timeout-method thread > gpurun_out/t_kdsvd.log 2>&1; echo "tests rc=$?"
grep -E "FAILED|passed|failed|Error" gpurun_out/t_kdsvd.log | head -12
timeout -k 10 300 python benchmarks/throughput.py --configs kdsvd_cifar_res32x4_res8x4 --steps 30 --warmup 10 || exit 1
PROF="configs/cifar100/kdsvd.yaml:r4_kdsvd2;configs/cifar100/nst.yaml:r4_nst2" bash scripts/gpu_run.sh
