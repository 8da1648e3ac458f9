set -o pipefail
mkdir -p gpurun_out; export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kdsvd.py -q --timeout 200 --timeout-method thread > gpurun_out/t_kdsvd2.log 2>&1; rc=$?; echo "kdsvd tests rc=$rc"; tail -1 gpurun_out/t_kdsvd2.log
[ $rc -ne 0 ] && exit 1
timeout -k 10 300 python benchmarks/throughput.py --configs kdsvd_cifar_res32x4_res8x4 --steps 100 --warmup 20 | cut -c1-100
