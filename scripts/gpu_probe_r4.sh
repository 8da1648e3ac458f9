set -o pipefail
mkdir -p gpurun_out; export PYTHONPATH=$PWD TMPDIR=/tmp
step() { local log=$1; shift; "$@" > gpurun_out/$log 2>&1; local rc=$?; tail -3 gpurun_out/$log | cut -c1-300; if [ $rc -ge 124 ]; then echo "FATAL rc=$rc in $log"; exit $rc; fi; return 0; }
step t_dot1.log timeout -k 10 400 python -u -m pytest tests/test_gpu_dot_single.py -x -v --timeout 200 --timeout-method thread
grep -E "Error|assert|PASS|FAIL" gpurun_out/t_dot1.log | head -20
step b_dot1.log timeout -k 10 300 python -u bench.py --steps 300 --warmup 30 --cfg configs/cifar100/dot/res32x4_res8x4.yaml
step b_dot0.log timeout -k 10 300 python -u bench.py --steps 300 --warmup 30 --cfg configs/cifar100/dot/res32x4_res8x4.yaml RUNTIME.DOT_SINGLE_PASS false
step t_e2e.log timeout -k 10 600 python -u -m pytest tests/test_gpu_e2e.py -x -q --timeout 200 --timeout-method thread -k "dot"
