set -o pipefail
mkdir -p gpurun_out; export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_multirank.py -q --timeout 800 --timeout-method thread > gpurun_out/t_multi2.log 2>&1; rc=$?; echo "multirank rc=$rc"
grep -E "passed|failed|assert" gpurun_out/t_multi2.log | head -5
