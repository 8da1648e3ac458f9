set -o pipefail
mkdir -p gpurun_out; export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_multirank.py -q --runxfail --timeout 600 --timeout-method thread > gpurun_out/t_multi.log 2>&1; rc=$?; echo "multirank rc=$rc"
tail -3 gpurun_out/t_multi.log
grep -E "FAILED|assert|rel" gpurun_out/t_multi.log | head -8
