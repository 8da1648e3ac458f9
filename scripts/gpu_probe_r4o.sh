set -o pipefail
mkdir -p gpurun_out; export PYTHONPATH=$PWD TMPDIR=/tmp
MDA_EVENTS_SYNC=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_multirank.py -k events -q --runxfail --timeout 500 --timeout-method thread > gpurun_out/t_multi_sync.log 2>&1; rc=$?; echo "events+sync rc=$rc"
grep -E "passed|failed|assert 0" gpurun_out/t_multi_sync.log | head -4
