set -o pipefail
mkdir -p gpurun_out; export PYTHONPATH=$PWD TMPDIR=/tmp
MDA_TEST_BUCKET_MB=1.0 timeout -k 10 400 python -u -m pytest tests/test_gpu_multirank.py -k events -q --runxfail --timeout 300 --timeout-method thread > gpurun_out/t_ev1.log 2>&1; echo "events vs split, both 1.0 MB rc=$?"
grep -E "passed|failed|assert 0" gpurun_out/t_ev1.log | head -3
MDA_TEST_BUCKET_MB=0.5 timeout -k 10 400 python -u -m pytest tests/test_gpu_multirank.py -k events -q --runxfail --timeout 300 --timeout-method thread > gpurun_out/t_ev2.log 2>&1; echo "events vs split, both 0.5 MB rc=$?"
grep -E "passed|failed|assert 0" gpurun_out/t_ev2.log | head -3
