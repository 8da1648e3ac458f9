export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 1140 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/gpu_full.log 2>&1; rc=$?
grep -E "passed|failed|error" gpurun_out/gpu_full.log | tail -3; exit $rc
