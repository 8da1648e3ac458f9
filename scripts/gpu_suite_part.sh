# One part of the GPU suite (PART=a: e2e + multirank; PART=b: everything else), one process.
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD TMPDIR=/tmp
if [ "$PART" = "a" ]; then
  FILES="tests/test_gpu_e2e.py tests/test_gpu_multirank.py"
else
  FILES=$(ls tests/test_gpu_*.py | grep -v "test_gpu_e2e.py\|test_gpu_multirank.py" | tr '\n' ' ')
fi
timeout -k 10 1080 python -u -m pytest $FILES -q --timeout 600 --timeout-method thread > gpurun_out/suite_$PART.log 2>&1
rc=$?; tail -15 gpurun_out/suite_$PART.log; exit $rc
