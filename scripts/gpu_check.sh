#!/bin/bash
# GPU check: full GPU test suite, 1-GPU bench, then (optionally) the RCCL probe.
# Each GPU step under its own time limit; stop at the first failure.
set -o pipefail
mkdir -p gpurun_out
T=${GPU_TEST_TIMEOUT:-900}
timeout -k 10 $T python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/gputest.log 2>&1
rc=$?; echo "pytest rc=$rc" | tee -a gpurun_out/gputest.log; tail -3 gpurun_out/gputest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 200 --warmup 20 > gpurun_out/bench.log 2>&1
rc=$?; cat gpurun_out/bench.log | tail -2; [ $rc -ne 0 ] && exit $rc
if [ -n "$RCCL_PROBE" ]; then
  timeout -k 10 120 python scripts/rccl_probe.py 2 > gpurun_out/rccl_probe.log 2>&1
  rc=$?; echo "probe rc=$rc" >> gpurun_out/rccl_probe.log; tail -8 gpurun_out/rccl_probe.log
fi
exit 0
