#!/bin/bash
# Iteration check: selected GPU test files ($TESTS), then throughput rows for $CONFIGS.
set -o pipefail
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-600} python -u -m pytest $TESTS -x -q --timeout 300 --timeout-method thread > gpurun_out/iter_tests.log 2>&1
  rc=$?; tail -15 gpurun_out/iter_tests.log; [ $rc -ne 0 ] && exit $rc
fi
if [ -n "$CONFIGS" ]; then
  timeout -k 10 ${BENCH_TIMEOUT:-600} python benchmarks/throughput.py --configs $CONFIGS --steps ${STEPS:-30} --warmup 10 > gpurun_out/iter_tp.log 2>&1
  rc=$?; grep -v "^\[WARN\]" gpurun_out/iter_tp.log | tail -12; [ $rc -ne 0 ] && exit $rc
fi
exit 0
