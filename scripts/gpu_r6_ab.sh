#!/bin/bash
# Round-6 A/B batch: BN apply kernel tests, then fresh-process bench arms
# (ARMS, ';'-separated env sets), then the 20-step driver command.
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD TMPDIR=/tmp
if [ -n "$TESTS" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-600} python -u -m pytest $TESTS -x -q --timeout 300 --timeout-method thread > gpurun_out/r6_tests.log 2>&1
  rc=$?; tail -4 gpurun_out/r6_tests.log; [ $rc -ne 0 ] && exit $rc
fi
if [ -n "$ARMS" ]; then
  ARMS="$ARMS" ROUNDS=${ROUNDS:-1} STEPS=${STEPS:-300} bash scripts/ab_env.sh 2>&1 | tail -12 || exit 1
fi
if [ -n "$SHORT" ]; then
  for i in $(seq 1 $SHORT); do
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 2>/dev/null | grep -o "\"ms_per_step\": [0-9.]*" || exit 1
  done
fi
exit 0
