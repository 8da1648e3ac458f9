#!/bin/bash
# One parameterised GPU iteration (replaces the round-2 one-off gpu_r2*.sh):
#   TESTS="<pytest files>"      GPU tests (one process, per-test timeout)
#   BENCH="<bench.py args>"     flagship bench line(s), ';'-separated arg sets
#   CONFIGS="<names>"           benchmarks/throughput.py rows
#   PROF="<cfg>[:tag[:args]];..." rocprofv3 kernel-trace summary + step timeline per entry
# Every GPU step has its own time limit; the first failure ends the script.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
if [ -n "$TESTS" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest $TESTS -x -q --timeout 180 --timeout-method thread > gpurun_out/run_tests.log 2>&1
  rc=$?; tail -15 gpurun_out/run_tests.log; [ $rc -ne 0 ] && exit $rc
fi
if [ -n "$BENCH" ]; then
  IFS=';' read -ra SETS <<< "$BENCH"
  i=0
  for a in "${SETS[@]}"; do
    timeout -k 10 ${BENCH_TIMEOUT:-300} python bench.py $a > gpurun_out/run_bench$i.log 2>&1
    rc=$?; grep -v "^\[WARN\]" gpurun_out/run_bench$i.log | tail -2 | cut -c1-400; [ $rc -ne 0 ] && exit $rc
    i=$((i+1))
  done
fi
if [ -n "$CONFIGS" ]; then
  timeout -k 10 ${TP_TIMEOUT:-600} python benchmarks/throughput.py --configs $CONFIGS --steps ${STEPS:-30} --warmup 10 > gpurun_out/run_tp.log 2>&1
  rc=$?; grep -v "^\[WARN\]" gpurun_out/run_tp.log | tail -14; [ $rc -ne 0 ] && exit $rc
fi
if [ -n "$PROF" ]; then
  # ';'-separated entries "cfg.yaml[:tag[:bench args]]" (TAG / EXTRA: defaults for the first)
  IFS=';' read -ra PROFS <<< "$PROF"
  for ent in "${PROFS[@]}"; do
    IFS=':' read -r cfg name extra <<< "$ent"
    name=${name:-${TAG:-$(basename $cfg .yaml)}}
    extra=${extra:-$EXTRA}
    timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_$name -o run -- python bench.py --cfg $cfg --steps 20 --warmup 10 $extra > gpurun_out/prof_$name.log 2>&1 || { tail -20 gpurun_out/prof_$name.log; exit 1; }
    python scripts/prof_summary.py gpurun_out/prof_$name/run_results.db --skip 12 --top ${TOP:-40} ${BYDISP:+--by-dispatch} --md gpurun_out/prof_${name}_summary.md > /dev/null; head -3 gpurun_out/prof_${name}_summary.md
    python scripts/step_timeline.py gpurun_out/prof_$name/run_results.db > gpurun_out/prof_${name}_timeline.txt
    tail -1 gpurun_out/prof_${name}_timeline.txt
    rm -f gpurun_out/prof_$name/run_results.db
  done
fi
exit 0
