# Quick GPU check: selected test files + bench + steady-state profile summary.
set -x
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_head.py} -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_quick.log 2>&1 ; rc=$?; tail -8 gpurun_out/pytest_quick.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --steps 200 --warmup 30 > gpurun_out/bench_quick.log 2>&1 || { tail -30 gpurun_out/bench_quick.log; exit 1; }
grep -h metric gpurun_out/bench_quick.log | cut -c1-200
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/prof_q -o run -- python bench.py --steps 20 --warmup 10 > gpurun_out/prof_q.log 2>&1 || { tail -20 gpurun_out/prof_q.log; exit 1; }
python scripts/prof_summary.py gpurun_out/prof_q/run_results.db --skip 12 --top 45 --md gpurun_out/prof_q_summary.md > /dev/null
python scripts/step_timeline.py gpurun_out/prof_q/run_results.db > gpurun_out/prof_q_timeline.txt
head -30 gpurun_out/prof_q_summary.md | cut -c1-160
