# Round-2 end-of-session check: full GPU suite, smoke, bench, wgrad-stream A/B under the look-ahead,
# full throughput table and a flagship kernel profile.
set -x
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 ; rc=$?; tail -4 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log | cut -c1-200
timeout -k 10 300 python bench.py > gpurun_out/bench_default.log 2>&1 || { tail -20 gpurun_out/bench_default.log; exit 1; }
grep -h metric gpurun_out/bench_default.log | cut -c1-250
for o in "RUNTIME.WGRAD_STREAM on" "RUNTIME.WGRAD_STREAM auto"; do
  timeout -k 10 300 python bench.py --steps 300 --warmup 30 $o > gpurun_out/bench_j.log 2>&1 || { tail -20 gpurun_out/bench_j.log; exit 1; }
  echo "$o"; grep -h metric gpurun_out/bench_j.log | cut -c100-200
done
rm -f gpurun_out/throughput.jsonl
timeout -k 10 900 python -u benchmarks/throughput.py --steps 100 --warmup 20 --out gpurun_out/throughput.jsonl > gpurun_out/throughput.log 2>&1 || { tail -30 gpurun_out/throughput.log; exit 1; }
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_flag -o run -- python bench.py --steps 50 --warmup 10 > gpurun_out/prof_flag.log 2>&1 || { tail -20 gpurun_out/prof_flag.log; exit 1; }
python scripts/prof_summary.py gpurun_out/prof_flag/run_results.db --skip 12 --top 45 --md gpurun_out/prof_flag_summary.md | head -3
python scripts/step_timeline.py gpurun_out/prof_flag/run_results.db > gpurun_out/prof_flag_timeline.txt 2>&1 || true
rm -f gpurun_out/prof_flag/run_results.db
