# Iteration loop on the GPU box: gpu tests, smoke, graph bench (A/B), steady-state rocprof.
# Extensions are built on the CPU container beforehand (the .so travels with the snapshot).
set -x
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 ; rc=$?; tail -8 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -30 gpurun_out/smoke.log; exit 1; }
timeout -k 10 300 python bench.py --steps 200 --warmup 30 > gpurun_out/bench_graph.log 2>&1 || { tail -30 gpurun_out/bench_graph.log; exit 1; }
timeout -k 10 300 python bench.py > gpurun_out/bench_default.log 2>&1 || { tail -30 gpurun_out/bench_default.log; exit 1; }
grep -h metric gpurun_out/bench_graph.log gpurun_out/bench_default.log | cut -c1-300
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_graph -o run -- python bench.py --steps 20 --warmup 10 > gpurun_out/prof_graph.log 2>&1 || { tail -20 gpurun_out/prof_graph.log; exit 1; }
python scripts/prof_summary.py gpurun_out/prof_graph/run_results.db --skip 12 --top 40 --md gpurun_out/prof_graph_summary.md | head -45
