# Iteration loop on the GPU box: build, gpu tests, graph bench (A/B), steady-state rocprof.
set -x
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { tail -30 gpurun_out/build.log; exit 1; }
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 ; rc=$?; tail -5 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --steps 200 --warmup 30 > gpurun_out/bench_graph.log 2>&1 || { tail -30 gpurun_out/bench_graph.log; exit 1; }
timeout -k 10 300 python bench.py --steps 200 --warmup 30 --no-train-kernels > gpurun_out/bench_graph_miopen.log 2>&1 || { tail -30 gpurun_out/bench_graph_miopen.log; exit 1; }
grep -h metric gpurun_out/bench_graph.log gpurun_out/bench_graph_miopen.log | cut -c1-260
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_graph -o run -- python bench.py --steps 20 --warmup 10 > gpurun_out/prof_graph.log 2>&1 || { tail -20 gpurun_out/prof_graph.log; exit 1; }
python scripts/prof_summary.py gpurun_out/prof_graph/run_results.db --skip 12 --top 40 --md gpurun_out/prof_graph_summary.md | head -45
