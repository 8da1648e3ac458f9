# First-path GPU check: build, gpu tests, smoke, bench (eager/graph), rocprof.
set -x
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 1
timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 ; echo "pytest rc=$?"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 30 --warmup 10 --no-graph > gpurun_out/bench_nograph.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 100 --warmup 20 > gpurun_out/bench_graph.log 2>&1 ; echo "bench rc=$?"
grep -h metric gpurun_out/bench_nograph.log gpurun_out/bench_graph.log
cd /tmp && export TMPDIR=/tmp && cd - &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_nograph -o run -- python bench.py --steps 10 --warmup 3 --no-graph > gpurun_out/prof_nograph.log 2>&1 ; echo "prof rc=$?"
