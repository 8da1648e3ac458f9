# Round-end check on a fresh box with the in-tree build: GPU tests, smoke,
# default bench, 200-step bench and a steady-state rocprofv3 kernel summary.
set -x
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 ; rc=$?; tail -25 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/bench_default.log 2>&1 || { tail -20 gpurun_out/bench_default.log; exit 1; }
timeout -k 10 300 python bench.py --steps 200 --warmup 30 > gpurun_out/bench_200.log 2>&1 || { tail -20 gpurun_out/bench_200.log; exit 1; }
grep -h metric gpurun_out/bench_default.log gpurun_out/bench_200.log | cut -c1-220
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_final -o run -- python bench.py --steps 50 --warmup 10 > gpurun_out/prof_final.log 2>&1 ; echo "prof rc=$?"
