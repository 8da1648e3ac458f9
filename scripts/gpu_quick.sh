# Quick GPU check after a conv-kernel change: build, conv/BN numerics tests,
# isolated kernel times (kernel trace of the microbench), bench A/B (halo on/off).
set -x
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { tail -30 gpurun_out/build.log; exit 1; }
timeout -k 10 300 python -m pytest tests/test_gpu_conv.py tests/test_gpu_train_layers.py -x -q > gpurun_out/pytest_quick.log 2>&1 ; rc=$?; tail -15 gpurun_out/pytest_quick.log; [ $rc -eq 0 ] || exit 1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/ktm -o run -- python scripts/conv_microbench.py --iters 20 --ops fwd,dgrad,wgrad > gpurun_out/ktm.log 2>&1 || { tail -20 gpurun_out/ktm.log; exit 1; }
python scripts/kernel_times.py gpurun_out/ktm/run_results.db "mespace)::conv"
timeout -k 10 300 python bench.py --steps 200 --warmup 30 > gpurun_out/bench_quick.log 2>&1 || { tail -30 gpurun_out/bench_quick.log; exit 1; }
MDA_CONV_HALO=0 timeout -k 10 300 python bench.py --steps 200 --warmup 30 > gpurun_out/bench_quick_nohalo.log 2>&1 || { tail -30 gpurun_out/bench_quick_nohalo.log; exit 1; }
grep -h metric gpurun_out/bench_quick.log gpurun_out/bench_quick_nohalo.log | cut -c1-200
