# Quick GPU check after a kernel change: build, conv/BN numerics tests, conv
# microbench with the LDS-DMA and register-staged conv kernels, bench A/B.
set -x
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { tail -30 gpurun_out/build.log; exit 1; }
timeout -k 10 300 python -m pytest tests/test_gpu_conv.py tests/test_gpu_train_layers.py -x -q > gpurun_out/pytest_quick.log 2>&1 ; rc=$?; tail -5 gpurun_out/pytest_quick.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python scripts/conv_microbench.py --iters 30 > gpurun_out/mb_glds.log 2>&1 || { tail -20 gpurun_out/mb_glds.log; exit 1; }
MDA_CONV_GLDS=0 timeout -k 10 200 python scripts/conv_microbench.py --iters 30 > gpurun_out/mb_reg.log 2>&1 || { tail -20 gpurun_out/mb_reg.log; exit 1; }
echo glds; cut -c1-200 gpurun_out/mb_glds.log; echo reg; cut -c1-200 gpurun_out/mb_reg.log
timeout -k 10 300 python bench.py --steps 200 --warmup 30 > gpurun_out/bench_quick.log 2>&1 || { tail -30 gpurun_out/bench_quick.log; exit 1; }
MDA_CONV_GLDS=0 timeout -k 10 300 python bench.py --steps 200 --warmup 30 > gpurun_out/bench_quick_reg.log 2>&1 || { tail -30 gpurun_out/bench_quick_reg.log; exit 1; }
grep -h metric gpurun_out/bench_quick.log gpurun_out/bench_quick_reg.log | cut -c1-200
