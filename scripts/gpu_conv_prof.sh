# Isolated conv kernel times (kernel trace of the per-shape microbench), LDS-DMA vs register-staged.
set -x
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/ktm_glds -o run -- python scripts/conv_microbench.py --iters 20 > gpurun_out/ktm_glds.log 2>&1 || { tail -20 gpurun_out/ktm_glds.log; exit 1; }
MDA_CONV_GLDS=0 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/ktm_reg -o run -- python scripts/conv_microbench.py --iters 20 --ops fwd,dgrad > gpurun_out/ktm_reg.log 2>&1 || { tail -20 gpurun_out/ktm_reg.log; exit 1; }
echo GLDS; python scripts/kernel_times.py gpurun_out/ktm_glds/run_results.db "mespace)::conv"
echo REG; python scripts/kernel_times.py gpurun_out/ktm_reg/run_results.db "mespace)::conv"
echo MIOPEN; python scripts/kernel_times.py gpurun_out/ktm_glds/run_results.db "ck::" | head -20
python scripts/kernel_times.py gpurun_out/ktm_glds/run_results.db "igemm" | head -20
python scripts/kernel_times.py gpurun_out/ktm_glds/run_results.db "Cijk" | head -20
