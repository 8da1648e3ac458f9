# Kernel-trace the bench with the LDS-DMA conv (default) and the register-staged conv (A/B).
set -x
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { tail -30 gpurun_out/build.log; exit 1; }
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/kt_glds -o run -- python bench.py --steps 20 --warmup 10 > gpurun_out/kt_glds.log 2>&1 || { tail -20 gpurun_out/kt_glds.log; exit 1; }
MDA_CONV_GLDS=0 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/kt_reg -o run -- python bench.py --steps 20 --warmup 10 > gpurun_out/kt_reg.log 2>&1 || { tail -20 gpurun_out/kt_reg.log; exit 1; }
echo GLDS; python scripts/kernel_times.py gpurun_out/kt_glds/run_results.db "mespace)::conv"
echo REG; python scripts/kernel_times.py gpurun_out/kt_reg/run_results.db "mespace)::conv"
python scripts/prof_summary.py gpurun_out/kt_glds/run_results.db --skip 12 --top 30 --md gpurun_out/prof_glds.md > /dev/null
python scripts/prof_summary.py gpurun_out/kt_reg/run_results.db --skip 12 --top 30 --md gpurun_out/prof_reg.md > /dev/null
head -3 gpurun_out/prof_glds.md gpurun_out/prof_reg.md
