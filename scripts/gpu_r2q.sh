# Kernel profile of the DOT step (dual-stream backwards + look-ahead + deferred reductions).
set -x
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_dotq -o run -- python bench.py --cfg configs/cifar100/dot/res32x4_res8x4.yaml --steps 20 --warmup 10 > gpurun_out/prof_dotq.log 2>&1 || { tail -20 gpurun_out/prof_dotq.log; exit 1; }
python scripts/prof_summary.py gpurun_out/prof_dotq/run_results.db --skip 12 --top 40 --md gpurun_out/prof_dotq_summary.md | head -3
rm -f gpurun_out/prof_dotq/run_results.db
