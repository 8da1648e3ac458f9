# Round-2 final numbers: every config's throughput (1 GPU) + kernel profiles of SP, RKD, DOT.
set -x
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_head.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_head.log 2>&1 ; rc=$?; tail -3 gpurun_out/pytest_head.log; [ $rc -eq 0 ] || exit 1
PYTHONPATH=. timeout -k 10 120 python -u scripts/head_microbench.py > gpurun_out/head_mb.log 2>&1 || { tail -20 gpurun_out/head_mb.log; exit 1; }
cat gpurun_out/head_mb.log
rm -f gpurun_out/throughput.jsonl
timeout -k 10 900 python -u benchmarks/throughput.py --steps 100 --warmup 20 --out gpurun_out/throughput.jsonl > gpurun_out/throughput.log 2>&1 || { tail -30 gpurun_out/throughput.log; exit 1; }
cut -c1-200 gpurun_out/throughput.jsonl
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for c in sp rkd dot/res32x4_res8x4; do
  name=$(echo $c | tr '/' '_')
  timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_$name -o run -- python bench.py --cfg configs/cifar100/$c.yaml --steps 20 --warmup 10 > gpurun_out/prof_$name.log 2>&1 || { tail -20 gpurun_out/prof_$name.log; exit 1; }
  python scripts/prof_summary.py gpurun_out/prof_$name/run_results.db --skip 12 --top 40 --md gpurun_out/prof_${name}_summary.md | cut -c1-160 | head -3
  rm -f gpurun_out/prof_$name/run_results.db
done
