# DOT dual-stream backward graphs + faster relation kernels: numerics, then A/B.
set -x
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_relation.py tests/test_gpu_e2e.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_f.log 2>&1 ; rc=$?; tail -5 gpurun_out/pytest_f.log; [ $rc -eq 0 ] || exit 1
for o in "RUNTIME.DOT_DUAL_STREAM True" "RUNTIME.DOT_DUAL_STREAM False" "RUNTIME.DOT_DUAL_STREAM True"; do
  timeout -k 10 300 python bench.py --cfg configs/cifar100/dot/res32x4_res8x4.yaml --steps 200 --warmup 30 $o > gpurun_out/bench_dot.log 2>&1 || { tail -20 gpurun_out/bench_dot.log; exit 1; }
  echo "$o"; grep -h metric gpurun_out/bench_dot.log | cut -c100-190
done
for c in sp rkd pkt; do
  timeout -k 10 300 python bench.py --cfg configs/cifar100/$c.yaml --steps 200 --warmup 30 > gpurun_out/bench_$c.log 2>&1 || { tail -20 gpurun_out/bench_$c.log; exit 1; }
  echo $c; grep -h metric gpurun_out/bench_$c.log | cut -c100-190
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_dotd -o run -- python bench.py --cfg configs/cifar100/dot/res32x4_res8x4.yaml --steps 20 --warmup 10 > gpurun_out/prof_dotd.log 2>&1 || { tail -20 gpurun_out/prof_dotd.log; exit 1; }
python scripts/prof_summary.py gpurun_out/prof_dotd/run_results.db --skip 12 --top 40 --md gpurun_out/prof_dotd_summary.md | cut -c1-160 | head -3
python scripts/kernel_times.py gpurun_out/prof_dotd/run_results.db "gram\|rkd\|relation" > /dev/null
rm -f gpurun_out/prof_dotd/run_results.db
