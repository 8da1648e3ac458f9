# Per-step loss traces of the configs that reported non-finite bench losses
# (OFD, ShuffleV1): torch fp32 eager vs native bf16 eager vs native bf16
# graph; then a fresh throughput row for every BASELINE config.
set -x
mkdir -p gpurun_out
for y in ${YAMLS:-configs/cifar100/ofd.yaml configs/cifar100/dkd/res32x4_shuv1.yaml}; do
  n=$(basename $y .yaml)
  timeout -k 10 300 python -u scripts/loss_trace.py $y ${STEPS:-40} > gpurun_out/trace_$n.log 2>&1 || { tail -30 gpurun_out/trace_$n.log; exit 1; }
  grep -E "graph=|  (0|1|5|10|20|30|39) " gpurun_out/trace_$n.log | cut -c1-120
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_detection.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_det.log 2>&1 || { tail -40 gpurun_out/pytest_det.log; exit 1; }
tail -3 gpurun_out/pytest_det.log
rm -f gpurun_out/throughput.jsonl
timeout -k 10 900 python -u benchmarks/throughput.py --steps 100 --warmup 20 --out gpurun_out/throughput.jsonl > gpurun_out/throughput.log 2>&1 || { tail -30 gpurun_out/throughput.log; exit 1; }
cut -c1-200 gpurun_out/throughput.jsonl
