# Fresh throughput row for every BASELINE/inset config (1 GPU).
set -x
mkdir -p gpurun_out
rm -f gpurun_out/throughput.jsonl
timeout -k 10 900 python -u benchmarks/throughput.py --steps 100 --warmup 20 --out gpurun_out/throughput.jsonl > gpurun_out/throughput.log 2>&1 || { tail -30 gpurun_out/throughput.log; exit 1; }
cut -c1-200 gpurun_out/throughput.jsonl
