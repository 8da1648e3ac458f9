set -o pipefail
mkdir -p gpurun_out; export PYTHONPATH=$PWD TMPDIR=/tmp
rm -f gpurun_out/r4_throughput_final.jsonl
timeout -k 10 1100 python benchmarks/throughput.py --configs all --steps 100 --warmup 20 --out gpurun_out/r4_throughput_final.jsonl | cut -c1-150
