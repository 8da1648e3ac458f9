export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 300 python benchmarks/throughput.py --configs dot_tiny_r18_mv2 --steps 60 --warmup 15 2>/dev/null | grep "^{" | cut -c1-220
timeout -k 10 200 python bench.py --cfg configs/imagenet/r34_r18/dot.yaml --batch 32 --steps 20 --warmup 5 RUNTIME.DOT_SINGLE_PASS False > gpurun_out/dot_r18_two.log 2>&1; tail -3 gpurun_out/dot_r18_two.log | cut -c1-300
