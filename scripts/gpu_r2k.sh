# Why DOT in benchmarks/throughput.py (after other configs in one process) is slower than bench.py.
set -x
mkdir -p gpurun_out
timeout -k 10 300 python -u benchmarks/throughput.py --configs dot_cifar_res32x4_res8x4 --steps 100 --warmup 20 > gpurun_out/tp_k1.log 2>&1 || { tail -20 gpurun_out/tp_k1.log; exit 1; }
grep config gpurun_out/tp_k1.log | cut -c1-120
timeout -k 10 300 python -u benchmarks/throughput.py --configs dkd_cifar_res32x4_res8x4,dot_cifar_res32x4_res8x4 --steps 100 --warmup 20 > gpurun_out/tp_k2.log 2>&1 || { tail -20 gpurun_out/tp_k2.log; exit 1; }
grep config gpurun_out/tp_k2.log | cut -c1-120
