# Steady-state kernel profiles of the ReviewKD and CRD inset methods (1 GPU).
set -x
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for c in reviewkd_cifar_res32x4_res8x4 crd_cifar_res32x4_res8x4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$c -o run -- python benchmarks/throughput.py --configs $c --steps 40 --warmup 10 > gpurun_out/prof_$c.log 2>&1 || { tail -20 gpurun_out/prof_$c.log; exit 1; }
done
