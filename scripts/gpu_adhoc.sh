set -o pipefail
mkdir -p gpurun_out; export PYTHONPATH=$PWD TMPDIR=/tmp
for cs in dot_cifar_res32x4_res8x4,dot_cifar_res32x4_res8x4 kd_cifar_res56_res20,dkd_cifar_res32x4_res8x4,dot_cifar_res32x4_res8x4; do
timeout -k 10 600 python benchmarks/throughput.py --configs $cs --steps 100 --warmup 20 > gpurun_out/tp_x.log 2>&1 || exit 1
echo "$cs: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/tp_x.log | tr '\n' ' ')"
done
