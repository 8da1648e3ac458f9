set -o pipefail
mkdir -p gpurun_out; export PYTHONPATH=$PWD TMPDIR=/tmp
step() { local log=$1; shift; "$@" > gpurun_out/$log 2>&1; local rc=$?; grep -v "WARN\|amdgpu.ids" gpurun_out/$log | tail -4 | cut -c1-400; if [ $rc -ge 124 ]; then echo "FATAL rc=$rc in $log"; exit $rc; fi; return 0; }
step t_b.log timeout -k 10 400 python -u -m pytest tests/test_gpu_deform.py tests/test_gpu_kdsvd.py -q --timeout 200 --timeout-method thread
grep -E "FAILED|passed|failed|assert" gpurun_out/t_b.log | head -12
step shuv1.log timeout -k 10 300 python -u scripts/debug/shuv1_dkd_loss.py
grep step gpurun_out/shuv1.log
step tp_bn.log timeout -k 10 300 python -u benchmarks/throughput.py --configs dot_cifar_res32x4_shuv2,dkd_cifar_res32x4_shuv1,dkd_cifar_vgg13_mv2,kd_cifar_res32x4_res8x4 --steps 60 --warmup 10
MDA_BN_BWD_PER=4 step tp_bn4.log timeout -k 10 300 python -u benchmarks/throughput.py --configs dot_cifar_res32x4_shuv2,dkd_cifar_res32x4_shuv1,dkd_cifar_vgg13_mv2,kd_cifar_res32x4_res8x4 --steps 60 --warmup 10
grep -h "{" gpurun_out/tp_bn.log gpurun_out/tp_bn4.log | cut -c1-160
timeout -k 10 700 bash scripts/gpu_conv_exp.sh > gpurun_out/conv_exp_run.log 2>&1; echo "conv_exp rc=$?"
PROF="configs/tiny_imagenet/dot/r18_mv2.yaml:r4_dot_tiny_mv2:--batch 256;configs/tiny_imagenet/dot/r18_shuv2.yaml:r4_dot_tiny_shuv2:--batch 256" bash scripts/gpu_run.sh
