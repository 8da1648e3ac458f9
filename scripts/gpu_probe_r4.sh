set -o pipefail
mkdir -p gpurun_out; export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_train_layers.py -q --timeout 200 --timeout-method thread > gpurun_out/t_c.log 2>&1; rc=$?; echo "tests rc=$rc"
grep -E "FAILED|passed|failed" gpurun_out/t_c.log | head -12
[ $rc -ge 124 ] && exit $rc
out=gpurun_out/stamps2.log; : > $out
for sh in 64,128,16,128 64,256,8,256 64,64,32,64; do
  echo "== $sh" >> $out
  timeout -k 10 60 python -u scripts/conv_stamps.py --shape $sh --runs 1 >> $out 2>&1 || { echo "rc=$?"; tail $out; exit 1; }
done
grep -v "amdgpu.ids" $out
timeout -k 10 200 python -u bench.py --steps 300 --warmup 30 > gpurun_out/b1.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --steps 300 --warmup 30 --cfg configs/cifar100/dot/res32x4_res8x4.yaml > gpurun_out/b2.log 2>&1 || exit 1
grep -h "{" gpurun_out/b1.log gpurun_out/b2.log | cut -c1-220
PROF="configs/cifar100/fitnet.yaml:r4_fitnet;configs/cifar100/vid.yaml:r4_vid;configs/cifar100/dkd/res32x4_res8x4.yaml:r4_flagship" bash scripts/gpu_run.sh
