set -o pipefail
mkdir -p gpurun_out; export PYTHONPATH=$PWD TMPDIR=/tmp
out=gpurun_out/kernarg.log; : > $out
for v in 0 1; do
  echo "== HIP_FORCE_DEV_KERNARG=$v" >> $out
  HIP_FORCE_DEV_KERNARG=$v timeout -k 10 60 python -u scripts/conv_stamps.py --shape 64,128,16,128 --runs 1 >> $out 2>&1 || { echo "rc=$?"; tail $out; exit 1; }
  HIP_FORCE_DEV_KERNARG=$v timeout -k 10 200 python -u bench.py --steps 300 --warmup 30 >> $out 2>&1 || { echo "rc=$?"; tail $out; exit 1; }
  HIP_FORCE_DEV_KERNARG=$v timeout -k 10 200 python -u bench.py --steps 300 --warmup 30 --cfg configs/cifar100/dot/res32x4_res8x4.yaml >> $out 2>&1 || { echo "rc=$?"; tail $out; exit 1; }
done
grep -v "WARN\|amdgpu.ids" $out | cut -c1-260
