# Halo conv phase breakdown (in-kernel stamps) and ring-depth A/B on the
# CIFAR teacher / student 3x3 shapes.  Each step has its own time limit.
set -o pipefail
mkdir -p gpurun_out; export PYTHONPATH=$PWD TMPDIR=/tmp
out=gpurun_out/conv_exp.log; : > $out
for sh in 64,128,16,128 64,256,8,256 64,64,32,64; do
  for ring in 3 8; do
    echo "== shape $sh ring $ring" >> $out
    MDA_HALO_RING=$ring timeout -k 10 60 python -u scripts/conv_stamps.py --shape $sh --runs 2 >> $out 2>&1 || { echo "rc=$? at $sh $ring"; tail -5 $out; exit 1; }
  done
done
for env in "MDA_HALO_RING=3" "MDA_HALO_RING=8" "MDA_CONV_HALO=0"; do
  echo "== microbench $env" >> $out
  env $env timeout -k 10 120 python -u scripts/conv_microbench.py --graph --ops fwd,dgrad --iters 30 >> $out 2>&1 || { echo "rc=$? at $env"; tail -5 $out; exit 1; }
done
grep -v "amdgpu.ids" $out | head -150
