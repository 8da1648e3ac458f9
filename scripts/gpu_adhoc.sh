set -o pipefail
mkdir -p gpurun_out; export PYTHONPATH=$PWD
timeout -k 10 400 python -u -m pytest tests/test_gpu_bn_dgrad_sums.py tests/test_gpu_bn_fused.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_bnb.log 2>&1; rc=$?; tail -15 gpurun_out/t_bnb.log; [ $rc -ne 0 ] && exit $rc
for b in 64 8; do
timeout -k 10 200 python scripts/debug/host_probe.py --batch $b > gpurun_out/hp_$b.log 2>&1 || { tail gpurun_out/hp_$b.log; exit 1; }
grep -v WARN gpurun_out/hp_$b.log
done
timeout -k 10 200 python bench.py --steps 300 --warmup 20 > gpurun_out/b.log 2>&1 || exit 1
tail -1 gpurun_out/b.log | cut -c 1-250
MDA_BN_DGRAD_SUMS=0 timeout -k 10 200 python bench.py --steps 300 --warmup 20 > gpurun_out/b0.log 2>&1 || exit 1
tail -1 gpurun_out/b0.log | cut -c 1-250
