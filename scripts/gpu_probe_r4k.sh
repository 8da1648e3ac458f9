set -o pipefail
mkdir -p gpurun_out; export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 300 --warmup 30 > gpurun_out/bench_k.log 2>&1 || { tail -5 gpurun_out/bench_k.log; exit 1; }
grep '^{' gpurun_out/bench_k.log | cut -c1-220
MDA_CONV1X1_MIN_M=100000000 timeout -k 10 300 python bench.py --steps 300 --warmup 30 > gpurun_out/bench_k2.log 2>&1 || { tail -5 gpurun_out/bench_k2.log; exit 1; }
grep '^{' gpurun_out/bench_k2.log | cut -c1-220
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_all.log 2>&1; rc=$?; echo "all gpu tests rc=$rc"
tail -3 gpurun_out/t_all.log
grep -E "FAILED|Error" gpurun_out/t_all.log | head -5
exit $rc
