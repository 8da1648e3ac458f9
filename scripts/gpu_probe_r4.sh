set -o pipefail
mkdir -p gpurun_out; export PYTHONPATH=$PWD TMPDIR=/tmp
step() { local log=$1; shift; "$@" > gpurun_out/$log 2>&1; local rc=$?; tail -3 gpurun_out/$log | cut -c1-300; if [ $rc -ge 124 ]; then echo "FATAL rc=$rc in $log"; exit $rc; fi; return 0; }
step tail.log timeout -k 10 120 python -u scripts/debug/tail_probe.py
cat gpurun_out/tail.log
step t_mr.log timeout -k 10 600 python -u -m pytest tests/test_gpu_multirank.py -x -q --timeout 580 --timeout-method thread -k "events"
grep -E "hipError|capture failed" gpurun_out/t_mr.log | head -5
