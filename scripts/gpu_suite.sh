set -o pipefail
mkdir -p gpurun_out; export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 1080 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/t_final.log 2>&1; rc=$?; echo "all gpu tests rc=$rc"
tail -2 gpurun_out/t_final.log
grep -E "^FAILED" gpurun_out/t_final.log | head -8
exit $rc
