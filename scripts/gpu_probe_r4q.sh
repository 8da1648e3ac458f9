set -o pipefail
mkdir -p gpurun_out; export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 600 python -u scripts/debug/multirank_determinism.py > gpurun_out/mr_det.log 2>&1; echo "rc=$?"
grep -E "vs" gpurun_out/mr_det.log
