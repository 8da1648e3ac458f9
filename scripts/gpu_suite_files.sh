# Selected GPU test files (FILES="..."), one process, then optionally PART=a.
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest $FILES -q --timeout 300 --timeout-method thread > gpurun_out/suite_files.log 2>&1
rc=$?; tail -6 gpurun_out/suite_files.log; [ $rc -eq 0 ] || exit $rc
if [ -n "$PART" ]; then bash scripts/gpu_suite_part.sh; fi
