set -x
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 1
for v in b32_hold; do
timeout -k 10 120 python -X faulthandler scripts/probe_variant.py $v > gpurun_out/probe_$v.log 2>&1 || { echo "FAIL $v"; tail -5 gpurun_out/probe_$v.log; exit 1; }
tail -1 gpurun_out/probe_$v.log
done
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 ; rc=$?; tail -5 gpurun_out/pytest_gpu.log; exit $rc
