set -o pipefail
mkdir -p gpurun_out; export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_virtual_residual.py tests/test_grad_reducer_cpu.py tests/test_host_sanitizer.py tests/test_kdsvd_gram.py tests/test_models.py tests/test_parity_reference.py tests/test_shufflenet_padding.py tests/test_tools.py tests/test_trainer_cpu.py -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/t_rest.log 2>&1; rc=$?; echo "rest gpu tests rc=$rc"
tail -3 gpurun_out/t_rest.log
grep -E "FAILED" gpurun_out/t_rest.log | head -5
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; echo "smoke rc=$?"; tail -2 gpurun_out/smoke.log
