export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_train_layers.py tests/test_gpu_bn_dgrad_sums.py -q -k "group or Group or shuffle or Shuffle" --timeout 300 --timeout-method thread > gpurun_out/grp.log 2>&1; rc=$?; tail -3 gpurun_out/grp.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_e2e.py -q -k "ShuffleV1" --timeout 500 --timeout-method thread > gpurun_out/grp_e2e.log 2>&1; rc=$?; tail -3 gpurun_out/grp_e2e.log; [ $rc -eq 0 ] || exit $rc
for arm in 1 0 1 0; do timeout -k 10 200 env MDA_GROUPED_BN=$arm python benchmarks/throughput.py --configs dkd_cifar_res32x4_shuv1 --steps 100 --warmup 20 2>/dev/null | grep -o '"ms_per_step": [0-9.]*' | sed "s/^/arm $arm /"; done
