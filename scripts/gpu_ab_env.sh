# conv numerics tests, then bench A/B of an env knob: AB_VAR=<name> (value 0 = off)
set -x
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_train_layers.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_conv.log 2>&1; rc=$?; tail -4 gpurun_out/pytest_conv.log; [ $rc -eq 0 ] || exit 1
for v in 1 0 1 0; do
  env ${AB_VAR}=$v timeout -k 10 200 python bench.py --steps 300 --warmup 30 > gpurun_out/ab_$v.log 2>&1 || { tail -20 gpurun_out/ab_$v.log; exit 1; }
  echo "${AB_VAR}=$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_$v.log)"
done
