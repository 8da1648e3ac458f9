export PYTHONPATH=$PWD TMPDIR=/tmp
for s in 64,256,8,256 64,128,16,128 64,64,32,64; do timeout -k 10 120 python scripts/wgrad_stamps.py --shape $s || exit 1; done > gpurun_out/wg_stamps.txt 2>&1; grep -v amdgpu gpurun_out/wg_stamps.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_train_layers.py -x -q --timeout 120 --timeout-method thread -k "dgrad_wgrad or conv_bn_act_train" > gpurun_out/t5.log 2>&1; rc=$?; tail -2 gpurun_out/t5.log; [ $rc -ne 0 ] && exit $rc
BENCH="--steps 300 --warmup 20" bash scripts/gpu_run.sh || exit 1
MDA_WGH_BLOCKS=256 BENCH="--steps 300 --warmup 20" bash scripts/gpu_run.sh || exit 1
MDA_WG_HALO=0 BENCH="--steps 300 --warmup 20" bash scripts/gpu_run.sh || exit 1
