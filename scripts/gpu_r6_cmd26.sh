export PYTHONPATH=$PWD TMPDIR=/tmp
TESTS="tests/test_gpu_train_layers.py::test_apply_ride_matches_separate tests/test_gpu_e2e.py::test_native_bf16_graph_matches_eager tests/test_gpu_e2e.py::test_graph_matches_eager tests/test_gpu_virtual_residual.py tests/test_gpu_conv1x1_stream.py" ARMS=" ;MDA_APPLY_RIDE=0" ROUNDS=2 bash scripts/gpu_r6_ab.sh || exit 1
ARMS=" ;MDA_APPLY_RIDE=0" ROUNDS=1 BENCH_ARGS="--cfg configs/cifar100/vanilla.yaml DISTILLER.STUDENT resnet8x4" bash scripts/gpu_r6_ab.sh
