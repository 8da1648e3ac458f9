export PYTHONPATH=$PWD TMPDIR=/tmp
TESTS="tests/test_gpu_train_layers.py tests/test_gpu_e2e.py::test_native_bf16_graph_matches_eager tests/test_gpu_e2e.py::test_partial_batch_between_replays_matches_eager tests/test_gpu_bn_dgrad_sums.py" ARMS=" ;MDA_WGRAD_RIDE=0" ROUNDS=2 bash scripts/gpu_r6_ab.sh || exit 1
ARMS=" ;MDA_WGRAD_RIDE=0" ROUNDS=1 BENCH_ARGS="--cfg configs/cifar100/vanilla.yaml DISTILLER.STUDENT resnet8x4" bash scripts/gpu_r6_ab.sh
