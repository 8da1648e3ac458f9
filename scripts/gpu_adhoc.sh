export PYTHONPATH=$PWD TMPDIR=/tmp
TESTS="tests/test_gpu_e2e.py tests/test_gpu_train_layers.py tests/test_gpu_conv_pair.py tests/test_gpu_head.py tests/test_gpu_bn_dgrad_sums.py" TEST_TIMEOUT=900 bash scripts/gpu_run.sh && \
ARMS="MDA_BN_FINISH=0 MDA_BN_BWD_FINISH=0 MDA_GLDS_DEEP=0 MDA_PACK_EXTRAS=0 MDA_HEAD_KSPLIT=1 MDA_HALO_PERM8=0;MDA_BN_FINISH=0 MDA_BN_BWD_FINISH=0;MDA_BN_BWD_FINISH=0;MDA_HALO_PERM8=0;MDA_X=1" ROUNDS=2 bash scripts/ab_env.sh | tail -5
