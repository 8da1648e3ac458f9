export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 300 python -u scripts/teacher_only.py 2>&1 | grep "^{" || exit 1
ARMS=" ;MDA_HALO_RING=8;MDA_GLDS_RING1_MAX=2;MDA_GLDS_RING1_MAX=8;MDA_CONV_XCD=0;MDA_CONV_KROT=0;MDA_CONV1X1_MIN_M=4096" ROUNDS=1 bash scripts/gpu_r6_ab.sh
