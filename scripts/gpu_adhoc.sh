set -o pipefail
mkdir -p gpurun_out; export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_bn_dgrad_sums.py tests/test_gpu_bn_fused.py tests/test_gpu_e2e.py tests/test_gpu_head.py tests/test_gpu_kdsvd.py -x -q --timeout 150 --timeout-method thread > gpurun_out/t_r.log 2>&1; rc=$?; tail -2 gpurun_out/t_r.log; [ $rc -ne 0 ] && { grep -E "assert|Error|FAILED" gpurun_out/t_r.log | head; exit $rc; }
run() { tag=$1; shift; timeout -k 10 200 "$@" > gpurun_out/q_$tag.log 2>&1 || { tail -3 gpurun_out/q_$tag.log; return 0; }; echo "$tag $(tail -1 gpurun_out/q_$tag.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["final_loss"])')"; }
run flag python bench.py --steps 300 --warmup 20
run flag_off env MDA_BN_DGRAD_SUMS=0 python bench.py --steps 300 --warmup 20
run flag2 python bench.py --steps 300 --warmup 20
run r50 python bench.py --steps 60 --warmup 10 --cfg configs/imagenet/r50_mv1/dkd.yaml
run r50_off env MDA_BN_DGRAD_SUMS=0 python bench.py --steps 60 --warmup 10 --cfg configs/imagenet/r50_mv1/dkd.yaml
run mv2 python bench.py --steps 100 --warmup 20 --cfg configs/cifar100/dkd/vgg13_mv2.yaml
run kdsvd python bench.py --steps 100 --warmup 20 --cfg configs/cifar100/kdsvd.yaml
