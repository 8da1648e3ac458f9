set -o pipefail
mkdir -p gpurun_out; export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_dwconv.py tests/test_gpu_e2e.py tests/test_gpu_train_layers.py -x -q --timeout 150 --timeout-method thread > gpurun_out/t_d.log 2>&1; rc=$?; tail -2 gpurun_out/t_d.log; [ $rc -ne 0 ] && { grep -E "assert|Error|FAILED" gpurun_out/t_d.log | head; exit $rc; }
run() { tag=$1; shift; timeout -k 10 200 "$@" > gpurun_out/q_$tag.log 2>&1 || { tail -3 gpurun_out/q_$tag.log; return 0; }; echo "$tag $(tail -1 gpurun_out/q_$tag.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["final_loss"])')"; }
run mv2 python bench.py --steps 100 --warmup 20 --cfg configs/cifar100/dkd/vgg13_mv2.yaml
run shuv1 python bench.py --steps 100 --warmup 20 --cfg configs/cifar100/dkd/res32x4_shuv1.yaml
run r50 python bench.py --steps 30 --warmup 10 --cfg configs/imagenet/r50_mv1/dkd.yaml
run flag python bench.py --steps 300 --warmup 20
