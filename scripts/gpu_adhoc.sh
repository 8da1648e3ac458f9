set -o pipefail
mkdir -p gpurun_out; export PYTHONPATH=$PWD TMPDIR=/tmp
run() { tag=$1; shift; timeout -k 10 200 "$@" > gpurun_out/q_$tag.log 2>&1 || { tail -3 gpurun_out/q_$tag.log; return 0; }; echo "$tag $(tail -1 gpurun_out/q_$tag.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"; }
run base python bench.py --steps 300 --warmup 20
run base2 python bench.py --steps 300 --warmup 20
run r50 python bench.py --steps 30 --warmup 10 --cfg configs/imagenet/r50_mv1/dkd.yaml
run r34 python bench.py --steps 30 --warmup 10 --batch 32 --cfg configs/imagenet/r34_r18/reviewkd.yaml
run mv2 python bench.py --steps 100 --warmup 20 --cfg configs/cifar100/dkd/vgg13_mv2.yaml
run shuv1 python bench.py --steps 100 --warmup 20 --cfg configs/cifar100/dkd/res32x4_shuv1.yaml
