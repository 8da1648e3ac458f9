set -o pipefail
mkdir -p gpurun_out; export PYTHONPATH=$PWD TMPDIR=/tmp
run() { tag=$1; shift; timeout -k 10 200 "$@" > gpurun_out/q_$tag.log 2>&1 || { tail -5 gpurun_out/q_$tag.log; exit 1; }; echo "$tag $(tail -1 gpurun_out/q_$tag.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"; }
for v in 32768 999999999; do
MDA_REG1X1_MIN_M=$v timeout -k 10 120 python scripts/conv_microbench.py --set cifar --shape 9 --ops fwd --graph --iters 30 > gpurun_out/cv.log 2>&1 || exit 1
echo "cifar1x1 $v $(grep shape gpurun_out/cv.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["fwd_us"])')"
MDA_REG1X1_MIN_M=$v run r50_$v python bench.py --steps 30 --warmup 10 --cfg configs/imagenet/r50_mv1/dkd.yaml
MDA_REG1X1_MIN_M=$v run flag_$v python bench.py --steps 300 --warmup 20
MDA_REG1X1_MIN_M=$v run mv2_$v python bench.py --steps 100 --warmup 20 --cfg configs/cifar100/dkd/vgg13_mv2.yaml
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_train_layers.py -x -q --timeout 150 --timeout-method thread > gpurun_out/t_c.log 2>&1; rc=$?; tail -2 gpurun_out/t_c.log; exit $rc
