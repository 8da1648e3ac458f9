set -o pipefail
mkdir -p gpurun_out; export PYTHONPATH=$PWD TMPDIR=/tmp
run() { tag=$1; shift; timeout -k 10 200 "$@" > gpurun_out/q_$tag.log 2>&1; rc=$?; if [ $rc -ne 0 ]; then tail -3 gpurun_out/q_$tag.log; case $rc in 124|134|137|139) exit $rc;; esac; return 0; fi; echo "$tag $(tail -1 gpurun_out/q_$tag.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["final_loss"])')"; }
run flag python bench.py --steps 300 --warmup 20
run flag_off env MDA_BN_DGRAD_SUMS=0 python bench.py --steps 300 --warmup 20
run flag2 python bench.py --steps 300 --warmup 20
run r50 python bench.py --steps 60 --warmup 10 --cfg configs/imagenet/r50_mv1/dkd.yaml
run mv2 python bench.py --steps 100 --warmup 20 --cfg configs/cifar100/dkd/vgg13_mv2.yaml
timeout -k 10 200 python -u scripts/debug/kdsvd_capture_probe.py bmm8 eig8 loss3_fwd_bwd || exit $?
run kdsvd python bench.py --steps 100 --warmup 20 --cfg configs/cifar100/kdsvd.yaml
