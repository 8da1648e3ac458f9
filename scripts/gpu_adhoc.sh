set -o pipefail
mkdir -p gpurun_out; export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_train_layers.py tests/test_gpu_e2e.py -x -q --timeout 150 --timeout-method thread > gpurun_out/t_c.log 2>&1; rc=$?; tail -2 gpurun_out/t_c.log; [ $rc -ne 0 ] && { grep -E "assert|Error|FAILED" gpurun_out/t_c.log | head; exit $rc; }
run() { tag=$1; shift; timeout -k 10 200 "$@" > gpurun_out/q_$tag.log 2>&1 || { tail -3 gpurun_out/q_$tag.log; return 0; }; echo "$tag $(tail -1 gpurun_out/q_$tag.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["final_loss"])')"; }
run flag python bench.py --steps 300 --warmup 20
run flag2 python bench.py --steps 300 --warmup 20
run r50 python bench.py --steps 30 --warmup 10 --cfg configs/imagenet/r50_mv1/dkd.yaml
PROF="configs/cifar100/dkd/res32x4_res8x4.yaml:r3_flagship_b" bash scripts/gpu_run.sh
grep wgrad_reduce gpurun_out/prof_r3_flagship_b_summary.md | cut -c1-100
