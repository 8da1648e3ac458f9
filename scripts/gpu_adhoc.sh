set -o pipefail
mkdir -p gpurun_out; export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_vid_nst.py -x -q --timeout 150 --timeout-method thread > gpurun_out/t_g.log 2>&1; rc=$?; tail -3 gpurun_out/t_g.log; [ $rc -ne 0 ] && { grep -E "Error|error|assert|FAILED" gpurun_out/t_g.log | head -30; exit $rc; }
run() { tag=$1; shift; timeout -k 10 200 "$@" > gpurun_out/q_$tag.log 2>&1 || { tail -5 gpurun_out/q_$tag.log; exit 1; }; echo "$tag $(tail -1 gpurun_out/q_$tag.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("final_loss"))')"; }
run nst python bench.py --steps 100 --warmup 20 --cfg configs/cifar100/nst.yaml
run flag python bench.py --steps 300 --warmup 20
