set -o pipefail
mkdir -p gpurun_out; export PYTHONPATH=$PWD TMPDIR=/tmp
run() { tag=$1; shift; timeout -k 10 200 "$@" > gpurun_out/q_$tag.log 2>&1 || { tail -5 gpurun_out/q_$tag.log; exit 1; }; echo "$tag $(tail -1 gpurun_out/q_$tag.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("host_ms_per_step"))')"; }
MDA_BN_FUSED=0 run r50_unfused python bench.py --steps 30 --warmup 10 --cfg configs/imagenet/r50_mv1/dkd.yaml
MDA_BN_FUSED=0 MDA_BN_DGRAD_SUMS=0 run r50_unfused_nosums python bench.py --steps 30 --warmup 10 --cfg configs/imagenet/r50_mv1/dkd.yaml
MDA_BN_DGRAD_SUMS=0 run r50_nosums python bench.py --steps 30 --warmup 10 --cfg configs/imagenet/r50_mv1/dkd.yaml
PROF="configs/imagenet/r50_mv1/dkd.yaml:r50b" bash scripts/gpu_run.sh
