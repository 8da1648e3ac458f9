set -o pipefail
mkdir -p gpurun_out; export PYTHONPATH=$PWD TMPDIR=/tmp
run() { tag=$1; shift; timeout -k 10 200 "$@" > gpurun_out/q_$tag.log 2>&1 || { tail -3 gpurun_out/q_$tag.log; return 0; }; echo "$tag $(tail -1 gpurun_out/q_$tag.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"; }
run base python bench.py --steps 300 --warmup 20
run glds0 env MDA_CONV_GLDS=0 python bench.py --steps 300 --warmup 20
run ring8 env MDA_HALO_RING=8 python bench.py --steps 300 --warmup 20
run tgt128 env MDA_CONV_TARGET=128 python bench.py --steps 300 --warmup 20
run tgt512 env MDA_CONV_TARGET=512 python bench.py --steps 300 --warmup 20
run r1max8 env MDA_GLDS_RING1_MAX=8 python bench.py --steps 300 --warmup 20
run narrow0 env MDA_HALO_NARROW=0 python bench.py --steps 300 --warmup 20
run halo2off env MDA_CONV_HALO2=0 python bench.py --steps 300 --warmup 20
run branch1 env MDA_BRANCH_STREAMS=1 python bench.py --steps 300 --warmup 20
run wgstream python bench.py --steps 300 --warmup 20 RUNTIME.WGRAD_STREAM on
run nodefer python bench.py --steps 300 --warmup 20 RUNTIME.WGRAD_DEFER False
run reg1x1all env MDA_REG1X1_MIN_M=0 python bench.py --steps 300 --warmup 20
run base2 python bench.py --steps 300 --warmup 20
