set -o pipefail
mkdir -p gpurun_out; export PYTHONPATH=$PWD TMPDIR=/tmp
run() { tag=$1; shift; timeout -k 10 200 "$@" > gpurun_out/q_$tag.log 2>&1 || { tail -3 gpurun_out/q_$tag.log; return 0; }; echo "$tag $(tail -1 gpurun_out/q_$tag.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["final_loss"])')"; }
for v in 1 0 1 0; do run ps$v env MDA_PACK_STREAM=$v python bench.py --steps 300 --warmup 20; done
timeout -k 10 300 python -u -m pytest tests/test_gpu_e2e.py -x -q --timeout 150 --timeout-method thread > gpurun_out/t_e.log 2>&1; rc=$?; tail -2 gpurun_out/t_e.log; exit $rc
