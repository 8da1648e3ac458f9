set -o pipefail
mkdir -p gpurun_out; export PYTHONPATH=$PWD TMPDIR=/tmp
run() { tag=$1; shift; timeout -k 10 200 "$@" > gpurun_out/q_$tag.log 2>&1; rc=$?; if [ $rc -ne 0 ]; then tail -3 gpurun_out/q_$tag.log; case $rc in 124|134|137|139) exit $rc;; esac; return 0; fi; echo "$tag $(tail -1 gpurun_out/q_$tag.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["final_loss"])')"; }
for t in 64 128 256; do
  MDA_EIG_THREADS=$t timeout -k 10 200 python -u -m pytest tests/test_gpu_kdsvd.py -x -q --timeout 150 --timeout-method thread -k "eigh or cpu" > gpurun_out/t_e$t.log 2>&1 || { tail -20 gpurun_out/t_e$t.log; exit 1; }
  tail -1 gpurun_out/t_e$t.log
  run kdsvd_t$t env MDA_EIG_THREADS=$t python bench.py --steps 100 --warmup 20 --cfg configs/cifar100/kdsvd.yaml
done
