# Native SP / PKT / RKD (csrc/relation.hip): numerics vs the PyTorch fp32 forms, then
# throughput of the three configs.
set -x
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_relation.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_rel.log 2>&1 ; rc=$?; tail -25 gpurun_out/pytest_rel.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 600 python -u benchmarks/throughput.py --configs rkd_cifar_res32x4_res8x4,sp_cifar_res32x4_res8x4,pkt_cifar_res32x4_res8x4,dkd_cifar_res32x4_shuv1 --steps 60 --warmup 15 --out gpurun_out/tp_rel.jsonl > gpurun_out/tp_rel.log 2>&1 || { tail -30 gpurun_out/tp_rel.log; exit 1; }
cut -c1-200 gpurun_out/tp_rel.jsonl
