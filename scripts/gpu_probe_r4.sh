set -o pipefail
mkdir -p gpurun_out; export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_vid_nst.py tests/test_gpu_kdsvd.py tests/test_gpu_embed.py -q --timeout 200 --timeout-method thread > gpurun_out/t_v.log 2>&1; echo "tests rc=$?"
grep -E "FAILED|passed|failed" gpurun_out/t_v.log | head -8
PROF="configs/cifar100/nst.yaml:r4_nst;configs/cifar100/kdsvd.yaml:r4_kdsvd;configs/cifar100/crd.yaml:r4_crd;configs/cifar100/at.yaml:r4_at" bash scripts/gpu_run.sh
