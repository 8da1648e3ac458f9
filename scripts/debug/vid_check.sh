export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_vid_nst.py -q --timeout 300 --timeout-method thread > gpurun_out/vid_t.log 2>&1; rc=$?; tail -2 gpurun_out/vid_t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python benchmarks/throughput.py --configs vid_cifar_res32x4_res8x4,vid_cifar_res32x4_res8x4 --steps 100 --warmup 20 2>/dev/null | grep -o '"ms_per_step": [0-9.]*'
PROF="configs/cifar100/vid.yaml:r6b_vid" TOP=6 bash scripts/gpu_run.sh > /dev/null 2>&1; grep "vid_finalize\|wall per step" gpurun_out/prof_r6b_vid_summary.md | cut -c1-120
