export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_dot_single.py -q -s --timeout 300 --timeout-method thread > gpurun_out/dot1.log 2>&1; rc=$?; grep -i "rel\|passed\|failed\|Error" gpurun_out/dot1.log | tail -20; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python benchmarks/throughput.py --configs dot_cifar_vgg13_vgg8,dkd_cifar_vgg13_vgg8,dkd_cifar_vgg13_mv2 --steps 100 --warmup 20 2>/dev/null | grep "^{" | cut -c1-200
timeout -k 10 200 python bench.py --cfg configs/imagenet/r34_r18/dot.yaml --batch 32 --steps 20 --warmup 5 2>/dev/null | grep "^{" | cut -c1-160
timeout -k 10 200 python bench.py --cfg configs/imagenet/r34_r18/dot.yaml --batch 32 --steps 20 --warmup 5 RUNTIME.DOT_SINGLE_PASS False 2>/dev/null | grep "^{" | cut -c1-160
