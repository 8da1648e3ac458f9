export PYTHONPATH=$PWD
run() { tag=$1; shift; timeout -k 10 150 "$@" > gpurun_out/ofd_$tag.log 2>&1 || { echo "$tag FAILED"; tail -5 gpurun_out/ofd_$tag.log; exit 1; }; echo "== $tag"; grep "^[0-9]" gpurun_out/ofd_$tag.log | cut -c1-120 | tail -9; }


timeout -k 10 400 python -u -m pytest tests/test_gpu_e2e.py -q -k "OFD or ofd or lookahead" --timeout 300 --timeout-method thread > gpurun_out/ofd_tests.log 2>&1; rc=$?; tail -4 gpurun_out/ofd_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python benchmarks/throughput.py --configs ofd_cifar_res32x4_res8x4,dkd_cifar_res32x4_res8x4 --steps 100 --warmup 20 2>/dev/null | grep "^{"
