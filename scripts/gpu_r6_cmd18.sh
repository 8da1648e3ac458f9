export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_multirank.py -k "not bitwise" -x -v --timeout 600 --timeout-method thread > gpurun_out/t_multirank.log 2>&1; rc=$?; tail -12 gpurun_out/t_multirank.log; [ $rc -ne 0 ] && exit $rc
for ws in auto off; do
  timeout -k 10 400 python benchmarks/throughput.py --configs reviewkd_imagenet_r34_r18,dkd_imagenet_r50_mv1 --steps 20 --warmup 8 --opts RUNTIME.WGRAD_STREAM $ws 2>/dev/null | grep "^{" | python -c "
import json,sys
for l in sys.stdin:
    r=json.loads(l); print('wgrad_stream=$ws', r.get('config'), r.get('ms_per_step'), r.get('host_idle_ms_per_step'), r.get('error',''))" || exit 1
done
