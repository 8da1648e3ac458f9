# halo-kernel defaults: flagship arms + the ImageNet configs with / without halo2
export PYTHONPATH=$PWD TMPDIR=/tmp
ARMS=" ;MDA_CONV_HALO2=1;MDA_HALO_RING=3;MDA_HALO_NARROW=0" ROUNDS=2 bash scripts/gpu_r6_ab.sh || exit 1
for h in 0 1; do
  MDA_CONV_HALO2=$h timeout -k 10 400 python benchmarks/throughput.py --configs reviewkd_imagenet_r34_r18,dkd_imagenet_r50_mv1 --steps 20 --warmup 8 2>/dev/null | grep "^{" | python -c "
import json,sys
for l in sys.stdin:
    r=json.loads(l); print('halo2=$h', r.get('config'), r.get('ms_per_step'), r.get('host_idle_ms_per_step'))" || exit 1
done
