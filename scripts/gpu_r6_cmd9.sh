export PYTHONPATH=$PWD TMPDIR=/tmp
for xg in 0 1 3 6; do
  for r in 1 2; do
    ms=$(timeout -k 10 200 python bench.py --steps 300 --warmup 30 RUNTIME.WGRAD_XGRAPH $xg 2>/dev/null | grep -o '"ms_per_step": [0-9.]*') || exit 1
    echo "xgraph=$xg run $r $ms"
  done
done
for xg in 0 3; do
  ms=$(timeout -k 10 200 python bench.py --steps 300 --warmup 30 --cfg configs/cifar100/vanilla.yaml DISTILLER.STUDENT resnet8x4 RUNTIME.WGRAD_XGRAPH $xg 2>/dev/null | grep -o '"ms_per_step": [0-9.]*') || exit 1
  echo "vanilla xgraph=$xg $ms"
done
ARMS=" ;MDA_CONV_HALO2=0;MDA_CONV_HALO=0" ROUNDS=1 bash scripts/gpu_r6_ab.sh
