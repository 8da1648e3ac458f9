set -o pipefail
mkdir -p gpurun_out; export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 100 python -u scripts/graph_external_event_probe.py > gpurun_out/extev.log 2>&1 || { cat gpurun_out/extev.log; exit 1; }
cat gpurun_out/extev.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_virtual_residual.py tests/test_gpu_head.py tests/test_gpu_bn_dgrad_sums.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_head.log 2>&1 || { tail -30 gpurun_out/t_head.log; exit 1; }
tail -2 gpurun_out/t_head.log
timeout -k 10 200 python -u scripts/dgrad_wgrad_overlap_probe.py > gpurun_out/ovl.log 2>&1 || { cat gpurun_out/ovl.log; exit 1; }
cat gpurun_out/ovl.log
for a in "base:" "novres:MDA_VIRTUAL_RES=0" "wgtile:MDA_WG_TILE=64128" "nopar:MDA_DGRAD_PARITY=0"; do
  n=${a%%:*}; e=${a#*:}
  env $e timeout -k 10 300 python bench.py --steps 300 > gpurun_out/b300.log 2>&1 || { tail -5 gpurun_out/b300.log; exit 1; }
  echo "$n $e: $(tail -1 gpurun_out/b300.log | cut -c150-200)"
  env $e timeout -k 10 300 python bench.py --steps 300 --cfg configs/cifar100/vanilla.yaml > gpurun_out/b300.log 2>&1 || { tail -5 gpurun_out/b300.log; exit 1; }
  echo "   vanilla: $(tail -1 gpurun_out/b300.log | cut -c150-200)"
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_multirank.py -x -q --timeout 580 --timeout-method thread -k "events" > gpurun_out/t_mr.log 2>&1 || { tail -30 gpurun_out/t_mr.log; exit 1; }
tail -2 gpurun_out/t_mr.log
