# Detection on the GPU: kernel + end-to-end tests, then the train_net bench at
# COCO shape (800x1067 synthetic, 2 images/GPU) for DKD and ReviewKD.
set -x
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_detection.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_det.log 2>&1 || { tail -40 gpurun_out/pytest_det.log; exit 1; }
tail -3 gpurun_out/pytest_det.log
for c in DKD/DKD-R18-R101 ReviewKD/ReviewKD-R18-R101 DKD/ReviewDKD-R50-R101; do
  timeout -k 10 300 python -u detection/train_net.py --config-file detection/configs/$c.yaml --bench ${STEPS:-20} --warmup 5 \
    SOLVER.IMS_PER_BATCH 2 RUNTIME.SYNTHETIC_SIZE "(800,1067)" ${EXTRA:-} > gpurun_out/detbench_$(basename $c).log 2>&1 || { tail -30 gpurun_out/detbench_$(basename $c).log; exit 1; }
  tail -1 gpurun_out/detbench_$(basename $c).log
done
