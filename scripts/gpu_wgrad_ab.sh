#!/bin/bash
# wgrad A/B: register-staged kernel vs LDS-DMA kernel (tile variants), ImageNet + CIFAR shapes.
set -o pipefail
mkdir -p gpurun_out
: timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_train_layers.py -x -q --timeout 120 --timeout-method thread -k "wgrad or train or stem" > gpurun_out/wg_tests.log 2>&1 || { tail -30 gpurun_out/wg_tests.log; exit 1; }
: 
for cfg in "old MDA_WG_GLDS=0" "auto X=1" "t64 MDA_WG_TILE=64064" "t64x128 MDA_WG_TILE=64128"; do
  set -- $cfg
  for st in imagenet cifar; do
    env $2 timeout -k 10 200 python scripts/conv_microbench.py --set $st --iters 20 --ops wgrad --graph > gpurun_out/wg_${1}_$st.log 2>&1 || { tail -5 gpurun_out/wg_${1}_$st.log; exit 1; }
  done
done
python - <<'PY'
import json
tags = ["old", "auto", "t64", "t64x128"]
for st in ("imagenet", "cifar"):
    rows = {}
    for t in tags:
        for line in open(f"gpurun_out/wg_{t}_{st}.log"):
            if line.startswith("{"):
                d = json.loads(line)
                rows.setdefault(tuple(d["shape"]), {})[t] = d["wgrad_us"]
    for k, v in rows.items():
        print(st, k, " ".join(f"{t}: {v.get(t, float('nan')):7.2f}" for t in tags))
PY
