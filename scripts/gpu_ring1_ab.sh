#!/bin/bash
# A/B of the single-stage glds variant threshold on the ImageNet conv shapes.
set -o pipefail
mkdir -p gpurun_out
for r in 0 1 2 4; do
  MDA_GLDS_RING1_MAX=$r timeout -k 10 200 python scripts/conv_microbench.py --set imagenet --iters 20 --ops fwd,dgrad > gpurun_out/ring1_$r.log 2>&1 || { tail -5 gpurun_out/ring1_$r.log; exit 1; }
done
python - <<'PY'
import json
rows = {}
for r in (0, 1, 2, 4):
    for line in open(f"gpurun_out/ring1_{r}.log"):
        if line.startswith("{"):
            d = json.loads(line)
            rows.setdefault(tuple(d["shape"]), {})[r] = (d["fwd_us"], d["dgrad_us"])
for k, v in rows.items():
    print(k, " ".join(f"r{r}: fwd {a:7.2f} dg {b:7.2f}" for r, (a, b) in v.items()))
PY
