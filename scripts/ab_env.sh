#!/bin/bash
# Interleaved A/B of environment-switched paths, one fresh process per run:
#   ARMS="A_ENV;B_ENV;..." ROUNDS=3 STEPS=500 bash scripts/ab_env.sh
# (each arm's env is a space-separated list of VAR=value; empty = defaults).
# In-process repeats drift with the stream / hardware-queue history, so every
# run is its own process.
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD TMPDIR=/tmp
IFS=';' read -ra A <<< "$ARMS"
for r in $(seq 1 ${ROUNDS:-3}); do
  i=0
  for arm in "${A[@]}"; do
    out=$(env $arm timeout -k 10 300 python bench.py --steps ${STEPS:-500} --warmup 30 ${BENCH_ARGS} 2>/dev/null | grep '^{') || exit 1
    ms=$(echo "$out" | python -c "import json,sys; print(json.loads(sys.stdin.read())['ms_per_step'])")
    echo "round $r arm $i [$arm] $ms"
    i=$((i+1))
  done
done | tee gpurun_out/ab_env.txt
python - <<'PY'
import collections, statistics
d = collections.defaultdict(list)
for line in open("gpurun_out/ab_env.txt"):
    p = line.split()
    arm = line[line.index("["):line.index("]") + 1]
    d[arm].append(float(p[-1]))
for k, v in d.items():
    print(f"{k:50s} median {statistics.median(v):.4f}  {v}")
PY
