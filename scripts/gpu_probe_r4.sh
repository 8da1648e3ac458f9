set -o pipefail
mkdir -p gpurun_out; export PYTHONPATH=$PWD TMPDIR=/tmp
out=gpurun_out/envsweep.log; : > $out
for e in "X=0" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=1" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=0" "HSA_ENABLE_SDMA=0"; do
  echo "== $e" >> $out
  env $e timeout -k 10 200 python -u bench.py --steps 300 --warmup 30 >> $out 2>&1 || { echo "rc=$? $e"; tail -5 $out; exit 1; }
done
grep -E "^==|ms_per_step" $out | sed 's/.*"ms_per_step": \([0-9.]*\).*/  \1 ms/'
MDA_EVENTS_SYNC=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_multirank.py -q --timeout 380 --timeout-method thread -k events > gpurun_out/t_ev.log 2>&1; echo "events(sync) rc=$?"
grep -E "passed|failed|assert|rel" gpurun_out/t_ev.log | head -5
timeout -k 10 900 python -u benchmarks/throughput.py --steps 60 --warmup 15 --out gpurun_out/r4_tp_all.jsonl > gpurun_out/tp_all.log 2>&1; echo "tp rc=$?"
grep "{" gpurun_out/tp_all.log | cut -c1-150
