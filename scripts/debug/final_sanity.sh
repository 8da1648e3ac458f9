export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1; rc=$?; tail -2 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench_default.log 2>&1; rc=$?; grep "^{" gpurun_out/bench_default.log | cut -c1-200; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_default.log; exit $rc; }
cat > /tmp/pg1.py <<'PY'
import os, torch, torch.distributed as dist
from mdistiller_ddp_amd.parallel.dist import nccl_options
torch.cuda.set_device(0)
dist.init_process_group("nccl", init_method="tcp://127.0.0.1:29511", rank=0, world_size=1, pg_options=nccl_options(), device_id=torch.device("cuda", 0))
t = torch.ones(1024, device="cuda")
dist.all_reduce(t)
torch.cuda.synchronize()
print("rccl world=1 high-priority pg ok", float(t.sum()))
dist.destroy_process_group()
PY
timeout -k 10 120 python /tmp/pg1.py > gpurun_out/pg1.log 2>&1; rc=$?; tail -2 gpurun_out/pg1.log; exit $rc
