"""A/B the throughput bench's mean loss for one config: torch fp32 eager vs
native bf16 eager vs native bf16 graph, same seed/steps as
benchmarks/throughput.py (tells a numerics bug from a diverging random-teacher
run)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from mdistiller_ddp_amd import benchmark  # noqa: E402

if __name__ == "__main__":
    yaml = sys.argv[1]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 100
    opts = sys.argv[3:]
    modes = os.environ.get("MODES", "torch:fp32:0,auto:bf16:0,auto:bf16:1")
    for m in modes.split(","):
        backend, dtype, graph = m.split(":")
        graph = graph == "1"
        r = benchmark.run(yaml, 64, steps, 20, opts=opts, use_graph=graph, backend=backend, dtype=dtype)
        print(json.dumps({"cfg": yaml, "backend": backend, "dtype": dtype, "graph": graph,
                          "opts": opts, "final_loss": r["final_loss"], "ms_per_step": r["ms_per_step"]}), flush=True)
