#!/usr/bin/env python
"""How much of the flagship step does the look-ahead teacher hide?

Builds the flagship TrainStep as bench.py does, then times (a) the full step,
(b) the captured look-ahead teacher graph replayed alone on its stream and
(c) the student's step graph replayed alone (teacher outputs left as they
are), each over K back-to-back replays.  overlap = (b) + (c) - (a).

usage: python scripts/teacher_only.py [--steps 300] [--warmup 30]
"""
import argparse
import json
import os
import sys
import time

os.environ.setdefault("HIP_FORCE_DEV_KERNARG", "1")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--warmup", type=int, default=30)
    ap.add_argument("--cfg", default="configs/cifar100/dkd/res32x4_res8x4.yaml")
    a = ap.parse_args()
    import torch
    from mdistiller_ddp_amd import benchmark
    from mdistiller_ddp_amd.engine import step as step_mod

    captured = {}
    Orig = step_mod.TrainStep

    class Spy(Orig):
        def __init__(self, *args, **kw):
            super().__init__(*args, **kw)
            captured["step"] = self

    step_mod.TrainStep = Spy
    r = benchmark.run(a.cfg, 64, a.steps, a.warmup, use_graph=True)
    st = captured["step"]
    out = {"full_step_ms": round(r["ms_per_step"], 4)}

    def timed(fn, stream):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with torch.cuda.stream(stream):
            for _ in range(a.steps):
                fn()
        torch.cuda.synchronize()
        return round(1000 * (time.perf_counter() - t0) / a.steps, 4)

    if st._tsplit is not None:
        g_tp, _, _, ts, _, _ = st._tsplit
        out["teacher_graph_ms"] = timed(g_tp.replay, ts)
    g1, g2 = st._graphs
    out["student_graph_ms"] = timed(g1.replay, torch.cuda.current_stream())
    if "teacher_graph_ms" in out:
        out["hidden_ms"] = round(out["teacher_graph_ms"] + out["student_graph_ms"] - out["full_step_ms"], 4)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
