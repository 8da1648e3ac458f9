#!/usr/bin/env python
"""Where does the short-run gap come from?  (round-6 probe for VERDICT r5 Weak #5)

Builds the flagship TrainStep exactly as ``bench.py`` does, runs W warm-up
steps, then times several back-to-back windows of K steps, each bracketed by
``synchronize`` like bench.py's timed region.  It also records one event pair
per step on the main stream for the first window, so a slow first replay
shows up as one long step rather than a uniformly slower window.

usage: python scripts/replay_ramp.py [--steps 20] [--warmup 5] [--windows 6]
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
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--windows", type=int, default=6)
    ap.add_argument("--cfg", default="configs/cifar100/dkd/res32x4_res8x4.yaml")
    ap.add_argument("--idle-sweep", default="", help="comma list of pre-window idle times in ms")
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import torch
    from mdistiller_ddp_amd import benchmark

    captured = {}
    orig_run = benchmark.run

    # reuse benchmark.run's set-up by intercepting the TrainStep it builds
    from mdistiller_ddp_amd.engine import step as step_mod
    Orig = step_mod.TrainStep

    class Spy(Orig):
        def __init__(self, *args, **kw):
            super().__init__(*args, **kw)
            captured["step"] = self

    benchmark_TrainStep = Spy
    step_mod.TrainStep = benchmark_TrainStep
    r = orig_run(a.cfg, 64, 1, a.warmup, use_graph=True)
    step = captured["step"]
    print("bench-style (1 timed step after warmup):", round(r["ms_per_step"], 4), flush=True)

    from mdistiller_ddp_amd.data.synthetic import SyntheticLoader
    dev = torch.device("cuda", 0)
    loader = SyntheticLoader("cifar100", 64, dev, steps_per_epoch=10 ** 9, pool=4, seed=0,
                             channels_last=True)
    it = iter(loader)
    cur = next(it)
    from mdistiller_ddp_amd.ops import _ext
    clk = torch.zeros(a.windows, a.steps + 1, device=dev)
    out = []
    for w in range(a.windows):
        evs = [torch.cuda.Event(enable_timing=True) for _ in range(a.steps + 1)] if w < 2 else None
        hot = w % 2 == 1  # odd windows: the GPU is kept busy (matmuls) right up to the window
        if hot:
            xx = torch.randn(4096, 4096, device=dev, dtype=torch.bfloat16)
            for _ in range(60):
                xx = (xx @ xx).clamp_(-1, 1)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        hts = []
        for i in range(a.steps):
            if evs:
                evs[i].record()
                _ext.call("mda_clock_probe", clk[w], i)
            h0 = time.perf_counter()
            nb = next(it)
            step.step(cur, next_batch=nb)
            cur = nb
            hts.append(time.perf_counter() - h0)
        if evs:
            evs[-1].record()
            _ext.call("mda_clock_probe", clk[w], a.steps)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        rec = {"window": w, "hot": hot, "ms_per_step": round(1000 * el / a.steps, 4)}
        if evs:
            rec["per_step_ms"] = [round(evs[i].elapsed_time(evs[i + 1]), 4) for i in range(a.steps)]
            rec["sclk_mhz"] = [round(v) for v in clk[w].tolist()]
            rec["host_enqueue_ms"] = [round(1000 * v, 3) for v in hts]
        out.append(rec)
        print(json.dumps(rec), flush=True)
        time.sleep(0.05)
    if a.idle_sweep:
        import gc
        res = {}
        for rep in range(a.reps):
            for idle in [float(v) for v in a.idle_sweep.split(",")]:
                torch.cuda.synchronize()
                if idle < 0:  # a gc.collect() in the gap, as bench.py had before its timed loop
                    t1 = time.perf_counter()
                    gc.collect()
                    idle_eff = 1000 * (time.perf_counter() - t1)
                else:
                    time.sleep(idle / 1000.0)
                    idle_eff = idle
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                t0 = time.perf_counter()
                for i in range(a.steps):
                    if i == 0:
                        e0.record()
                    nb = next(it)
                    step.step(cur, next_batch=nb)
                    cur = nb
                    if i == 0:
                        e1.record()
                torch.cuda.synchronize()
                ms = 1000 * (time.perf_counter() - t0) / a.steps
                res.setdefault(idle, []).append((round(ms, 4), round(e0.elapsed_time(e1), 3),
                                                 round(idle_eff, 1)))
        for k, v in res.items():
            print(json.dumps({"idle_ms": k, "runs (ms/step, first-step ms, idle ms)": v}), flush=True)
    # long window for the steady-state reference
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(300):
        nb = next(it)
        step.step(cur, next_batch=nb)
        cur = nb
    torch.cuda.synchronize()
    print(json.dumps({"window": "300", "ms_per_step": round(1000 * (time.perf_counter() - t0) / 300, 4)}))


if __name__ == "__main__":
    main()
