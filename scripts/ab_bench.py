#!/usr/bin/env python
"""Interleaved A/B of Python-switchable kernel paths on one box / process:
rounds of (arm A, arm B, ...) flagship runs (mdistiller_ddp_amd.benchmark.run),
median ms/step per arm.  Box-to-box spread is ~1-2 %; this compares arms
under the same clocks.

    python scripts/ab_bench.py --arms merge=1;merge=0 [--rounds 3] [--steps 300]
    knobs: merge (shortcut dgrad merge)
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def apply(knobs):
    from mdistiller_ddp_amd.ops import hip_train as H
    for k, v in knobs.items():
        on = v not in ("0", "false", "off")
        if k == "merge":
            H.set_dgrad_merge(on)
        else:
            raise SystemExit(f"unknown knob {k}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arms", required=True, help="';'-separated arms of ','-separated knob=v")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--cfg", default="configs/cifar100/dkd/res32x4_res8x4.yaml")
    ap.add_argument("--batch", type=int, default=64)
    a = ap.parse_args()
    from mdistiller_ddp_amd import benchmark
    arms = [dict(kv.split("=") for kv in arm.split(",") if kv) for arm in a.arms.split(";")]
    res = {i: [] for i in range(len(arms))}
    for r in range(a.rounds):
        for i, knobs in enumerate(arms):
            apply(knobs)
            out = benchmark.run(a.cfg, a.batch, a.steps, a.warmup)
            res[i].append(out["ms_per_step"])
            print(json.dumps({"round": r, "arm": knobs, "ms_per_step": round(out["ms_per_step"], 4)}),
                  flush=True)
    for i, knobs in enumerate(arms):
        print(f"arm {knobs}: median {statistics.median(res[i]):.4f} ms/step  all {[round(v, 4) for v in res[i]]}")


if __name__ == "__main__":
    main()
