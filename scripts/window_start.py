#!/usr/bin/env python
"""Kernel timeline of the first steps of each timed window (scripts/replay_ramp.py
under ``rocprofv3 --kernel-trace``): windows are found by the idle gap
(> --gap-ms) before them; prints per-step wall / busy for the first steps of a
window and the first step's kernels with their gaps.

usage: python scripts/window_start.py DB [--gap-ms 20] [--steps 4]
"""
import argparse
import glob
import re
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--gap-ms", type=float, default=20.0)
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--step-kernel", default=r"sgd_kernel")
    a = ap.parse_args()
    c = sqlite3.connect(glob.glob(a.db)[0])
    rows = c.execute("select name, start, end from kernels order by start").fetchall()
    rx = re.compile(a.step_kernel)
    starts = [i for i in range(1, len(rows)) if rows[i][1] - rows[i - 1][2] > a.gap_ms * 1e6]
    for w, i0 in enumerate(starts[-4:]):
        print(f"== window at kernel {i0}: idle gap before {(rows[i0][1] - rows[i0 - 1][2]) / 1e6:.2f} ms")
        i = i0
        for s in range(a.steps):
            j = i
            while j < len(rows) and not rx.search(rows[j][0]):
                j += 1
            seg = rows[i:j + 1]
            if not seg:
                break
            busy = sum(e - b for _, b, e in seg) / 1e3
            print(f"  step {s}: wall {(seg[-1][2] - seg[0][1]) / 1e3:8.1f} us  kernels {len(seg):4d}  "
                  f"sum-dur {busy:8.1f} us")
            if s == 0 or s == a.steps - 1:
                prev = seg[0][1]
                for name, b, e in seg[:12]:
                    nm = re.sub(r"\(anonymous namespace\)::", "", name)[:70]
                    print(f"      +{(b - seg[0][1]) / 1e3:8.1f} dur {(e - b) / 1e3:7.1f} gap {(b - prev) / 1e3:6.1f}  {nm}")
                    prev = e
            i = j + 1


if __name__ == "__main__":
    main()
