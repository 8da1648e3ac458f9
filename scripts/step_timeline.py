#!/usr/bin/env python
"""Print one steady-state step's kernel sequence from a rocprofv3 kernel-trace DB:
start offset, duration, gap to previous kernel, grid/workgroup, VGPRs, name.

usage: python scripts/step_timeline.py DB [--step N] [--step-kernel REGEX]
"""
import argparse
import glob
import re
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--step", type=int, default=-2, help="which step (python index over step markers)")
    ap.add_argument("--step-kernel", default=r"sgd_kernel|dot_kernel|adam_kernel")
    ap.add_argument("--width", type=int, default=90)
    a = ap.parse_args()
    db = glob.glob(a.db)[0]
    c = sqlite3.connect(db)
    rows = c.execute("select name, start, end, grid_x, grid_y, grid_z, workgroup_x, vgpr_count, "
                     "accum_vgpr_count, lds_size from kernels order by start").fetchall()
    rx = re.compile(a.step_kernel)
    marks = [i for i, r in enumerate(rows) if rx.search(r[0])]
    hi = marks[a.step]
    lo = marks[a.step - 1] if a.step - 1 >= -len(marks) else 0
    seg = rows[lo + 1:hi + 1]
    t0 = seg[0][1]
    prev = rows[lo][2]
    tot = 0
    for name, s, e, gx, gy, gz, wx, vg, ag, lds in seg:
        d = (e - s) / 1000
        tot += d
        nm = re.sub(r"\(anonymous namespace\)::", "", name)[: a.width]
        blocks = (gx // max(wx, 1)) * gy * gz
        print(f"{(s - t0) / 1000:8.1f} {d:7.1f} gap{(s - prev) / 1000:6.1f}  blk{blocks:6d} v{vg:3d}+{ag:3d} "
              f"lds{lds:6d}  {nm}")
        prev = e
    print(f"step wall {(seg[-1][2] - t0) / 1000:.1f} us, busy {tot:.1f} us, {len(seg)} kernels")


if __name__ == "__main__":
    main()
