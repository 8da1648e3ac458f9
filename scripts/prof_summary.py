#!/usr/bin/env python
"""Summarise a rocprofv3 ``--kernel-trace`` database over the steady-state steps.

The window is delimited by the per-step optimizer kernel (``--step-kernel``,
default the fused SGD kernel): kernels that start after the end of its
``--skip``-th dispatch and end at/before its last dispatch are counted, and
per-step times are divided by the number of steps in the window.

usage: python scripts/prof_summary.py DB [--skip W] [--step-kernel REGEX] [--top N] [--md OUT]
"""
import argparse
import glob
import re
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--skip", type=int, default=3)
    ap.add_argument("--step-kernel", default=r"sgd_kernel|dot_kernel|adam_kernel")
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--md", default=None)
    ap.add_argument("--by-dispatch", action="store_true",
                    help="also list one step's dispatches in order with their grid sizes")
    args = ap.parse_args()
    dbs = glob.glob(args.db) if "*" in args.db else [args.db]
    c = sqlite3.connect(dbs[0])
    rows = c.execute("select name, start, end, duration from kernels order by start").fetchall()
    rx = re.compile(args.step_kernel)
    marks = [r for r in rows if rx.search(r[0])]
    if len(marks) <= args.skip + 1:
        raise SystemExit(f"only {len(marks)} step markers found")
    t0 = marks[args.skip][2]
    t1 = marks[-1][2]
    nsteps = len(marks) - 1 - args.skip
    win = [r for r in rows if r[1] >= t0 and r[2] <= t1]
    agg = {}
    for name, s, e, d in win:
        a = agg.setdefault(name, [0, 0.0])
        a[0] += 1
        a[1] += d / 1000.0
    busy = sum(v[1] for v in agg.values()) / nsteps
    wall = (t1 - t0) / 1000.0 / nsteps
    lines = [f"steps in window: {nsteps}; wall per step {wall:.1f} us; kernel-busy per step {busy:.1f} us;"
             f" kernels per step {sum(v[0] for v in agg.values()) / nsteps:.1f}",
             "", "| us/step | % | calls/step | kernel |", "|---:|---:|---:|---|"]
    for name, (n, tot) in sorted(agg.items(), key=lambda kv: -kv[1][1])[: args.top]:
        short = name if len(name) < 110 else name[:107] + "..."
        lines.append(f"| {tot / nsteps:.1f} | {100 * tot / nsteps / busy:.1f} | {n / nsteps:.1f} | `{short}` |")
    if args.by_dispatch:
        cols = [r[1] for r in c.execute("PRAGMA table_info(kernels)").fetchall()]
        gcols = [x for x in cols if "grid" in x.lower() or "workgroup" in x.lower()]
        sel = ", ".join(["name", "start", "end", "duration"] + gcols)
        last = [m for m in marks][-2:]
        step = c.execute(f"select {sel} from kernels where start >= ? and end <= ? order by start",
                         (last[0][2], last[1][2])).fetchall()
        lines += ["", f"one step in dispatch order ({', '.join(gcols)}):", "",
                  "| start us | us | kernel | grid |", "|---:|---:|---|---|"]
        for r in step:
            short = r[0] if len(r[0]) < 70 else r[0][:67] + "..."
            lines.append(f"| {(r[1] - last[0][2]) / 1000:.1f} | {r[3] / 1000:.1f} | `{short}` | "
                         f"{' '.join(str(v) for v in r[4:])} |")
    text = "\n".join(lines)
    print(text)
    if args.md:
        with open(args.md, "w") as f:
            f.write(text + "\n")


if __name__ == "__main__":
    main()
