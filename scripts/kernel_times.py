#!/usr/bin/env python
"""Median kernel duration per (kernel, grid) from a rocprofv3 kernel-trace DB."""
import collections
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
flt = sys.argv[2] if len(sys.argv) > 2 else ""
rows = c.execute("select name, grid_x, duration from kernels").fetchall()
agg = collections.defaultdict(list)
for n, g, d in rows:
    if flt in n:
        agg[(n[:70], g)].append(d / 1000.0)
for (n, g), v in sorted(agg.items()):
    v.sort()
    print(f"{n:70s} grid={g:8d} n={len(v):4d} med={v[len(v)//2]:8.2f}us min={v[0]:8.2f}us")
