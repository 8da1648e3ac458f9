#!/usr/bin/env python
"""Average duration per kernel name from a rocprofv3 --kernel-trace DB.
usage: python scripts/kstats.py DB [--top N] [--filter REGEX]"""
import argparse
import glob
import re
import sqlite3

ap = argparse.ArgumentParser()
ap.add_argument("db")
ap.add_argument("--top", type=int, default=30)
ap.add_argument("--filter", default=None)
a = ap.parse_args()
db = glob.glob(a.db)[0]
c = sqlite3.connect(db)
rows = c.execute("select name, duration from kernels").fetchall()
agg = {}
for n, d in rows:
    if a.filter and not re.search(a.filter, n):
        continue
    x = agg.setdefault(n, [0, 0.0, []])
    x[0] += 1
    x[1] += d
    x[2].append(d)
for n, (k, tot, ds) in sorted(agg.items(), key=lambda kv: -kv[1][1])[: a.top]:
    ds.sort()
    print(f"{k:6d} avg {tot / k / 1000:8.2f} us  med {ds[len(ds) // 2] / 1000:8.2f} us  {n[:120]}")
