#!/usr/bin/env python
"""Median per-dispatch PMC counter values of kernels matching a pattern,
from rocprofv3 ``--pmc`` CSV output (``*counter_collection.csv``).

usage: python scripts/pmc_summary.py ROOT DIRGLOB KERNEL_SUBSTR
"""
import collections
import csv
import glob
import os
import sys

root, dglob, pat = sys.argv[1], sys.argv[2], sys.argv[3]
vals = collections.defaultdict(list)
for d in sorted(glob.glob(os.path.join(root, dglob))):
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if pat in row["Kernel_Name"]:
                    vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
for k in sorted(vals):
    v = sorted(vals[k])
    print(f"{pat:12s} {k:28s} n={len(v):4d} med={v[len(v)//2]:.4g}")
