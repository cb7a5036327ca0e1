#!/usr/bin/env python3
"""Mean of one PMC counter per dispatch for kernels whose name contains a
substring (rocprofv3 --pmc counter_collection.csv).  Diagnostic helper.

  python3 tools/pmc_kernel_mean.py DIR SUBSTRING"""
import csv
import glob
import sys
from collections import defaultdict

d, sub = sys.argv[1], sys.argv[2]
acc = defaultdict(lambda: defaultdict(float))
for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if sub in r["Kernel_Name"]:
            acc[(r["Kernel_Name"][:60], r["Counter_Name"])][r["Dispatch_Id"]] += float(r["Counter_Value"])
for (k, c), v in sorted(acc.items()):
    print("%-60s %-12s dispatches %3d mean %.4g" % (k, c, len(v), sum(v.values()) / len(v)))
