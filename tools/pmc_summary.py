#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSV passes: per-kernel mean counter value per dispatch."""
import csv
import glob
import os
import sys
from collections import defaultdict

root = sys.argv[1]
acc = defaultdict(lambda: defaultdict(list))
for path in sorted(glob.glob(os.path.join(root, "p*", "**", "*counter_collection.csv"), recursive=True)):
    per = defaultdict(lambda: defaultdict(float))
    for row in csv.DictReader(open(path)):
        k = row.get("Kernel_Name", "?")
        disp = row.get("Dispatch_Id", "0")
        per[(k, disp)][row["Counter_Name"]] += float(row["Counter_Value"])
    for (k, disp), cs in per.items():
        for c, v in cs.items():
            acc[k][c].append(v)
for k, cs in acc.items():
    short = k.split("(")[0][-60:]
    print("kernel:", short)
    for c in sorted(cs):
        vals = cs[c]
        print("  %-24s mean %.6g over %d dispatches" % (c, sum(vals) / len(vals), len(vals)))
