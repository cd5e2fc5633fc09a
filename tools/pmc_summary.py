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


def name(k):
    """Full template name without the argument list and the anonymous-namespace tag
    (round 5's summaries cut every name at "(anonymous namespace)": "void mipgpu::")."""
    k = k.replace("(anonymous namespace)::", "")
    if k.endswith(")") and "(" in k:
        depth = 0
        for i in range(len(k) - 1, -1, -1):  # the matching "(" of the final ")"
            depth += k[i] == ")"
            depth -= k[i] == "("
            if depth == 0:
                k = k[:i]
                break
    return k


for k, cs in acc.items():
    print("kernel:", name(k))
    for c in sorted(cs):
        vals = cs[c]
        print("  %-24s mean %.6g over %d dispatches" % (c, sum(vals) / len(vals), len(vals)))
