"""Summarise rocprofv3 --pmc counter CSVs under a directory: per kernel (template instance), the
mean value per dispatch of every counter, and the dispatch count.  Usage: pmc_kernels.py DIR"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

vals = defaultdict(lambda: defaultdict(list))
for path in glob.glob(os.path.join(sys.argv[1], "**", "*counter_collection*.csv"), recursive=True):
    with open(path) as f:
        for row in csv.DictReader(f):
            name = row.get("Kernel_Name", "")
            m = re.search(r"k_(?:march|range|frame)<ocn::([^(]*?)>\(", name) or re.search(r"ocn::(\w+)\(", name)
            k = m.group(1) if m else name[:80]
            vals[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
out = {k: {c: round(sum(v) / len(v), 1) for c, v in d.items()} | {"dispatches": max(len(v) for v in d.values())}
       for k, d in vals.items()}
print(json.dumps(out, indent=1, sort_keys=True))
