"""Summarise rocprofv3 --pmc CSVs: mean FETCH_SIZE / WRITE_SIZE (KB) per dispatch per kernel,
converted to bytes.  FETCH_SIZE on gfx950 counts 64 B per memory-side read request
(MI355X_MICROARCH.md 'HBM'); the conversion factor is calibrated in DESIGN.md against a
kernel with exactly known traffic (the pointwise sw_next_step part of fused C1)."""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

root = sys.argv[1]
vals = defaultdict(lambda: defaultdict(list))
for path in glob.glob(os.path.join(root, "**", "*counter_collection*.csv"), recursive=True):
    with open(path) as f:
        for row in csv.DictReader(f):
            name = row.get("Kernel_Name", "")
            m = re.search(r"k_range<ocn::(\w+(?:<\w+>)?)>|ocn::(\w+)\(", name)
            k = (m.group(1) or m.group(2)) if m else name[:60]
            vals[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
out = {}
for k, d in vals.items():
    out[k] = {c: {"mean_kb": sum(v) / len(v), "dispatches": len(v)} for c, v in d.items()}
print(json.dumps(out, indent=1, sort_keys=True))
