"""Summarise scripts/gpu_sq.sh's counter passes: per kernel (by name substring), the counters
summed over its dispatches, and per wave."""
import csv
import glob
import os
import sys
from collections import defaultdict


def main(out, pattern="MarchStep"):
    tot = defaultdict(float)
    disp = defaultdict(set)
    for f in glob.glob(os.path.join(out, "g*", "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            name = row.get("Kernel_Name", "")
            if pattern not in name:
                continue
            ctr = row["Counter_Name"]
            tot[ctr] += float(row["Counter_Value"])
            disp[ctr].add(row.get("Dispatch_Id"))
    if not tot:
        print("no dispatches of", pattern)
        return
    waves = tot.get("SQ_WAVES", 0.0)
    for k in sorted(tot):
        per = f"  per wave {tot[k] / waves:12.1f}" if waves else ""
        print(f"{k:28s} {tot[k]:16.0f}  dispatches {len(disp[k]):3d}{per}")


if __name__ == "__main__":
    main(sys.argv[1], *(sys.argv[2:3]))
