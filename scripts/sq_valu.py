"""VALU issue of the one-pass step from a rocprofv3 SQ counter pass over bench.py, written as the
JSON bench.py reads for roofline.valu.

    python scripts/sq_valu.py <sq pmc dir> --box NXxNY --blocks BXxBY > profiles/sq_valu.json

Counters (one pass, scripts/gpu_sq_valu.sh): SQ_WAVES, SQ_INSTS_VALU, SQ_ACTIVE_INST_VALU,
SQ_WAVE_CYCLES, SQ_BUSY_CYCLES, SQ_WAIT_INST_ANY, SQ_WAIT_ANY, SQ_ACTIVE_INST_ANY, per dispatch of
the known-constant one-pass kernel (k_march<MarchStep<P2, false, true, X2>>: the steps between a
call's first and last).  SQ_*_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles
(MI355X_MICROARCH.md); a wave64 VALU instruction occupies its SIMD for one quad-cycle (f64
included: 16 lanes per cycle at full rate).  The JSON is stamped with ocn_build_id() and the
workload; bench.py reports roofline.valu only when both match the run it times."""
import argparse
import csv
import glob
import json
import os
import sys
from collections import defaultdict

PATTERN = "MarchStepILb1ELb0ELb1E"   # P2, !LAST, ZF (any X2)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("sq")
    ap.add_argument("--box", required=True)
    ap.add_argument("--blocks", required=True)
    a = ap.parse_args()
    tot, disp, names = defaultdict(float), defaultdict(set), set()
    for f in glob.glob(os.path.join(a.sq, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            name = row.get("Kernel_Name", "")
            mangled = name.replace("ocn::", "").replace("<", "I").replace(" ", "")
            if "MarchStep<true, false, true" not in name and PATTERN not in mangled:
                continue
            names.add(name)
            tot[row["Counter_Name"]] += float(row["Counter_Value"])
            disp[row["Counter_Name"]].add(row.get("Dispatch_Id"))
    if not tot:
        raise SystemExit("no dispatches of the one-pass kernel")
    n = max(len(v) for v in disp.values())
    per = {k: v / n for k, v in tot.items()}
    waves = per.get("SQ_WAVES", 0.0)
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
    from ocean_model_arch_amd._lib import build_id
    out = {"source": "rocprofv3 --pmc SQ counters (one pass) over bench.py; per dispatch of the one-pass kernel",
           "build_id": build_id(), "box": [int(v) for v in a.box.lower().split("x")],
           "blocks": [int(v) for v in a.blocks.lower().split("x")], "kernel": sorted(names), "dispatches": n,
           "per_launch": {k: round(v) for k, v in sorted(per.items())},
           "per_wave": {k: round(v / waves, 1) for k, v in sorted(per.items())} if waves else {}}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
