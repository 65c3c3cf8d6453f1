"""VALU issue of the one-pass step from a rocprofv3 SQ counter pass over bench.py, written as the
JSON bench.py reads for roofline.valu.

    python scripts/sq_valu.py <sq pmc dir> --box NXxNY --blocks BXxBY > profiles/sq_valu.json

Counters (one pass, scripts/gpu_sq_valu.sh): SQ_WAVES, SQ_INSTS_VALU, SQ_ACTIVE_INST_VALU,
SQ_WAVE_CYCLES, SQ_BUSY_CYCLES, SQ_WAIT_INST_ANY, SQ_WAIT_ANY, SQ_ACTIVE_INST_ANY, per dispatch of
the known-constant one-pass kernels (k_march<MarchStep<true, false, true, false, false, PAIR>>: tau a
power of two, not a last step, h_r / mu / forcing / fallback values known, one block; PAIR = two steps
per launch) that ran -- the
first call's gated-off variant launches (their workgroups return at once) are left out.  SQ_*_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles
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

# the known-constant one-pass kernels (P2, !LAST, ZF, !X2, h_r a constant): a single step and two
# steps per launch (PAIR)
KERNELS = {"onepass": "MarchStep<true, false, true, false, false, false>",
           "onepass2": "MarchStep<true, false, true, false, false, true>"}


def summary(sq, kernel):
    # per dispatch (counters summed over the dimensions rocprofv3 reports them in)
    disp = defaultdict(lambda: defaultdict(float))
    for f in glob.glob(os.path.join(sq, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if row.get("Kernel_Name", "").startswith(f"void ocn::k_march<ocn::{kernel}"):
                disp[row.get("Dispatch_Id")][row["Counter_Name"]] += float(row["Counter_Value"])
    if not disp:
        return None
    # the launches that ran: with the device-side variant choice the first call also launches the
    # variants whose workgroups see another verdict and return at once
    top = max(d.get("SQ_INSTS_VALU", 0.0) for d in disp.values())
    ran = [d for d in disp.values() if d.get("SQ_INSTS_VALU", 0.0) > 0.5 * top]
    n = len(ran)
    per = {k: sum(d.get(k, 0.0) for d in ran) / n for k in ran[0]}
    waves = per.get("SQ_WAVES", 0.0)
    return {"kernel": kernel, "dispatches": n, "per_launch": {k: round(v) for k, v in sorted(per.items())},
            "per_wave": {k: round(v / waves, 1) for k, v in sorted(per.items())} if waves else {}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("sq")
    ap.add_argument("--box", required=True)
    ap.add_argument("--blocks", required=True)
    a = ap.parse_args()
    kern = {stage: s for stage, k in KERNELS.items() if (s := summary(a.sq, k))}
    if not kern:
        raise SystemExit("no dispatches of the one-pass kernels")
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
    from ocean_model_arch_amd._lib import build_id
    out = {"source": "rocprofv3 --pmc SQ counters (one pass) over bench.py; per dispatch of the one-pass kernels",
           "build_id": build_id(), "box": [int(v) for v in a.box.lower().split("x")],
           "blocks": [int(v) for v in a.blocks.lower().split("x")], "kernels": kern}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
