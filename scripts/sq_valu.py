"""VALU issue of the one-pass step from a rocprofv3 SQ counter pass over bench.py, written as the
JSON bench.py reads for roofline.valu.

    python scripts/sq_valu.py <sq pmc dir> --box NXxNY --blocks BXxBY > profiles/sq_valu.json

Counters (one pass, scripts/gpu_sq_valu.sh): SQ_WAVES, SQ_INSTS_VALU, SQ_ACTIVE_INST_VALU,
SQ_WAVE_CYCLES, SQ_BUSY_CYCLES, SQ_WAIT_INST_ANY, SQ_WAIT_ANY, SQ_ACTIVE_INST_ANY and GRBM_GUI_ACTIVE
(the effective clock of each dispatch), per dispatch of
the known-constant one-pass kernels (k_march<MarchStep<true, false, true, false, false, PAIR, false>>: tau a
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
KERNELS = {"onepass": "MarchStep<true, false, true, false, false, false, false>",
           "onepass2": "MarchStep<true, false, true, false, false, true, false>"}


def summary(sq, kernel):
    # per dispatch (counters summed over the dimensions rocprofv3 reports them in)
    disp = defaultdict(lambda: defaultdict(float))
    dur = {}
    for f in glob.glob(os.path.join(sq, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if row.get("Kernel_Name", "").startswith(f"void ocn::k_march<ocn::{kernel}"):
                disp[row.get("Dispatch_Id")][row["Counter_Name"]] += float(row["Counter_Value"])
                if row.get("Start_Timestamp") and row.get("End_Timestamp"):
                    dur[row.get("Dispatch_Id")] = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-9
    if not disp:
        return None
    # the effective shader clock of each dispatch: GRBM_GUI_ACTIVE (summed over the 8 XCDs) / 8 / its
    # time (MI355X_MICROARCH.md 'DVFS give-back')
    for i, d in disp.items():
        if "GRBM_GUI_ACTIVE" in d and dur.get(i):
            d["clock_ghz"] = d.pop("GRBM_GUI_ACTIVE") / 8.0 / dur[i] / 1e9
            d["launch_ms"] = dur[i] * 1e3
    # the launches that ran: with the device-side variant choice the first call also launches the
    # variants whose workgroups see another verdict and return at once
    # (a pass without SQ_INSTS_VALU: another counter of the launches' work)
    work = next((k for k in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU")
                 if any(k in d for d in disp.values())), "SQ_WAVES")
    top = max(d.get(work, 0.0) for d in disp.values())
    ran = [d for d in disp.values() if d.get(work, 0.0) > 0.5 * top]
    n = len(ran)
    per = {k: sum(d.get(k, 0.0) for d in ran) / n for k in ran[0]}
    clk = {k: per.pop(k) for k in ("clock_ghz", "launch_ms") if k in per}
    waves = per.get("SQ_WAVES", 0.0)
    out = {"kernel": kernel, "dispatches": n, "per_launch": {k: round(v) for k, v in sorted(per.items())},
           "per_wave": {k: round(v / waves, 1) for k, v in sorted(per.items())} if waves else {}}
    if clk:   # mean over the pass's dispatches (counter passes serialize dispatches: profiled clocks)
        out["clock"] = {k: round(v, 4) for k, v in clk.items()}
        out["clock"]["per_dispatch_ghz"] = [round(d["clock_ghz"], 3) for d in ran if "clock_ghz" in d]
    return out


def merged(dirs, kernel):
    """summary() of each counter pass (its own run of the same command: the same launches), merged:
    the per-launch means of every counter any pass collected (SQ_WAVES, in several, must agree)."""
    outs = [s for d in dirs if (s := summary(d, kernel))]
    if not outs:
        return None
    out = outs[0]
    for o in outs[1:]:
        for k, v in o["per_launch"].items():
            out["per_launch"].setdefault(k, v)
        for k, v in o["per_wave"].items():
            out["per_wave"].setdefault(k, v)
        out.setdefault("clock", o.get("clock"))
        out["dispatches_per_pass"] = out.get("dispatches_per_pass", [outs[0]["dispatches"]]) + [o["dispatches"]]
    pl = out["per_launch"]
    # VALU instructions by class (SQ_INSTS_VALU_* passes): the f64 arithmetic the reference's order
    # requires vs the rest (integer / address arithmetic, conversions, moves, DPP shifts, selects)
    f64 = [k for k in ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64",
                       "SQ_INSTS_VALU_TRANS_F64") if k in pl]
    if f64 and pl.get("SQ_INSTS_VALU"):
        tot = pl["SQ_INSTS_VALU"]
        cls = {k[len("SQ_INSTS_VALU_"):].lower(): pl[k] for k in pl if k.startswith("SQ_INSTS_VALU_")}
        known = sum(cls.values())
        out["valu_classes"] = {"per_launch": cls, "f64": sum(pl[k] for k in f64),
                               "f64_frac": round(sum(pl[k] for k in f64) / tot, 4),
                               "unclassified": round(tot - known), "unclassified_frac": round((tot - known) / tot, 4),
                               "note": "SQ_INSTS_VALU_<class> counters; unclassified = SQ_INSTS_VALU - their sum "
                                       "(moves, DPP shifts, selects, compares, bit ops)"}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("sq", nargs="+", help="one directory per counter pass of the same command")
    ap.add_argument("--box", required=True)
    ap.add_argument("--blocks", required=True)
    a = ap.parse_args()
    kern = {stage: s for stage, k in KERNELS.items() if (s := merged(a.sq, k))}
    if not kern:
        raise SystemExit("no dispatches of the one-pass kernels")
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
    from ocean_model_arch_amd._lib import LIB_PATH, build_id
    from ocean_model_arch_amd import _codeobj
    for rec in kern.values():   # the profiled machine code (bench.py profile_match)
        args = rec["kernel"][rec["kernel"].index("<") + 1:rec["kernel"].rindex(">")]
        rec["symbol"] = _codeobj.march_step_symbol(args)
        rec["code_sha"] = _codeobj.kernel_code_sha(LIB_PATH, rec["symbol"])
    out = {"source": "rocprofv3 --pmc SQ counters (one pass) over bench.py; per dispatch of the one-pass kernels",
           "build_id": build_id(), "box": [int(v) for v in a.box.lower().split("x")],
           "blocks": [int(v) for v in a.blocks.lower().split("x")], "kernels": kern}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
