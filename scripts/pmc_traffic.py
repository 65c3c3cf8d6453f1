"""HBM bytes per launch of the fused-step kernels from rocprofv3 FETCH_SIZE / WRITE_SIZE passes
over bench.py (scripts/pmc.sh), written as the JSON bench.py reads for roofline.traffic.

    python scripts/pmc_traffic.py <pmc dir> <stenbench pmc dir> <cells> --box NXxNY --blocks BXxBY [--compact]
        > profiles/pmc_traffic.json

The JSON is stamped with the library's ocn_build_id() (run this on the tree that was profiled) and
the workload (box, block grid, cells per block); bench.py reports roofline.traffic only when all
of them match the run it is timing.

FETCH_SIZE on gfx950 under-counts wide streaming reads (MI355X_MICROARCH.md 'HBM': half the
bytes at 16 B/lane); our kernels read 8 B/lane.  The read scale is therefore calibrated on the
stencil microbenchmark's pointwise kernel k_bench<0,0> (scripts/stenbench.hip), whose reads are
exactly 20 arrays x 4094^2 x 8 B in the same 64 x 4-thread, 8-B-per-lane pattern; the write
scale on the same kernel's 2 x 4094^2 x 8 B of stores (the guide calls WRITE_SIZE exact for
16-B-per-lane stores only).  Counter values are KiB."""
import argparse
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

STAGE = {"KFusedA": "fused_a", "KFusedB": "fused_b", "MarchFusedB": "fused_b", "KFusedC1": "fused_c1",
         "KHhInit": "hh_init", "MarchHhInit": "hh_init", "MarchFusedA": "fused_a", "MarchCA": "fused_ca", "MarchStep": "onepass"}


def values(root):
    """{kernel name: {counter: [bytes per dispatch]}}"""
    vals = defaultdict(lambda: defaultdict(list))
    for path in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(path)):
            vals[row["Kernel_Name"]][row["Counter_Name"]].append(float(row["Counter_Value"]) * 1024.0)
    return vals


def means(root):
    return {k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in values(root).items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("pmc")
    ap.add_argument("sten")
    ap.add_argument("cells", type=int)
    ap.add_argument("--box", required=True)
    ap.add_argument("--blocks", required=True)
    ap.add_argument("--compact", action="store_true")
    a = ap.parse_args()
    pmc, sten, cells, compact = a.pmc, a.sten, a.cells, a.compact
    cal = [v for k, v in means(sten).items() if "k_bench<0, 0>" in k][0]
    exact_read, exact_write = 20 * 4094 * 4094 * 8.0, 2 * 4094 * 4094 * 8.0
    scale = exact_read / cal["FETCH_SIZE"]
    wscale = exact_write / cal["WRITE_SIZE"]
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
    from ocean_model_arch_amd._lib import build_id
    out = {"source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes) over bench.py; read scale {scale:.4f} "
                     f"calibrated on stenbench k_bench<0,0> ({exact_read:.0f} B read exactly), write scale "
                     f"{wscale:.4f} ({exact_write:.0f} B written)",
           "build_id": build_id(), "box": [int(v) for v in a.box.lower().split("x")],
           "blocks": [int(v) for v in a.blocks.lower().split("x")],
           "fetch_scale": scale, "write_scale": wscale, "kernels": {}}
    # every dispatch of every template instance of a stage's kernel (e.g. MarchFusedB<true, true>
    # and <false, false>), averaged per dispatch like bench.py's per-launch timing
    agg = defaultdict(lambda: {"FETCH_SIZE": [], "WRITE_SIZE": [], "names": set(), "full": set()})
    for k, d in values(pmc).items():
        m = re.search(r"ocn::(\w+)", k.replace("k_range<ocn::", "").replace("k_march<ocn::", ""))
        name = m.group(1) if m else k
        stage = STAGE.get(name)
        t = re.search(r"MarchStep<([^>]*)>", k)
        targs = [a.strip() for a in t.group(1).split(",")] if t else []
        if targs[5:6] == ["true"]:   # MarchStep PAIR: two steps (LAST: the second is the call's last)
            stage, name = ("onepass2_last", "MarchStep(pair, last)") if targs[1:2] == ["true"] else \
                ("onepass2", "MarchStep(pair)")
        if not stage:
            continue
        for c in ("FETCH_SIZE", "WRITE_SIZE"):
            agg[stage][c] += d.get(c, [])
        agg[stage]["names"].add(name)
        agg[stage]["full"].add(k)
    for stage, d in agg.items():
        # the launches that ran: the one-pass step's first call also launches the variants the device
        # verdict does not select, whose workgroups return at once (a few KB each) -- left out
        for c in ("FETCH_SIZE", "WRITE_SIZE"):
            top = max(d[c], default=0.0)
            d[c] = [v for v in d[c] if v > 0.05 * top]
        if not d["FETCH_SIZE"] or not d["WRITE_SIZE"]:
            continue
        rd = sum(d["FETCH_SIZE"]) / len(d["FETCH_SIZE"]) * scale
        wr = sum(d["WRITE_SIZE"]) / len(d["WRITE_SIZE"]) * wscale
        out["kernels"][stage] = {"kernel": "/".join(sorted(d["names"])), "dispatches": len(d["WRITE_SIZE"]),
                                 "cells": cells, "compact": compact, "fetch_bytes": round(rd), "write_bytes": round(wr),
                                 "hbm_bytes_per_launch": round(rd + wr)}
        if len(d["full"]) == 1:   # one kernel instance: its machine code (bench.py profile_match)
            from ocean_model_arch_amd._lib import LIB_PATH
            from ocean_model_arch_amd import _codeobj
            hit = _codeobj.sha_by_demangled(LIB_PATH, d["full"])
            if hit:
                out["kernels"][stage]["symbol"], out["kernels"][stage]["code_sha"] = next(iter(hit.values()))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
