"""Synchronising HIP calls of a scripts/psy_loop.py run, from its rocprofv3 --hip-trace output.

    python3 scripts/psy_trace_summary.py DIR LOG [N]

DIR: the rocprofv3 output directory (its *hip_api_trace.csv), LOG: psy_loop.py's stdout (the
LOOP_BEGIN / LOOP_END markers, CLOCK_MONOTONIC ns).  Prints, for the calls that wait for the device
(hipStreamSynchronize, hipDeviceSynchronize, hipEventSynchronize, blocking hipMemcpy*), how many were
made inside the loop and outside it, and the loop's per-step count of every HIP call.
"""
import csv
import glob
import json
import os
import sys

SYNCING = ("hipStreamSynchronize", "hipDeviceSynchronize", "hipEventSynchronize", "hipMemcpy", "hipMemcpy2D",
           "hipMemcpyDtoH", "hipMemcpyHtoD", "hipMemcpyDtoD", "hipStreamQuery")


def main():
    d, log = sys.argv[1], sys.argv[2]
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 50
    marks = {}
    for ln in open(log):
        p = ln.split()
        if len(p) == 2 and p[0] in ("LOOP_BEGIN", "LOOP_END"):
            marks[p[0]] = int(p[1])
    files = glob.glob(os.path.join(d, "**", "*hip_api_trace.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no hip_api_trace.csv under {d}")
    inside, outside, per = {}, {}, {}
    for f in files:
        for r in csv.DictReader(open(f)):
            name = r.get("Function") or r.get("Kernel_Name") or r.get("Operation")
            t = int(r.get("Start_Timestamp", 0))
            ins = marks.get("LOOP_BEGIN", 0) <= t <= marks.get("LOOP_END", 1 << 62)
            if ins:
                per[name] = per.get(name, 0) + 1
            if name in SYNCING:
                (inside if ins else outside)[name] = (inside if ins else outside).get(name, 0) + 1
    out = {"steps": n, "syncing_calls_inside_loop": inside, "syncing_calls_outside_loop": outside,
           "hip_calls_per_step_inside_loop": {k: round(v / n, 2) for k, v in sorted(per.items())}}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
