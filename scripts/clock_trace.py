"""Effective shader clock per launch from a rocprofv3 counter pass with the kernel trace
(--pmc GRBM_GUI_ACTIVE --kernel-trace, scripts/gpu_clock.sh): GRBM_GUI_ACTIVE is summed over the 8
XCDs, so clock = GRBM_GUI_ACTIVE / 8 / launch time (MI355X_MICROARCH.md, 'DVFS give-back').

    python3 scripts/clock_trace.py <counter_collection.csv> [kernel substring] > clock.txt
"""
import csv
import sys


def main():
    path = sys.argv[1]
    pat = sys.argv[2] if len(sys.argv) > 2 else "MarchStep"
    rows = [r for r in csv.DictReader(open(path)) if r.get("Counter_Name") == "GRBM_GUI_ACTIVE"]
    rows.sort(key=lambda r: int(r.get("Start_Timestamp") or r.get("Dispatch_Id")))
    t0 = None
    print(f"{'t (ms)':>9} {'launch (us)':>12} {'GHz':>6}  kernel")
    for r in rows:
        if pat not in r["Kernel_Name"]:
            continue
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        t0 = s if t0 is None else t0
        dur = (e - s) * 1e-9
        ghz = float(r["Counter_Value"]) / 8.0 / dur / 1e9 if dur > 0 else float("nan")
        print(f"{(s - t0) * 1e-6:9.3f} {dur * 1e6:12.1f} {ghz:6.3f}  {r['Kernel_Name'][:90]}")


if __name__ == "__main__":
    main()
