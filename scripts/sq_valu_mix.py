"""Render an SQ pass summary (scripts/sq_valu.py's JSON, e.g. profiles/sq_valu.json) as the
per-kernel mix table of profiles/*/sq_mix.txt: each counter per launch and per wave, then the
fractions of a wave's quad-cycles (SQ_WAVE_CYCLES) spent issuing VALU, waiting on dependencies
(SQ_WAIT_INST_ANY) and waiting on memory (SQ_WAIT_ANY), and the SIMD's VALU busy fraction at the
launch's occupancy (waves per SIMD x a wave's VALU-active share).

usage: python scripts/sq_valu_mix.py profiles/sq_valu.json [--waves-per-simd 2] > profiles/rNN/sq_mix.txt
"""
import argparse
import json


def render(d, waves_per_simd):
    out = [f"# {d.get('source', '')}", f"# build {d.get('build_id')}  box {d.get('box')}  blocks {d.get('blocks')}"]
    for name, k in d["kernels"].items():
        pl, pw = k["per_launch"], k["per_wave"]
        out.append("")
        out.append(f"[{name}] {k.get('kernel', '')}  dispatches {k.get('dispatches')}")
        for c in sorted(pl):
            out.append(f"{c:<28}{pl[c]:>16.0f}  per launch   {pw.get(c, 0.0):>12.1f}  per wave")
        cyc = pw["SQ_WAVE_CYCLES"]
        valu, dep, mem = pw["SQ_ACTIVE_INST_VALU"] / cyc, pw["SQ_WAIT_INST_ANY"] / cyc, pw["SQ_WAIT_ANY"] / cyc
        out.append(f"wave quad-cycles: VALU active {valu:.3f}  WAIT_INST_ANY {dep:.3f}  WAIT_ANY {mem:.3f}")
        out.append(f"SIMD VALU busy at {waves_per_simd} waves per SIMD: {min(1.0, waves_per_simd * valu):.3f}")
    return "\n".join(out) + "\n"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("summary")
    ap.add_argument("--waves-per-simd", type=int, default=2)
    a = ap.parse_args()
    with open(a.summary) as f:
        print(render(json.load(f), a.waves_per_simd), end="")


if __name__ == "__main__":
    main()
