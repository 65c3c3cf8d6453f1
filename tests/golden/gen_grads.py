"""Generate tests/golden/grads_bs_tr_s180.npz: the reference model's own local output.

Runs the unmodified reference model (oracle/_ref/model, built by oracle/ref.mk from
/root/reference with AMD flang; this container only) on the Black Sea basin with one tracer,
tau = 1 s, 0.0025 days (216 steps), local output every minute (ocean_run.par lines 3 and 6; everything else as
shipped), and stores what it wrote under RESULTS/: ssh.dat / ff1.dat (4 records: steps 0, 60,
120, 180), hhq.dat (1 record) as float32 arrays, and the three .ctl descriptors as text.

    python tests/golden/gen_grads.py
"""
import os
import shutil
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
from tests.golden import gen_golden as G  # noqa: E402

MODEL = os.path.join(REPO, "oracle", "_ref", "model")
DAYS, PERIOD_MIN = "0.0025", 1.0   # 216 steps of 1 s


def main():
    subprocess.check_call(["make", "-s", "-f", os.path.join(REPO, "oracle", "ref.mk")], cwd=REPO,
                          stdout=subprocess.DEVNULL)
    d = tempfile.mkdtemp()
    try:
        os.makedirs(os.path.join(d, "RESULTS"))
        open(os.path.join(d, "basin.par"), "w").write(G.BASIN_TMPL.format(**G.BS))
        open(os.path.join(d, "sw.par"), "w").write(G.SW_TMPL.format(**dict(dict(tr=1, trn=1), **G.SW_DEFAULT)))
        open(os.path.join(d, "parallel.par"), "w").write(G.PAR_TMPL.format(bx=1, by=1))
        lines = open(os.path.join(G.REF, "ocean_run.par")).read().splitlines(True)
        lines[2] = f"{DAYS:>14} : Duration of the run (in days)\n"
        lines[5] = f"{PERIOD_MIN:>13} : Periodicity for writing local  instantaneous data (in minutes)\n"
        open(os.path.join(d, "ocean_run.par"), "w").write("".join(lines))
        subprocess.check_call([MODEL], cwd=d, env=dict(os.environ, OMP_NUM_THREADS="1"),
                              stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        nx, ny = G.BS["nx"] - 4, G.BS["ny"] - 4
        out = {"meta/days": np.array(DAYS), "meta/period_min": np.float32(PERIOD_MIN),
               "meta/sw": np.array(repr(dict(tr=1, trn=1, **G.SW_DEFAULT)))}
        for nm in ("ssh", "ff1", "hhq"):
            raw = np.fromfile(os.path.join(d, "RESULTS", nm + ".dat"), dtype="<f4")
            out[f"dat/{nm}"] = raw.reshape(-1, ny, nx)
            out[f"ctl/{nm}"] = np.array(open(os.path.join(d, "RESULTS", nm + ".ctl")).read())
    finally:
        shutil.rmtree(d)
    np.savez_compressed(os.path.join(HERE, "grads_bs_tr_s180.npz"), **out)
    print({k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
