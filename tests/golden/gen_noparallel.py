"""Fixtures from the reference built in _MPP_NO_PARALLEL_MODE_ (test infrastructure, build container only).

BASELINE.json's north star names the reference's CPU _MPP_NO_PARALLEL_MODE_ run; the golden fixtures
(gen_golden.py, oracle/ref.mk) come from its default build, macros/mpp_macros.fi:22-23
(_MPP_SORTED_BLOCKS_, _MPP_BLOCK_MODE_: the block loop of envoke as an OpenMP loop,
core/kernel_interface.f90:72-84, run with one thread).  The mode is a #define in that header, so this
script builds the reference once more from a scratch copy of its tree OUTSIDE the repository
(/tmp/ocn_ref_noparallel) in which that single line reads _MPP_NO_PARALLEL_MODE_ (the header's own
documented alternative, :9-10), runs the same cases, and stores the SHA-256 digests of every field of
every block as e2e_<case>_noparallel.npz.  tests/test_oracle_pinned.py checks they equal the default
build's fixtures.  Nothing of the reference enters the repository; only the digests.

    python tests/golden/gen_noparallel.py
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
from tests.golden import gen_golden as G  # noqa: E402

SCRATCH = "/tmp/ocn_ref_noparallel"
OUT = "/tmp/ocn_ref_noparallel_out"
CASES = ["box70x54_b3x2_s20", "bs_b4x2_s60", "bs_b4x2_tr_s60"]


def build():
    if os.path.exists(SCRATCH):
        shutil.rmtree(SCRATCH)
    shutil.copytree(G.REF, SCRATCH, ignore=shutil.ignore_patterns(".git", "work"))
    hdr = os.path.join(SCRATCH, "macros", "mpp_macros.fi")
    txt = open(hdr).read()
    assert txt.count("\n#define _MPP_BLOCK_MODE_\n") == 1, "unexpected mpp_macros.fi"
    open(hdr, "w").write(txt.replace("\n#define _MPP_BLOCK_MODE_\n", "\n#define _MPP_NO_PARALLEL_MODE_\n"))
    subprocess.check_call(["make", "-s", "-f", os.path.join(REPO, "oracle", "ref.mk"), f"REF={SCRATCH}", f"OUT={OUT}",
                           f"{OUT}/ref_driver"], cwd=REPO, stdout=subprocess.DEVNULL)
    return os.path.join(OUT, "ref_driver")


def main():
    drv = build()
    G.REFDRV = drv
    for name in CASES:
        basin, sw, bxy, steps, _ = G.CASES[name]
        G.gen_e2e(name + "_noparallel", basin, sw, bxy, steps, "sha")
        # keep the digests and the metadata only
        path = os.path.join(HERE, f"e2e_{name}_noparallel.npz")
        z = np.load(path)
        keep = {k: z[k] for k in z.files if "/sha/" in k or k.startswith("meta/") or k.endswith("/info")}
        np.savez_compressed(path, **keep)
        print("kept", path, os.path.getsize(path))
    shutil.rmtree(SCRATCH, ignore_errors=True)
    shutil.rmtree(OUT, ignore_errors=True)


if __name__ == "__main__":
    main()
