"""The Fortran host (host/fortran, ISO_C_BINDING over libocn_sw) on the golden cases.

The driver reads the reference's positional basin.par / sw.par / parallel.par, runs the
reference-shaped Fortran PSy layer (envoke -> envoke_<stage>_kernel -> extern "C" HIP entry),
and dumps every field in the oracle/ref_driver.f90 format; each field must hash identically
to the unmodified reference run."""
import hashlib
import os
import subprocess

import numpy as np
import pytest

from tests.golden import cases
from tests.golden.refdump import read_dump

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DRIVER = os.path.join(REPO, "host", "fortran", "ocn_sw_driver")

BASIN = """{nx} : nx
{ny} : ny
1 : nz
0 : px
0 : py
{dxst!r} : dxst
{dyst!r} : dyst
{rlon!r} : rlon
{rlat!r} : rlat
0 : xgr
0 : ygr
{curve_grid} : curve grid
0.0 : rot lon
0.0 : rot lat
90.0 :
60.0 :
90.0 :
-90.0 :
{mask} : mask
{topo} : topography
"""


def write_case(d, case):
    b = case["basin"]
    mask = "none"
    if case["mask"] is not None:
        mask = os.path.join(d, "mask.txt")
        m = case["mask"]
        with open(mask, "w") as f:
            f.write("mask written from tests/golden (reference data/BS/mask_bs4km.txt)\n")
            for n in range(b["ny"] - 1, -1, -1):
                f.write("".join(str(int(v)) for v in m[:, n]) + "\n")
    topo = "none"
    if case.get("topography") is not None:   # the basin.par line-20 real(4) file (init_data.f90:115-120)
        topo = os.path.join(d, "topo.dat")
        np.asarray(case["topography"], dtype=np.float32).ravel(order="F").tofile(topo)
    open(os.path.join(d, "basin.par"), "w").write(BASIN.format(mask=mask, topo=topo, **b))
    s = case["sw"]
    open(os.path.join(d, "sw.par"), "w").write(
        f"{s['full_free_surface']} : ffs\n{s['trans_terms']} : trans\n{s['ksw_lat']} : ksw\n"
        f"{s['time_smooth']!r} : ts\n1000.0 : lvisc\n{s.get('use_tracers', 0)} : tracers\n"
        f"{s.get('tracer_num', 1)} : n\nnone : ssh\n")
    bx, by = case["bxy"]
    open(os.path.join(d, "parallel.par"), "w").write(f"0 : m\nnone : f\n{bx} : bx\n{by} : by\n0\n0\nnone\n0\n0\n")


def test_fortran_host_builds():
    if not os.path.exists(DRIVER):
        subprocess.check_call(["make", "-s", "-f", os.path.join(REPO, "host", "fortran", "Makefile")], cwd=REPO)
    assert os.access(DRIVER, os.X_OK)


@pytest.mark.gpu
@pytest.mark.parametrize("name,mode", [("box70x54_b3x2_s20", "stages"), ("bs_b4x2_s60", "stages"),
                                       ("box48x40_flags000_s10", "native"), ("bs_b1x1_s60", "native"),
                                       ("box40x32_tr2_s5", "stages"), ("bs_b4x2_tr_s60", "native"),
                                       ("box70x54_b1x1_s20", "psy"), ("box70x54_b3x2_tr_s20", "psy"),
                                       ("bs_b1x1_s604", "psy"), ("box70x54_topo_b3x2_s20", "psy"),
                                       ("bs_topo_b4x2_s60", "stages")])
def test_fortran_host_matches_reference(tmp_path, name, mode):
    """stages = the reference's envoke stages over the kernel-layer entries; psy = the same PSy
    time loop (one expl_shallow_water per step, model.f90:146) in its fused form, one
    ocn_ctx_step(ctx, tau, 1) per step; native = one ocn_ctx_step call for the whole run."""
    case = cases.load_e2e(name)
    write_case(str(tmp_path), case)
    args = [DRIVER, str(case["steps"]), "dump.bin"] + ([mode] if mode != "psy" else [])
    r = subprocess.run(args, cwd=tmp_path, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    z = case["z"]
    bad = []
    for info, f in read_dump(os.path.join(tmp_path, "dump.bin")):
        for nm, a in f.items():
            key = f"b{info['bm']}_{info['bn']}/sha/{nm}"
            if key in z.files:
                h = hashlib.sha256(np.ascontiguousarray(a.ravel(order="F")).tobytes()).hexdigest()
                if h != str(z[key]):
                    bad.append(f"({info['bm']},{info['bn']}):{nm}")
    assert not bad, f"{name}/{mode}: {bad}"
