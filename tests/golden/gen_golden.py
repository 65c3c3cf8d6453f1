"""Generate the golden fixtures in tests/golden/ from the COMPILED REFERENCE.

Run in the build container only (needs /root/reference and `make -f oracle/ref.mk`):

    python tests/golden/gen_golden.py

Two kinds of fixtures:

1. ``kernels_<tag>.npz`` -- per-kernel known-answer vectors.  Seeded random inputs
   (numpy default_rng) on one block; every output array starts as random "poison" so the
   fixture also pins the kernel's exact write set.  Outputs come from calling the reference
   kernels themselves in ``oracle/_ref/libref.so`` through ctypes (every argument by
   reference, arrays Fortran-ordered; module variables ``config_sw_module::time_smooth`` /
   ``full_free_surface`` set through their symbols).

2. ``e2e_<case>.npz`` -- end-to-end state after N steps of the unmodified reference model
   (``oracle/ref_driver.f90``: model.f90's init + N x expl_shallow_water), one block grid.
   Small cases keep every field of every block; large cases keep SHA-256 digests of every
   field of every block plus the prognostic arrays.
"""
from __future__ import annotations

import ctypes as C
import hashlib
import os
import shutil
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
from tests.golden.refdump import read_dump, R4_FIELDS, R8_FIELDS  # noqa: E402

REF = "/root/reference"
REFLIB = os.path.join(REPO, "oracle", "_ref", "libref.so")
REFDRV = os.path.join(REPO, "oracle", "_ref", "ref_driver")

# ---------------------------------------------------------------- per-kernel fixtures
# argument lists: (name, kind) with kind r4/r8 input "i", output "o" (poisoned), in/out "io"
KERNELS = {
    # kernel/shallow_water/vel_ssh.f90:69
    "sw_update_ssh": ("_QMvelssh_sw_modulePsw_update_ssh_kernel", ["tau"],
                      [("lu", "r4"), ("dx", "r4"), ("dy", "r4"), ("dxh", "r4"), ("dyh", "r4"),
                       ("hhu", "r8"), ("hhv", "r8"), ("sshn", "r8o"), ("sshp", "r8"), ("ubrtr", "r8"),
                       ("vbrtr", "r8")]),
    # vel_ssh.f90:108
    "sw_update_uv": ("_QMvelssh_sw_modulePsw_update_uv", ["tau"],
                     [("lcu", "r4"), ("lcv", "r4"), ("dxt", "r4"), ("dyt", "r4"), ("dxh", "r4"),
                      ("dyh", "r4"), ("dxb", "r4"), ("dyb", "r4"),
                      ("hhu", "r8"), ("hhu_n", "r8"), ("hhu_p", "r8"), ("hhv", "r8"), ("hhv_n", "r8"),
                      ("hhv_p", "r8"), ("hhh", "r8"), ("ssh", "r8"),
                      ("ubrtr", "r8"), ("ubrtrn", "r8o"), ("ubrtrp", "r8"),
                      ("vbrtr", "r8"), ("vbrtrn", "r8o"), ("vbrtrp", "r8"),
                      ("r_diss", "r4"), ("rlh_s", "r4"),
                      ("RHSx", "r8"), ("RHSy", "r8"), ("RHSx_adv", "r8"), ("RHSy_adv", "r8"),
                      ("RHSx_dif", "r8"), ("RHSy_dif", "r8")]),
    # vel_ssh.f90:197
    "sw_next_step": ("_QMvelssh_sw_modulePsw_next_step", ["time_smooth"],
                     [("lu", "r4"), ("lcu", "r4"), ("lcv", "r4"),
                      ("ssh", "r8o"), ("sshn", "r8o"), ("sshp", "r8o"),
                      ("ubrtr", "r8o"), ("ubrtrn", "r8o"), ("ubrtrp", "r8o"),
                      ("vbrtr", "r8o"), ("vbrtrn", "r8o"), ("vbrtrp", "r8o")]),
    # vel_ssh.f90:247
    "uv_trans_vort": ("_QMvelssh_sw_modulePuv_trans_vort_kernel", [],
                      [("luu", "r4"), ("dxt", "r4"), ("dyt", "r4"), ("dxb", "r4"), ("dyb", "r4"),
                       ("ubrtr", "r8"), ("vbrtr", "r8"), ("vort", "r8o"), ("nlev", "int")]),
    # vel_ssh.f90:283
    "uv_trans": ("_QMvelssh_sw_modulePuv_trans_kernel", [],
                 [("lcu", "r4"), ("lcv", "r4"), ("luu", "r4"), ("dxh", "r4"), ("dyh", "r4"),
                  ("ubrtr", "r8"), ("vbrtr", "r8"), ("vort", "r8"), ("hhq", "r8"), ("hhu", "r8"),
                  ("hhv", "r8"), ("hhh", "r8"), ("RHSx_adv", "r8o"), ("RHSy_adv", "r8o"), ("nlev", "int")]),
    # vel_ssh.f90:375
    "uv_diff2": ("_QMvelssh_sw_modulePuv_diff2_kernel", [],
                 [("lcu", "r4"), ("lcv", "r4"), ("dx", "r4"), ("dy", "r4"), ("dxt", "r4"), ("dyt", "r4"),
                  ("dxh", "r4"), ("dyh", "r4"), ("dxb", "r4"), ("dyb", "r4"),
                  ("mu", "r8"), ("str_t", "r8"), ("str_s", "r8"), ("hhq", "r8"), ("hhu", "r8"),
                  ("hhv", "r8"), ("hhh", "r8"), ("RHSx_dif", "r8o"), ("RHSy_dif", "r8o"), ("nlev", "int")]),
    # kernel/shallow_water/mixing.f90:14
    "stress_components": ("_QMmixing_modulePstress_components_kernel", [],
                          [("lu", "r4"), ("luu", "r4"), ("dx", "r4"), ("dy", "r4"), ("dxt", "r4"),
                           ("dyt", "r4"), ("dxh", "r4"), ("dyh", "r4"), ("dxb", "r4"), ("dyb", "r4"),
                           ("ubrtrp", "r8"), ("vbrtrp", "r8"), ("str_t", "r8o"), ("str_s", "r8o"),
                           ("nlev", "int")]),
    # kernel/shallow_water/depth.f90:14 (module var full_free_surface)
    "hh_init": ("_QMdepth_modulePhh_init_kernel", [],
                [("lu", "r4"), ("llu", "r4"), ("llv", "r4"), ("luh", "r4"),
                 ("dx", "r4"), ("dy", "r4"), ("dxt", "r4"), ("dyt", "r4"), ("dxh", "r4"), ("dyh", "r4"),
                 ("dxb", "r4"), ("dyb", "r4"),
                 ("hhq", "r8o"), ("hhq_p", "r8o"), ("hhq_n", "r8o"), ("hhu", "r8o"), ("hhu_p", "r8o"),
                 ("hhu_n", "r8o"), ("hhv", "r8o"), ("hhv_p", "r8o"), ("hhv_n", "r8o"),
                 ("hhh", "r8o"), ("hhh_p", "r8o"), ("hhh_n", "r8o"),
                 ("ssh", "r8"), ("sshp", "r8"), ("hhq_rest", "r8")]),
    # depth.f90:101
    "hh_update": ("_QMdepth_modulePhh_update_kernel", [],
                  [("lu", "r4"), ("llu", "r4"), ("llv", "r4"), ("luh", "r4"),
                   ("dx", "r4"), ("dy", "r4"), ("dxt", "r4"), ("dyt", "r4"), ("dxh", "r4"), ("dyh", "r4"),
                   ("dxb", "r4"), ("dyb", "r4"),
                   ("hhq_n", "r8o"), ("hhu_n", "r8o"), ("hhv_n", "r8o"), ("hhh_n", "r8o"),
                   ("ssh", "r8"), ("hhq_rest", "r8")]),
    # kernel/tracer/leapfrog_tracer.f90:13 (factor_mu passed as 1.0d0 by tracer_interface.f90:47)
    "tran_diff_fluxes": ("_QMtracer_modulePtran_diff_fluxes_kernel", [],
                         [("lcu", "r4"), ("lcv", "r4"), ("dxt", "r4"), ("dyt", "r4"), ("dxh", "r4"), ("dyh", "r4"),
                          ("hhu", "r8"), ("hhv", "r8"), ("ff1", "r8"), ("ff1p", "r8"), ("ubrtr", "r8"),
                          ("vbrtr", "r8"), ("mu", "r8"), ("factor_mu", "f64"), ("flux_x", "r8o"),
                          ("flux_y", "r8o")]),
    # leapfrog_tracer.f90:94
    "tran_diff_tracer": ("_QMtracer_modulePtran_diff_tracer_kernel", [],
                         [("lu", "r4"), ("dx", "r4"), ("dy", "r4"), ("tau", "f64"), ("hhq_n", "r8"),
                          ("hhq_p", "r8"), ("flux_x", "r8"), ("flux_y", "r8"), ("ff1p", "r8"), ("ff1n", "r8o")]),
    # leapfrog_tracer.f90:138
    "tracer_next_step": ("_QMtracer_modulePtracer_next_step_kernel", ["time_smooth"],
                         [("lu", "r4"), ("ff1n", "r8"), ("ff1p", "r8o"), ("ff1", "r8o")]),
    # depth.f90:164 (module var time_smooth)
    "hh_shift": ("_QMdepth_modulePhh_shift_kernel", [],
                 [("lu", "r4"), ("llu", "r4"), ("llv", "r4"), ("luh", "r4"),
                  ("hhq", "r8o"), ("hhq_p", "r8o"), ("hhq_n", "r8o"), ("hhu", "r8o"), ("hhu_p", "r8o"),
                  ("hhu_n", "r8o"), ("hhv", "r8o"), ("hhv_p", "r8o"), ("hhv_n", "r8o"),
                  ("hhh", "r8o"), ("hhh_p", "r8o"), ("hhh_n", "r8o")]),
}

# Block geometries for the kernel fixtures: (nxs, nxe, nys, nye) with arrays start-2..end+2
GEOMS = {"b66x50": (3, 68, 3, 52), "b1x1": (3, 3, 3, 3), "b130x7": (3, 132, 3, 9)}


def random_state(rng: np.random.Generator, shape, ref) -> dict[str, np.ndarray]:
    """Seeded inputs: metrics U(240,260) r4, depths U(99,101), velocities/SSH
    U(-0.1,0.1), Coriolis U(1e-4,1.1e-4); RHS, stresses, mu, r_diss random too so every
    term of every kernel is exercised.  Masks: random T mask (85 % sea) and the U/V/H masks
    derived from it by the reference's own lu_lv_init_kernel (grid_kernels.f90:40)."""
    def f4(lo, hi):
        return np.asfortranarray(rng.uniform(lo, hi, shape).astype(np.float32))

    def f8(lo, hi):
        return np.asfortranarray(rng.uniform(lo, hi, shape))

    s = {}
    s["lu"] = np.asfortranarray((rng.random(shape) < 0.85).astype(np.float32))
    for nm in ("luh", "luu", "llu", "llv", "lcu", "lcv"):
        s[nm] = np.zeros(shape, np.float32, order="F")
    bx1, by1 = 1, 1
    bx2, by2 = shape[0], shape[1]
    ib = [C.byref(C.c_int(v)) for v in (bx1, bx2, by1, by2)]
    ref._QMgrid_kernels_modulePlu_lv_init_kernel(*ib, *[s[n].ctypes.data_as(C.c_void_p)
                                                         for n in ("lu", "luh", "luu", "llu", "llv", "lcu", "lcv")])
    for nm in ("dx", "dy", "dxt", "dyt", "dxh", "dyh", "dxb", "dyb"):
        s[nm] = f4(240.0, 260.0)
    s["rlh_s"] = f4(1.0e-4, 1.1e-4)
    s["r_diss"] = f4(0.0, 1.0e-4)
    for nm in ("hhq", "hhq_p", "hhq_n", "hhu", "hhu_p", "hhu_n", "hhv", "hhv_p", "hhv_n",
               "hhh", "hhh_p", "hhh_n", "hhq_rest"):
        s[nm] = f8(99.0, 101.0)
    for nm in ("ssh", "sshn", "sshp", "ubrtr", "ubrtrn", "ubrtrp", "vbrtr", "vbrtrn", "vbrtrp"):
        s[nm] = f8(-0.1, 0.1)
    for nm in ("RHSx", "RHSy", "RHSx_adv", "RHSy_adv", "RHSx_dif", "RHSy_dif"):
        s[nm] = f8(-1.0e-3, 1.0e-3)
    s["vort"] = f8(-1.0e-5, 1.0e-5)
    s["str_t"] = f8(-1.0e-4, 1.0e-4)
    s["str_s"] = f8(-1.0e-4, 1.0e-4)
    s["mu"] = f8(0.0, 1.0e3)
    # tracer state (drawn last: the inputs of the SW kernels above are unchanged by it)
    for nm in ("ff1", "ff1p", "ff1n"):
        s[nm] = f8(0.0, 0.5)
    for nm in ("flux_x", "flux_y"):
        s[nm] = f8(-1.0e-3, 1.0e-3)
    return s


def gen_kernels(ref, tag, geom, seed):
    nxs, nxe, nys, nye = geom
    bx1, bx2, by1, by2 = nxs - 2, nxe + 2, nys - 2, nye + 2
    shape = (bx2 - bx1 + 1, by2 - by1 + 1)
    rng = np.random.default_rng(seed)
    state = random_state(rng, shape, ref)
    out = {"geom": np.array([nxs, nxe, nys, nye, bx1, bx2, by1, by2], np.int32),
           "tau": np.float64(1.0), "time_smooth": np.float64(0.5), "full_free_surface": np.int32(1),
           "factor_mu": np.float64(0.7)}
    for nm, a in state.items():
        out["in/" + nm] = a
    C.c_double.in_dll(ref, "_QMconfig_sw_moduleEtime_smooth").value = 0.5
    C.c_int.in_dll(ref, "_QMconfig_sw_moduleEfull_free_surface").value = 1
    for kname, (sym, scalars, args) in KERNELS.items():
        work = {nm: a.copy(order="F") for nm, a in state.items()}
        cargs = [C.byref(C.c_int(v)) for v in (nxs, nxe, nys, nye, bx1, bx2, by1, by2)]
        for sc in scalars:
            cargs.append(C.byref(C.c_double(float(out[sc]))))
        for nm, kind in args:
            if kind == "int":
                cargs.append(C.byref(C.c_int(1)))
            elif kind == "f64":
                cargs.append(C.byref(C.c_double(float(out[nm]))))
            else:
                cargs.append(work[nm].ctypes.data_as(C.c_void_p))
        getattr(ref, sym)(*cargs)
        for nm, kind in args:
            if kind.endswith("o"):
                out[f"{kname}/{nm}"] = work[nm]
    path = os.path.join(HERE, f"kernels_{tag}.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, os.path.getsize(path))


# ---------------------------------------------------------------- end-to-end fixtures
BASIN_TMPL = """{nx} : nx
{ny} : ny
1 : nz
0 : periodicity x
0 : periodicity y
{dxst} : dxst
{dyst} : dyst
{rlon} : rlon
{rlat} : rlat
0 : xgr_type
0 : ygr_type
{curve} : curve_grid
0.0d0 : rotation_on_lon
0.0d0 : rotation_on_lat
90.0d0 : x_pole
60.0d0 : y_pole
90.0d0 : p_pole
-90.0d0 : q_pole
{mask} : mask
{topo} : topography
"""
SW_TMPL = """{ffs} : full free surface
{trans} : trans terms
{ksw} : ksw_lat
{ts} : time smooth
1.0d+03 : lvisc_2
{tr} : tracers
{trn} : tracer num
none : ssh init
"""
PAR_TMPL = """0 : mod
none : file
{bx} : bppnx
{by} : bppny
0 : dbg
0 : mode
none : out
0 : dlb
0 : dlb
"""

BOX = dict(dxst="0.00312d0", dyst="0.00225d0", rlon="34.751560d0", rlat="44.801125d0", curve=1, mask="none",
           topo="none")
BS = dict(nx=289, ny=163, dxst="0.05d0", dyst="0.04d0", rlon="27.525d0", rlat="40.940d0", curve=1,
          mask=os.path.join(REF, "data/BS/mask_bs4km.txt"), topo="none")


def topography(nx, ny):
    """A synthetic bottom topography (real(4), the (nx-4) x (ny-4) interior points, Fortran order):
    depths between 20 and 100 m varying along both axes -- the reference reads it as its
    basin.par line-20 file (control/init_data.f90:115-120)."""
    i = np.arange(nx - 4, dtype=np.float64)[:, None] / (nx - 4)
    j = np.arange(ny - 4, dtype=np.float64)[None, :] / (ny - 4)
    h = 20.0 + 80.0 * (0.5 + 0.25 * np.sin(2 * np.pi * 1.5 * i + 0.3) + 0.25 * np.cos(2 * np.pi * 2.3 * j))
    return np.asfortranarray(h.astype(np.float32))
SW_DEFAULT = dict(ffs=1, trans=1, ksw=1, ts="0.5d0")

# name -> (basin, sw, (bppnx, bppny), steps, keep_full_arrays)
CASES = {
    "box40x32_b2x2_s5": (dict(BOX, nx=40, ny=32), SW_DEFAULT, (2, 2), 5, True),
    "box70x54_b1x1_s20": (dict(BOX, nx=70, ny=54), SW_DEFAULT, (1, 1), 20, True),
    "box70x54_b3x2_s20": (dict(BOX, nx=70, ny=54), SW_DEFAULT, (3, 2), 20, False),
    "box48x40_flags000_s10": (dict(BOX, nx=48, ny=40), dict(ffs=0, trans=0, ksw=0, ts="0.5d0"), (1, 1), 10, True),
    "box48x40_cart_s10": (dict(BOX, nx=48, ny=40, curve=0), dict(SW_DEFAULT, ts="0.25d0"), (1, 1), 10, True),
    "bs_b1x1_s60": (BS, SW_DEFAULT, (1, 1), 60, False),
    "bs_b4x2_s60": (BS, SW_DEFAULT, (4, 2), 60, False),
    # tracers (config 5 = BS + 1 tracer on 4x2 blocks)
    "box40x32_tr2_s5": (dict(BOX, nx=40, ny=32), dict(SW_DEFAULT, tr=1, trn=2), (2, 1), 5, True),
    "box70x54_b3x2_tr_s20": (dict(BOX, nx=70, ny=54), dict(SW_DEFAULT, tr=1, trn=1), (3, 2), 20, False),
    "bs_b4x2_tr_s60": (BS, dict(SW_DEFAULT, tr=1, trn=1), (4, 2), 60, False),
    # the shipped run length (ocean_run.par: 0.007 days = 604 steps), SURVEY.md 8(c) tolerance
    "bs_b1x1_s604": (BS, SW_DEFAULT, (1, 1), 604, False),
    "bs_b4x2_tr_s604": (BS, dict(SW_DEFAULT, tr=1, trn=1), (4, 2), 604, False),
    # step 0 (init_grid_data + init_ocean_data only): pins the device-side initial state
    "box70x54_b1x1_s0": (dict(BOX, nx=70, ny=54), SW_DEFAULT, (1, 1), 0, True),
    "box48x40_cart_s0": (dict(BOX, nx=48, ny=40, curve=0), dict(SW_DEFAULT, ts="0.25d0"), (1, 1), 0, True),
    "bs_b4x2_tr_s0": (BS, dict(SW_DEFAULT, tr=1, trn=1), (4, 2), 0, False),
    # BASELINE.json configs at full size: SHA-256 digests only ("sha"), streamed from the dump
    "box1024_b1x1_s10": (dict(BOX, nx=1028, ny=1028), SW_DEFAULT, (1, 1), 10, "sha"),      # C2
    "box2048_b2x2_s4": (dict(BOX, nx=2052, ny=2052), SW_DEFAULT, (2, 2), 4, "sha"),        # C3
    "box4096_b1x1_s6": (dict(BOX, nx=4100, ny=4100), SW_DEFAULT, (1, 1), 6, "sha"),        # the bench workload
    "box4096_b4x2_s4": (dict(BOX, nx=4100, ny=4100), SW_DEFAULT, (4, 2), 4, "sha"),        # C4
    # C3 / C4 long enough for pairs of x2 steps over ranks with the bench's cadence (a 2-step call
    # that votes with the known-constant verdict, then one call of 8 or 10 steps: 4 / 5 x4 pairs)
    "box2048_b2x2_s10": (dict(BOX, nx=2052, ny=2052), SW_DEFAULT, (2, 2), 10, "sha"),      # C3
    "box4096_b4x2_s12": (dict(BOX, nx=4100, ny=4100), SW_DEFAULT, (4, 2), 12, "sha"),      # C4
    # the reference's shipped default run: basin.par 1525 x 1115, mask and topography none, sw.par,
    # ocean_run.par's tau = 1 s for 0.007 days = 604 steps (model.f90:135-160); one block as
    # parallel.par ships it, and 2 x 2 blocks (odd, non-64-aligned block sizes)
    "box1521x1111_b1x1_s604": (dict(BOX, nx=1525, ny=1115), SW_DEFAULT, (1, 1), 604, "sha"),
    "box1521x1111_b2x2_s604": (dict(BOX, nx=1525, ny=1115), SW_DEFAULT, (2, 2), 604, "sha"),
    # a non-uniform rest depth (basin.par line 20 file): the one-pass steps' general variant
    "box70x54_topo_b1x1_s20": (dict(BOX, nx=70, ny=54, topo="wave"), SW_DEFAULT, (1, 1), 20, True),
    "box70x54_topo_b3x2_s20": (dict(BOX, nx=70, ny=54, topo="wave"), SW_DEFAULT, (3, 2), 20, False),
    "bs_topo_b4x2_s60": (dict(BS, topo="wave"), SW_DEFAULT, (4, 2), 60, False),
}
PROGNOSTIC = ["ssh", "sshp", "ubrtr", "ubrtrp", "vbrtr", "vbrtrp", "ff1_1", "ff1p_1"]


def digest(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a.ravel(order="F")).tobytes()).hexdigest()


def digest_dump(path):
    """read_dump's layout, but every field only as its SHA-256 (memory-mapped, for the
    multi-GB dumps of the full-size boxes): each field record is already the Fortran-ordered
    array, so its bytes are what digest() hashes."""
    from tests.golden.refdump import R4_FIELDS as r4, R8_FIELDS as r8
    raw = np.memmap(path, dtype=np.uint8, mode="r")
    pos = 0

    def take(nbytes):
        nonlocal pos
        a = raw[pos:pos + nbytes]
        pos += nbytes
        return a

    bcount, ntr = (int(v) for v in take(8).view("<i4"))
    out = []
    for _ in range(bcount):
        bm, bn, nxs, nxe, nys, nye, bx1, bx2, by1, by2 = (int(v) for v in take(40).view("<i4"))
        n = (bx2 - bx1 + 1) * (by2 - by1 + 1)
        names = [(nm, 4) for nm in r4] + [(nm, 8) for nm in r8]
        if ntr > 0:
            names += [(nm, 8) for nm in ["flux_x", "flux_y"] +
                      [f"{p}_{t}" for t in range(1, ntr + 1) for p in ("ff1", "ff1p", "ff1n")]]
        f = {nm: hashlib.sha256(memoryview(take(n * es))).hexdigest() for nm, es in names}
        out.append((dict(bm=bm, bn=bn, nxs=nxs, nxe=nxe, nys=nys, nye=nye, bx1=bx1, bx2=bx2, by1=by1, by2=by2), f))
    assert pos == raw.size, (pos, raw.size)
    return out


def gen_e2e(name, basin, sw, bxy, steps, full):
    d = tempfile.mkdtemp()
    topo = None
    try:
        if basin.get("topo", "none") != "none":
            topo = topography(basin["nx"], basin["ny"])
            topo.ravel(order="F").tofile(os.path.join(d, "topo.dat"))
        open(os.path.join(d, "basin.par"), "w").write(
            BASIN_TMPL.format(**dict(basin, topo="topo.dat" if topo is not None else "none")))
        open(os.path.join(d, "sw.par"), "w").write(SW_TMPL.format(**dict(dict(tr=0, trn=1), **sw)))
        open(os.path.join(d, "parallel.par"), "w").write(PAR_TMPL.format(bx=bxy[0], by=bxy[1]))
        env = dict(os.environ, OMP_NUM_THREADS="1")
        subprocess.check_call([REFDRV, str(steps), "dump.bin"], cwd=d, env=env,
                              stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        if full == "sha":
            blocks = digest_dump(os.path.join(d, "dump.bin"))
        else:
            blocks = read_dump(os.path.join(d, "dump.bin"))
    finally:
        shutil.rmtree(d)
    out = {"meta/basin": np.array(repr({k: v for k, v in basin.items() if k not in ("mask", "topo")} |
                                         {"mask": "BS" if basin["mask"] != "none" else "none"})),
           "meta/sw": np.array(repr(sw)), "meta/bxy": np.array(bxy, np.int32), "meta/steps": np.int32(steps)}
    if topo is not None:
        out["in/topo"] = topo
    if basin["mask"] != "none":
        from oracle.oracle import read_mask_file
        m = read_mask_file(basin["mask"], basin["nx"], basin["ny"])
        out["in/mask_packed"] = np.packbits(m.ravel(order="F").astype(np.uint8))
    for info, f in blocks:
        key = f"{info['bm']}_{info['bn']}"
        out[f"b{key}/info"] = np.array([info[k] for k in ("nxs", "nxe", "nys", "nye", "bx1", "bx2", "by1", "by2")],
                                       np.int32)
        for nm, a in f.items():
            out[f"b{key}/sha/{nm}"] = np.array(a if isinstance(a, str) else digest(a))
            if full is True or (full is False and nm in PROGNOSTIC):
                out[f"b{key}/{nm}"] = a
    path = os.path.join(HERE, f"e2e_{name}.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, os.path.getsize(path))


def main(which):
    """which: nothing = everything; otherwise "kernels" and/or e2e case names."""
    subprocess.check_call(["make", "-s", "-f", os.path.join(REPO, "oracle", "ref.mk")], cwd=REPO)
    ref = C.CDLL(REFLIB)
    if not which or "kernels" in which:
        for i, (tag, geom) in enumerate(GEOMS.items()):
            gen_kernels(ref, tag, geom, 1234 + i)
    for name, (basin, sw, bxy, steps, full) in CASES.items():
        if not which or name in which:
            gen_e2e(name, basin, sw, bxy, steps, full)


if __name__ == "__main__":
    main(sys.argv[1:])
