"""The product's stencil functors (ocean_model_arch_amd/csrc/sw_stencils.h -- the code the HIP
kernels run) executed on the host by tests/native/stencil_host.cpp with every array access
bounds-checked, against the compiled reference's golden outputs.

Catches, on the CPU and before anything reaches the GPU: out-of-bounds accesses (a GPU memory
fault), write-set mistakes, arithmetic-order mistakes, and errors in the fused regrouping of
the step (fused A/B/C1 + hh_init with three halo exchanges must give the reference's state bit
for bit).  Halo exchanges between blocks use the oracle's block copies."""
import ctypes as C
import hashlib
import os
import subprocess

import numpy as np
import pytest

from oracle import oracle as O
from tests.golden import cases

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(REPO, "tests", "native", "libstencil_host.so")

R4 = ["lu", "luu", "luh", "lcu", "lcv", "llu", "llv", "dx", "dy", "dxt", "dyt", "dxh", "dyh", "dxb", "dyb",
      "rlh_s", "r_diss"]
R8 = ["ssh", "sshn", "sshp", "ubrtr", "ubrtrn", "ubrtrp", "vbrtr", "vbrtrn", "vbrtrp", "hhq", "hhq_p", "hhq_n",
      "hhu", "hhu_p", "hhu_n", "hhv", "hhv_p", "hhv_n", "hhh", "hhh_p", "hhh_n", "hhq_rest", "vort", "str_t",
      "str_s", "mu", "RHSx", "RHSy", "RHSx_adv", "RHSy_adv", "RHSx_dif", "RHSy_dif"]
STAGE = {n: i for i, n in enumerate(cases.KERNEL_NAMES)}
STAGE_IDS = {"sw_update_ssh": 0, "hh_update": 1, "uv_trans_vort": 2, "uv_trans": 3, "stress_components": 4,
             "uv_diff2": 5, "sw_update_uv": 6, "sw_next_step": 7, "hh_shift": 8, "hh_init": 9}
FUSED_A, FUSED_B, FUSED_C1, CHECK = 11, 12, 13, 10


class Block(C.Structure):
    _fields_ = [(n, C.c_int32) for n in ("nx_start", "nx_end", "ny_start", "ny_end", "bnd_x1", "bnd_x2",
                                         "bnd_y1", "bnd_y2")] + [("pitch", C.c_int64)]


class SwParams(C.Structure):
    _fields_ = [("full_free_surface", C.c_int32), ("trans_terms", C.c_int32), ("ksw_lat", C.c_int32),
                ("time_smooth", C.c_double), ("lvisc_2", C.c_double)]


@pytest.fixture(scope="module")
def hst():
    subprocess.check_call(["make", "-s", "-f", os.path.join(REPO, "tests", "native", "Makefile")], cwd=REPO)
    L = C.CDLL(LIB)
    L.hst_stage.restype = C.c_long
    L.hst_stage.argtypes = [C.c_int, C.POINTER(Block), C.c_void_p, C.c_int, C.c_void_p, C.c_void_p,
                            C.POINTER(SwParams), C.c_double, C.POINTER(C.c_int32), C.c_int, C.c_int]
    L.hst_split_ok.argtypes = [C.c_int] * 8
    L.hst_tracer.restype = C.c_long
    L.hst_tracer.argtypes = [C.c_int, C.POINTER(Block), C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_int,
                             C.c_double, C.c_double, C.c_double]
    L.hst_tracer_step.restype = C.c_long
    L.hst_tracer_step.argtypes = [C.POINTER(Block), C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_int, C.c_double,
                                  C.c_double, C.c_uint, C.c_void_p, C.c_void_p]
    L.hst_prepare.restype = C.c_int
    L.hst_prepare.argtypes = [C.POINTER(Block), C.c_void_p, C.c_void_p, C.c_void_p]
    return L


def table(arrs, ntr=0, kernel_names=False):
    """Field table indexed like ocn_field_slot: the SW fields, then (tracers) flux_x, flux_y and
    ff1/ff1p/ff1n per tracer (named ff1, ff1p, ff1n in the kernel fixtures)."""
    names = R4 + R8
    if ntr:
        names = names + ["flux_x", "flux_y"] + (["ff1", "ff1p", "ff1n"] if kernel_names else
                                                [f"{p}_{k}" for k in range(1, ntr + 1) for p in ("ff1", "ff1p", "ff1n")])
    t = (C.c_void_p * len(names))()
    for i, n in enumerate(names):
        t[i] = arrs[n].ctypes.data
    return t


def blk(g):
    nxs, nxe, nys, nye, bx1, bx2, by1, by2 = (int(v) for v in g)
    return Block(nxs, nxe, nys, nye, bx1, bx2, by1, by2, bx2 - bx1 + 1)


def bits_equal(a, b):
    return np.ascontiguousarray(a.ravel(order="F")).tobytes() == np.ascontiguousarray(b.ravel(order="F")).tobytes()


@pytest.mark.parametrize("geom", cases.KERNEL_GEOMS)
def test_tracer_functors_match_reference(hst, geom):
    z = cases.load_kernels(geom)
    b = blk(z["geom"])
    bad = []
    for st, kname in enumerate(cases.TRACER_KERNEL_NAMES):
        arrs = {k[3:]: z[k].copy(order="F") for k in z.files if k.startswith("in/")}
        t = table(arrs, 1, True)
        oob = hst.hst_tracer(st, C.byref(b), t, len(t), None, None, 1, float(z["tau"]),
                             float(z["time_smooth"]), float(z["factor_mu"]))
        assert oob == 0, f"{kname}: {oob} out-of-bounds accesses"
        for nm in [k.split("/", 1)[1] for k in z.files if k.startswith(kname + "/")]:
            if not bits_equal(arrs[nm], z[f"{kname}/{nm}"]):
                bad.append(f"{kname}:{nm}")
    assert not bad, bad


@pytest.mark.parametrize("geom", cases.KERNEL_GEOMS)
def test_stage_functors_match_reference(hst, geom):
    z = cases.load_kernels(geom)
    b = blk(z["geom"])
    sw = SwParams(int(z["full_free_surface"]), 1, 1, float(z["time_smooth"]), 1000.0)
    bad = []
    for kname in cases.KERNEL_NAMES:
        arrs = {k[3:]: z[k].copy(order="F") for k in z.files if k.startswith("in/")}
        nbad = C.c_int32(0)
        t = table(arrs)
        oob = hst.hst_stage(STAGE_IDS[kname], C.byref(b), t, len(t), None, None, C.byref(sw), float(z["tau"]),
                            C.byref(nbad), 1, 0)
        assert oob == 0, f"{kname}: {oob} out-of-bounds accesses"
        for nm in [k.split("/", 1)[1] for k in z.files if k.startswith(kname + "/")]:
            if not bits_equal(arrs[nm], z[f"{kname}/{nm}"]):
                bad.append(f"{kname}:{nm}")
    assert not bad, bad


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a.ravel(order="F")).tobytes()).hexdigest()


N_ROW_FIELDS = len(R4) - 7 + 4      # dx .. r_diss, then the 4 stress_components ratios (sw_stencils.h kRowTable)


def compact_tables(hst, om):
    """Host-built compact static fields (sw_stencils.h Prepare) of every block; rows the
    stencils must not read are NaN so that a wrong row index cannot go unnoticed."""
    out = []
    for k, b in enumerate(om.blocks):
        blk_ = Block(*b.args, b.bx2 - b.bx1 + 1)
        shape = om.f[k]["lu"].shape
        bits = np.zeros(shape[0] * shape[1], dtype=np.uint8)
        # + the one-pass step's per-row reciprocals (sw_stencils.h recip_offset / row_table_floats)
        rows = np.full(((N_ROW_FIELDS * shape[1] + 1) & ~1) + 2 * 7 * shape[1], np.nan, dtype=np.float32)
        flags = hst.hst_prepare(C.byref(blk_), table(om.f[k]), bits.ctypes.data, rows.ctypes.data)
        out.append((bits, rows, flags))
    return out


def host_step(hst, om, mode, nbad, last=True, tabs=None, first=True):
    sw_o = om.sw
    sw = SwParams(sw_o.full_free_surface, sw_o.trans_terms, sw_o.ksw_lat, sw_o.time_smooth, sw_o.lvisc_2)
    ntr = sw_o.tracer_num if sw_o.use_tracers > 0 else 0
    blocks = [(Block(*b.args, b.bx2 - b.bx1 + 1), table(om.f[k], ntr)) for k, b in enumerate(om.blocks)]
    compact = mode in ("compact", "overlap_early", "overlap_late")

    def tracers():
        """expl_tracer (control/tracer.f90:33-62) after the SW step."""
        for t in range(1, ntr + 1):
            for st, sync in ((0, ["flux_x", "flux_y"]), (1, [f"ff1n_{t}"]), (2, [])):
                for k, (b, tb) in enumerate(blocks):
                    bits, rows = (tabs[k][0].ctypes.data, tabs[k][1].ctypes.data) if compact else (None, None)
                    oob = hst.hst_tracer(st, C.byref(b), tb, len(tb), bits, rows, t, 1.0, sw_o.time_smooth, 1.0)
                    assert oob == 0, f"tracer stage {st}: {oob} out-of-bounds accesses"
                for f in sync:
                    om.sync(f)

    def each(stage, tau=1.0, full=1, part=0):
        for k, (b, t) in enumerate(blocks):
            bits, rows = (tabs[k][0].ctypes.data, tabs[k][1].ctypes.data) if compact else (None, None)
            oob = hst.hst_stage(stage, C.byref(b), t, len(t), bits, rows, C.byref(sw), tau, C.byref(nbad), full, part)
            assert oob == 0, f"stage {stage}: {oob} out-of-bounds accesses"

    def syncs(names):
        for f in names:
            om.sync(f)

    # ocn_ctx.hip one_step_fused: "reuse" steps skip hh_update (hun/hvn/hhn = previous hu/hv/hh)
    reuse = sw.full_free_surface == 1 and not first and not last
    fa = 2 * int(reuse)
    fb = int(last) | 2 * int(reuse)
    sa = ["sshn"] + (["hhu_n", "hhv_n", "hhh_n"] if sw.full_free_surface > 0 and not reuse else []) + \
         (["vort"] if sw.trans_terms > 0 else []) + (["str_t", "str_s"] if sw.ksw_lat > 0 else [])
    sb = (["hhu_p", "hhv_p", "hhh_p"] if sw.trans_terms > 0 else []) + ["vbrtrn", "ubrtrn"]
    if mode in ("overlap_early", "overlap_late"):
        # ocn_ctx.hip one_step_fused with OCN_OPT_OVERLAP: each exchange runs concurrently with
        # the inner launches; emulate it completing as early and as late as possible
        early = mode == "overlap_early"
        FR, IN = 1, 2
        each(FUSED_A, full=fa, part=FR)
        if early: syncs(sa)
        each(FUSED_A, full=fa, part=IN)
        each(FUSED_B, full=fb, part=IN)
        if not early: syncs(sa)
        each(FUSED_B, full=fb, part=FR)
        if early: syncs(sb)
        each(FUSED_C1, part=IN)
        if not early: syncs(sb)
        each(FUSED_C1, part=FR)
        if sw.full_free_surface > 0:
            each(STAGE_IDS["hh_init"], full=int(last or ntr > 0), part=FR)
            if early: syncs(["hhu", "hhv", "hhh"])
            each(STAGE_IDS["hh_init"], full=int(last or ntr > 0), part=IN)
            if not early: syncs(["hhu", "hhv", "hhh"])
        tracers()
        return
    if mode != "stages":
        each(FUSED_A, full=fa)
        for f in sa:
            om.sync(f)
        each(FUSED_B, full=fb)
        for f in (["hhu_p", "hhv_p", "hhh_p"] if sw.trans_terms > 0 else []) + ["vbrtrn", "ubrtrn"]:
            om.sync(f)
        each(FUSED_C1)
        if sw.full_free_surface > 0:
            each(STAGE_IDS["hh_init"], full=int(last or ntr > 0))      # tracers read hhq_p every step
            for f in ("hhu", "hhv", "hhh"):
                om.sync(f)
    else:
        syncs = {"sw_update_ssh": ["sshn"], "hh_update": ["hhu_n", "hhv_n", "hhh_n"], "uv_trans_vort": ["vort"],
                 "uv_trans": ["hhu_p", "hhv_p", "hhh_p"], "stress_components": ["str_t", "str_s"],
                 "sw_update_uv": ["vbrtrn", "ubrtrn"], "hh_init": ["hhu", "hhv", "hhh"]}
        order = ["sw_update_ssh"] + (["hh_update"] if sw.full_free_surface > 0 else []) + \
                (["uv_trans_vort", "uv_trans"] if sw.trans_terms > 0 else []) + \
                (["stress_components", "uv_diff2"] if sw.ksw_lat > 0 else []) + ["sw_update_uv", "sw_next_step"] + \
                (["hh_shift", "hh_init"] if sw.full_free_surface > 0 else [])
        for st in order:
            each(STAGE_IDS[st])
            for f in syncs.get(st, []):
                om.sync(f)
        each(CHECK)
    tracers()


@pytest.mark.parametrize("mode", ["compact", "fused", "stages", "overlap_early", "overlap_late"])
@pytest.mark.parametrize("name", cases.E2E_CASES + cases.TRACER_E2E_CASES)
def test_host_step_matches_reference(hst, name, mode):
    """The whole run as one ocn_ctx_step call: hh_init's time-invariant stores are skipped on
    every step but the last (fused modes); "compact" reads masks / metrics from the compact
    tables, which must be exact for these grids (no curvilinear metrics)."""
    case = cases.load_e2e(name)
    b = case["basin"]
    om = O.OracleModel(O.BasinConfig(nx=b["nx"], ny=b["ny"], dxst=b["dxst"], dyst=b["dyst"], rlon=b["rlon"],
                                     rlat=b["rlat"], curve_grid=b["curve_grid"], mask=case["mask"]),
                       O.SWConfig(**case["sw"]), *case["bxy"]).init()
    nbad = C.c_int32(0)
    tabs = None
    if mode in ("compact", "overlap_early", "overlap_late"):
        tabs = compact_tables(hst, om)
        assert all(t[2] & 3 == 0 for t in tabs), [t[2] for t in tabs]   # 4 = sea on the halo ring: fine
    for s in range(case["steps"]):
        host_step(hst, om, mode, nbad, last=s == case["steps"] - 1, tabs=tabs, first=s == 0)
    assert nbad.value == 0
    z = case["z"]
    bad = []
    for k, blkk in enumerate(om.blocks):
        for nm, a in om.f[k].items():
            key = f"b{blkk.bm}_{blkk.bn}/sha/{nm}"
            if key in z.files and _sha(a) != str(z[key]):
                bad.append(f"({blkk.bm},{blkk.bn}):{nm}")
    assert not bad, f"{name}: {bad}"


@pytest.mark.parametrize("what,flag", [("none", 0), ("metric", 2), ("mask", 1)])
def test_compact_tables_detect_inexact_fields(hst, what, flag):
    """Prepare must refuse (flags) real(4) fields the compact tables cannot hold exactly: a metric
    that varies along a row inside [nx_start-1, nx_end+1], a mask value other than 0.0 / 1.0."""
    om = O.OracleModel(O.BasinConfig(nx=40, ny=36), O.SWConfig(), 2, 1).init()
    for k in range(len(om.blocks)):
        if what == "metric":
            om.f[k]["dyh"][3, 4] = np.nextafter(om.f[k]["dyh"][3, 4], np.float32(2e9))
        elif what == "mask":
            om.f[k]["llv"][5, 5] = 0.5
    tabs = compact_tables(hst, om)
    assert [t[2] & 3 for t in tabs] == [flag] * len(om.blocks)
    # OCN_COMPACT_RING_SEA: the blocks' shared edge puts sea points on each block's halo ring
    assert all(t[2] & 4 for t in tabs)


def test_ring_sea_flag_on_closed_box(hst):
    """One block of the closed box: the halo ring is the land frame, so the role-flip steps may
    skip a8 / a9 on the ring (Prepare leaves OCN_COMPACT_RING_SEA clear); the Black Sea basin's
    single block too, when no sea touches its ring."""
    om = O.OracleModel(O.BasinConfig(nx=40, ny=36), O.SWConfig(), 1, 1).init()
    assert compact_tables(hst, om)[0][2] == 0


def test_compact_row_window_is_what_the_stencils_read(hst):
    """A metric varying only outside [nx_start-1, nx_end+1] (the outer halo column, never read)
    keeps the compact tables usable, and the run stays bitwise equal to the 2-D path."""
    om = O.OracleModel(O.BasinConfig(nx=40, ny=36), O.SWConfig(), 1, 1).init()
    om.f[0]["dx"][0, :] *= np.float32(3.0)          # column bnd_x1 = nx_start - 2
    tabs = compact_tables(hst, om)
    assert tabs[0][2] & 3 == 0
    ref = O.OracleModel(O.BasinConfig(nx=40, ny=36), O.SWConfig(), 1, 1).init()
    ref.f[0]["dx"][0, :] *= np.float32(3.0)
    nbad = C.c_int32(0)
    for s in range(4):
        host_step(hst, om, "compact", nbad, last=s == 3, tabs=tabs, first=s == 0)
        host_step(hst, ref, "stages", nbad)
    for nm in ref.f[0]:
        assert bits_equal(om.f[0][nm], ref.f[0][nm]), nm


@pytest.mark.parametrize("r,inner", [((1, 40, 1, 30), (3, 38, 3, 28)), ((2, 9, 2, 9), (3, 8, 3, 8)),
                                     ((5, 6, 5, 6), (6, 5, 6, 5)), ((0, 63, 0, 0), (1, 62, 1, -1)),
                                     ((3, 70, 3, 70), (0, 100, 0, 100)), ((3, 70, 3, 70), (10, 20, 50, 60))])
def test_frame_inner_split_partitions_the_range(hst, r, inner):
    """The halo-overlap split: frame + inner cover every point of the launch range exactly once."""
    assert hst.hst_split_ok(*r, *inner) == 1


def _own_bits(om, b):
    """sw_stencils.h own_class bits of block b's halo points that neighbour blocks own."""
    own = 0
    for d, (dm, dn) in O.DIRS.items():
        if d in b.nbr:
            own |= 1 << ((2 if dm > 0 else 0 if dm < 0 else 1) * 3 + (2 if dn > 0 else 0 if dn < 0 else 1))
    return own


@pytest.mark.parametrize("compact", [False, True])
@pytest.mark.parametrize("name", cases.TRACER_E2E_CASES)
def test_tracer_step_matches_expl_tracer(hst, name, compact):
    """The tracer step (sw_stencils.h TracerStep, one launch per tracer in one-pass sequences) on the
    state a step leaves, against the oracle's expl_tracer (control/tracer.f90:33-62: the three stages
    with hh_init's stored depths and their exchanges) on the same state: its ffn and filtered ffp at
    every interior sea point bit for bit, after a few steps (a moving state, nonzero fluxes)."""
    case = cases.load_e2e(name)
    b = case["basin"]
    om = O.OracleModel(O.BasinConfig(nx=b["nx"], ny=b["ny"], dxst=b["dxst"], dyst=b["dyst"], rlon=b["rlon"],
                                     rlat=b["rlat"], curve_grid=b["curve_grid"], mask=case["mask"]),
                       O.SWConfig(**case["sw"]), *case["bxy"]).init()
    om.run(3)
    tau, ts = 1.0, om.sw.time_smooth
    # step 4's shallow-water part (model.f90:146), then expl_tracer on copies
    ntr = om.sw.tracer_num
    expl = om.expl_tracer
    om.expl_tracer = lambda tau=1.0: None
    om.step(tau)
    om.expl_tracer = expl
    state = [{nm: a.copy(order="F") for nm, a in f.items()} for f in om.f]
    tabs = compact_tables(hst, om) if compact else None
    om.expl_tracer(tau)
    bad = []
    for k, blkk in enumerate(om.blocks):
        g = blkk.args
        bb = blk(g)
        for t in range(1, ntr + 1):
            ffn_out = state[k][f"ff1n_{t}"].copy(order="F")
            ffp_out = state[k][f"ff1p_{t}"].copy(order="F")
            tab = table(state[k], ntr)
            bits, rows = (tabs[k][0].ctypes.data, tabs[k][1].ctypes.data) if compact else (None, None)
            oob = hst.hst_tracer_step(C.byref(bb), tab, len(tab), bits, rows, t, tau, ts, _own_bits(om, blkk),
                                      ffn_out.ctypes.data, ffp_out.ctypes.data)
            assert oob == 0, oob
            lu = om.f[k]["lu"] > 0.5
            inner = np.zeros_like(lu)
            inner[g[0] - g[4]:g[1] - g[4] + 1, g[2] - g[6]:g[3] - g[6] + 1] = True
            sea = lu & inner
            for nm, got, want in ((f"ff1n_{t}", ffn_out, om.f[k][f"ff1n_{t}"]), (f"ff1p_{t}", ffp_out, om.f[k][f"ff1p_{t}"]),
                                  (f"ff1_{t}", ffn_out, om.f[k][f"ff1_{t}"])):
                if got[sea].tobytes() != want[sea].tobytes():
                    bad.append(f"({blkk.bm},{blkk.bn}):{nm} {int((got[sea] != want[sea]).sum())}/{int(sea.sum())}")
    assert not bad, bad


@pytest.mark.parametrize("which", ["llu", "llv", "luh"])
def test_compact_tables_flag_inconsistent_sea_masks(hst, which):
    """The one-pass step divides its hh_init averages by the sea count without a zero case
    (sw_kernels.hip rcp_sea): Prepare flags (OCN_COMPACT_DIVISOR_RANGE: no one-pass steps) an
    llu / llv / luh set where lu_lv_init would not set it -- no sea point among the average's
    corners (grid_kernels.f90:60-86) -- and nothing for the masks lu_lv_init forms."""
    om = O.OracleModel(O.BasinConfig(nx=40, ny=36), O.SWConfig(), 1, 1).init()
    assert compact_tables(hst, om)[0][2] & 8 == 0
    f = om.f[0]
    for nm in ("lu", "luh", "luu", "llu", "llv", "lcu", "lcv"):   # a land square of 3 x 3 points
        f[nm][10:13, 10:13] = 0.0
    f[which][11, 11] = 1.0
    assert compact_tables(hst, om)[0][2] & 8 == 8
