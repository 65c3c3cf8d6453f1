"""Pin the CPU oracle (oracle/sw_oracle.c + oracle/oracle.py) against the compiled
reference's own outputs (tests/golden, made by tests/golden/gen_golden.py).

Bar: bitwise equality of every output array (halos and untouched cells included)."""
import ctypes as C
import hashlib

import numpy as np
import pytest

from oracle import oracle as O
from tests.golden import cases

# oracle entry point + argument names (same order as the reference kernel, see gen_golden.KERNELS)
ORC_ARGS = {
    "sw_update_ssh": ("orc_sw_update_ssh", ["tau"], ["lu", "dx", "dy", "dxh", "dyh", "hhu", "hhv", "sshn",
                                                     "sshp", "ubrtr", "vbrtr"]),
    "sw_update_uv": ("orc_sw_update_uv", ["tau"], ["lcu", "lcv", "dxt", "dyt", "dxh", "dyh", "dxb", "dyb",
                                                   "hhu", "hhu_n", "hhu_p", "hhv", "hhv_n", "hhv_p", "hhh", "ssh",
                                                   "ubrtr", "ubrtrn", "ubrtrp", "vbrtr", "vbrtrn", "vbrtrp",
                                                   "r_diss", "rlh_s", "RHSx", "RHSy", "RHSx_adv", "RHSy_adv",
                                                   "RHSx_dif", "RHSy_dif"]),
    "sw_next_step": ("orc_sw_next_step", ["time_smooth"], ["lu", "lcu", "lcv", "ssh", "sshn", "sshp", "ubrtr",
                                                           "ubrtrn", "ubrtrp", "vbrtr", "vbrtrn", "vbrtrp"]),
    "uv_trans_vort": ("orc_uv_trans_vort", [], ["luu", "dxt", "dyt", "dxb", "dyb", "ubrtr", "vbrtr", "vort"]),
    "uv_trans": ("orc_uv_trans", [], ["lcu", "lcv", "luu", "dxh", "dyh", "ubrtr", "vbrtr", "vort", "hhq", "hhu",
                                      "hhv", "hhh", "RHSx_adv", "RHSy_adv"]),
    "uv_diff2": ("orc_uv_diff2", [], ["lcu", "lcv", "dx", "dy", "dxt", "dyt", "dxh", "dyh", "dxb", "dyb", "mu",
                                      "str_t", "str_s", "hhq", "hhu", "hhv", "hhh", "RHSx_dif", "RHSy_dif"]),
    "stress_components": ("orc_stress_components", [], ["lu", "luu", "dx", "dy", "dxt", "dyt", "dxh", "dyh",
                                                        "dxb", "dyb", "ubrtrp", "vbrtrp", "str_t", "str_s"]),
    "hh_init": ("orc_hh_init", ["ffs"], ["lu", "llu", "llv", "luh", "dx", "dy", "dxt", "dyt", "dxh", "dyh",
                                         "dxb", "dyb", "hhq", "hhq_p", "hhq_n", "hhu", "hhu_p", "hhu_n", "hhv",
                                         "hhv_p", "hhv_n", "hhh", "hhh_p", "hhh_n", "ssh", "sshp", "hhq_rest"]),
    "hh_update": ("orc_hh_update", [], ["lu", "llu", "llv", "luh", "dx", "dy", "dxt", "dyt", "dxh", "dyh", "dxb",
                                        "dyb", "hhq_n", "hhu_n", "hhv_n", "hhh_n", "ssh", "hhq_rest"]),
    # kernel/tracer/leapfrog_tracer.f90; "@x" = the fixture's scalar x passed in place
    "tran_diff_fluxes": ("orc_tran_diff_fluxes", [], ["lcu", "lcv", "dxt", "dyt", "dxh", "dyh", "hhu", "hhv", "ff1",
                                                     "ff1p", "ubrtr", "vbrtr", "mu", "@factor_mu", "flux_x",
                                                     "flux_y"]),
    "tran_diff_tracer": ("orc_tran_diff_tracer", [], ["lu", "dx", "dy", "@tau", "hhq_n", "hhq_p", "flux_x", "flux_y",
                                                     "ff1p", "ff1n"]),
    "tracer_next_step": ("orc_tracer_next_step", ["time_smooth"], ["lu", "ff1n", "ff1p", "ff1"]),
    "hh_shift": ("orc_hh_shift", ["time_smooth"], ["lu", "llu", "llv", "luh", "hhq", "hhq_p", "hhq_n", "hhu",
                                                   "hhu_p", "hhu_n", "hhv", "hhv_p", "hhv_n", "hhh", "hhh_p",
                                                   "hhh_n"]),
}


def bits_equal(a, b):
    a = np.ascontiguousarray(np.asarray(a).ravel(order="F"))
    b = np.ascontiguousarray(np.asarray(b).ravel(order="F"))
    return a.dtype == b.dtype and a.shape == b.shape and a.tobytes() == b.tobytes()


def run_oracle_kernel(z, kname):
    L = O.lib()
    geom = [int(v) for v in z["geom"]]
    work = {k[3:]: z[k].copy(order="F") for k in z.files if k.startswith("in/")}
    sym, scalars, names = ORC_ARGS[kname]
    sc = []
    for s in scalars:
        if s == "ffs":
            sc.append(C.c_int(int(z["full_free_surface"])))
        else:
            sc.append(C.c_double(float(z[s])))
    getattr(L, sym)(*geom, *sc, *[C.c_double(float(z[n[1:]])) if n[0] == "@" else work[n].ctypes.data_as(C.c_void_p)
                                  for n in names])
    return work


@pytest.mark.parametrize("geom", cases.KERNEL_GEOMS)
@pytest.mark.parametrize("kname", cases.KERNEL_NAMES + cases.TRACER_KERNEL_NAMES)
def test_oracle_kernel_matches_reference(geom, kname):
    z = cases.load_kernels(geom)
    work = run_oracle_kernel(z, kname)
    outs = [k.split("/", 1)[1] for k in z.files if k.startswith(kname + "/")]
    assert outs, kname
    for nm in outs:
        assert bits_equal(work[nm], z[f"{kname}/{nm}"]), f"{kname}:{nm} differs from the reference"


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a.ravel(order="F")).tobytes()).hexdigest()


def build_oracle_model(case):
    b = case["basin"]
    basin = O.BasinConfig(nx=b["nx"], ny=b["ny"], dxst=b["dxst"], dyst=b["dyst"], rlon=b["rlon"],
                          rlat=b["rlat"], curve_grid=b["curve_grid"], mask=case["mask"],
                            topography=case.get("topography"))
    sw = O.SWConfig(**case["sw"])
    return O.OracleModel(basin, sw, *case["bxy"])


@pytest.mark.parametrize("name", cases.E2E_CASES + cases.TRACER_E2E_CASES + cases.LONG_CASES + cases.INIT_CASES
                         + cases.FULLSIZE_CASES + cases.TOPO_CASES + ["box2048_b2x2_s10"])
def test_oracle_end_to_end_matches_reference(name):
    case = cases.load_e2e(name)
    z = case["z"]
    m = build_oracle_model(case).init().run(case["steps"])
    blocks = cases.e2e_blocks(z)
    assert len(blocks) == len(m.blocks)
    checked = set()
    for k, blk in enumerate(m.blocks):
        info = blocks[(blk.bm, blk.bn)]
        assert list(info) == list(blk.args)
        for nm, a in m.f[k].items():
            key = f"b{blk.bm}_{blk.bn}/sha/{nm}"
            if key not in z.files:
                continue
            assert _sha(a) == str(z[key]), f"{name}: block ({blk.bm},{blk.bn}) field {nm} differs"
            checked.add(nm)
    assert len(checked) >= 49, f"{name}: only {len(checked)} fields checked"
    if case["sw"].get("use_tracers", 0) > 0:
        assert {"flux_x", "flux_y", "ff1_1", "ff1p_1", "ff1n_1"} <= checked


def test_uniform_decomposition_sizes():
    # decomposition.f90:448-482 on BS x-size 285 over 4 blocks: 71/71/71/72
    assert O.uniform_sizes(285, 4) == [71, 71, 71, 72]
    assert O.uniform_sizes(159, 2) == [79, 80]
    assert sum(O.uniform_sizes(1024, 8)) == 1024


def test_oracle_threads_over_blocks_match_reference():
    """The all-cores CPU baseline's mode (threads over blocks, kernel_interface.f90:84-88) gives the
    reference's results bit for bit."""
    name = "box70x54_b3x2_s20"
    case = cases.load_e2e(name)
    b = case["basin"]
    basin = O.BasinConfig(nx=b["nx"], ny=b["ny"], dxst=b["dxst"], dyst=b["dyst"], rlon=b["rlon"],
                          rlat=b["rlat"], curve_grid=b["curve_grid"], mask=case["mask"],
                            topography=case.get("topography"))
    m = O.OracleModel(basin, O.SWConfig(**case["sw"]), *case["bxy"], threads=3).init().run(case["steps"])
    m.pool.shutdown()
    z = case["z"]
    for k, blk in enumerate(m.blocks):
        for nm, a in m.f[k].items():
            key = f"b{blk.bm}_{blk.bn}/sha/{nm}"
            if key in z.files:
                assert _sha(a) == str(z[key]), f"block ({blk.bm},{blk.bn}) field {nm} differs"


@pytest.mark.parametrize("name", ["box70x54_b3x2_s20", "bs_b4x2_s60", "bs_b4x2_tr_s60"])
def test_noparallel_build_matches_block_build(name):
    """BASELINE.json's north star names the reference's _MPP_NO_PARALLEL_MODE_ CPU run; the fixtures
    come from its default _MPP_BLOCK_MODE_ build (one thread).  tests/golden/gen_noparallel.py built
    the reference once more with that one macro switched (macros/mpp_macros.fi:23) and ran the same
    multi-block cases: every field of every block has the same digest."""
    a = cases.load_e2e(name)["z"]
    b = np.load(cases.HERE + f"/e2e_{name}_noparallel.npz")
    sha_a = {k for k in a.files if "/sha/" in k}
    sha_b = {k for k in b.files if "/sha/" in k}
    assert sha_a == sha_b and len(sha_a) >= 49
    diff = [k for k in sha_a if str(a[k]) != str(b[k])]
    assert not diff, diff
