"""Access to the golden fixtures (no dependency on /root/reference at run time)."""
import ast
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))

E2E_CASES = ["box40x32_b2x2_s5", "box70x54_b1x1_s20", "box70x54_b3x2_s20",
             "box48x40_flags000_s10", "box48x40_cart_s10", "bs_b1x1_s60", "bs_b4x2_s60"]
TRACER_E2E_CASES = ["box40x32_tr2_s5", "box70x54_b3x2_tr_s20", "bs_b4x2_tr_s60"]
# the shipped run length (ocean_run.par: 604 steps), Black Sea, 1 block / 4x2 blocks + 1 tracer
LONG_CASES = ["bs_b1x1_s604", "bs_b4x2_tr_s604"]
# step 0: init_grid_data + init_ocean_data only (the initial state)
INIT_CASES = ["box70x54_b1x1_s0", "box48x40_cart_s0", "bs_b4x2_tr_s0"]
# BASELINE.json configs at full size (SHA-256 digests of every field of every block only):
# C2 1024^2 1 block, C3 2048^2 2x2 blocks, the bench workload 4096^2 1 block, C4 4096^2 4x2 blocks
FULLSIZE_CASES = ["box1024_b1x1_s10", "box2048_b2x2_s4", "box4096_b1x1_s6", "box4096_b4x2_s4"]
# C3 / C4 long enough for x4 pairs over ranks with the bench's cadence (tests/test_gpu_x4.py)
FULLSIZE_RANK_CASES = ["box2048_b2x2_s10", "box4096_b4x2_s12"]
# the reference's shipped default run (basin.par 1525 x 1115, 604 steps) on 1 and 2 x 2 blocks
SHIPPED_CASES = ["box1521x1111_b1x1_s604", "box1521x1111_b2x2_s604"]
# a non-uniform rest depth read from a basin.par topography file (control/init_data.f90:115-120)
TOPO_CASES = ["box70x54_topo_b1x1_s20", "box70x54_topo_b3x2_s20", "bs_topo_b4x2_s60"]
KERNEL_GEOMS = ["b66x50", "b1x1", "b130x7"]
KERNEL_NAMES = ["sw_update_ssh", "sw_update_uv", "sw_next_step", "uv_trans_vort", "uv_trans",
                "uv_diff2", "stress_components", "hh_init", "hh_update", "hh_shift"]
TRACER_KERNEL_NAMES = ["tran_diff_fluxes", "tran_diff_tracer", "tracer_next_step"]


def _f(s):
    return float(str(s).replace("d", "e").replace("D", "e"))


def load_e2e(name):
    """-> dict(basin=..., sw=..., bxy=(bx, by), steps=N, mask=int32 (nx,ny) or None, z=npz)."""
    z = np.load(os.path.join(HERE, f"e2e_{name}.npz"))
    b = ast.literal_eval(str(z["meta/basin"]))
    sw = ast.literal_eval(str(z["meta/sw"]))
    basin = dict(nx=int(b["nx"]), ny=int(b["ny"]), dxst=_f(b["dxst"]), dyst=_f(b["dyst"]),
                 rlon=_f(b["rlon"]), rlat=_f(b["rlat"]), curve_grid=int(b["curve"]))
    mask = None
    if "in/mask_packed" in z.files:
        n = basin["nx"] * basin["ny"]
        mask = np.unpackbits(z["in/mask_packed"])[:n].astype(np.int32).reshape(
            (basin["nx"], basin["ny"]), order="F")
    swc = dict(full_free_surface=int(sw["ffs"]), trans_terms=int(sw["trans"]), ksw_lat=int(sw["ksw"]),
               time_smooth=_f(sw["ts"]))
    if int(sw.get("tr", 0)) > 0:
        swc.update(use_tracers=int(sw["tr"]), tracer_num=int(sw["trn"]))
    topo = z["in/topo"] if "in/topo" in z.files else None
    return dict(basin=basin, sw=swc, bxy=tuple(int(v) for v in z["meta/bxy"]), steps=int(z["meta/steps"]),
                mask=mask, topography=topo, z=z)


def e2e_blocks(z):
    """-> {(bm, bn): info int32[8]} for the blocks in an e2e fixture."""
    out = {}
    for k in z.files:
        if k.endswith("/info"):
            bm, bn = k[1:].split("/")[0].split("_")
            out[(int(bm), int(bn))] = z[k]
    return out


def load_kernels(geom):
    return np.load(os.path.join(HERE, f"kernels_{geom}.npz"))
