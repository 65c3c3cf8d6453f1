"""CPU oracle for the shallow-water barotropic step -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this module.  It is the parity checker, never the thing measured or shipped.

It restates, on the host, the reference's algorithm layer and its storage:

* decomposition: ``core/decomposition.f90:427-503`` (uniform blocks, interior 3..nx-2,
  arrays start-2..end+2), land-block removal (``:614-669``), 8-neighbour maps (``:976-1062``);
* init: ``control/init_data.f90:29-125`` (masks, metrics, Coriolis, 100 m depth, Gaussian SSH,
  hh_init, zero velocities, mu=0);
* one step: ``control/shallow_water/shallow_water.f90:22-94`` with the per-stage syncs of
  ``interface/shallow_water/sw_interface.f90`` (table in SURVEY.md section 3);
* halo exchange: ``shared/mpp/syncborder_block2D_gen_all.fi`` (block-to-block copies; one
  process holding every block gives bitwise the same result as MPI ranks).

Compute is delegated to ``oracle/liboracle.so`` (``oracle/sw_oracle.c``), a scalar C
restatement of each reference kernel.  Pinned against the compiled reference via the
fixtures in ``tests/golden``.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from dataclasses import dataclass, field

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

R4_FIELDS = ["lu", "luu", "luh", "lcu", "lcv", "llu", "llv",
             "dx", "dy", "dxt", "dyt", "dxh", "dyh", "dxb", "dyb", "rlh_s", "r_diss"]
R8_FIELDS = ["ssh", "sshn", "sshp", "ubrtr", "ubrtrn", "ubrtrp", "vbrtr", "vbrtrn", "vbrtrp",
             "hhq", "hhq_p", "hhq_n", "hhu", "hhu_p", "hhu_n", "hhv", "hhv_p", "hhv_n",
             "hhh", "hhh_p", "hhh_n", "hhq_rest", "vort", "str_t", "str_s", "mu",
             "RHSx", "RHSy", "RHSx_adv", "RHSy_adv", "RHSx_dif", "RHSy_dif"]
AUX_R4 = ["lu1", "rlh_c"]


def lib():
    """Load (building if needed) oracle/liboracle.so."""
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liboracle.so")
        src = os.path.join(_HERE, "sw_oracle.c")
        if not os.path.exists(path) or os.path.getmtime(path) < os.path.getmtime(src):
            subprocess.check_call(["make", "-s", "-f", os.path.join(_HERE, "Makefile")])
        _LIB = C.CDLL(path)
        _LIB.orc_check_ssh_err.restype = C.c_long
    return _LIB


# --------------------------------------------------------------------------- configs
@dataclass
class BasinConfig:
    """configs/basinpar.f90:53-91 (positional basin.par lines 1-20)."""
    nx: int
    ny: int
    dxst: float = 0.00312
    dyst: float = 0.00225
    rlon: float = 34.751560
    rlat: float = 44.801125
    curve_grid: int = 1
    rotation_on_lon: float = 0.0
    rotation_on_lat: float = 0.0
    mask: np.ndarray | None = None   # int32 (nx, ny) Fortran order; None -> box, io.f90:49-59
    # bottom topography: float32 (nx-4, ny-4) interior points (basin.par line 20), None -> 100 m
    topography: np.ndarray | None = None

    def global_mask(self) -> np.ndarray:
        if self.mask is not None:
            return np.asfortranarray(self.mask.astype(np.int32))
        m = np.zeros((self.nx, self.ny), dtype=np.int32, order="F")
        m[:2, :] = 1; m[-2:, :] = 1; m[:, :2] = 1; m[:, -2:] = 1
        return m


@dataclass
class SWConfig:
    """configs/sw.f90:34-41, defaults = shipped sw.par."""
    full_free_surface: int = 1
    trans_terms: int = 1
    ksw_lat: int = 1
    time_smooth: float = 0.5
    lvisc_2: float = 1.0e3
    use_tracers: int = 0
    tracer_num: int = 1


def tracer_fields(sw: SWConfig) -> list[str]:
    """core/ocean.f90:38-41, 90-100: flux_x, flux_y and ff1/ff1p/ff1n per tracer (1-based)."""
    if sw.use_tracers <= 0:
        return []
    return ["flux_x", "flux_y"] + [f"{p}_{k}" for k in range(1, sw.tracer_num + 1) for p in ("ff1", "ff1p", "ff1n")]


def read_mask_file(path: str, nx: int, ny: int) -> np.ndarray:
    """tools/io.f90:61-70: first line comment, then ny rows of nx digits, top row (n=ny) first."""
    with open(path, "r", newline=None) as f:
        lines = [ln.rstrip("\r\n") for ln in f]
    rows = lines[1:1 + ny]
    m = np.zeros((nx, ny), dtype=np.int32, order="F")
    for r, ln in enumerate(rows):
        n = ny - 1 - r
        m[:, n] = [int(ch) for ch in ln[:nx]]
    return m


# --------------------------------------------------------------------------- decomposition
DIRS = {1: (1, 0), 2: (-1, 0), 3: (0, 1), 4: (0, -1), 5: (1, 1), 6: (1, -1), 7: (-1, 1), 8: (-1, -1)}


@dataclass
class Block:
    bm: int
    bn: int
    nxs: int
    nxe: int
    nys: int
    nye: int
    bx1: int
    bx2: int
    by1: int
    by2: int
    nbr: dict = field(default_factory=dict)   # dir -> local index of neighbour block

    @property
    def shape(self):
        return (self.bx2 - self.bx1 + 1, self.by2 - self.by1 + 1)

    @property
    def args(self):
        return (self.nxs, self.nxe, self.nys, self.nye, self.bx1, self.bx2, self.by1, self.by2)


def uniform_sizes(total: int, parts: int) -> list[int]:
    """decomposition.f90:448-482: floor(remaining/remaining_parts), last block takes the rest."""
    sizes, acc = [], 0
    for i in range(1, parts + 1):
        s = total - acc if i == parts else int(np.floor(float(np.float32(total - acc) / np.float32(parts - i + 1))))
        if s <= 0:
            raise ValueError("Error in decomposition to uniform blocks: size <= 0")
        sizes.append(s); acc += s
    return sizes


def decompose(nx: int, ny: int, bnx: int, bny: int, mask: np.ndarray) -> list[Block]:
    """Uniform block grid bnx x bny on one process; all-land blocks are dropped."""
    xs, ys = uniform_sizes(nx - 4, bnx), uniform_sizes(ny - 4, bny)
    x0 = np.concatenate([[0], np.cumsum(xs)[:-1]]); y0 = np.concatenate([[0], np.cumsum(ys)[:-1]])
    blocks, where = [], {}
    for bm in range(1, bnx + 1):
        for bn in range(1, bny + 1):
            nxs = 3 + int(x0[bm - 1]); nxe = nxs + xs[bm - 1] - 1
            nys = 3 + int(y0[bn - 1]); nye = nys + ys[bn - 1] - 1
            sea = (1 - mask[nxs - 1:nxe, nys - 1:nye]).sum()
            if sea == 0:
                continue
            where[(bm, bn)] = len(blocks)
            blocks.append(Block(bm, bn, nxs, nxe, nys, nye, nxs - 2, nxe + 2, nys - 2, nye + 2))
    for b in blocks:
        for d, (dm, dn) in DIRS.items():
            k = where.get((b.bm + dm, b.bn + dn))
            if k is not None:
                b.nbr[d] = k
    return blocks


# --------------------------------------------------------------------------- model
def _p(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


class OracleModel:
    """Per-block field storage (ocean_type/grid_type restated) + the SW algorithm layer."""

    def __init__(self, basin: BasinConfig, sw: SWConfig = SWConfig(), bnx: int = 1, bny: int = 1, threads: int = 1):
        """threads > 1: the kernel calls of a stage run over the blocks on that many host threads
        (the reference's OpenMP mode, core/kernel_interface.f90:84-88 `!$omp do schedule(static,1)`
        over blocks; the C kernels release the GIL); halo copies stay serial."""
        self.basin, self.sw = basin, sw
        self.pool = None
        if threads > 1:
            from concurrent.futures import ThreadPoolExecutor
            self.pool = ThreadPoolExecutor(max_workers=threads)
        self.mask = basin.global_mask()
        self.blocks = decompose(basin.nx, basin.ny, bnx, bny, self.mask)
        self.f: list[dict[str, np.ndarray]] = []
        for b in self.blocks:
            d = {}
            for name in R4_FIELDS + AUX_R4:
                d[name] = np.zeros(b.shape, dtype=np.float32, order="F")
            for name in R8_FIELDS + tracer_fields(sw):
                d[name] = np.zeros(b.shape, dtype=np.float64, order="F")
            self.f.append(d)
        self.L = lib()

    # ---------------------------------------------------------------- halo sync
    def sync(self, name: str):
        """shared/mpp/syncborder_block2D_gen_all.fi: every block's 8 halo regions from its neighbours."""
        for k, b in enumerate(self.blocks):
            for d, kn in b.nbr.items():
                s = self.blocks[kn]
                self.L.orc_halo_copy(d, *b.args, _p(self.f[k][name]), *s.args, _p(self.f[kn][name]))

    # ---------------------------------------------------------------- init
    def init(self):
        self.init_grid()
        self.init_ocean()
        return self

    def init_grid(self):
        """control/init_data.f90:96-125 (gridcon, basinpar, 100 m rest depth)."""
        L, bc = self.L, self.basin
        mask = self.mask
        for k, b in enumerate(self.blocks):
            f = self.f[k]
            L.orc_lu_init(b.bx1, b.bx2, b.by1, b.by2, bc.nx, _p(mask), _p(f["lu"]), _p(f["lu1"]))
        self.sync_r4("lu")
        for k, b in enumerate(self.blocks):
            f = self.f[k]
            L.orc_lu_lv_init(b.bx1, b.bx2, b.by1, b.by2, _p(f["lu"]), _p(f["luh"]), _p(f["luu"]),
                             _p(f["llu"]), _p(f["llv"]), _p(f["lcu"]), _p(f["lcv"]))
        for nm in ("luh", "luu", "lcu", "llu", "lcv", "llv"):
            self.sync_r4(nm)
        for k, b in enumerate(self.blocks):
            f = self.f[k]
            xt = np.zeros(b.shape[0]); xu = np.zeros(b.shape[0])
            yt = np.zeros(b.shape[1]); yv = np.zeros(b.shape[1])
            L.orc_grid_init(*b.args, 3, 3, C.c_double(bc.rlon), C.c_double(bc.rlat),
                            C.c_double(bc.dxst), C.c_double(bc.dyst), bc.curve_grid,
                            C.c_double(bc.rotation_on_lon), C.c_double(bc.rotation_on_lat),
                            _p(xt), _p(yt), _p(xu), _p(yv),
                            *[_p(f[n]) for n in ("dx", "dy", "dxt", "dyt", "dxh", "dyh", "dxb", "dyb")],
                            _p(f["rlh_s"]), _p(f["rlh_c"]))
            if bc.topography is None:
                f["hhq_rest"][...] = 100.0   # init_data.f90:112-114
            else:   # init_data.f90:115-120: read_data2D_real4 (io.f90:130-171) on the block interior,
                t = np.zeros(b.shape, dtype=np.float32, order="F")   # zero where |lu| < 0.5, then real(., wp8)
                t[b.nxs - b.bx1:b.nxe - b.bx1 + 1, b.nys - b.by1:b.nye - b.by1 + 1] = \
                    bc.topography[b.nxs - 3:b.nxe - 2, b.nys - 3:b.nye - 2]
                t[np.abs(f["lu"]) < 0.5] = 0.0
                f["hhq_rest"][...] = t.astype(np.float64)
        if bc.topography is not None:
            self.sync("hhq_rest")

    def sync_r4(self, name: str):
        """sync() on an r4 field (same geometry as the r8 one, done in numpy)."""
        for k, b in enumerate(self.blocks):
            for d, kn in b.nbr.items():
                s = self.blocks[kn]
                dst, src = self.f[k][name], self.f[kn][name]
                hx, hy, sx, sy = _halo_slices(d, b, s)
                dst[hx, hy] = src[sx, sy]

    def init_ocean(self):
        """control/init_data.f90:29-94."""
        L, bc = self.L, self.basin
        for k, b in enumerate(self.blocks):
            f = self.f[k]
            L.orc_gaussian_elimination(*b.args, _p(f["lu"]), _p(f["ssh"]), C.c_double(1.0),
                                       bc.nx // 2, bc.ny // 2)
        self.sync("ssh")
        for f in self.f:
            f["sshn"][...] = f["ssh"]; f["sshp"][...] = f["ssh"]
        self.stage_hh_init()
        for f in self.f:
            for nm in ("ubrtr", "ubrtrn", "ubrtrp", "vbrtr", "vbrtrn", "vbrtrp"):
                f[nm][...] = 0.0
            f["mu"][...] = self.sw.lvisc_2
            f["mu"][...] = 0.0
        if self.sw.use_tracers > 0:                    # init_data.f90:80-90
            for t in range(1, self.sw.tracer_num + 1):
                for k, b in enumerate(self.blocks):
                    L.orc_gaussian_elimination(*b.args, _p(self.f[k]["lu"]), _p(self.f[k][f"ff1_{t}"]),
                                               C.c_double(0.5), bc.nx // 2, bc.ny // 2)
                self.sync(f"ff1_{t}")
                for f in self.f:
                    f[f"ff1n_{t}"][...] = f[f"ff1_{t}"]; f[f"ff1p_{t}"][...] = f[f"ff1_{t}"]
            for f in self.f:
                f["flux_x"][...] = 0.0; f["flux_y"][...] = 0.0

    # ---------------------------------------------------------------- stages (a1..a10)
    def _each(self, fn, *names, scalars=(), tau=None):
        """fn(bounds, scalars..., arrays...) per block; the names "TAU" / "ONE" pass tau / 1.0d0 by value."""
        def one(k):
            b, f = self.blocks[k], self.f[k]
            fn(*b.args, *scalars, *[C.c_double(tau) if n == "TAU" else C.c_double(1.0) if n == "ONE" else _p(f[n])
                                    for n in names])
        if self.pool is None:
            for k in range(len(self.blocks)):
                one(k)
        else:
            list(self.pool.map(one, range(len(self.blocks))))

    def stage_sw_update_ssh(self, tau):
        self._each(self.L.orc_sw_update_ssh, "lu", "dx", "dy", "dxh", "dyh", "hhu", "hhv",
                   "sshn", "sshp", "ubrtr", "vbrtr", scalars=(C.c_double(tau),))
        self.sync("sshn")

    def stage_hh_update(self):
        self._each(self.L.orc_hh_update, "lu", "llu", "llv", "luh", "dx", "dy", "dxt", "dyt", "dxh",
                   "dyh", "dxb", "dyb", "hhq_n", "hhu_n", "hhv_n", "hhh_n", "ssh", "hhq_rest")
        for nm in ("hhu_n", "hhv_n", "hhh_n"):
            self.sync(nm)

    def stage_uv_trans_vort(self):
        self._each(self.L.orc_uv_trans_vort, "luu", "dxt", "dyt", "dxb", "dyb", "ubrtr", "vbrtr", "vort")
        self.sync("vort")

    def stage_uv_trans(self):
        self._each(self.L.orc_uv_trans, "lcu", "lcv", "luu", "dxh", "dyh", "ubrtr", "vbrtr", "vort",
                   "hhq", "hhu", "hhv", "hhh", "RHSx_adv", "RHSy_adv")
        for nm in ("hhu_p", "hhv_p", "hhh_p"):
            self.sync(nm)

    def stage_stress_components(self):
        self._each(self.L.orc_stress_components, "lu", "luu", "dx", "dy", "dxt", "dyt", "dxh", "dyh",
                   "dxb", "dyb", "ubrtrp", "vbrtrp", "str_t", "str_s")
        self.sync("str_t"); self.sync("str_s")

    def stage_uv_diff2(self):
        self._each(self.L.orc_uv_diff2, "lcu", "lcv", "dx", "dy", "dxt", "dyt", "dxh", "dyh", "dxb", "dyb",
                   "mu", "str_t", "str_s", "hhq", "hhu", "hhv", "hhh", "RHSx_dif", "RHSy_dif")

    def stage_sw_update_uv(self, tau):
        self._each(self.L.orc_sw_update_uv, "lcu", "lcv", "dxt", "dyt", "dxh", "dyh", "dxb", "dyb",
                   "hhu", "hhu_n", "hhu_p", "hhv", "hhv_n", "hhv_p", "hhh", "ssh",
                   "ubrtr", "ubrtrn", "ubrtrp", "vbrtr", "vbrtrn", "vbrtrp", "r_diss", "rlh_s",
                   "RHSx", "RHSy", "RHSx_adv", "RHSy_adv", "RHSx_dif", "RHSy_dif",
                   scalars=(C.c_double(tau),))
        self.sync("vbrtrn"); self.sync("ubrtrn")

    def stage_sw_next_step(self):
        self._each(self.L.orc_sw_next_step, "lu", "lcu", "lcv", "ssh", "sshn", "sshp", "ubrtr", "ubrtrn",
                   "ubrtrp", "vbrtr", "vbrtrn", "vbrtrp", scalars=(C.c_double(self.sw.time_smooth),))

    def stage_hh_shift(self):
        self._each(self.L.orc_hh_shift, "lu", "llu", "llv", "luh", "hhq", "hhq_p", "hhq_n", "hhu", "hhu_p",
                   "hhu_n", "hhv", "hhv_p", "hhv_n", "hhh", "hhh_p", "hhh_n",
                   scalars=(C.c_double(self.sw.time_smooth),))

    def stage_hh_init(self):
        self._each(self.L.orc_hh_init, "lu", "llu", "llv", "luh", "dx", "dy", "dxt", "dyt", "dxh", "dyh",
                   "dxb", "dyb", "hhq", "hhq_p", "hhq_n", "hhu", "hhu_p", "hhu_n", "hhv", "hhv_p", "hhv_n",
                   "hhh", "hhh_p", "hhh_n", "ssh", "sshp", "hhq_rest",
                   scalars=(C.c_int(self.sw.full_free_surface),))
        for nm in ("hhu", "hhv", "hhh"):
            self.sync(nm)

    # ---------------------------------------------------------------- tracers (control/tracer.f90)
    def stage_tran_diff_fluxes(self, t: int):
        """interface/tracer/tracer_interface.f90:28-59 (factor_mu = 1.0d0) + sync flux_x, flux_y."""
        self._each(self.L.orc_tran_diff_fluxes, "lcu", "lcv", "dxt", "dyt", "dxh", "dyh", "hhu", "hhv",
                   f"ff1_{t}", f"ff1p_{t}", "ubrtr", "vbrtr", "mu", "ONE", "flux_x", "flux_y")
        self.sync("flux_x"); self.sync("flux_y")

    def stage_tran_diff_tracer(self, t: int, tau: float):
        """tracer_interface.f90:61-86 + sync ff1n."""
        self._each(self.L.orc_tran_diff_tracer, "lu", "dx", "dy", "TAU", "hhq_n", "hhq_p", "flux_x", "flux_y",
                   f"ff1p_{t}", f"ff1n_{t}", tau=tau)
        self.sync(f"ff1n_{t}")

    def stage_tracer_next_step(self, t: int):
        """tracer_interface.f90:88-104 (no sync)."""
        self._each(self.L.orc_tracer_next_step, "lu", f"ff1n_{t}", f"ff1p_{t}", f"ff1_{t}",
                   scalars=(C.c_double(self.sw.time_smooth),))

    def expl_tracer(self, tau: float = 1.0):
        """control/tracer.f90:33-62."""
        if self.sw.use_tracers > 0:
            for t in range(1, self.sw.tracer_num + 1):
                self.stage_tran_diff_fluxes(t)
                self.stage_tran_diff_tracer(t, tau)
                self.stage_tracer_next_step(t)

    def check_ssh_err(self) -> int:
        bad = 0
        for k, b in enumerate(self.blocks):
            bad += self.L.orc_check_ssh_err(*b.args, _p(self.f[k]["lu"]), _p(self.f[k]["ssh"]))
        return bad

    def step(self, tau: float = 1.0):
        """One model time step (model.f90:146-160): expl_shallow_water (shallow_water.f90:22-94), then expl_tracer."""
        sw = self.sw
        self.stage_sw_update_ssh(tau)
        if sw.full_free_surface > 0:
            self.stage_hh_update()
        if sw.trans_terms > 0:
            self.stage_uv_trans_vort()
            self.stage_uv_trans()
        if sw.ksw_lat > 0:
            self.stage_stress_components()
            self.stage_uv_diff2()
        self.stage_sw_update_uv(tau)
        self.stage_sw_next_step()
        if sw.full_free_surface > 0:
            self.stage_hh_shift()
            self.stage_hh_init()
        if self.check_ssh_err():
            raise FloatingPointError("SIGFPRE predict error (check_ssh_err_kernel)")
        self.expl_tracer(tau)                          # model.f90:156

    def run(self, steps: int, tau: float = 1.0):
        for _ in range(steps):
            self.step(tau)
        return self


def _halo_slices(d, b: Block, s: Block):
    """Numpy slices (0-based, into the block arrays) for halo dir d of b, filled from s."""
    def r(lo, hi, base):
        return slice(lo - base, hi - base + 1)
    if d == 1:   hx, hy, sx, sy = (b.nxe + 1, b.nxe + 1), (b.nys, b.nye), (s.nxs, s.nxs), (s.nys, s.nye)
    elif d == 2: hx, hy, sx, sy = (b.nxs - 1, b.nxs - 1), (b.nys, b.nye), (s.nxe, s.nxe), (s.nys, s.nye)
    elif d == 3: hx, hy, sx, sy = (b.nxs, b.nxe), (b.nye + 1, b.nye + 1), (s.nxs, s.nxe), (s.nys, s.nys)
    elif d == 4: hx, hy, sx, sy = (b.nxs, b.nxe), (b.nys - 1, b.nys - 1), (s.nxs, s.nxe), (s.nye, s.nye)
    elif d == 5: hx, hy, sx, sy = (b.nxe + 1,) * 2, (b.nye + 1,) * 2, (s.nxs,) * 2, (s.nys,) * 2
    elif d == 6: hx, hy, sx, sy = (b.nxe + 1,) * 2, (b.nys - 1,) * 2, (s.nxs,) * 2, (s.nye,) * 2
    elif d == 7: hx, hy, sx, sy = (b.nxs - 1,) * 2, (b.nye + 1,) * 2, (s.nxe,) * 2, (s.nys,) * 2
    else:        hx, hy, sx, sy = (b.nxs - 1,) * 2, (b.nys - 1,) * 2, (s.nxe,) * 2, (s.nye,) * 2
    return r(*hx, b.bx1), r(*hy, b.by1), r(*sx, s.bx1), r(*sy, s.by1)
