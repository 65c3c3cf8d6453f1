"""Run configuration: the reference's positional ``.par`` files.

``readpar`` semantics (legacy/service/read_write_parameters.f90:7-42): one value per line,
the value is the first lexeme of the line; anything after it is a comment.  Fortran ``d``
exponents (``1.0d+03``) are accepted.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np


def _lexemes(path: str) -> list[str]:
    out = []
    with open(path, "r") as f:
        for ln in f:
            s = ln.strip()
            out.append(s.split()[0] if s else "")
    return out


def _real(s: str) -> float:
    return float(s.replace("d", "e").replace("D", "e"))


@dataclass
class BasinConfig:
    """configs/basinpar.f90:53-91 (basin.par lines 1-20)."""
    nx: int
    ny: int
    dxst: float = 0.00312
    dyst: float = 0.00225
    rlon: float = 34.751560
    rlat: float = 44.801125
    curve_grid: int = 1
    rotation_on_lon: float = 0.0
    rotation_on_lat: float = 0.0
    mask_file_name: str = "none"
    mask: np.ndarray | None = field(default=None, repr=False)   # int32 (nx, ny) Fortran order
    topography_file_name: str = "none"
    # bottom topography: float32 (nx-4, ny-4) interior points, Fortran order (None: 100 m everywhere)
    topography: np.ndarray | None = field(default=None, repr=False)

    @classmethod
    def from_par(cls, path: str) -> "BasinConfig":
        c = _lexemes(path)
        cfg = cls(nx=int(c[0]), ny=int(c[1]), dxst=_real(c[5]), dyst=_real(c[6]), rlon=_real(c[7]),
                  rlat=_real(c[8]), curve_grid=int(c[11]), rotation_on_lon=_real(c[12]),
                  rotation_on_lat=_real(c[13]), mask_file_name=c[18],
                  topography_file_name=c[19] if len(c) > 19 and c[19] else "none")
        if int(c[9]) != 0 or int(c[10]) != 0:
            raise NotImplementedError("non-uniform (levels) grids: only xgr_type = ygr_type = 0 are supported")
        if cfg.curve_grid not in (0, 1):
            raise NotImplementedError("curve_grid = 2 (distorted sphere) is not supported")
        if cfg.mask_file_name != "none":
            cfg.mask = read_mask(cfg.mask_file_name, cfg.nx, cfg.ny)
        if cfg.topography_file_name != "none":
            cfg.topography = read_topography(cfg.topography_file_name, cfg.nx, cfg.ny)
        return cfg


@dataclass
class SWConfig:
    """configs/sw.f90:34-41 (sw.par lines 1-7); defaults = the shipped sw.par."""
    full_free_surface: int = 1
    trans_terms: int = 1
    ksw_lat: int = 1
    time_smooth: float = 0.5
    lvisc_2: float = 1.0e3
    use_tracers: int = 0
    tracer_num: int = 1

    @classmethod
    def from_par(cls, path: str) -> "SWConfig":
        c = _lexemes(path)
        if len(c) > 7 and c[7].strip().lower() != "none":
            raise NotImplementedError("ssh_init_file_name other than 'none' is not supported")
        return cls(full_free_surface=int(c[0]), trans_terms=int(c[1]), ksw_lat=int(c[2]),
                   time_smooth=_real(c[3]), lvisc_2=_real(c[4]), use_tracers=int(c[5]), tracer_num=int(c[6]))


@dataclass
class ParallelConfig:
    """configs/parallel.f90:34-42 with _DD_MANUAL_BLOCK_GRID_: bppnx x bppny = total block grid."""
    bppnx: int = 1
    bppny: int = 1
    mod_decomposition: int = 0

    @classmethod
    def from_par(cls, path: str) -> "ParallelConfig":
        c = _lexemes(path)
        cfg = cls(mod_decomposition=int(c[0]), bppnx=int(c[2]), bppny=int(c[3]))
        if cfg.mod_decomposition != 0:
            raise NotImplementedError("only uniform decomposition (mod_decomposition = 0) is supported")
        return cfg


def read_mask(path: str, nx: int, ny: int) -> np.ndarray:
    """tools/io.f90:61-70: a comment line, then ny rows of nx digits, top row (n = ny) first."""
    with open(path, "r") as f:
        lines = [ln.rstrip("\r\n") for ln in f]
    m = np.zeros((nx, ny), dtype=np.int32, order="F")
    for r, ln in enumerate(lines[1:1 + ny]):
        m[:, ny - 1 - r] = [int(ch) for ch in ln[:nx]]
    return m


def read_topography(path: str, nx: int, ny: int) -> np.ndarray:
    """tools/io.f90:84-176 read_data2D_real4 (record 1): a raw real(4) file of the (nx-4) x (ny-4)
    interior points (nxb = mmm = 3 .. nxe = mm = nx-2), Fortran order, native byte order."""
    a = np.fromfile(path, dtype=np.float32, count=(nx - 4) * (ny - 4))
    if a.size != (nx - 4) * (ny - 4):
        raise ValueError(f"{path}: {a.size} values, (nx-4)*(ny-4) = {(nx - 4) * (ny - 4)} expected")
    return a.reshape((nx - 4, ny - 4), order="F")


def box_config(n: int, **kw) -> BasinConfig:
    """Synthetic N x N interior box of SURVEY.md 8(d): nx = ny = N + 4, closed 2-cell land frame,
    flat 100 m bottom, spherical grid with the shipped basin.par steps and origin."""
    return BasinConfig(nx=n + 4, ny=n + 4, **kw)
