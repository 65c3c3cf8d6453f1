"""Host-side view of the decomposition and the halo schedule (no GPU needed).

``decompose(basin, par, rank, nranks)`` returns the blocks a process owns, exactly as the
device context makes them (core/decomposition.f90: uniform blocks, land blocks dropped,
create_uniform_decomposition's block -> process map, _MPP_SORTED_BLOCKS_ numbering).
``halo_schedule(...)`` returns the copies / messages one halo exchange performs
(shared/mpp/syncborder_block2D_gen_all.fi semantics), as used by libocn_sw over RCCL.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from ._lib import FIELD_ID, check, lib
from .config import BasinConfig, ParallelConfig
from .model import BlockInfo


def _c_args(basin: BasinConfig, par: ParallelConfig, rank: int, nranks: int):
    cb = _lib.OcnBasin(basin.nx, basin.ny, basin.dxst, basin.dyst, basin.rlon, basin.rlat, basin.curve_grid,
                       basin.rotation_on_lon, basin.rotation_on_lat)
    cd = _lib.OcnDecomp(par.bppnx, par.bppny, nranks, rank, 0)
    mask = None if basin.mask is None else np.asfortranarray(basin.mask.astype(np.int32))
    return cb, cd, mask


def decompose(basin: BasinConfig, par: ParallelConfig, rank: int = 0, nranks: int = 1) -> list[BlockInfo]:
    cb, cd, mask = _c_args(basin, par, rank, nranks)
    mp = None if mask is None else mask.ctypes.data_as(C.c_void_p)
    n = C.c_int32()
    check(lib().ocn_decompose(C.byref(cb), C.byref(cd), mp, None, 0, C.byref(n)), "ocn_decompose")
    out = (_lib.OcnBlockInfo * max(1, n.value))()
    check(lib().ocn_decompose(C.byref(cb), C.byref(cd), mp, out, n.value, C.byref(n)), "ocn_decompose")
    res = []
    for k in range(n.value):
        g = out[k].geom
        res.append(BlockInfo(k, out[k].bm, out[k].bn, g.nx_start, g.nx_end, g.ny_start, g.ny_end, g.bnd_x1, g.bnd_x2,
                             g.bnd_y1, g.bnd_y2, g.pitch, tuple(out[k].nbr_rank), tuple(out[k].nbr_k)))
    return res


def halo_schedule(basin: BasinConfig, par: ParallelConfig, fields: list[str], rank: int = 0,
                  nranks: int = 1) -> list[dict]:
    cb, cd, mask = _c_args(basin, par, rank, nranks)
    mp = None if mask is None else mask.ctypes.data_as(C.c_void_p)
    ids = (C.c_int32 * len(fields))(*[FIELD_ID[f] for f in fields])
    n = C.c_int32()
    check(lib().ocn_halo_schedule(C.byref(cb), C.byref(cd), mp, ids, len(fields), None, 0, C.byref(n)),
          "ocn_halo_schedule")
    out = (_lib.OcnHaloMsg * max(1, n.value))()
    check(lib().ocn_halo_schedule(C.byref(cb), C.byref(cd), mp, ids, len(fields), out, n.value, C.byref(n)),
          "ocn_halo_schedule")
    inv = {v: k for k, v in FIELD_ID.items()}
    return [dict(kind=m.kind, peer=m.peer, k=m.k, k_src=m.k_src, field=inv[m.field],
                 dst=(m.dst_x0, m.dst_x1, m.dst_y0, m.dst_y1), src=(m.src_x0, m.src_x1, m.src_y0, m.src_y1),
                 count=m.count, offset=m.offset) for m in out[:n.value]]
