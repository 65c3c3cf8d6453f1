"""Tracer PSy wrappers -- mirror of interface/tracer/tracer_interface.f90.

``TracerInterface(model).envoke_<stage>_kernel(k, param)`` passes block k's bounds and the
device pointers the reference passes (tracer ``param.data_id``) to the kernel-layer C-ABI
entry; ``envoke_<stage>_sync`` exchanges the halos the reference syncs after that stage.
"""
from __future__ import annotations

import ctypes as C

from ._lib import check, lib

# stage -> (C entry, argument list in reference order); "{k}" = data_id, "%x" = scalar x
KERNEL_ARGS = {
    "tran_diff_fluxes": ("ocn_tran_diff_fluxes",                          # tracer_interface.f90:28-47
                         ["lcu", "lcv", "dxt", "dyt", "dxh", "dyh", "hhu", "hhv", "ff1_{k}", "ff1p_{k}", "ubrtr",
                          "vbrtr", "mu", "%factor_mu", "flux_x", "flux_y"]),
    "tran_diff_tracer": ("ocn_tran_diff_tracer",                          # :61-76
                         ["lu", "dx", "dy", "%tau", "hhq_n", "hhq_p", "flux_x", "flux_y", "ff1p_{k}", "ff1n_{k}"]),
    "tracer_next_step": ("ocn_tracer_next_step",                          # :88-98
                         ["%time_smooth", "lu", "ff1n_{k}", "ff1p_{k}", "ff1_{k}"]),
}

SYNC_LISTS = {
    "tran_diff_fluxes": ["flux_x", "flux_y"],          # :49-55
    "tran_diff_tracer": ["ff1n_{k}"],                  # :78-83
    "tracer_next_step": [],                            # :100-104
}


class TracerInterface:
    def __init__(self, model):
        self.model = model
        L = lib()
        self._fn = {st: getattr(L, sym) for st, (sym, _) in KERNEL_ARGS.items()}
        self._cblocks = [b.c_block() for b in model.blocks]
        self._ptrs = [{nm: C.c_void_p(model.field_ptr(b.k, nm)) for nm in model.field_names} for b in model.blocks]
        for st in KERNEL_ARGS:
            setattr(self, f"envoke_{st}_kernel", self._make_kernel(st))
            setattr(self, f"envoke_{st}_sync", self._make_sync(st))

    def _make_kernel(self, stage):
        sym, names = KERNEL_ARGS[stage]
        fn = self._fn[stage]

        def kernel(k, param):
            p = self._ptrs[k]
            args = []
            for n in names:
                if n == "%factor_mu":
                    args.append(C.c_double(1.0))          # tracer_interface.f90:47 passes 1.0d0
                elif n == "%tau":
                    args.append(C.c_double(param.tau))
                elif n == "%time_smooth":
                    args.append(C.c_double(param.time_smooth))
                else:
                    args.append(p[n.format(k=param.data_id)])
            check(fn(C.byref(self._cblocks[k]), *args, C.c_void_p(self.model.stream)), sym)
        kernel.__name__ = f"envoke_{stage}_kernel"
        return kernel

    def _make_sync(self, stage):
        fields = SYNC_LISTS[stage]

        def sync(k, sync_parameters):
            for f in fields:
                self.model.sync(f.format(k=sync_parameters.data_id))
        sync.__name__ = f"envoke_{stage}_sync"
        return sync
