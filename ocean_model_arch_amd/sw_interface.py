"""Per-kernel PSy wrappers -- mirror of interface/shallow_water/sw_interface.f90.

``ShallowWaterInterface(model).envoke_<stage>_kernel(k, param)`` unpacks block k's bounds and
the device pointers of the fields the reference passes (same fields, same order) and calls the
kernel-layer C-ABI entry (include/ocn_sw.h) on the model's stream.  ``envoke_<stage>_sync``
calls the halo exchange on the fields the reference syncs after that stage.
"""
from __future__ import annotations

import ctypes as C

from ._lib import check, lib

# stage -> (C entry, scalar params, field arguments in reference order)
KERNEL_ARGS = {
    "sw_update_ssh": ("ocn_sw_update_ssh", ("tau",),                      # sw_interface.f90:310-328
                      ["lu", "dx", "dy", "dxh", "dyh", "hhu", "hhv", "sshn", "sshp", "ubrtr", "vbrtr"]),
    "hh_update": ("ocn_hh_update", (),                                    # :145-169
                  ["lu", "llu", "llv", "luh", "dx", "dy", "dxt", "dyt", "dxh", "dyh", "dxb", "dyb",
                   "hhq_n", "hhu_n", "hhv_n", "hhh_n", "ssh", "hhq_rest"]),
    "uv_trans_vort": ("ocn_uv_trans_vort", (),                            # :211-228
                      ["luu", "dxt", "dyt", "dxb", "dyb", "ubrtr", "vbrtr", "vort"]),
    "uv_trans": ("ocn_uv_trans", (),                                      # :238-261
                 ["lcu", "lcv", "luu", "dxh", "dyh", "ubrtr", "vbrtr", "vort", "hhq", "hhu", "hhv", "hhh",
                  "RHSx_adv", "RHSy_adv"]),
    "stress_components": ("ocn_stress_components", (),                    # :110-133
                          ["lu", "luu", "dx", "dy", "dxt", "dyt", "dxh", "dyh", "dxb", "dyb", "ubrtrp", "vbrtrp",
                           "str_t", "str_s"]),
    "uv_diff2": ("ocn_uv_diff2", (),                                      # :273-300
                 ["lcu", "lcv", "dx", "dy", "dxt", "dyt", "dxh", "dyh", "dxb", "dyb", "mu", "str_t", "str_s",
                  "hhq", "hhu", "hhv", "hhh", "RHSx_dif", "RHSy_dif"]),
    "sw_update_uv": ("ocn_sw_update_uv", ("tau",),                        # :337-374
                     ["lcu", "lcv", "dxt", "dyt", "dxh", "dyh", "dxb", "dyb", "hhu", "hhu_n", "hhu_p", "hhv",
                      "hhv_n", "hhv_p", "hhh", "ssh", "ubrtr", "ubrtrn", "ubrtrp", "vbrtr", "vbrtrn", "vbrtrp",
                      "r_diss", "rlh_s", "RHSx", "RHSy", "RHSx_adv", "RHSy_adv", "RHSx_dif", "RHSy_dif"]),
    "sw_next_step": ("ocn_sw_next_step", ("time_smooth",),                # :384-401
                     ["lu", "lcu", "lcv", "ssh", "sshn", "sshp", "ubrtr", "ubrtrn", "ubrtrp", "vbrtr", "vbrtrn",
                      "vbrtrp"]),
    "hh_shift": ("ocn_hh_shift", ("time_smooth",),                        # :181-201
                 ["lu", "llu", "llv", "luh", "hhq", "hhq_p", "hhq_n", "hhu", "hhu_p", "hhu_n", "hhv", "hhv_p",
                  "hhv_n", "hhh", "hhh_p", "hhh_n"]),
    "hh_init": ("ocn_hh_init", ("full_free_surface",),                    # :42-75
                ["lu", "llu", "llv", "luh", "dx", "dy", "dxt", "dyt", "dxh", "dyh", "dxb", "dyb", "hhq", "hhq_p",
                 "hhq_n", "hhu", "hhu_p", "hhu_n", "hhv", "hhv_p", "hhv_n", "hhh", "hhh_p", "hhh_n", "ssh",
                 "sshp", "hhq_rest"]),
}

# fields exchanged after each stage (sw_interface.f90 envoke_*_sync)
SYNC_LISTS = {
    "sw_update_ssh": ["sshn"],                       # :77-83
    "hh_update": ["hhu_n", "hhv_n", "hhh_n"],        # :171-178
    "uv_trans_vort": ["vort"],                       # :231-235
    "uv_trans": ["hhu_p", "hhv_p", "hhh_p"],         # :264-270 (lazy update)
    "stress_components": ["str_t", "str_s"],         # :136-142
    "uv_diff2": [],
    "sw_update_uv": ["vbrtrn", "ubrtrn"],            # :376-381
    "sw_next_step": [],
    "hh_shift": [],
    "hh_init": ["hhu", "hhv", "hhh"],                # :82-90
}


class ShallowWaterInterface:
    def __init__(self, model):
        self.model = model
        L = lib()
        self._fn = {st: getattr(L, sym) for st, (sym, _, _) in KERNEL_ARGS.items()}
        self._cblocks = [b.c_block() for b in model.blocks]
        # device pointers resolved once per block (storage never moves)
        self._ptrs = [{nm: C.c_void_p(model.field_ptr(b.k, nm)) for nm in model.field_names} for b in model.blocks]
        for st in KERNEL_ARGS:
            setattr(self, f"envoke_{st}_kernel", self._make_kernel(st))
            setattr(self, f"envoke_{st}_sync", self._make_sync(st))

    def _make_kernel(self, stage):
        sym, scalars, names = KERNEL_ARGS[stage]
        fn = self._fn[stage]
        sw = self.model.sw

        def kernel(k, param):
            sc = []
            for s in scalars:
                if s == "tau":
                    sc.append(C.c_double(param.tau))
                elif s == "time_smooth":
                    sc.append(C.c_double(param.time_smooth))
                else:
                    sc.append(C.c_int32(sw.full_free_surface))
            p = self._ptrs[k]
            check(fn(C.byref(self._cblocks[k]), *sc, *[p[n] for n in names], C.c_void_p(self.model.stream)), sym)
        kernel.__name__ = f"envoke_{stage}_kernel"
        return kernel

    def _make_sync(self, stage):
        fields = SYNC_LISTS[stage]

        def sync(k, sync_parameters):
            for f in fields:
                self.model.sync(f)
        sync.__name__ = f"envoke_{stage}_sync"
        return sync

