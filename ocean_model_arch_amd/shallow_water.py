"""Algorithm layer -- mirror of control/shallow_water/shallow_water.f90:22-94.

``expl_shallow_water(model, tau)`` sequences the stages through ``envoke`` exactly as the
reference does (same order, same flag gates).  This is the PSyKAl-shaped host path; the
native ``OceanModel.step`` runs the same sequence inside libocn_sw (optionally as a hipGraph).
"""
from __future__ import annotations

from .kernel_interface import KernelParameters, envoke
from .sw_interface import ShallowWaterInterface


def expl_shallow_water(model, tau: float, iface: ShallowWaterInterface | None = None):
    iface = iface or ShallowWaterInterface(model)
    sw = model.sw
    p = KernelParameters()
    p.clear()
    p.tau = tau
    p.time_smooth = sw.time_smooth

    def run(stage):
        envoke(model, getattr(iface, f"envoke_{stage}_kernel"), getattr(iface, f"envoke_{stage}_sync"), p)

    run("sw_update_ssh")
    if sw.full_free_surface > 0:
        run("hh_update")
    if sw.trans_terms > 0:
        run("uv_trans_vort")
        run("uv_trans")
    if sw.ksw_lat > 0:
        run("stress_components")
        run("uv_diff2")
    run("sw_update_uv")
    run("sw_next_step")
    if sw.full_free_surface > 0:
        run("hh_shift")
        run("hh_init")
    model.stage("check_ssh_err", tau)
