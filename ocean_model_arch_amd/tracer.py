"""Tracer algorithm layer -- mirror of control/tracer.f90:33-62 (expl_tracer)."""
from __future__ import annotations

from .kernel_interface import KernelParameters, envoke
from .tracer_interface import TracerInterface


def expl_tracer(model, tau: float, iface: TracerInterface | None = None):
    sw = model.sw
    if sw.use_tracers <= 0:
        return
    iface = iface or TracerInterface(model)
    p = KernelParameters()
    for k in range(1, sw.tracer_num + 1):
        p.clear()
        p.tau = tau
        p.time_smooth = sw.time_smooth
        p.data_id = k
        for stage in ("tran_diff_fluxes", "tran_diff_tracer", "tracer_next_step"):
            envoke(model, getattr(iface, f"envoke_{stage}_kernel"), getattr(iface, f"envoke_{stage}_sync"), p)
