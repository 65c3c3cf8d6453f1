"""Local output in the reference's own format: float32 GrADS records + .ctl descriptors.

Mirrors the output layer around the hot path:

* ``local_output``   -- control/output.f90:32-174 (hhq once, ssh every record, ff1(tracer_num)
  with tracers);
* ``write_data``     -- tools/io.f90:276-386 write_data2D_real4: record ``nrec`` of a
  direct-access file holding the global interior ``(nx-4) x (ny-4)`` real(4), Fortran order, first
  filled with ``undef`` by the master, then every block writes its interior (land -> undef);
* ``ctl_file_write`` -- legacy/service/rw_ctl_file.f90:9-145, byte for byte (Fortran edit
  descriptors restated below);
* ``LocalOutputTime`` -- the local-output period and record header of tools/time_manager.f90:212-241.

The real(8) -> real(4) conversion and the land mask are applied on the device
(``ocn_ctx_output_r4``); only the packed interior crosses PCIe.  Multi-rank runs pass a
``barrier`` callable (e.g. ``torch.distributed.barrier``) for the master's fill, as the reference
does with its collective ``mpi_file_open``.
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass

import numpy as np

UNDEF = np.float32(-1.0e32)        # shared/system.f90:10
MONTHS = ["JAN", "FEB", "MAR", "APR", "MAY", "JUN", "JUL", "AUG", "SEP", "OCT", "NOV", "DEC"]


# ---------------------------------------------------------------- Fortran edit descriptors
def fortran_e(x: float, w: int, d: int) -> str:
    """Ew.d: 0.ddddE+ee, right-justified in w."""
    if x == 0.0:
        return ("0." + "0" * d + "E+00").rjust(w)
    m = f"{abs(x):.{d - 1}e}"
    digits, ex = m.split("e")
    s = ("-" if x < 0 else "") + "0." + digits.replace(".", "") + "E" + f"{int(ex) + 1:+03d}"
    return s.rjust(w)


def fortran_g(x: float, w: int = 15, d: int = 8) -> str:
    """Gw.d: F(w-4).(d-k) plus 4 blanks when 0.1 <= |x| < 10**d (k = decimal exponent), else Ew.d."""
    if x == 0.0:
        return f"{0.0:.{d - 1}f}".rjust(w - 4) + " " * 4
    k = int(f"{abs(x):.{d - 1}e}".split("e")[1]) + 1     # after rounding to d significant digits
    if 0 <= k <= d:
        return f"{x:.{d - k}f}".rjust(w - 4) + " " * 4
    return fortran_e(x, w, d)


def sec_to_yr_mo_hr_mn(sec: float):
    """rw_ctl_file.f90:169-191 in default-real (float32) arithmetic."""
    f = np.float32
    yr_sec, mo_sec = f(360.0 * 86400.0), f(30.0 * 86400.0)
    s = f(sec) + f(0.10)
    nyr = int(s / yr_sec); s = f(s - f(nyr) * yr_sec)
    nmo = int(s / mo_sec); s = f(s - f(nmo) * mo_sec)
    ndy = int(s / f(86400.0)); s = f(s - f(ndy) * f(86400.0))
    nhr = int(s / f(3600.0)); s = f(s - f(nhr) * f(3600.0))
    nmn = int(s / f(60.0))
    return nyr, nmo, ndy, nhr, nmn


def _def_line(axis: str, n: int, gtype: int, x0, h) -> str:
    if gtype == 0:   # '(a,i6,a,2(g15.8,5x))' -- the trailing 5x writes nothing
        return f"{axis}DEF  {n:6d}  LINEAR   " + fortran_g(x0[0]) + " " * 5 + fortran_g(h)
    # '(a,i6,a,7(g15.8,1x)/(22x,7(g15.8,1x)))'
    vals = [fortran_g(v) for v in x0[:n]]
    rows = [" ".join(vals[i:i + 7]) for i in range(0, len(vals), 7)]
    return f"{axis}DEF  {n:6d}  LEVELS  " + rows[0] + "".join("\n" + " " * 22 + r for r in rows[1:])


def ctl_file_write(fname: str, undef, nx, ny, nz, nt, xtype, x0, hx, ytype, y0, hy, ztype, z0, hz,
                   yr_type, year0, month0, day0, hour0, minute0, ht, title, varname):
    """rw_ctl_file.f90:9-145: the GrADS descriptor next to data file `fname` (.dat -> .ctl)."""
    base = os.path.splitext(fname)[0]
    namectl, namedat2 = base + ".ctl", os.path.basename(base + ".dat")
    lines = ["DSET    ^" + namedat2.ljust(128), "TITLE    " + title,
             "UNDEF   " + fortran_e(float(undef), 12, 5) + "  ! gap value",
             _def_line("X", nx, xtype, x0, hx), _def_line("Y", ny, ytype, y0, hy), _def_line("Z", nz, ztype, z0, hz)]
    nyr, nmo, ndy, nhr, nmn = sec_to_yr_mo_hr_mn(ht)
    tf, k = next(((t, v) for t, v in (("yr", nyr), ("mo", nmo), ("dy", ndy), ("hr", nhr), ("mn", nmn)) if v != 0),
                 ("  ", 0))
    lines.append(f"TDEF  {nt:6d}  LINEAR  {hour0:02d}:{minute0:02d}Z{day0:02d}{MONTHS[month0 - 1]}{year0:04d}"
                 + " " * 5 + f"{k:4d}{tf}")
    if yr_type == 0:
        lines.append("OPTIONS  365_DAY_CALENDAR")
    lines += ["VARS 1  ! Number of variables", f"{varname}        {nz:5d}  1 VARIABLES ", "ENDVARS", ""]
    with open(namectl, "w") as fh:
        fh.write("\n".join(lines) + "\n")


# ---------------------------------------------------------------- data records
def _rank_barrier(model, barrier):
    """The ordering io.f90 gets from its collective mpi_file_open / write_all: with several
    processes, rank 0's undef fill must precede every rank's block writes.  Defaults to
    torch.distributed.barrier when a process group is up; refuses to run unordered."""
    if barrier is not None or model.nranks <= 1:
        return barrier
    try:
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized():
            return dist.barrier
    except ImportError:
        pass
    raise ValueError("write_data with nranks > 1 needs a barrier (no torch.distributed process group is initialised)")


def write_data(model, path: str, fname: str, nrec: int, name: str, barrier=None):
    """io.f90:276-386 write_data2D_real4 of field `name` (real(8) fields are converted like
    bufwp4%copy_from_real8) into record nrec (1-based) of path/fname."""
    barrier = _rank_barrier(model, barrier)
    nx, ny = model.basin.nx, model.basin.ny
    nxb, nxe, nyb, nye = 3, nx - 2, 3, ny - 2           # mmm, mm, nnn, nn (basinpar)
    gw = nxe - nxb + 1
    recl = gw * (nye - nyb + 1) * 4
    fn = os.path.join(path, fname)
    if model.rank == 0:                                  # io.f90:306-311: the record, all undef
        os.makedirs(path, exist_ok=True)
        with open(fn, "r+b" if os.path.exists(fn) else "w+b") as fh:
            fh.seek((nrec - 1) * recl)
            fh.write(np.full(recl // 4, UNDEF, dtype="<f4").tobytes())
    if barrier is not None:
        barrier()
    with open(fn, "r+b") as fh:                          # io.f90:318-356: every block's interior
        for b in model.blocks:
            a = model.output_r4(b.k, name, float(UNDEF))
            for j in range(a.shape[1]):
                fh.seek((nrec - 1) * recl + ((b.ny_start + j - nyb) * gw + (b.nx_start - nxb)) * 4)
                fh.write(np.ascontiguousarray(a[:, j], dtype="<f4").tobytes())
    if barrier is not None:
        barrier()


@dataclass
class LocalOutputTime:
    """time_manager.f90:212-241: local output period (steps) and the record header."""
    period_steps: int
    year: int
    month: int
    day: int
    hour: int
    minute: int
    tstep: float          # loc_data_tstep, seconds (real(4))
    calendar: int = 1     # yr_type

    @classmethod
    def from_period(cls, wr_period_min: float, time_step_s: float = 1.0, init_year: int = 2012, calendar: int = 1):
        f = np.float32
        step_m = f(time_step_s) / f(60.0)
        p = max(min(f(wr_period_min), f(1440.0)), step_m)
        return cls(period_steps=int(math.floor(p / step_m + f(0.5))), year=init_year, month=1,
                   day=int(p / f(1440.0)) + 1, hour=int(p / f(60.0)) % 24, minute=int(p) % 60,
                   tstep=float(p * f(60.0)), calendar=calendar)


def local_output(model, nrec: int, t: LocalOutputTime, path: str = "RESULTS/", barrier=None):
    """output.f90:32-174 for record nrec: hhq (nrec = 1 only), ssh, ff1(tracer_num) with tracers."""
    b = model.basin
    x0, y0 = [b.rlon], [b.rlat]

    def ctl(fname, nt, ztype, title, var):
        if model.rank == 0:
            ctl_file_write(os.path.join(path, fname), UNDEF, b.nx - 4, b.ny - 4, 1, nt, 0, x0, b.dxst, 0, y0,
                           b.dyst, ztype, [0.0], 1.0, t.calendar, t.year, t.month, t.day, t.hour, t.minute,
                           t.tstep, title, var)

    if nrec == 1:
        write_data(model, path, "hhq.dat", nrec, "hhq_rest", barrier)
        ctl("hhq.dat", nrec, 1, "HHQ, m", "hhq")
    write_data(model, path, "ssh.dat", nrec, "ssh", barrier)
    ctl("ssh.dat", nrec, 0, "SSH, m", "ssh")
    if model.sw.use_tracers > 0:
        write_data(model, path, "ff1.dat", nrec, f"ff1_{model.sw.tracer_num}", barrier)
        ctl("ff1.dat", nrec, 0, "ff1 (last)", "ff1")


def run(model, nsteps: int, tau: float, t: LocalOutputTime, path: str = "RESULTS/", barrier=None):
    """model.f90:114-193: output the initial state, then step, writing record
    step / period + 1 every `period_steps` steps."""
    local_output(model, 1, t, path, barrier)
    done = 0
    while done < nsteps:
        n = min(t.period_steps - done % t.period_steps, nsteps - done)
        model.step(n, tau=tau).synchronize()
        done += n
        if done % t.period_steps == 0:
            local_output(model, done // t.period_steps + 1, t, path, barrier)
    return model
