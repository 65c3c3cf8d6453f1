"""Local output in the reference's GrADS format (ocean_model_arch_amd/output.py).

Pinned to the reference's own output: tests/golden/grads_bs_tr_s180.npz holds the RESULTS/
files the unmodified reference model wrote (tests/golden/gen_grads.py): Black Sea basin, one
tracer, records at steps 0, 60, 120, 180.

* CPU: the .ctl descriptors byte for byte, the Fortran edit descriptors, the output period.
* GPU: the .dat records (device-side real(8) -> real(4) + land undef, block subarrays written
  into the shared records) bit for bit, on 1 and 4x2 blocks.
"""
import os

import numpy as np
import pytest

from tests.golden import cases

HERE = os.path.dirname(os.path.abspath(__file__))
FIX = os.path.join(HERE, "golden", "grads_bs_tr_s180.npz")
BS = dict(nx=289, ny=163, dxst=0.05, dyst=0.04, rlon=27.525, rlat=40.940)


def test_fortran_edit_descriptors():
    from ocean_model_arch_amd.output import fortran_e, fortran_g
    assert fortran_e(-1.0e32, 12, 5) == "-0.10000E+33"
    assert fortran_g(27.525) == "  27.525000    "
    assert fortran_g(0.05) == " 0.50000000E-01"
    assert fortran_g(0.0) == "  0.0000000    "
    assert fortran_g(1.0) == "  1.0000000    "
    assert fortran_g(0.5) == " 0.50000000    "
    assert fortran_g(123456789.0) == " 0.12345679E+09"


def test_local_output_time():
    from ocean_model_arch_amd.output import LocalOutputTime
    t = LocalOutputTime.from_period(1.0, 1.0, 2012)           # ocean_run.par as shipped, tau = 1 s
    assert (t.period_steps, t.year, t.month, t.day, t.hour, t.minute, t.tstep) == (60, 2012, 1, 1, 0, 1, 60.0)
    t = LocalOutputTime.from_period(90.0, 30.0, 2000)
    assert (t.period_steps, t.day, t.hour, t.minute, t.tstep) == (180, 1, 1, 30, 5400.0)


@pytest.mark.parametrize("var", ["ssh", "ff1", "hhq"])
def test_ctl_matches_reference(tmp_path, var):
    from ocean_model_arch_amd.output import UNDEF, LocalOutputTime, ctl_file_write
    z = np.load(FIX)
    nt = z[f"dat/{var}"].shape[0]
    t = LocalOutputTime.from_period(float(z["meta/period_min"]))
    title = {"ssh": "SSH, m", "ff1": "ff1 (last)", "hhq": "HHQ, m"}[var]
    ctl_file_write(str(tmp_path / f"{var}.dat"), UNDEF, BS["nx"] - 4, BS["ny"] - 4, 1, nt, 0, [BS["rlon"]], BS["dxst"],
                   0, [BS["rlat"]], BS["dyst"], 1 if var == "hhq" else 0, [0.0], 1.0, t.calendar, t.year, t.month,
                   t.day, t.hour, t.minute, t.tstep, title, var)
    assert (tmp_path / f"{var}.ctl").read_text() == str(z[f"ctl/{var}"])


@pytest.mark.gpu
@pytest.mark.parametrize("bxy", [(1, 1), (4, 2)])
def test_grads_records_match_reference(tmp_path, bxy):
    import ocean_model_arch_amd as amd
    from ocean_model_arch_amd.output import LocalOutputTime, run
    case = cases.load_e2e("bs_b4x2_tr_s60")                    # Black Sea basin, mask, sw.par + 1 tracer
    b = case["basin"]
    basin = amd.BasinConfig(nx=b["nx"], ny=b["ny"], dxst=b["dxst"], dyst=b["dyst"], rlon=b["rlon"], rlat=b["rlat"],
                            curve_grid=b["curve_grid"], mask=case["mask"])
    m = amd.OceanModel(basin, amd.SWConfig(**case["sw"]), amd.ParallelConfig(*bxy)).init()
    z = np.load(FIX)
    nrec = z["dat/ssh"].shape[0]
    t = LocalOutputTime.from_period(float(z["meta/period_min"]))
    run(m, (nrec - 1) * t.period_steps, 1.0, t, str(tmp_path))
    m.close()
    bad = []
    for var in ("ssh", "ff1", "hhq"):
        got = np.fromfile(tmp_path / f"{var}.dat", dtype="<f4").reshape(z[f"dat/{var}"].shape)
        ref = z[f"dat/{var}"]
        for r in range(ref.shape[0]):
            if got[r].tobytes() != ref[r].tobytes():
                bad.append(f"{var} record {r + 1}: {int((got[r] != ref[r]).sum())} values differ")
        if (tmp_path / f"{var}.ctl").read_text() != str(z[f"ctl/{var}"]):
            bad.append(f"{var}.ctl")
    assert not bad, bad
