"""The Fortran host (host/fortran, ISO_C_BINDING over libocn_sw) on the golden cases.

The driver reads the reference's positional basin.par / sw.par / parallel.par, runs the
reference-shaped Fortran PSy layer (envoke -> envoke_<stage>_kernel -> extern "C" HIP entry),
and dumps every field in the oracle/ref_driver.f90 format; each field must hash identically
to the unmodified reference run."""
import hashlib
import os
import subprocess

import numpy as np
import pytest

from tests.golden import cases
from tests.golden.refdump import read_dump

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DRIVER = os.path.join(REPO, "host", "fortran", "ocn_sw_driver")

BASIN = """{nx} : nx
{ny} : ny
1 : nz
0 : px
0 : py
{dxst!r} : dxst
{dyst!r} : dyst
{rlon!r} : rlon
{rlat!r} : rlat
0 : xgr
0 : ygr
{curve_grid} : curve grid
0.0 : rot lon
0.0 : rot lat
90.0 :
60.0 :
90.0 :
-90.0 :
{mask} : mask
{topo} : topography
"""


def write_case(d, case):
    b = case["basin"]
    mask = "none"
    if case["mask"] is not None:
        mask = os.path.join(d, "mask.txt")
        m = case["mask"]
        with open(mask, "w") as f:
            f.write("mask written from tests/golden (reference data/BS/mask_bs4km.txt)\n")
            for n in range(b["ny"] - 1, -1, -1):
                f.write("".join(str(int(v)) for v in m[:, n]) + "\n")
    topo = "none"
    if case.get("topography") is not None:   # the basin.par line-20 real(4) file (init_data.f90:115-120)
        topo = os.path.join(d, "topo.dat")
        np.asarray(case["topography"], dtype=np.float32).ravel(order="F").tofile(topo)
    open(os.path.join(d, "basin.par"), "w").write(BASIN.format(mask=mask, topo=topo, **b))
    s = case["sw"]
    open(os.path.join(d, "sw.par"), "w").write(
        f"{s['full_free_surface']} : ffs\n{s['trans_terms']} : trans\n{s['ksw_lat']} : ksw\n"
        f"{s['time_smooth']!r} : ts\n1000.0 : lvisc\n{s.get('use_tracers', 0)} : tracers\n"
        f"{s.get('tracer_num', 1)} : n\nnone : ssh\n")
    bx, by = case["bxy"]
    open(os.path.join(d, "parallel.par"), "w").write(f"0 : m\nnone : f\n{bx} : bx\n{by} : by\n0\n0\nnone\n0\n0\n")


def test_fortran_host_builds():
    if not os.path.exists(DRIVER):
        subprocess.check_call(["make", "-s", "-f", os.path.join(REPO, "host", "fortran", "Makefile")], cwd=REPO)
    assert os.access(DRIVER, os.X_OK)


@pytest.mark.gpu
@pytest.mark.parametrize("name,mode", [("box70x54_b3x2_s20", "stages"), ("bs_b4x2_s60", "stages"),
                                       ("box48x40_flags000_s10", "native"), ("bs_b1x1_s60", "native"),
                                       ("box40x32_tr2_s5", "stages"), ("bs_b4x2_tr_s60", "native"),
                                       ("box70x54_b1x1_s20", "psy"), ("box70x54_b3x2_tr_s20", "psy"),
                                       ("bs_b1x1_s604", "psy"), ("box70x54_topo_b3x2_s20", "psy"),
                                       ("bs_topo_b4x2_s60", "stages")])
def test_fortran_host_matches_reference(tmp_path, name, mode):
    """stages = the reference's envoke stages over the kernel-layer entries; psy = the same PSy
    time loop (one expl_shallow_water per step, model.f90:146) in its fused form, one
    ocn_ctx_step(ctx, tau, 1) per step; native = one ocn_ctx_step call for the whole run."""
    case = cases.load_e2e(name)
    write_case(str(tmp_path), case)
    args = [DRIVER, str(case["steps"]), "dump.bin"] + ([mode] if mode != "psy" else [])
    r = subprocess.run(args, cwd=tmp_path, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    z = case["z"]
    bad = []
    for info, f in read_dump(os.path.join(tmp_path, "dump.bin")):
        for nm, a in f.items():
            key = f"b{info['bm']}_{info['bn']}/sha/{nm}"
            if key in z.files:
                h = hashlib.sha256(np.ascontiguousarray(a.ravel(order="F")).tobytes()).hexdigest()
                if h != str(z[key]):
                    bad.append(f"({info['bm']},{info['bn']}):{nm}")
    assert not bad, f"{name}/{mode}: {bad}"


DRIVER_MPI = os.path.join(REPO, "host", "fortran", "ocn_sw_driver_mpi")
PLAN_FIELDS = ["sshn", "ssh", "ubrtr", "vbrtr"]


def read_plan(path):
    """The driver's `plan` file: this rank's blocks (ocn_decompose) and one exchange's schedule."""
    blocks, msgs, head = [], [], None
    for ln in open(path):
        w = ln.split()
        if w[0] == "rank":
            head = (int(w[1]), int(w[3]), int(w[5]))
        elif w[0] == "block":
            v = [int(x) for x in w[1:]]
            blocks.append((v[0], v[1], v[2], v[3], v[4], v[5], tuple(v[6:14]), tuple(v[14:22])))
        elif w[0] == "msg":
            msgs.append(tuple(int(x) for x in w[1:]))
    return head, blocks, msgs


def expected_plan(case, rank, nranks):
    """The same through the Python host (ocean_model_arch_amd.domain over the same library entries)."""
    from ocean_model_arch_amd import domain
    from ocean_model_arch_amd._lib import FIELD_ID
    import ocean_model_arch_amd as amd
    basin = amd.BasinConfig(**case["basin"], mask=case["mask"])
    par = amd.ParallelConfig(*case["bxy"])
    blocks = [(b.bm, b.bn, b.nx_start, b.nx_end, b.ny_start, b.ny_end, tuple(b.nbr_rank), tuple(b.nbr_k))
              for b in domain.decompose(basin, par, rank, nranks)]
    msgs = [(m["kind"], m["peer"], m["k"], m["k_src"], FIELD_ID[m["field"]], *m["dst"], *m["src"], m["count"],
             m["offset"]) for m in domain.halo_schedule(basin, par, PLAN_FIELDS, rank, nranks)]
    return blocks, msgs


@pytest.mark.parametrize("name,nranks", [("box70x54_b3x2_s20", 3), ("box70x54_b3x2_s20", 6), ("bs_b4x2_s60", 2),
                                         ("bs_b4x2_s60", 4),
                                         ("bs_b4x2_s60", 8)])
@pytest.mark.parametrize("launcher", ["env", "mpi"])
def test_fortran_ranks_derive_the_decomposition(tmp_path, name, nranks, launcher):
    """Multi-rank Fortran host (mpp_init, shared/mpp/mpp.f90:64-221): N driver processes, each told its
    rank by RANK / WORLD_SIZE (torch.distributed.run's variables) or by MPI (mpiexec -n N, MPICH), derive
    the same blocks -- dealt as create_uniform_decomposition deals them, core/decomposition.f90:614-669 --
    and the same halo schedule as the library's ocn_decompose / ocn_halo_schedule give each rank.
    Host only: the `plan` mode stops before any device call."""
    case = cases.load_e2e(name)
    write_case(str(tmp_path), case)
    if launcher == "env":
        if not os.path.exists(DRIVER):
            pytest.skip("driver not built")
        procs = []
        for r in range(nranks):
            env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(nranks), LOCAL_RANK="0")
            procs.append(subprocess.Popen([DRIVER, "plan", "plan"], cwd=tmp_path, env=env,
                                          stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
        for p in procs:
            out, _ = p.communicate(timeout=120)
            assert p.returncode == 0, out
    else:
        mpiexec = "/opt/conda/bin/mpiexec"
        if not (os.path.exists(DRIVER_MPI) and os.path.exists(mpiexec)):
            pytest.skip("MPI driver or mpiexec not present")
        r = subprocess.run([mpiexec, "-n", str(nranks), DRIVER_MPI, "plan", "plan"], cwd=tmp_path,
                           capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stdout + r.stderr
    for r in range(nranks):
        head, blocks, msgs = read_plan(os.path.join(tmp_path, f"plan.r{r}"))
        want_b, want_m = expected_plan(case, r, nranks)
        assert head == (r, nranks, len(want_b)), head
        assert blocks == want_b, (r, blocks, want_b)
        assert msgs == want_m, r
    # every sea block is owned by exactly one rank
    owned = [b[:2] for r in range(nranks) for b in read_plan(os.path.join(tmp_path, f"plan.r{r}"))[1]]
    assert len(owned) == len(set(owned)) == len(cases.e2e_blocks(case["z"]))


@pytest.mark.gpu
@pytest.mark.parametrize("name,mode", [("box70x54_b1x1_s20", "psy"), ("bs_b1x1_s60", "psy"),
                                       ("box70x54_b3x2_s20", "native")])
@pytest.mark.parametrize("launcher", ["env", "mpi"])
def test_fortran_host_rccl_one_rank_matches_reference(tmp_path, name, mode, launcher):
    """The multi-rank Fortran host's communicator path on one GPU: the driver run as rank 0 of 1 --
    from WORLD_SIZE=1 or from `mpiexec -n 1` of the MPI build -- attaches an RCCL communicator
    (OCN_ATTACH_COMM=1: rank 0's unique id, ocn_ctx_attach_comm) and arms the watchdog, so every
    exchange, vote and synchronize goes through the RCCL branch; every field bitwise the reference's."""
    case = cases.load_e2e(name)
    write_case(str(tmp_path), case)
    env = dict(os.environ, OCN_ATTACH_COMM="1", OCN_WATCHDOG="60")
    args = [str(case["steps"]), "dump.bin"] + ([mode] if mode != "psy" else [])
    if launcher == "env":
        cmd = [DRIVER] + args
        env.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    else:
        if not (os.path.exists(DRIVER_MPI) and os.path.exists("/opt/conda/bin/mpiexec")):
            pytest.skip("MPI driver or mpiexec not present")
        cmd = ["/opt/conda/bin/mpiexec", "-n", "1", DRIVER_MPI] + args
    r = subprocess.run(cmd, cwd=tmp_path, capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    z = case["z"]
    bad, seen = [], 0
    for info, f in read_dump(os.path.join(tmp_path, "dump.bin")):
        for nm, a in f.items():
            key = f"b{info['bm']}_{info['bn']}/sha/{nm}"
            if key in z.files:
                seen += 1
                h = hashlib.sha256(np.ascontiguousarray(a.ravel(order="F")).tobytes()).hexdigest()
                if h != str(z[key]):
                    bad.append(f"({info['bm']},{info['bn']}):{nm}")
    assert seen > 0 and not bad, f"{name}/{mode}/{launcher}: {bad}"
