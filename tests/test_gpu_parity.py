"""GPU parity: the HIP path (libocn_sw.so, through its C ABI) against the reference.

* per-kernel: every kernel-layer entry on the golden random inputs of the compiled
  reference (tests/golden/kernels_*.npz) -- bitwise, untouched cells included;
* end-to-end: init + N steps on the golden cases (1 and several blocks on one GPU) against
  the SHA-256 of every field of every block of the unmodified reference run -- bitwise;
* larger sizes: against the CPU oracle (pinned to the reference by tests/test_oracle_pinned.py);
* full size (BASELINE 4096^2): size-independent properties (decomposition invariance,
  graph == eager, finite & bounded state).

Tolerance: none.  The path computes in fp64 with the reference's evaluation order and
-ffp-contract=off, so every comparison is bit-for-bit.
"""
import hashlib

import numpy as np
import pytest

from tests.golden import cases

pytestmark = pytest.mark.gpu


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a.ravel(order="F")).tobytes()).hexdigest()


def bits_equal(a, b):
    return a.dtype == b.dtype and a.shape == b.shape and \
        np.ascontiguousarray(a.ravel(order="F")).tobytes() == np.ascontiguousarray(b.ravel(order="F")).tobytes()


class OracleTwin:
    """The CPU oracle (oracle/oracle.py: the reference's algorithm layer over oracle/sw_oracle.c,
    pinned bit for bit to the compiled reference by tests/test_oracle_pinned.py) run beside a GPU
    model on the same box and block grid and given the same uploads -- so the parity corners the
    golden fixtures do not reach (arbitrary uploaded state, a forcing, tau changes, calls split
    anywhere) are checked against the reference's algorithm, not only between two HIP paths."""

    def __init__(self, n, blocks=(1, 1), tracers=0, mask=None):
        from oracle import oracle as O
        sw = O.SWConfig(use_tracers=1, tracer_num=tracers) if tracers else O.SWConfig()
        self.om = O.OracleModel(O.BasinConfig(nx=n + 4, ny=n + 4, mask=mask), sw, *blocks).init()

    def k(self, b):
        return [i for i, ob in enumerate(self.om.blocks) if (ob.bm, ob.bn) == (b.bm, b.bn)][0]

    def upload(self, b, nm, a):
        self.om.f[self.k(b)][nm][...] = a

    def run(self, steps, tau=1.0):
        self.om.run(steps, tau)

    def mismatches(self, m, names=None):
        """Fields of GPU model m that differ from the oracle's (every field by default)."""
        bad = []
        for b in m.blocks:
            f = self.om.f[self.k(b)]
            for nm in names or f:
                if nm in ("lu1", "rlh_c"):
                    continue
                if not bits_equal(m.download(b.k, nm), f[nm]):
                    bad.append(f"({b.bm},{b.bn}):{nm}")
        return bad


@pytest.fixture(scope="module")
def amd():
    import ocean_model_arch_amd as amd
    amd.lib()
    return amd


def model_for_geom(amd, z):
    nxs, nxe, nys, nye, bx1, bx2, by1, by2 = (int(v) for v in z["geom"])
    assert (nxs, nys, bx1, by1) == (3, 3, 1, 1)
    m = amd.OceanModel(amd.BasinConfig(nx=bx2, ny=by2))
    b = m.blocks[0]
    assert (b.nx_start, b.nx_end, b.ny_start, b.ny_end, b.bnd_x1, b.bnd_x2) == (nxs, nxe, nys, nye, bx1, bx2)
    return m


@pytest.mark.parametrize("geom", cases.KERNEL_GEOMS)
def test_kernels_match_reference(amd, geom):
    from ocean_model_arch_amd.kernel_interface import KernelParameters
    from ocean_model_arch_amd.sw_interface import ShallowWaterInterface
    z = cases.load_kernels(geom)
    m = model_for_geom(amd, z)
    inputs = {k[3:]: z[k] for k in z.files if k.startswith("in/") and k[3:] in m.field_names}
    iface = ShallowWaterInterface(m)
    p = KernelParameters(tau=float(z["tau"]), time_smooth=float(z["time_smooth"]))
    assert int(z["full_free_surface"]) == m.sw.full_free_surface
    failures = []
    for kname in cases.KERNEL_NAMES:
        for nm, a in inputs.items():
            m.upload(0, nm, a)
        getattr(iface, f"envoke_{kname}_kernel")(0, p)
        m.synchronize()
        outs = [k.split("/", 1)[1] for k in z.files if k.startswith(kname + "/")]
        for nm in outs:
            if not bits_equal(m.download(0, nm), z[f"{kname}/{nm}"]):
                failures.append(f"{kname}:{nm}")
    m.close()
    assert not failures, f"{geom}: differs from the reference: {failures}"


TRACER_IN = {"ff1": "ff1_1", "ff1p": "ff1p_1", "ff1n": "ff1n_1", "flux_x": "flux_x", "flux_y": "flux_y"}


@pytest.mark.parametrize("geom", cases.KERNEL_GEOMS)
def test_tracer_kernels_match_reference(amd, geom):
    """ocn_tran_diff_fluxes / ocn_tran_diff_tracer / ocn_tracer_next_step (kernel layer, called
    through the C ABI with the fixture's scalars, factor_mu = 0.7) on the reference's outputs."""
    import ctypes as C
    z = cases.load_kernels(geom)
    nxs, nxe, nys, nye, bx1, bx2, by1, by2 = (int(v) for v in z["geom"])
    m = amd.OceanModel(amd.BasinConfig(nx=bx2, ny=by2), amd.SWConfig(use_tracers=1, tracer_num=1))
    L = amd.lib()
    blk = m.blocks[0].c_block()
    inputs = {TRACER_IN.get(k[3:], k[3:]): z[k] for k in z.files if k.startswith("in/")}
    P = lambda nm: C.c_void_p(m.field_ptr(0, nm))      # noqa: E731
    calls = {
        "tran_diff_fluxes": lambda: L.ocn_tran_diff_fluxes(
            C.byref(blk), *[P(n) for n in ("lcu", "lcv", "dxt", "dyt", "dxh", "dyh", "hhu", "hhv", "ff1_1", "ff1p_1",
                                           "ubrtr", "vbrtr", "mu")], C.c_double(float(z["factor_mu"])),
            P("flux_x"), P("flux_y"), C.c_void_p(m.stream)),
        "tran_diff_tracer": lambda: L.ocn_tran_diff_tracer(
            C.byref(blk), P("lu"), P("dx"), P("dy"), C.c_double(float(z["tau"])),
            *[P(n) for n in ("hhq_n", "hhq_p", "flux_x", "flux_y", "ff1p_1", "ff1n_1")], C.c_void_p(m.stream)),
        "tracer_next_step": lambda: L.ocn_tracer_next_step(
            C.byref(blk), C.c_double(float(z["time_smooth"])), P("lu"), P("ff1n_1"), P("ff1p_1"), P("ff1_1"),
            C.c_void_p(m.stream)),
    }
    failures = []
    for kname in cases.TRACER_KERNEL_NAMES:
        for nm, a in inputs.items():
            m.upload(0, nm, a)
        assert calls[kname]() == 0, kname
        m.synchronize()
        for key in [k for k in z.files if k.startswith(kname + "/")]:
            nm = key.split("/", 1)[1]
            if not bits_equal(m.download(0, TRACER_IN.get(nm, nm)), z[key]):
                failures.append(f"{kname}:{nm}")
    m.close()
    assert not failures, f"{geom}: differs from the reference: {failures}"


def build_model(amd, case, graph=False, fused=True, compact=True, overlap=None, march=True, flip=True,
                recompute=True, rank=0, nranks=1, onepass=True, onepass_last=True, x2=True, batch=True):
    b = case["basin"]
    basin = amd.BasinConfig(nx=b["nx"], ny=b["ny"], dxst=b["dxst"], dyst=b["dyst"], rlon=b["rlon"], rlat=b["rlat"],
                            curve_grid=b["curve_grid"], mask=case["mask"],
                            topography=case.get("topography"))
    sw = amd.SWConfig(**case["sw"])
    par = amd.ParallelConfig(bppnx=case["bxy"][0], bppny=case["bxy"][1])
    m = amd.OceanModel(basin, sw, par, rank=rank, nranks=nranks)
    m.set_fused(fused)
    m.set_compact(compact)
    if overlap is not None:
        m.set_overlap(overlap)
    m.set_march(march)
    m.set_flip(flip)
    m.set_recompute(recompute)
    m.set_onepass(onepass)
    m.set_onepass_last(onepass_last)
    m.set_x2(x2)
    m.set_batch(batch)
    if graph:
        m.set_graph(True)
    return m


def compare_case(m, case, name, whole=True):
    """SHA of every field of every block of model m against the fixture; whole = m holds every
    block of the fixture (else: one rank's share)."""
    z = case["z"]
    blocks = cases.e2e_blocks(z)
    if whole:
        assert len(blocks) == len(m.blocks), name
    bad = []
    for b in m.blocks:
        info = blocks[(b.bm, b.bn)]
        assert [b.nx_start, b.nx_end, b.ny_start, b.ny_end, b.bnd_x1, b.bnd_x2, b.bnd_y1, b.bnd_y2] == list(info)
        for key in z.files:
            pre = f"b{b.bm}_{b.bn}/sha/"
            if key.startswith(pre):
                nm = key[len(pre):]
                if _sha(m.download(b.k, nm)) != str(z[key]):
                    bad.append(f"({b.bm},{b.bn}):{nm}")
    return bad


@pytest.mark.parametrize("mode", ["compact", "nox2", "noonepass", "nolast", "norecompute", "noflip", "pointwise",
                                  "fused", "stages", "stages_compact", "serial", "overlap2", "nobatch"])
@pytest.mark.parametrize("name", cases.E2E_CASES + cases.TRACER_E2E_CASES + cases.LONG_CASES + cases.TOPO_CASES)
def test_end_to_end_matches_reference(amd, name, mode):
    """compact = the default: the fused step reading the compact static fields, fused A / B /
    hh_init as register marches, role-flip steps, tracer runs included (hh_init fused with the next
    step's A, fused B recomputing hhq / hhu_p / hhv_p), halo exchanges overlapped
    with inner launches in the standard steps when there are several blocks;
    nox2 = compact with the one-pass steps of several blocks as hybrid steps (role-flip bands along
    the exchanged sides, two exchanges per step) instead of x2 steps (one 2-deep state exchange,
    the whole interior marched); nolast = compact with a standard last step where exchanges or ring
    work make the one-pass last step a hybrid one (so no x2 steps either); norecompute = compact without the recompute steps; noflip = compact with
    standard steps only;
    pointwise = compact with every launch one thread per point; overlap2 = compact with the
    role-flip steps' exchanges overlapped too (OCN_OPT_OVERLAP = 2); fused =
    the 4-launch step on the 2-D real(4) arrays; serial = compact without the overlap; stages =
    the reference's 11 envoke stages on the 2-D real(4) arrays (the ocn_<stage> kernel entries);
    stages_compact = the 11 stages over the compact tables (hh_init as the register march); nobatch = compact with one launch per block and launch group
    (every other mode batches the blocks of a device, OCN_OPT_BATCH)."""
    case = cases.load_e2e(name)
    compact = mode in ("compact", "nox2", "noonepass", "nolast", "norecompute", "noflip", "serial", "pointwise",
                       "overlap2", "nobatch", "stages_compact")
    m = build_model(amd, case, fused=mode not in ("stages", "stages_compact"), compact=compact,
                    overlap=2 if mode == "overlap2" else int(mode != "serial"),
                    march=mode != "pointwise", flip=mode != "noflip", recompute=mode != "norecompute",
                    onepass=mode != "noonepass", onepass_last=mode != "nolast", x2=mode != "nox2",
                    batch=mode != "nobatch")
    m.init().step(case["steps"], tau=1.0, check_every=1).synchronize()
    assert m.compact_active == compact
    bad = compare_case(m, case, name)
    flip_used, one_used, x2_used = m.flip_active, m.onepass_active, m.x2_active
    m.close()
    assert not bad, f"{name}: fields differ from the reference: {bad}"
    if mode in ("compact", "nox2", "noonepass", "nolast", "norecompute", "serial", "overlap2", "nobatch"):   # tracer runs included
        assert flip_used, f"{name}: role-flip steps not used"
    full_sw = case["sw"]["trans_terms"] > 0 and case["sw"]["ksw_lat"] > 0 and not case["sw"].get("use_tracers", 0)
    one_block = tuple(case["bxy"]) == (1, 1)
    if mode == "compact" and one_block and full_sw:
        assert one_used, f"{name}: one-pass steps not used"
    if mode in ("compact", "nobatch") and not one_block and full_sw and case["steps"] >= 3:
        assert x2_used, f"{name}: x2 steps not used"
    if mode in ("nox2", "nolast"):
        assert not x2_used


@pytest.mark.parametrize("name", cases.TOPO_CASES)
def test_topography_variants_match_reference(amd, name):
    """A non-uniform rest depth from a basin.par topography file (control/init_data.f90:115-120):
    the one-pass steps run their known-constant variant that reads h_r (OCN_KC_KNOWN_HR; the
    forcing and fallback values known zeros, mu uniform) -- and with OCN_OPT_KNOWN_CONSTANTS 0 the
    general variant -- on one block, and with x2 steps (h_r's second halo ring from the neighbours)
    on several, bitwise against the reference run that read the same file; also in 1-step calls
    (lazy tail)."""
    case = cases.load_e2e(name)
    for kc, calls in ((True, [case["steps"]]), (True, [1] * case["steps"]), (False, [case["steps"]])):
        m = build_model(amd, case).set_known_constants(kc).init()
        for n in calls:
            m.step(n, tau=1.0, check_every=1)
        m.synchronize()
        one, zero, hr, x2 = m.onepass_active, m.onepass_zero, m.onepass_hr, m.x2_active
        bad = compare_case(m, case, name)
        m.close()
        assert not bad, f"{name} ({len(calls)} calls, kc {kc}): fields differ from the reference: {bad}"
        assert one and not zero and hr == kc, (one, zero, hr, kc)
        assert x2 == ("_b1x1_" not in name), x2


@pytest.mark.parametrize("calls", ["7,1,12", "1x20"])
@pytest.mark.parametrize("graph", [False, True], ids=["stream", "graph"])
@pytest.mark.parametrize("name", ["box70x54_b3x2_s20", "box70x54_b1x1_s20"])
def test_split_step_calls_match_reference(amd, graph, name, calls):
    """The run split over several ocn_ctx_step calls -- down to the reference's own cadence of one
    expl_shallow_water per call (model.f90:146): same final state as one call and as the
    reference.  One block: every call after the first continues the one-pass sequence and leaves
    its tail pending (OCN_OPT_LAZY_TAIL), formed when the fields are read."""
    case = cases.load_e2e(name)
    m = build_model(amd, case, graph=graph).init()
    split = [7, 1, 12] if calls == "7,1,12" else [1] * 20
    pend = []
    for n in split:
        m.step(n, tau=1.0, check_every=0)
        pend.append(m.tail_pending)
    m.synchronize()
    bad = compare_case(m, case, name)
    pending_after = m.tail_pending
    m.close()
    assert not bad, f"{name}: fields differ from the reference: {bad}"
    assert not pending_after   # the downloads formed the tail
    assert all(pend), pend     # one block, or x2 steps between the blocks: the tail stays pending


def test_lazy_tail_interleaved_with_reads(amd):
    """1-step calls on one block with the fields read (tail formed) after some of them and a
    field written in between: every read sees the reference's state of that step, and the run
    ends bitwise equal to the one-call run with the same upload."""
    case = cases.load_e2e("box70x54_b1x1_s20")
    a = build_model(amd, case).init()
    b = build_model(amd, case).init()
    b.set_lazy_tail(False)
    for s in range(1, 13):
        a.step(1, check_every=1)
        b.step(1, check_every=1)
        if s in (3, 4, 9):
            for nm in ("ssh", "vort", "str_t", "hhu", "hhq", "sshp", "ubrtrp"):
                assert bits_equal(a.download(0, nm), b.download(0, nm)), (s, nm)
        if s == 6:   # a forcing change between steps (the known-constant check must see it)
            r = np.zeros(a.blocks[0].shape)
            r[10:20, 10:20] = 1.0e-7
            a.upload(0, "RHSx", r)
            b.upload(0, "RHSx", r)
    a.synchronize(); b.synchronize()
    bad = [nm for nm in a.field_names if not bits_equal(a.download(0, nm), b.download(0, nm))]
    assert a.onepass_active
    a.close(); b.close()
    assert not bad, bad


@pytest.mark.parametrize("what", ["metric", "mask"])
def test_compact_fallback_is_exact(amd, what):
    """real(4) fields the compact tables cannot represent (a metric varying along a row, a mask
    value other than 0/1): the fused step must detect it, read the 2-D arrays, and still match
    the oracle run on the same modified fields bit for bit."""
    from oracle import oracle as O
    n, bxy, steps = 96, (2, 1), 6
    om = O.OracleModel(O.BasinConfig(nx=n + 4, ny=n + 4), O.SWConfig(), *bxy).init()
    m = amd.OceanModel(amd.box_config(n), amd.SWConfig(), amd.ParallelConfig(*bxy)).init()
    for b in m.blocks:
        k = [i for i, ob in enumerate(om.blocks) if (ob.bm, ob.bn) == (b.bm, b.bn)][0]
        if what == "metric":
            a = om.f[k]["dx"]
            a *= (1.0 + 1.0e-4 * np.arange(a.shape[0], dtype=np.float32))[:, None]
            nm = "dx"
        else:
            a = om.f[k]["lu"]
            a[a.shape[0] // 2, a.shape[1] // 2] = 0.75
            nm = "lu"
        m.upload(b.k, nm, a)
    m.step(steps).synchronize()
    assert not m.compact_active
    om.run(steps)
    bad = []
    for b in m.blocks:
        k = [i for i, ob in enumerate(om.blocks) if (ob.bm, ob.bn) == (b.bm, b.bn)][0]
        for nm, a in om.f[k].items():
            if nm in ("lu1", "rlh_c"):
                continue
            if not bits_equal(m.download(b.k, nm), a):
                bad.append(f"({b.bm},{b.bn}):{nm}")
    m.close()
    assert not bad, bad


def test_flip_falls_back_when_pairs_disagree(amd):
    """Role-flip steps need ssh/sshn, ubrtr/ubrtrn, vbrtr/vbrtrn to agree outside their write
    sets (sw_stencils.h Coherence).  A state where sshn differs from ssh on a land point and
    ubrtrn from ubrtr on the halo must be detected on the device and run with standard steps:
    same result bit for bit as a run with OCN_OPT_FLIP off.  A coherent upload keeps flip on and
    still matches."""
    n, steps = 96, 6
    out = {}
    for flip in (True, False):
        for kind in ("incoherent", "coherent"):
            m = amd.OceanModel(amd.box_config(n)).set_flip(flip).init()
            s, u = m.download(0, "sshn"), m.download(0, "ubrtrn")
            if kind == "incoherent":
                s[0, 0] += 0.25         # bnd corner: outside every write set
                u[1, 5] = 1.0e-3        # halo column
            m.upload(0, "sshn", s)
            m.upload(0, "ubrtrn", u)
            m.step(steps).synchronize()
            out[(flip, kind)] = {nm: m.download(0, nm) for nm in ("ssh", "sshn", "sshp", "ubrtr", "ubrtrn",
                                                                   "ubrtrp", "vbrtr", "vbrtrn", "vbrtrp", "hhu",
                                                                   "hhv", "hhh", "hhq", "vort", "str_t", "str_s")}
            m.close()
    for kind in ("incoherent", "coherent"):
        bad = [nm for nm, a in out[(True, kind)].items() if not bits_equal(a, out[(False, kind)][nm])]
        assert not bad, f"{kind}: flip vs standard steps differ in {bad}"
    assert out[(True, "incoherent")]["sshn"][0, 0] != out[(True, "incoherent")]["ssh"][0, 0]


@pytest.mark.parametrize("kind", ["sea", "land"])
def test_flip_falls_back_when_halo_disagrees(amd, kind):
    """With halo exchanges, role-flip steps also need the halo ring of ssh (and ubrtr, vbrtr,
    hhu, hhv, hhq_rest) to hold the neighbours' values (ocn_ctx.hip check_coherence).  A state
    whose ssh and sshn differ there (kind = sea: a sea point of the ring between two blocks, which
    the exchange and a8 overwrite; land: a land point of that ring, where the standard step keeps
    ssh and the swapped one would not) must run with
    standard steps, bit for bit as with OCN_OPT_FLIP off; the unmodified state uses them."""
    n, steps = 96, 6
    par = amd.ParallelConfig(2, 1)
    probe = amd.OceanModel(amd.box_config(n), par=par)
    xe = [x for x in probe.blocks if x.bm == 1][0].nx_end
    probe.close()
    mask = np.zeros((n + 4, n + 4), dtype=np.int32)   # the closed box with a 2-cell land frame ...
    mask[:2, :] = mask[-2:, :] = mask[:, :2] = mask[:, -2:] = 1
    mask[xe, n // 2 - 3:n // 2 + 3] = 1               # ... and an island on the column right of block 1
    out, used = {}, {}
    for flip in (True, False):
        for mod in (True, False):
            m = amd.OceanModel(amd.box_config(n, mask=mask), par=par).set_flip(flip).init()
            b = [x for x in m.blocks if x.bm == 1][0]
            if mod:   # the halo column right of block (1, 1) (its neighbour's first interior column):
                # ssh and sshn changed alike, so the pairs still agree on the block itself
                i = b.nx_end + 1 - b.bnd_x1
                lu = m.download(b.k, "lu")[i, b.ny_start - b.bnd_y1:b.ny_end - b.bnd_y1 + 1]
                rows = np.flatnonzero(lu == (1.0 if kind == "sea" else 0.0))
                assert rows.size, kind
                j = b.ny_start - b.bnd_y1 + int(rows[rows.size // 2])
                for nm in ("ssh", "sshn"):
                    a = m.download(b.k, nm)
                    a[i, j] += 0.125
                    m.upload(b.k, nm, a)
            m.step(steps).synchronize()
            used[(flip, mod)] = m.flip_active
            out[(flip, mod)] = [{nm: m.download(x.k, nm) for nm in ("ssh", "sshn", "sshp", "ubrtr", "ubrtrn",
                                                                     "vbrtr", "vbrtrn", "hhu", "hhv", "hhh")}
                                for x in m.blocks]
            m.close()
    for mod in (True, False):
        bad = [(k, nm) for k, d in enumerate(out[(True, mod)]) for nm, a in d.items()
               if not bits_equal(a, out[(False, mod)][k][nm])]
        assert not bad, f"modified={mod}: flip vs standard steps differ in {bad}"
    assert used[(True, False)] and not used[(True, True)]


@pytest.mark.parametrize("name", ["box70x54_b3x2_s20", "bs_b1x1_s60"])
def test_graph_step_matches_reference(amd, name):
    case = cases.load_e2e(name)
    m = build_model(amd, case, graph=True)
    m.init().step(case["steps"], tau=1.0, check_every=0).synchronize()
    bad = compare_case(m, case, name)
    m.close()
    assert not bad, f"{name} (hipGraph): fields differ: {bad}"


def test_psykal_host_path_matches_reference(amd):
    """Reference-shaped host: expl_shallow_water -> envoke -> envoke_<stage>_kernel -> C ABI entry."""
    from ocean_model_arch_amd.shallow_water import expl_shallow_water
    from ocean_model_arch_amd.sw_interface import ShallowWaterInterface
    case = cases.load_e2e("box70x54_b3x2_s20")
    m = build_model(amd, case)
    m.init()
    iface = ShallowWaterInterface(m)
    for _ in range(case["steps"]):
        expl_shallow_water(m, 1.0, iface)
    m.synchronize()
    bad = compare_case(m, case, "psykal")
    m.close()
    assert not bad, bad


def test_psykal_tracer_path_matches_reference(amd):
    """expl_shallow_water + expl_tracer through the Python PSy layers (tracer_interface mirror)."""
    from ocean_model_arch_amd.shallow_water import expl_shallow_water
    from ocean_model_arch_amd.sw_interface import ShallowWaterInterface
    from ocean_model_arch_amd.tracer import expl_tracer
    from ocean_model_arch_amd.tracer_interface import TracerInterface
    case = cases.load_e2e("box70x54_b3x2_tr_s20")
    m = build_model(amd, case)
    m.init()
    iface, tiface = ShallowWaterInterface(m), TracerInterface(m)
    for _ in range(case["steps"]):
        expl_shallow_water(m, 1.0, iface)
        expl_tracer(m, 1.0, tiface)
    m.synchronize()
    bad = compare_case(m, case, "psykal tracers")
    m.close()
    assert not bad, bad


def _oracle_state(n, bxy, steps):
    from oracle import oracle as O
    om = O.OracleModel(O.BasinConfig(nx=n + 4, ny=n + 4), O.SWConfig(), *bxy).init().run(steps)
    return om


@pytest.mark.parametrize("n,bxy,steps,fused,overlap", [(256, (1, 1), 10, True, 1), (1024, (1, 1), 3, True, 1),
                                                        (300, (3, 2), 8, True, 1), (300, (3, 2), 8, False, 1),
                                                        (1024, (2, 2), 4, True, 1), (1024, (2, 2), 4, True, 2),
                                                        (520, (3, 2), 6, True, 2), (520, (3, 2), 6, True, 0)])
def test_larger_boxes_match_oracle(amd, n, bxy, steps, fused, overlap):
    """Against the oracle on boxes whose blocks are wide enough for the halo-overlap split of the
    march launches (inner part 64 columns / 8 rows inside the interior, frame bands around it)."""
    om = _oracle_state(n, bxy, steps)
    m = amd.OceanModel(amd.box_config(n), amd.SWConfig(), amd.ParallelConfig(*bxy)).set_fused(fused)
    m.set_overlap(overlap)
    m.init().step(steps).synchronize()
    bad = []
    for b in m.blocks:
        k = [i for i, ob in enumerate(om.blocks) if (ob.bm, ob.bn) == (b.bm, b.bn)][0]
        for nm, a in om.f[k].items():
            if nm in ("lu1", "rlh_c"):
                continue
            if not bits_equal(m.download(b.k, nm), a):
                bad.append(f"({b.bm},{b.bn}):{nm}")
    m.close()
    assert not bad, bad


def _interior(m, nm):
    """Assemble the global interior of field nm from all blocks."""
    nx, ny = m.basin.nx, m.basin.ny
    g = np.full((nx, ny), np.nan)
    for b in m.blocks:
        a = m.download(b.k, nm)
        g[b.nx_start - 1:b.nx_end, b.ny_start - 1:b.ny_end] = \
            a[b.nx_start - b.bnd_x1:b.nx_end - b.bnd_x1 + 1, b.ny_start - b.bnd_y1:b.ny_end - b.bnd_y1 + 1]
    return g


def test_full_size_decomposition_invariance(amd):
    """BASELINE box 4096^2: one block vs a 2 x 2 block grid on one GPU give bitwise-identical interiors
    (the reference's own property: 1 vs 4 vs 8 ranks are bit-identical)."""
    n, steps = 4096, 3
    a = amd.OceanModel(amd.box_config(n)).init().step(steps).synchronize()
    ga = {nm: _interior(a, nm) for nm in ("ssh", "ubrtr", "vbrtr", "sshp", "hhu", "hhh")}
    a.close()
    b = amd.OceanModel(amd.box_config(n), par=amd.ParallelConfig(2, 2)).init().step(steps).synchronize()
    for nm, ref in ga.items():
        got = _interior(b, nm)
        assert np.isfinite(ref[2:-2, 2:-2]).all()
        assert bits_equal(got, ref), nm
    # the Gaussian hump starts to spread: bounded, nonzero velocities after 3 steps
    assert 0.0 < np.nanmax(np.abs(ga["ubrtr"])) < 1.0
    b.close()


@pytest.mark.parametrize("nsteps", [1, 3])
def test_blowup_is_reported(amd, nsteps):
    """check_ssh_err_kernel (vel_ssh.f90:40-67): |ssh| >= 1e4 on a sea point must fail the step
    (nsteps = 3: the check inside the role-flip steps' fused B)."""
    m = amd.OceanModel(amd.box_config(64)).init()
    s = m.download(0, "ssh")
    s[10, 10] = 2.0e4
    for nm in ("ssh", "sshn", "sshp"):
        m.upload(0, nm, s)
    with pytest.raises(amd.OcnError):
        m.step(nsteps, check_every=1).synchronize()
    m.close()


@pytest.mark.parametrize("blocks", [(1, 1), (2, 2)])
def test_onepass_with_nonzero_fallback_values(amd, blocks):
    """The one-pass step where D takes the arrays' values (mask 0, outside a stage's range) when
    those are not zero, and with a forcing (sw_kernels.hip MarchStep ZF = false: loaded, not the
    constant 0): hhu, hhv, hhh, vort and the stresses set to nonzero values on the land frame and
    the halo, RHSx / RHSy on the sea, then
    the same call with one-pass steps and with the round-1 role-flip path (pinned to the
    reference by the other tests), bit for bit."""
    n, steps = 96, 8
    out = {}
    for onepass in (True, False):
        m = amd.OceanModel(amd.box_config(n), par=amd.ParallelConfig(*blocks)).set_onepass(onepass)
        m.init()
        ref = OracleTwin(n, blocks)
        for b in m.blocks:
            lu = m.download(b.k, "lu")
            for nm, v in (("hhu", 0.25), ("hhv", 0.5), ("hhh", 0.75), ("vort", 1e-3), ("str_t", 2e-3),
                          ("str_s", 3e-3), ("hhu_p", 0.125), ("hhv_p", 0.375)):
                a = m.download(b.k, nm)
                a[lu < 0.5] = v            # land and the land halo
                m.upload(b.k, nm, a)
                ref.upload(b, nm, a)
            for nm, v in (("RHSx", 2e-7), ("RHSy", -3e-7)):   # a wind forcing on the sea
                a = m.download(b.k, nm)
                a[lu > 0.5] = v
                m.upload(b.k, nm, a)
                ref.upload(b, nm, a)
        m.step(steps, tau=1.0, check_every=1).synchronize()
        assert m.onepass_active == onepass
        ref.run(steps)
        out[onepass] = ref.mismatches(m)
        m.close()
    assert not out[True], f"one-pass with nonzero fallback values differs from the oracle: {out[True]}"
    assert not out[False], f"role-flip path with nonzero fallback values differs from the oracle: {out[False]}"


@pytest.mark.gpu
def test_known_constants_option(amd):
    """OCN_OPT_KNOWN_CONSTANTS 0: the one-pass steps run their general variant (h_r, mu, the
    forcing and D's fallback values read from the arrays) -- the same results bit for bit as the
    known-constant variant the check selects by default."""
    n, steps = 130, 9
    ref = OracleTwin(n)
    ref.run(steps)
    for kc in (True, False):
        m = amd.OceanModel(amd.box_config(n)).set_known_constants(kc)
        m.init()
        m.step(steps, tau=1.0, check_every=1).synchronize()
        assert m.onepass_active and m.onepass_zero == kc
        bad = ref.mismatches(m)
        m.close()
        assert not bad, f"one-pass variant (known constants {kc}) differs from the oracle: {bad}"


@pytest.mark.parametrize("what", ["forcing", "mu", "h_r"])
def test_graph_replay_sees_uploads_between_calls(amd, what):
    """Graph replay (OCN_OPT_GRAPH) with a field uploaded between two step calls that changes the
    one-pass variant's preconditions (a forcing, a new uniform mu, a new uniform h_r): the replayed
    steps must see the new values (the known-constant variant reads them from device memory, the
    device check picks the variant, the captured step's key holds the variant mode) -- bitwise as
    the same run on the stream."""
    n = 96
    for graph in (True, False):
        m = amd.OceanModel(amd.box_config(n)).init()
        ref = OracleTwin(n)
        m.set_graph(graph)
        m.step(6, check_every=1).synchronize()
        ref.run(6)
        b = m.blocks[0]
        if what == "forcing":
            a = np.zeros(b.shape)
            a[20:40, 30:50] = 2.5e-7
            nm = "RHSx"
        else:
            nm = "mu" if what == "mu" else "hhq_rest"
            a = np.full(b.shape, 3.0 if what == "mu" else 80.0)
        m.upload(0, nm, a)
        ref.upload(b, nm, a)
        m.step(5, check_every=1)
        m.step(4, check_every=1).synchronize()
        ref.run(9)
        assert m.onepass_active
        bad = ref.mismatches(m)
        m.close()
        assert not bad, f"graph {graph}: steps after a {what} upload differ from the oracle: {bad}"


@pytest.mark.gpu
@pytest.mark.parametrize("kc", [True, False])
def test_onepass_rows_rerun_with_ieee_divisions(amd, kc):
    """Dividends below udiv's range (|x| < 2^-900: velocities of ~1e-290 on 20 rows) make
    the one-pass step re-run those rows with IEEE divisions (sw_kernels.hip MarchStep::iteration,
    a wave-uniform branch no other test takes); the results must still be the role-flip path's
    bit for bit, in both variants (known constants / general)."""
    n, steps = 130, 6
    for onepass in (True, False):
        m = amd.OceanModel(amd.box_config(n)).set_onepass(onepass).set_known_constants(kc)
        m.init()
        ref = OracleTwin(n)
        rng = np.random.default_rng(7)
        for nms in (("ubrtr", "ubrtrn"), ("ubrtrp",), ("vbrtr", "vbrtrn"), ("vbrtrp",)):
            a = m.download(0, nms[0])
            a[:, 40:60] = 1e-290 * (1.0 + rng.random(a[:, 40:60].shape))   # rows 40..59 (at rest: 0 before)
            for nm in nms:   # both buffers of a role-flip pair (they agree, as the reference leaves them)
                m.upload(0, nm, a)
                ref.upload(m.blocks[0], nm, a)
        m.step(steps, tau=1.0, check_every=1).synchronize()
        assert m.onepass_active == onepass
        ref.run(steps)
        bad = ref.mismatches(m)
        m.close()
        assert not bad, f"rows with dividends below udiv's range (one-pass {onepass}) differ from the oracle: {bad}"


def test_second_buffers_across_calls(amd):
    """One-pass calls leave sshp / ubrtrp / vbrtrp in their second buffers between calls (no
    copies back at a call's end).  A raw pointer handed out afterwards holds the current values,
    later calls keep returning them there, and the run equals one that never handed one out."""
    import ctypes as C
    hip = C.CDLL("libamdhip64.so")
    names = ("sshp", "ubrtrp", "vbrtrp")
    m = amd.OceanModel(amd.box_config(130)).init()
    m.step(6, tau=1.0).synchronize()
    assert m.onepass_active
    ptr = {nm: m.field_ptr(0, nm) for nm in names}
    m.synchronize()
    b = m.blocks[0]
    w, h = b.shape

    def raw(nm):
        a = np.zeros((h, b.pitch), dtype=np.float64)
        assert hip.hipMemcpy(a.ctypes.data_as(C.c_void_p), C.c_void_p(ptr[nm]), C.c_size_t(a.nbytes), 2) == 0
        return np.asfortranarray(a[:, :w].T)

    for nm in names:
        assert bits_equal(raw(nm), m.download(0, nm)), nm
    m.step(5, tau=1.0).synchronize()
    for nm in names:
        assert bits_equal(raw(nm), m.download(0, nm)), nm
    ref = amd.OceanModel(amd.box_config(130)).init()
    ref.step(6, tau=1.0).step(5, tau=1.0).synchronize()
    bad = [nm for nm in m.field_names if not bits_equal(m.download(0, nm), ref.download(0, nm))]
    m.close()
    ref.close()
    assert not bad, bad


def test_user_sync_of_second_buffer_fields(amd):
    """ocn_ctx_sync of sshp / ubrtrp / vbrtrp between one-pass calls (their values in the second
    buffers after an odd number of one-pass steps) and after they return home (ocn_ctx_field):
    the halo plan follows the field's current buffer."""
    m = amd.OceanModel(amd.box_config(130), par=amd.ParallelConfig(2, 2)).init()
    nx = ny = 134
    f = lambda i, j: i * 10000.0 + j   # noqa: E731

    def check_sync(nm):
        for b in m.blocks:
            i = np.arange(b.bnd_x1, b.bnd_x2 + 1)[:, None]
            j = np.arange(b.bnd_y1, b.bnd_y2 + 1)[None, :]
            inner = (i >= b.nx_start) & (i <= b.nx_end) & (j >= b.ny_start) & (j <= b.ny_end)
            m.upload(b.k, nm, np.asfortranarray(np.where(inner, f(i, j), -1.0)))
        m.sync(nm)
        m.synchronize()
        for b in m.blocks:
            i = np.arange(b.bnd_x1, b.bnd_x2 + 1)[:, None]
            j = np.arange(b.bnd_y1, b.bnd_y2 + 1)[None, :]
            # the 1-wide halo ring inside the global interior receives the neighbours' values
            ring = (i >= b.nx_start - 1) & (i <= b.nx_end + 1) & (j >= b.ny_start - 1) & (j <= b.ny_end + 1)
            glob = ring & (i >= 3) & (i <= nx - 2) & (j >= 3) & (j <= ny - 2)
            assert bits_equal(m.download(b.k, nm), np.asfortranarray(np.where(glob, f(i, j), -1.0))), (nm, b.k)

    m.step(5, tau=1.0).synchronize()
    assert m.onepass_active
    for nm in ("sshp", "ubrtrp", "vbrtrp"):
        check_sync(nm)
    m.init().step(5, tau=1.0).synchronize()   # (the patterns are no state to step from)
    for nm in ("sshp", "ubrtrp", "vbrtrp"):
        m.field_ptr(0, nm)   # the values return to the fields' own buffers
        check_sync(nm)
    m.close()


@pytest.mark.parametrize("name", ["bs_b4x2_tr_s60", "box70x54_b3x2_s20"])
def test_block_batching_cuts_launches(amd, name):
    """OCN_OPT_BATCH: with several blocks on the device each launch group goes out once for all of
    them -- fewer launches per step than one per block, and the same bits (the e2e `nobatch` mode
    covers the unbatched path against the reference too)."""
    case = cases.load_e2e(name)
    counts, digests = [], []
    for batch in (False, True):
        m = build_model(amd, case, batch=batch).init()
        m.step(2, tau=1.0, check_every=1).synchronize()    # the one-time checks and tables
        n0 = amd._lib.launch_count()
        m.step(case["steps"] - 2, tau=1.0, check_every=1).synchronize()
        counts.append(amd._lib.launch_count() - n0)
        digests.append(compare_case(m, case, name))
        m.close()
    assert digests == [[], []], digests
    assert counts[1] < counts[0], counts


@pytest.mark.parametrize("name", ["box70x54_b3x2_s20", "bs_b4x2_tr_s60"])
def test_rccl_single_rank_matches_reference(amd, name):
    """RCCL on the hardware: one pool box has one GPU and RCCL refuses two ranks on one device, so
    the production communicator is exercised as a world of one -- ncclCommInitRank through
    ocn_ctx_attach_comm, the step's vote as ncclAllReduce, the halo plans' grouped calls (all
    exchanges local) and the per-call h_r refresh of a communicating context -- bitwise against the
    reference fixture."""
    case = cases.load_e2e(name)
    m = build_model(amd, case)
    m.attach_comm(amd.make_unique_id())
    m.init().step(case["steps"], tau=1.0, check_every=1).synchronize()
    bad = compare_case(m, case, name)
    flip = m.flip_active
    m.close()
    assert not bad, f"{name}: fields differ from the reference over an RCCL communicator: {bad}"
    assert flip
