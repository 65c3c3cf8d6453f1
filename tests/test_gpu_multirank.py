"""GPU parity of the multi-rank path (one block per rank, halos between ranks) and of the
BASELINE.json configurations at full size, against the reference.

The ranks run as contexts of this one process on the one GPU, joined by the library's loopback
transport (ocn_ctx_attach_loopback), each driven by its own host thread.  The loopback replaces
only the two RCCL calls (ncclRecv/ncclSend of an exchange, the ncclAllReduce of the role-flip
vote); the device pack / unpack of every message, the per-peer plans per buffer role, the
merged hh_init + A exchange and the overlap forks are the production code that an 8-GPU run
over RCCL executes.  Reference behaviour replaced: core/kernel_interface.f90:174-184
(_GPU_MULTI_: block k on device k-1) and shared/mpp/syncborder_block2D_gen_all.fi:100-129.

Tolerance: none (bitwise SHA-256 of every field of every block vs the unmodified reference run).
"""
import numpy as np
import pytest

from tests.golden import cases
from tests.test_gpu_parity import bits_equal, build_model, compare_case

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def amd():
    import ocean_model_arch_amd as amd
    amd.lib()
    return amd


def run_ranks_case(amd, case, nranks, steps=None, calls=None, **opts):
    """The fixture's block grid over `nranks` loopback ranks; returns the models (caller closes)."""
    models = [build_model(amd, case, rank=r, nranks=nranks, **opts) for r in range(nranks)]
    amd.OceanModel.attach_loopback(models)
    calls = calls or [steps if steps is not None else case["steps"]]

    def body(m):
        m.init()
        for n in calls:
            m.step(n, tau=1.0, check_every=1)
        m.synchronize()
        return m.flip_active, m.x2_active

    used = amd.run_ranks(models, body)
    run_ranks_case.x2 = [u[1] for u in used]
    return models, [u[0] for u in used]


def check_ranks(models, case, name):
    bad, nblocks = [], 0
    for m in models:
        bad += compare_case(m, case, name, whole=False)
        nblocks += len(m.blocks)
    assert nblocks == len(cases.e2e_blocks(case["z"])), name
    return bad


MODES = {   # name -> build_model options
    "default": {},                            # role-flip steps; exchanges overlapped per OCN_OPT_OVERLAP default
    "overlap0": dict(overlap=0),
    "overlap1": dict(overlap=1),
    "overlap2": dict(overlap=2),
    "noflip": dict(flip=False),
    "noflip_overlap0": dict(flip=False, overlap=0),
    "norecompute": dict(recompute=False),
    "nolast": dict(onepass_last=False),
    "nox2": dict(x2=False),                   # hybrid one-pass steps: CA / B bands, two exchanges per step
    "nox2_overlap0": dict(x2=False, overlap=0),
    "stages": dict(fused=False),
}


@pytest.mark.parametrize("mode", list(MODES))
@pytest.mark.parametrize("name,nranks", [("box70x54_b3x2_s20", 6), ("bs_b4x2_s60", 8), ("bs_b4x2_tr_s60", 8),
                                         ("box40x32_b2x2_s5", 4)])
def test_ranks_match_reference(amd, name, nranks, mode):
    case = cases.load_e2e(name)
    models, flips = run_ranks_case(amd, case, nranks, **MODES[mode])
    try:
        bad = check_ranks(models, case, name)
        levels = {m.overlap_level for m in models}
    finally:
        for m in models:
            m.close()
    assert not bad, f"{name} over {nranks} ranks ({mode}): fields differ from the reference: {bad}"
    if mode == "default":   # OCN_OPT_OVERLAP auto: remote peers -> role-flip exchanges overlapped
        assert levels == {2}, levels
    x2 = run_ranks_case.x2
    assert len(set(flips)) == 1 and len(set(x2)) == 1, "ranks ran different kinds of steps"
    if mode in ("default", "overlap0", "overlap1", "overlap2", "norecompute", "nox2"):   # tracer runs included
        assert flips[0], f"{name}: role-flip steps not used over ranks"
    if mode == "default" and "_tr_" not in name and case["steps"] >= 3:
        assert x2[0], f"{name}: x2 steps not used over ranks"
    if mode.startswith("nox2") or mode == "nolast":
        assert not x2[0]


def test_ranks_split_calls_match_reference(amd):
    """Several ocn_ctx_step calls per rank (each call votes again over the ranks)."""
    case = cases.load_e2e("box70x54_b3x2_s20")
    models, _ = run_ranks_case(amd, case, 6, calls=[7, 1, 12])
    try:
        bad = check_ranks(models, case, "split")
    finally:
        for m in models:
            m.close()
    assert not bad, bad


def test_ranks_604_steps_tracer_match_reference(amd):
    """Config 5 at the shipped run length: Black Sea + 1 tracer, 4x2 blocks, one per rank."""
    case = cases.load_e2e("bs_b4x2_tr_s604")
    models, _ = run_ranks_case(amd, case, 8)
    try:
        bad = check_ranks(models, case, "bs_b4x2_tr_s604")
    finally:
        for m in models:
            m.close()
    assert not bad, bad


@pytest.mark.parametrize("kind", ["sea", "land"])
def test_ranks_flip_falls_back_when_halo_disagrees(amd, kind):
    """test_gpu_parity.test_flip_falls_back_when_halo_disagrees with the island on a RANK
    boundary: rank 0's check finds the disagreement, the vote (the loopback's ncclAllReduce)
    makes both ranks run standard steps, bit for bit as with OCN_OPT_FLIP off."""
    n, steps = 96, 6
    par = amd.ParallelConfig(2, 1)
    probe = amd.OceanModel(amd.box_config(n), par=par)
    xe = [x for x in probe.blocks if x.bm == 1][0].nx_end
    probe.close()
    mask = np.zeros((n + 4, n + 4), dtype=np.int32)
    mask[:2, :] = mask[-2:, :] = mask[:, :2] = mask[:, -2:] = 1
    mask[xe, n // 2 - 3:n // 2 + 3] = 1
    out, used = {}, {}
    for flip in (True, False):
        for mod in (True, False):
            models = [amd.OceanModel(amd.box_config(n, mask=mask), par=par, rank=r, nranks=2).set_flip(flip)
                      for r in range(2)]
            amd.OceanModel.attach_loopback(models)
            amd.run_ranks(models, lambda m: m.init())
            m0 = models[0]
            b = m0.blocks[0]
            assert b.bm == 1
            if mod:
                i = b.nx_end + 1 - b.bnd_x1
                lu = m0.download(b.k, "lu")[i, b.ny_start - b.bnd_y1:b.ny_end - b.bnd_y1 + 1]
                rows = np.flatnonzero(lu == (1.0 if kind == "sea" else 0.0))
                assert rows.size, kind
                j = b.ny_start - b.bnd_y1 + int(rows[rows.size // 2])
                for nm in ("ssh", "sshn"):
                    a = m0.download(b.k, nm)
                    a[i, j] += 0.125
                    m0.upload(b.k, nm, a)
            flips = amd.run_ranks(models, lambda m: m.step(steps).synchronize().flip_active)
            assert len(set(flips)) == 1
            used[(flip, mod)] = flips[0]
            out[(flip, mod)] = [{nm: m.download(x.k, nm) for nm in ("ssh", "sshn", "sshp", "ubrtr", "ubrtrn",
                                                                     "vbrtr", "vbrtrn", "hhu", "hhv", "hhh")}
                                for m in models for x in m.blocks]
            for m in models:
                m.close()
    for mod in (True, False):
        bad = [(k, nm) for k, d in enumerate(out[(True, mod)]) for nm, a in d.items()
               if not bits_equal(a, out[(False, mod)][k][nm])]
        assert not bad, f"modified={mod}: flip vs standard steps differ in {bad}"
    assert used[(True, False)] and not used[(True, True)]


def test_ranks_upload_on_one_rank_votes_together(amd):
    """A field uploaded on one rank only (its hh_init depths then no longer match the state, so that
    rank alone could not start the call with a one-pass step): the vote (loopback ncclAllReduce)
    carries that condition too, so every rank runs the same kind of first step and the exchange
    sequences match -- the run completes, equal bit for bit to the same upload in one process."""
    n, steps = 96, 6
    par = amd.ParallelConfig(2, 1)
    outs = {}
    for ranks in (2, 1):
        models = [amd.OceanModel(amd.box_config(n), par=par, rank=r, nranks=ranks) for r in range(ranks)]
        if ranks > 1:
            amd.OceanModel.attach_loopback(models)
            amd.run_ranks(models, lambda m: m.init().step(3).synchronize())
        else:
            models[0].init().step(3).synchronize()
        m0 = [m for m in models if any(b.bm == 1 for b in m.blocks)][0]
        k = [b.k for b in m0.blocks if b.bm == 1][0]
        a = m0.download(k, "ssh")
        a[10:14, 20:24] += 1.0e-3     # sea points of block (1, 1) only
        m0.upload(k, "ssh", a)
        if ranks > 1:
            amd.run_ranks(models, lambda m: m.step(steps).synchronize())
        else:
            models[0].step(steps).synchronize()
        outs[ranks] = {(b.bm, b.bn): {nm: m.download(b.k, nm) for nm in ("ssh", "ubrtr", "vbrtr", "hhu", "sshp")}
                       for m in models for b in m.blocks}
        for m in models:
            m.close()
    bad = [(key, nm) for key, d in outs[2].items() for nm, a in d.items() if not bits_equal(a, outs[1][key][nm])]
    assert not bad, bad


def test_ranks_blowup_stops_every_rank(amd):
    """check_ssh_err_kernel on one rank (vel_ssh.f90:52-66 abort_model -> mpi_abort on the cart
    communicator, shared/errors.f90:16-37): |ssh| >= 1e4 on one sea point of one block of 8 ranks --
    every rank raises OcnError (OCN_ERR_BLOWUP) from the same synchronize (the counts are reduced
    over the ranks), and no rank waits for a peer (no 120 s rendezvous timeout)."""
    import time
    n, nranks, hot = 128, 8, 5
    par = amd.ParallelConfig(4, 2)
    models = [amd.OceanModel(amd.box_config(n), par=par, rank=r, nranks=nranks) for r in range(nranks)]
    amd.OceanModel.attach_loopback(models)

    def body(m):
        m.init().step(2).synchronize()
        if m.rank == hot:
            k = m.blocks[0].k
            s = m.download(k, "ssh")
            s[s.shape[0] // 2, s.shape[1] // 2] = 2.0e4
            for nm in ("ssh", "sshn", "sshp"):
                m.upload(k, nm, s)
        t0 = time.perf_counter()
        try:
            m.step(3, check_every=1).synchronize()
        except amd.OcnError as e:
            return ("raised", str(e), time.perf_counter() - t0)
        return ("ok", "", time.perf_counter() - t0)

    try:
        res = amd.run_ranks(models, body)
    finally:
        for m in models:
            m.close()
    assert [r[0] for r in res] == ["raised"] * nranks, res
    assert all("1e4" in r[1] for r in res), res
    assert max(r[2] for r in res) < 60.0, res


# ---------------------------------------------------------------- BASELINE.json configs, full size
def _full(amd, name, **opts):
    case = cases.load_e2e(name)
    m = build_model(amd, case, **opts)
    return case, m


@pytest.mark.parametrize("variant", ["bench", "graph", "noflip", "noonepass"])
def test_bench_workload_matches_reference(amd, variant):
    """The bench's exact workload and options (bench.py: 4096^2 box, 1 block, stage-timing events
    on, one call whose steps are first / one-pass x 4 / CA + last) vs the reference's 6-step run;
    noonepass: the recompute steps instead."""
    case, m = _full(amd, "box4096_b1x1_s6", graph=variant == "graph", flip=variant != "noflip",
                    onepass=variant != "noonepass")
    try:
        m.init()
        if variant == "bench":
            m.set_stage_timing(True)
        m.step(case["steps"], tau=1.0, check_every=1).synchronize()
        if variant == "bench":
            assert m.flip_active and m.onepass_active
        if variant == "noonepass":
            assert m.flip_active and m.recompute_active
        bad = compare_case(m, case, "box4096")
    finally:
        m.close()
    assert not bad, f"4096^2 ({variant}): fields differ from the reference: {bad}"


@pytest.mark.parametrize("x2", [True, False], ids=["x2", "nox2"])
@pytest.mark.parametrize("name", ["box1024_b1x1_s10", "box2048_b2x2_s4", "box4096_b4x2_s4"])
def test_fullsize_blocks_match_reference(amd, name, x2):
    """C2 (1024^2), C3 (2048^2 as 2x2 blocks) and C4 (4096^2 as 4x2 blocks) in one process:
    every block on the GPU, local halo copies; the one-pass steps of the block grids with one 2-deep
    state exchange each (x2) or as hybrid steps (nox2)."""
    if not x2 and "_b1x1_" in name:
        pytest.skip("one block: no exchange")
    case, m = _full(amd, name, x2=x2)
    try:
        m.init().step(case["steps"], tau=1.0, check_every=1).synchronize()
        used = m.x2_active
        bad = compare_case(m, case, name)
    finally:
        m.close()
    assert not bad, f"{name}: fields differ from the reference: {bad}"
    assert used == (x2 and "_b1x1_" not in name)


@pytest.mark.parametrize("calls", ["one", "per_step"])
@pytest.mark.parametrize("name", cases.SHIPPED_CASES)
def test_shipped_default_run_matches_reference(amd, name, calls):
    """The reference's shipped run (basin.par 1525 x 1115: a non-power-of-two, non-64-aligned box;
    ocean_run.par: tau = 1 s for 604 steps, model.f90:135-160) on one block and on 2 x 2 blocks
    (odd block sizes, x2 steps), in one ocn_ctx_step call and in 604 calls of one step (the
    reference's own cadence), bitwise against the unmodified reference run."""
    case, m = _full(amd, name)
    try:
        m.init()
        for n in ([case["steps"]] if calls == "one" else [1] * case["steps"]):
            m.step(n, tau=1.0, check_every=1)
        m.synchronize()
        one, x2 = m.onepass_active, m.x2_active
        bad = compare_case(m, case, name)
    finally:
        m.close()
    assert not bad, f"{name} ({calls}): fields differ from the reference: {bad}"
    assert one and x2 == ("_b2x2_" in name), (one, x2)


@pytest.mark.parametrize("name,nranks", [("box2048_b2x2_s4", 4), ("box4096_b4x2_s4", 8), ("box1521x1111_b2x2_s604", 4)])
def test_fullsize_ranks_match_reference(amd, name, nranks):
    """C3 and C4 as BASELINE.json runs them: one block per rank, halos between ranks."""
    case = cases.load_e2e(name)
    models, flips = run_ranks_case(amd, case, nranks)
    try:
        bad = check_ranks(models, case, name)
    finally:
        for m in models:
            m.close()
    assert not bad, f"{name} over {nranks} ranks: fields differ from the reference: {bad}"
    assert all(flips) and all(run_ranks_case.x2)


@pytest.mark.parametrize("name", cases.INIT_CASES)
def test_initial_state_matches_reference(amd, name):
    """ocn_ctx_init_state (init_grid_data + init_ocean_data) vs the reference's step-0 state."""
    case = cases.load_e2e(name)
    m = build_model(amd, case)
    try:
        m.init().synchronize()
        bad = compare_case(m, case, name)
    finally:
        m.close()
    assert not bad, f"{name}: initial fields differ from the reference: {bad}"


@pytest.mark.parametrize("name,nranks", [("bs_topo_b4x2_s60", 8), ("box70x54_topo_b3x2_s20", 6)])
def test_ranks_topography_match_reference(amd, name, nranks):
    """A topography (non-uniform h_r) over loopback ranks: x2 steps with the h_r-reading
    known-constant variant, h_r's second halo ring exchanged from the neighbour ranks every call
    (refresh_hrx), the verdicts voted -- bitwise against the reference run that read the file."""
    case = cases.load_e2e(name)
    models, flips = run_ranks_case(amd, case, nranks)
    try:
        bad = check_ranks(models, case, name)
        hr = {m.onepass_hr for m in models}
    finally:
        for m in models:
            m.close()
    assert not bad, f"{name} over {nranks} ranks: fields differ from the reference: {bad}"
    assert run_ranks_case.x2 == [True] * nranks and hr == {True}, (run_ranks_case.x2, hr)


@pytest.mark.parametrize("tracers,seed", [(0, 600), (0, 601), (2, 600), (2, 601), (1, 602), (1, 603)])
def test_random_rank_sequences_match_oracle(amd, tracers, seed):
    """Seeded random sequences of host entries (calls, tau changes, synchronize, reads, uploads of
    ssh, u, mu, RHSx, hhq_n and h_r, option toggles incl. the overlap level) run by every rank of 4
    loopback ranks (2x2 blocks: the RCCL path's plans, votes and exchanges) on its block, then
    replayed on the oracle: every field of every block, and every read, bitwise."""
    _ranks_sequence(amd, seed, 20, tracers=tracers)


def _ranks_sequence(amd, seed, nops=20, tracers=0, n=120, grid=(2, 2)):
    """The same over loopback ranks (one block per rank, the RCCL path's plans, votes and
    exchanges): every rank runs the same seeded op list on its block; the oracle replays it after."""
    import numpy as np
    from tests.test_gpu_parity import OracleTwin, bits_equal
    rng = np.random.default_rng(seed)
    nranks = grid[0] * grid[1]
    ops = []
    for _ in range(nops):
        op = str(rng.choice(["step", "step", "step", "tau", "sync", "read", "ssh", "hr", "kc", "uv", "mu", "rhs",
                             "hqn", "opt"]))
        if op in ("step", "tau"):
            ops.append((op, int(rng.integers(1, 8)), 0.5 if op == "tau" else 1.0))
        elif op == "read":
            ops.append((op, str(rng.choice(["ssh", "ubrtr", "hhu_n", "hhq", "vort", "sshp", "hhq_n"]))))
        elif op == "opt":
            w = str(rng.choice(["onepass", "tracer_step", "lazy_tail", "flip", "overlap", "co_launch", "x4"]))
            # (overlap: 2, 1 or auto -- the measured choice, ov_begin; x4: off, auto, always)
            ops.append((op, w, int(rng.integers(0, 3 if w in ("overlap", "x4") else 2))))
        elif op == "kc":
            ops.append((op, int(rng.integers(0, 2))))
        else:
            ops.append((op,))
    sw = amd.SWConfig(use_tracers=1, tracer_num=tracers) if tracers else amd.SWConfig()
    models = [amd.OceanModel(amd.box_config(n), sw=sw, par=amd.ParallelConfig(*grid), rank=r, nranks=nranks)
              for r in range(nranks)]
    amd.OceanModel.attach_loopback(models)
    rec = {}

    def smooth(a, amp):
        i, j = np.meshgrid(np.arange(a.shape[0]), np.arange(a.shape[1]), indexing="ij")
        return amp * np.exp(-((i - a.shape[0] / 2) ** 2 + (j - a.shape[1] / 2) ** 2) / (a.size / 40.0))

    fn = {"ssh": ("ssh", lambda a: a + np.where(np.arange(a.size).reshape(a.shape, order="F") == a.size // 2, 1e-3, 0.0)),
          "hr": ("hhq_rest", lambda a: a + smooth(a, 2.0)), "uv": ("ubrtr", lambda a: a + smooth(a, 1.0e-4)),
          "mu": ("mu", lambda a: a + smooth(a, 50.0)), "rhs": ("RHSx", lambda a: a + smooth(a, 1.0e-7)),
          "hqn": ("hhq_n", lambda a: a + 1.0)}

    def body(m):
        m.init().step(2, check_every=1).synchronize()
        for i, op in enumerate(ops):
            if op[0] in ("step", "tau"):
                m.step(op[1], tau=op[2], check_every=1)
            elif op[0] == "sync":
                m.synchronize()
            elif op[0] == "read":
                for b in m.blocks:
                    rec[(i, b.bm, b.bn)] = m.download(b.k, op[1])
            elif op[0] == "kc":
                m.set_known_constants(bool(op[1]))
            elif op[0] == "opt":
                if op[1] == "overlap":
                    m.set_overlap((2, 1, -1)[op[2]])
                elif op[1] == "x4":
                    m.set_x4((0, 1, 3)[op[2]])
                else:
                    {"onepass": m.set_onepass, "tracer_step": m.set_tracer_step, "lazy_tail": m.set_lazy_tail,
                     "flip": m.set_flip, "co_launch": m.set_co_launch}[op[1]](bool(op[2]))
            else:
                nm, f = fn[op[0]]
                for b in m.blocks:
                    a = f(m.download(b.k, nm))
                    m.upload(b.k, nm, a)
                    rec[(i, b.bm, b.bn)] = a
        out = {}
        for b in m.blocks:
            for nm in m.field_names:
                if nm in ("lu1", "rlh_c"):
                    continue
                out[(b.bm, b.bn, nm)] = m.download(b.k, nm)
        return out

    try:
        res = amd.run_ranks(models, body)
    finally:
        for m in models:
            m.close()
    ref = OracleTwin(n, grid, tracers)
    om = ref.om
    ob = {(b.bm, b.bn): k for k, b in enumerate(om.blocks)}
    ref.run(2)
    bad = []
    for i, op in enumerate(ops):
        if op[0] in ("step", "tau"):
            ref.run(op[1], op[2])
        elif op[0] == "read":
            for (bm, bn), k in ob.items():
                if (i, bm, bn) in rec and not bits_equal(rec[(i, bm, bn)], om.f[k][op[1]]):
                    bad.append(f"read {op[1]} ({bm},{bn}) at op {i}")
        elif op[0] in fn:
            nm = fn[op[0]][0]
            for (bm, bn), k in ob.items():
                om.f[k][nm][...] = rec[(i, bm, bn)]
    for out in res:
        for (bm, bn, nm), a in out.items():
            if nm in om.f[ob[(bm, bn)]] and not bits_equal(a, om.f[ob[(bm, bn)]][nm]):
                bad.append(f"({bm},{bn}):{nm}")
    if bad:
        raise AssertionError(f"ranks: fields differ from the oracle: {bad[:12]} ({ops})")




# ---------------------------------------------------------------- watchdog and exchange statistics
def test_watchdog_ends_every_rank_when_one_stalls(amd):
    """One rank of four never reaches its step (it sleeps): every other rank is blocked in the
    exchange's rendezvous.  Their watchdogs (ocn_ctx_set_watchdog, 2 s) end them: each raises OcnError
    with the watchdog's message (the call and the last completed exchange id) well inside the 120 s
    rendezvous bound; the stalled rank, arriving later, fails too -- no rank hangs."""
    import time
    n, T, stalled = 96, 2.0, 2
    ms = [amd.OceanModel(amd.box_config(n), par=amd.ParallelConfig(2, 2), rank=r, nranks=4) for r in range(4)]
    amd.OceanModel.attach_loopback(ms)
    try:
        def init(m):
            m.set_watchdog(T)
            m.init()
            m.step(3, check_every=1).synchronize()
        amd.run_ranks(ms, init)

        def body(m):
            if m.rank == stalled:
                time.sleep(3 * T)
            t0 = time.perf_counter()
            try:
                m.step(5, check_every=1)
                m.synchronize()
            except amd.OcnError as e:
                return str(e), time.perf_counter() - t0
            return None, time.perf_counter() - t0
        out = amd.run_ranks(ms, body)
        info = ms[0].comm_info()
    finally:
        for m in ms:
            m.close()
    for r, (msg, dt) in enumerate(out):
        assert msg is not None, f"rank {r} did not fail"
        if r != stalled:   # its own watchdog's message, or the group a peer's watchdog failed
            assert "ocn watchdog: rank" in msg or "loopback transport" in msg, msg
            assert dt < T + 8.0, (r, dt)
    fired = [msg for r, (msg, _) in enumerate(out) if r != stalled and "ocn watchdog: rank" in msg]
    assert fired and all("last completed exchange id" in m for m in fired), out
    assert info["transport"] == "loopback" and info["exchanges"] > 0 and info["exchanges_done"] >= 0, info


def test_exchange_stats_and_comm_info(amd):
    """With stage timing on, every exchange with a remote peer is one OCN_TIMER_EXCHANGE record (its
    count = the exchanges comm_info counts), and each overlapped x2 step one OCN_TIMER_EXPOSED record
    -- what bench.py's `rccl` object reports for an N-GPU run; results stay bitwise."""
    case = cases.load_e2e("box70x54_b3x2_s20")
    models = [build_model(amd, case, rank=r, nranks=6) for r in range(6)]
    amd.OceanModel.attach_loopback(models)

    def body(m):
        m.init()
        m.step(2, tau=1.0, check_every=1).synchronize()
        m.set_stage_timing(True)
        m.stage_times()
        x0 = m.comm_info()["exchanges"]
        m.step(18, tau=1.0, check_every=1)
        m.synchronize()
        st = m.stage_stats()
        return st, m.comm_info()["exchanges"] - x0, m.x2_active, m.overlap_level
    try:
        out = amd.run_ranks(models, body)
        bad = check_ranks(models, case, "box70x54_b3x2_s20")
    finally:
        for m in models:
            m.close()
    assert not bad, bad
    for st, groups, x2, level in out:
        assert x2 and level == 2, (x2, level)
        ex = st.get("exchange")
        # (17 one-pass steps: 8 pairs of x2 steps with one 4-deep exchange each + 1 x2 step, then the last
        # step's exchanges, the h_r refresh and the vote's two compare-mode exchanges)
        assert ex and ex[1] == groups and groups >= 10 and ex[2] >= ex[0] / ex[1] > 0, (ex, groups)
        # (overlap auto: the measured choice runs one pair of the call in sequence -- ocn_ctx.hip ov_begin)
        assert "exposed" in st and st["exposed"][1] >= 8, st.get("exposed")
