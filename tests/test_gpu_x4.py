"""GPU parity of the pairs of x2 steps (OCN_OPT_X4, ocn_ctx.hip one_step_x4): blocks with halo
exchanges run two one-pass steps per launch with ONE exchange of the state four points deep per two
steps -- the launch's first step also updates the two halo rings neighbour blocks own, as they do --
bitwise against the reference fixtures (its step exchanges 15 fields at 7 sync points per step:
shared/mpp/syncborder_block2D_gen_all.fi:100-129 after every stage, core/kernel_interface.f90:105-117).

The pairs run the known-constant variant the host has chosen, so every run makes a first short call
and a synchronize() (the check's verdict reaches the host), then the rest.  One process with several
blocks (local copies, the lazy call tail: pairs across calls) and loopback ranks (the RCCL path's
plans, exchanges and vote; one call per run after the first).  Tolerance: none.
"""
import pytest

from tests.golden import cases
from tests.test_gpu_parity import build_model, compare_case

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def amd():
    import ocean_model_arch_amd as amd
    amd.lib()
    return amd


def _run_blocks(amd, name, calls, x4=True, overlap=None):
    case = cases.load_e2e(name)
    m = build_model(amd, case, overlap=overlap).set_x4(x4).init()
    used = []
    try:
        m.step(calls[0], tau=1.0, check_every=1)
        m.synchronize()   # the known-constant verdict reaches the host
        for n in calls[1:]:
            m.step(n, tau=1.0, check_every=1)
            used.append(m.x4_active)
        m.synchronize()
        bad = compare_case(m, case, name)
    finally:
        m.close()
    return bad, used


@pytest.mark.parametrize("name,calls", [("box70x54_b3x2_s20", [2, 18]), ("box70x54_b3x2_s20", [2, 5, 1, 1, 3, 8]),
                                        ("box70x54_b3x2_s20", [1] * 20), ("bs_b4x2_s60", [2, 58]),
                                        ("bs_b4x2_s60", [3, 1, 1, 1, 54]), ("box40x32_b2x2_s5", [2, 3]),
                                        ("box2048_b2x2_s4", [1, 3]), ("box4096_b4x2_s4", [1, 3]),
                                        ("box2048_b2x2_s10", [2, 8]), ("box4096_b4x2_s12", [2, 10])])
def test_x4_blocks_match_reference(amd, name, calls):
    """Several blocks in one process (local halo copies): pairs of x2 steps inside calls and across
    calls (the reference's 1-step cadence: a pair every second call), every field bitwise."""
    bad, used = _run_blocks(amd, name, calls)
    assert not bad, f"{name} {calls}: fields differ from the reference: {bad}"
    assert any(used), used


@pytest.mark.parametrize("name,calls", [("box70x54_b3x2_s20", [2, 18]), ("bs_b4x2_s60", [2, 5, 1, 52]),
                                        ("box4096_b4x2_s4", [1, 3])])
def test_x4_overlapped_blocks_match_reference(amd, name, calls):
    """OCN_OPT_OVERLAP 2 (the default with remote peers): each block's inner pair on the compute stream
    beside the 4-deep exchange, then the bands around it on the comm stream -- bitwise."""
    bad, used = _run_blocks(amd, name, calls, overlap=2)
    assert not bad, f"{name} {calls}: fields differ from the reference: {bad}"
    assert any(used), used


@pytest.mark.parametrize("name,calls", [("box70x54_b3x2_tr_s20", [2, 18]), ("box70x54_b3x2_tr_s20", [2, 5, 1, 1, 3, 8]),
                                        ("box70x54_b3x2_tr_s20", [1] * 20), ("bs_b4x2_tr_s60", [2, 58]),
                                        ("bs_b4x2_tr_s60", [3, 1, 1, 1, 54]), ("bs_b4x2_tr_s604", [2, 602])])
@pytest.mark.parametrize("overlap", [None, 2])
def test_x4_tracer_blocks_match_reference(amd, name, calls, overlap):
    """Tracer runs with x4 pairs (one_step_x4 with tracer steps): the exchange carries the tracers 2
    deep, the pending tracer step runs over the interior and the halo ring neighbours own (co-launched
    with the pair), the pair's producers write the first step's state for the second tracer step --
    two SW steps and two tracer steps per exchange, every field bitwise (control/tracer.f90:33-62 after
    each step, leapfrog_tracer.f90:13-170)."""
    bad, used = _run_blocks(amd, name, calls, x4=3, overlap=overlap)
    assert not bad, f"{name} {calls}: fields differ from the reference: {bad}"
    assert any(used), used


def test_x4_tracer_runs_in_one_process_default_to_x2(amd):
    """OCN_OPT_X4 auto (1): a tracer run whose exchanges are all local copies keeps the x2 steps (the
    pair's second tracer step costs a launch more than the exchange it saves), bitwise."""
    bad, used = _run_blocks(amd, "box70x54_b3x2_tr_s20", [2, 18])
    assert not bad and not any(used), (bad, used)


@pytest.mark.parametrize("name,calls", [("box70x54_topo_b3x2_s20", [2, 18]), ("box70x54_topo_b3x2_s20", [2, 5, 1, 1, 3, 8]),
                                        ("bs_topo_b4x2_s60", [2, 58])])
@pytest.mark.parametrize("overlap", [None, 2])
def test_x4_topography_blocks_match_reference(amd, name, calls, overlap):
    """A rest depth read from a topography file (control/init_data.f90:115-120): the pairs run the
    h_r-read variant (OCN_KC_KNOWN_HR) with h_r's copy exchanged four rings deep (refresh_hrx) -- every
    field bitwise."""
    bad, used = _run_blocks(amd, name, calls, overlap=overlap)
    assert not bad, f"{name} {calls}: fields differ from the reference: {bad}"
    assert any(used), used


def test_x4_off_is_the_x2_path(amd):
    bad, used = _run_blocks(amd, "box70x54_b3x2_s20", [2, 18], x4=False)
    assert not bad and not any(used), (bad, used)


def _run_ranks(amd, name, nranks, calls, overlap=None, co=None):
    """One block per loopback rank, the bench's cadence (a first call, a synchronize: the
    known-constant verdict reaches every host, so the next call's vote can choose the pairs), then
    the remaining calls, complete() and a synchronize.  Returns (differing fields, per rank the
    x4_active of each later call, per rank whether a later call co-launched a march and a tracer step)."""
    case = cases.load_e2e(name)
    models = [build_model(amd, case, rank=r, nranks=nranks, overlap=overlap) for r in range(nranks)]
    if co is not None:
        for m in models:
            m.set_co_launch(co)
    amd.OceanModel.attach_loopback(models)

    def body(m):
        m.init()
        m.step(calls[0], tau=1.0, check_every=1)
        m.synchronize()
        used, co_used = [], False
        for n in calls[1:]:
            m.step(n, tau=1.0, check_every=1)
            used.append(m.x4_active)
            co_used = co_used or m.co_launched
        m.complete()
        m.synchronize()
        return used, co_used

    try:
        res = amd.run_ranks(models, body)
        bad = []
        for m in models:
            bad += compare_case(m, case, name, whole=False)
    finally:
        for m in models:
            m.close()
    return bad, [r[0] for r in res], [r[1] for r in res]


@pytest.mark.parametrize("name,nranks,calls", [("box70x54_b3x2_s20", 6, [2, 18]), ("bs_b4x2_s60", 8, [2, 58]),
                                               ("box40x32_b2x2_s5", 4, [2, 3]), ("box70x54_b3x2_s20", 6, [2, 7, 3, 8]),
                                               ("bs_b4x2_tr_s60", 8, [2, 58]), ("box70x54_b3x2_tr_s20", 6, [2, 7, 3, 8]),
                                               ("box70x54_topo_b3x2_s20", 6, [2, 18]), ("bs_topo_b4x2_s60", 8, [2, 58])])
def test_x4_ranks_match_reference(amd, name, nranks, calls):
    """One block per loopback rank: the exchange is the RCCL path's (device pack / unpack, per-peer
    messages 4 deep), the decision every rank's (the vote's x4 word), every field bitwise.  (With a
    communicator a call runs pairs after a call of 2 or more steps has voted with the verdict known.)"""
    bad, used, _ = _run_ranks(amd, name, nranks, calls)
    assert not bad, f"{name} over {nranks} ranks {calls}: fields differ from the reference: {bad}"
    assert all(any(u) for u in used) and all(u == used[0] for u in used), used


@pytest.mark.parametrize("overlap", [1, 2])
@pytest.mark.parametrize("name,nranks,calls", [("box2048_b2x2_s10", 4, [2, 8]), ("box4096_b4x2_s12", 8, [2, 10])])
def test_x4_fullsize_ranks_match_reference(amd, name, nranks, calls, overlap):
    """BASELINE configs 3 and 4 at full size, one block per loopback rank, exactly as a multi-GPU bench
    run executes them: the warm-up call, then one long call of x4 pairs (every rank asserts it ran
    them), complete(); overlap 2 = the inner pair beside the 4-deep exchange then the bands (the
    default with peers), overlap 1 = exchange then the whole pair.  Every field of every block
    bitwise against the reference's 4 / 8-block run (shared/mpp/syncborder_block2D_gen_all.fi:100-129,
    core/kernel_interface.f90:105-117)."""
    bad, used, _ = _run_ranks(amd, name, nranks, calls, overlap=overlap)
    assert not bad, f"{name} over {nranks} ranks, overlap {overlap}: fields differ from the reference: {bad}"
    assert all(all(u) for u in used), used


@pytest.mark.parametrize("overlap", [1, 2])
@pytest.mark.parametrize("name,calls", [("bs_b4x2_tr_s60", [2, 58]), ("bs_b4x2_tr_s604", [2, 602])])
def test_x4_tracer_ranks_co_launch_match_reference(amd, name, calls, overlap):
    """Config 5 (Black Sea + tracer, 8 blocks) over 8 loopback ranks with x4 pairs and the tracer steps:
    the tracers exchanged 2 deep with the state, the pending tracer step co-launched with the pair
    (overlap 2: in the bands' launch after the exchange; overlap 1: with the whole pair) -- every rank
    ran the pairs and the co-launch, every field bitwise (control/tracer.f90:33-62,
    interface/tracer/tracer_interface.f90:52-98)."""
    bad, used, co = _run_ranks(amd, name, 8, calls, overlap=overlap, co=True)
    assert not bad, f"{name} over 8 ranks, overlap {overlap}: fields differ from the reference: {bad}"
    assert all(all(u) for u in used), used
    assert all(co), co


def test_x4_counts_blowup_like_single_launches(amd):
    """check_ssh_err (vel_ssh.f90:40-67) in the pairs: each point counted once per step -- a producer
    counts its workgroup's interior points, never the halo points it updates for a neighbour: the same
    count as the x2 single launches."""
    import numpy as np
    msgs = []
    for x4 in (True, False):
        m = amd.OceanModel(amd.box_config(120), par=amd.ParallelConfig(3, 2)).set_x4(x4).init()
        m.step(2, check_every=1).synchronize()
        for b in m.blocks:   # a hot patch straddling the block boundaries
            s = m.download(b.k, "ssh")
            i = np.arange(b.bnd_x1, b.bnd_x2 + 1)[:, None]
            j = np.arange(b.bnd_y1, b.bnd_y2 + 1)[None, :]
            s[(abs(i - 42) < 9) & (abs(j - 62) < 9)] = 2.0e4
            for nm in ("ssh", "sshn", "sshp"):
                m.upload(b.k, nm, s)
        m.step(2, check_every=0).synchronize()   # the re-check's verdict reaches the host
        with pytest.raises(amd.OcnError) as e:
            m.step(5, check_every=1)
            used = m.x4_active
            m.synchronize()
        msgs.append(str(e.value))
        m.close()
        assert used == x4
    assert msgs[0] == msgs[1], msgs


@pytest.mark.parametrize("delay_us", [0, 600])
def test_overlap_choice_is_measured_and_voted(amd, delay_us):
    """OCN_OPT_OVERLAP auto with peers on other ranks (ocn_ctx.hip ov_begin): one x2 step in sequence
    and the next overlapped, each timed; the next call's vote max-reduces both times and every rank
    keeps the faster form -- every rank decides, all the same, the level is the one the compared
    times pick, and an injected 600 us wait before each exchange (a slow link) is in the measured
    sequential step.  (Which form wins is not asserted: four loopback ranks share one GPU, and their
    step times carry the other ranks' work and the transport's cross-rank waits.)  Either way every
    field bitwise against the reference's 4-block run (core/kernel_interface.f90:105-117 is the
    reference's own overlap mode)."""
    name, calls = "box2048_b2x2_s10", [4, 2, 4]
    case = cases.load_e2e(name)
    models = [build_model(amd, case, rank=r, nranks=4) for r in range(4)]
    for m in models:
        m.set_exchange_delay(delay_us)
    amd.OceanModel.attach_loopback(models)

    def body(m):
        m.init()
        infos = []
        for n in calls:
            m.step(n, tau=1.0, check_every=1)
            infos.append(m.overlap_info())
        m.complete()
        m.synchronize()
        return infos

    try:
        infos = amd.run_ranks(models, body)
        bad = []
        for m in models:
            bad += compare_case(m, case, name, whole=False)
    finally:
        for m in models:
            m.close()
    assert not bad, f"{name} delay {delay_us}: fields differ from the reference: {bad}"
    last = [i[-1] for i in infos]
    print("overlap", delay_us, last)
    assert all(i["state"] == 3 for i in last), last
    assert len({i["level"] for i in last}) == 1 and len({(i["seq_ms"], i["overlapped_ms"]) for i in last}) == 1, last
    i0 = last[0]
    assert i0["level"] == (2 if i0["overlapped_ms"] < i0["seq_ms"] else 1), last
    if delay_us:
        assert i0["seq_ms"] > delay_us * 1e-3 and i0["overlapped_ms"] > 0.0, last
