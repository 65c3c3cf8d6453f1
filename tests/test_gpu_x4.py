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
                                        ("box2048_b2x2_s4", [1, 3]), ("box4096_b4x2_s4", [1, 3])])
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
    bad, used = _run_blocks(amd, name, calls, overlap=overlap)
    assert not bad, f"{name} {calls}: fields differ from the reference: {bad}"
    assert any(used), used


def test_x4_off_is_the_x2_path(amd):
    bad, used = _run_blocks(amd, "box70x54_b3x2_s20", [2, 18], x4=False)
    assert not bad and not any(used), (bad, used)


@pytest.mark.parametrize("name,nranks,calls", [("box70x54_b3x2_s20", 6, [2, 18]), ("bs_b4x2_s60", 8, [2, 58]),
                                               ("box40x32_b2x2_s5", 4, [2, 3]), ("box70x54_b3x2_s20", 6, [2, 7, 3, 8]),
                                               ("bs_b4x2_tr_s60", 8, [2, 58]), ("box70x54_b3x2_tr_s20", 6, [2, 7, 3, 8])])
def test_x4_ranks_match_reference(amd, name, nranks, calls):
    """One block per loopback rank: the exchange is the RCCL path's (device pack / unpack, per-peer
    messages 4 deep), the decision every rank's (the vote's x4 word), every field bitwise.  (With a
    communicator a call runs pairs after a call of 2 or more steps has voted with the verdict known:
    the full-size C3 / C4 fixtures, 4 steps, are too short for that -- their blocks run the pairs in one
    process above, and over ranks in the random rank sequences.)"""
    case = cases.load_e2e(name)
    models = [build_model(amd, case, rank=r, nranks=nranks) for r in range(nranks)]
    amd.OceanModel.attach_loopback(models)

    def body(m):
        m.init()
        m.step(calls[0], tau=1.0, check_every=1)
        m.synchronize()
        used = []
        for n in calls[1:]:
            m.step(n, tau=1.0, check_every=1)
            used.append(m.x4_active)
        m.synchronize()
        return used

    try:
        used = amd.run_ranks(models, body)
        bad = []
        for m in models:
            bad += compare_case(m, case, name, whole=False)
    finally:
        for m in models:
            m.close()
    assert not bad, f"{name} over {nranks} ranks {calls}: fields differ from the reference: {bad}"
    assert all(any(u) for u in used) and all(u == used[0] for u in used), used


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
