"""GPU parity of the multi-step launch (OCN_OPT_MULTI, sw_kernels.hip k_march_multi): the one-pass
steps of a call of a small single block -- the Black Sea basin as one block, config 1 on the GPU --
in ONE launch with a grid-wide barrier between the steps, bitwise against the reference
fixtures (model.f90:135-160 runs expl_shallow_water once per step; the launch runs the same steps).

A multi-step launch needs an open sequence (OCN_OPT_LAZY_TAIL: the call continues a one-pass sequence)
and the variant chosen on the host, so the runs below make a first short call and a synchronize()
first.  Tolerance: none (fp64, the reference's order).
"""
import pytest

from tests.golden import cases
from tests.test_gpu_parity import OracleTwin, build_model, compare_case

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def amd():
    import ocean_model_arch_amd as amd
    amd.lib()
    return amd


def _run(amd, name, calls, multi=True, timing=False):
    case = cases.load_e2e(name)
    m = build_model(amd, case).set_multi(multi).init()
    used, times = [], {}
    try:
        m.step(calls[0], tau=1.0, check_every=1)
        m.synchronize()   # the known-constant verdict reaches the host
        if timing:
            m.set_stage_timing(True)
            m.stage_times()
        for n in calls[1:]:
            m.step(n, tau=1.0, check_every=1)
            used.append(m.multi_active)
        if timing:
            times = m.stage_times()
        bad = compare_case(m, case, name)
    finally:
        m.close()
    return bad, used, times


@pytest.mark.parametrize("name,calls", [("bs_b1x1_s60", [2, 58]), ("bs_b1x1_s60", [1, 7, 1, 2, 49]),
                                        ("bs_b1x1_s604", [4, 300, 300]), ("box70x54_b1x1_s20", [3, 17]),
                                        ("box48x40_cart_s10", [2, 3, 5]), ("box70x54_topo_b1x1_s20", [2, 18])])
def test_multi_steps_match_reference(amd, name, calls):
    bad, used, times = _run(amd, name, calls, timing=True)
    assert not bad, f"{name} {calls}: fields differ from the reference: {bad}"
    assert used == [n >= 2 for n in calls[1:]], used
    assert times.get("onepass_multi", (0, 0))[1] == sum(n >= 2 for n in calls[1:]), times


def test_multi_off_is_per_step(amd):
    bad, used, times = _run(amd, "bs_b1x1_s60", [2, 58], multi=False, timing=True)
    assert not bad and used == [False] and "onepass_multi" not in times, (bad, used, times)


def test_multi_counts_blowup_like_single_launches(amd):
    """check_ssh_err_kernel (vel_ssh.f90:40-67) inside the multi-step launch: every step counts its
    points, as single launches do -- the same error message (count) either way."""
    msgs = []
    for multi in (True, False):
        m = amd.OceanModel(amd.box_config(100)).set_multi(multi).init()
        m.step(2, check_every=1).synchronize()
        s = m.download(0, "ssh")
        s[30:60, 40:70] = 2.0e4
        for nm in ("ssh", "sshn", "sshp"):
            m.upload(0, nm, s)
        m.step(3, check_every=0).synchronize()   # the re-check's verdict reaches the host
        with pytest.raises(amd.OcnError) as e:
            m.step(4, check_every=1).synchronize()
        used = m.multi_active
        msgs.append(str(e.value))
        m.close()
        assert used == multi
    assert msgs[0] == msgs[1], msgs


def test_multi_with_uploads_and_forcing_matches_oracle(amd):
    """The multi-step launch in its general variant (a forcing on the sea: RHSx read) and across an
    upload between calls, against the oracle given the same uploads."""
    import numpy as np
    n = 120
    m = amd.OceanModel(amd.box_config(n)).init()
    ref = OracleTwin(n)
    b = m.blocks[0]
    m.step(2, check_every=1).synchronize()
    ref.run(2)
    a = np.zeros(b.shape)
    a[m.download(0, "lu") > 0.5] = 3e-7
    m.upload(0, "RHSx", a)
    ref.upload(b, "RHSx", a)
    m.step(2, check_every=1).synchronize()
    m.step(9, check_every=1)
    used = m.multi_active
    m.synchronize()
    ref.run(11)
    bad = ref.mismatches(m)
    zero = m.onepass_zero
    m.close()
    assert used and not zero, (used, zero)
    assert not bad, f"multi-step launch (general variant) differs from the oracle: {bad}"


# ---------------------------------------------------------------- tracer steps (OCN_OPT_TRACER_STEP)
@pytest.mark.parametrize("calls", ["one", "split", "per_step"])
@pytest.mark.parametrize("name", ["box40x32_tr2_s5", "box70x54_b3x2_tr_s20", "bs_b4x2_tr_s60", "bs_b4x2_tr_s604"])
def test_tracer_steps_match_reference(amd, name, calls):
    """Tracer runs with one-pass steps: expl_tracer (control/tracer.f90:33-62) of each step as one
    launch per tracer (sw_stencils.h TracerStep: hh_init's depths formed from the state), run with the
    next step after its exchange (x2 steps carry the tracers one point deep); the last step the
    standard stages -- bitwise against the reference, in one call, split calls and 1-step calls."""
    case = cases.load_e2e(name)
    steps = case["steps"]
    plan = {"one": [steps], "split": [2, steps - 5, 3] if steps > 5 else [2, steps - 2],
            "per_step": [1] * steps}[calls]
    m = build_model(amd, case).init()
    used = []
    try:
        for n in plan:
            m.step(n, tau=1.0, check_every=1)
            used.append(m.tracer_step_active)
        m.synchronize()
        bad = compare_case(m, case, name)
        x2 = m.x2_active
    finally:
        m.close()
    assert not bad, f"{name} ({calls}): fields differ from the reference: {bad}"
    assert used[0], used
    if "tr2" not in name:   # several blocks: the x2 steps carry the tracers
        assert x2, name


@pytest.mark.parametrize("co", [True, False])
@pytest.mark.parametrize("name", ["box70x54_b3x2_tr_s20", "bs_b4x2_tr_s60"])
def test_tracer_step_co_launch_matches_reference(amd, name, co):
    """OCN_OPT_CO_LAUNCH (ocn_ctx.hip one_step_x2, sw_kernels.hip k_march_tracer_b): each x2 step's march
    and the previous state's tracer step as one launch (on), or two on two streams (off) -- bitwise
    against the reference either way; the co-launch runs once the known-constant verdict is on the
    host (a first call and a synchronize)."""
    case = cases.load_e2e(name)
    steps = case["steps"]
    m = build_model(amd, case).set_co_launch(co).init()
    used = []
    try:
        m.step(2, tau=1.0, check_every=1).synchronize()
        for n in (steps - 5, 1, 2):
            m.step(n, tau=1.0, check_every=1)
            used.append(m.co_launched)
        m.synchronize()
        bad = compare_case(m, case, name)
    finally:
        m.close()
    assert not bad, f"{name} (co-launch {co}): fields differ from the reference: {bad}"
    assert any(used) == co, used


def test_tracer_steps_off_is_the_role_flip_path(amd):
    case = cases.load_e2e("bs_b4x2_tr_s60")
    m = build_model(amd, case).set_tracer_step(False).init()
    try:
        m.step(case["steps"], tau=1.0, check_every=1).synchronize()
        bad = compare_case(m, case, "bs_b4x2_tr_s60")
        used, one = m.tracer_step_active, m.onepass_active
    finally:
        m.close()
    assert not bad and not used and not one, (bad, used, one)


def test_tracer_steps_launches(amd):
    """Config 5's layout on one GPU (Black Sea + tracer, 4x2 blocks): x2 steps with the tracer steps,
    block-batched -- a few launches per step instead of the role-flip path's 22."""
    case = cases.load_e2e("bs_b4x2_tr_s60")
    m = build_model(amd, case).init()
    try:
        m.step(4, tau=1.0, check_every=1).synchronize()
        n0 = amd._lib.launch_count()
        m.step(40, tau=1.0, check_every=1)
        per_step = (amd._lib.launch_count() - n0) / 40
        used, x2 = m.tracer_step_active, m.x2_active
        m.synchronize()
    finally:
        m.close()
    assert used and x2, (used, x2)
    assert per_step <= 4, per_step   # (co-launched march + tracer step: 3.3 -> ~2.3)


@pytest.mark.parametrize("path", ["tracer_steps", "role_flip", "fused"])
def test_tracers_after_rest_depth_upload_match_oracle(amd, path):
    """tran_diff_tracer reads hhq_n, which every hh_init sets to h_r (depth.f90:14-99) -- after an
    upload of a non-uniform h_r the role-flip steps' fused hh_init + A (which does not store it)
    must not leave the tracers the old one (ocn_ctx.hip expl_tracer, hqn_stale): calls of 2 and 3
    steps after the upload, every field against the oracle given the same upload."""
    import numpy as np
    from tests.test_gpu_parity import OracleTwin
    n = 100
    sw = amd.SWConfig(use_tracers=1, tracer_num=2)
    m = amd.OceanModel(amd.box_config(n), sw=sw)
    if path != "tracer_steps":
        m.set_tracer_step(False)
    if path == "fused":
        m.set_onepass(False)
    m.init()
    ref = OracleTwin(n, (1, 1), 2)
    try:
        m.step(2, check_every=1).synchronize()
        ref.run(2)
        h = m.download(0, "hhq_rest")
        i, j = np.meshgrid(np.arange(h.shape[0]), np.arange(h.shape[1]), indexing="ij")
        h = h + 2.0 * np.exp(-((i - 52.0) ** 2 + (j - 40.0) ** 2) / 300.0)
        m.upload(0, "hhq_rest", h)
        ref.upload(m.blocks[0], "hhq_rest", h)
        for k in (2, 3):
            m.step(k, check_every=1)
            ref.run(k)
        bad = ref.mismatches(m)
    finally:
        m.close()
    assert not bad, f"{path}: fields differ from the oracle: {bad}"


def test_tracer_steps_after_inconsistent_mu_upload_match_oracle(amd):
    """Tracer steps form tran_diff_fluxes' fluxes at the halo points neighbour blocks own (the
    reference computes them there and exchanges them, tracer.f90:33-62) from mu at those points: a
    per-block mu whose halos are not the neighbours' values (an upload) must not be used -- the
    x2 check covers mu's first halo ring for tracer runs (ocn_ctx.hip check_coherence), and the
    run takes the role-flip path: every field against the oracle, in calls of 2."""
    import numpy as np
    from tests.test_gpu_parity import OracleTwin
    n, blocks = 120, (3, 2)
    m = amd.OceanModel(amd.box_config(n), sw=amd.SWConfig(use_tracers=1, tracer_num=2),
                       par=amd.ParallelConfig(*blocks)).init()
    ref = OracleTwin(n, blocks, 2)
    try:
        m.step(2, check_every=1).synchronize()
        ref.run(2)
        for b in m.blocks:   # a bump per block, centred in it: the halos differ from the neighbours
            a = m.download(b.k, "mu")
            i, j = np.meshgrid(np.arange(a.shape[0]), np.arange(a.shape[1]), indexing="ij")
            a = a + 50.0 * np.exp(-((i - a.shape[0] / 2) ** 2 + (j - a.shape[1] / 2) ** 2) / (a.size / 40.0))
            m.upload(b.k, "mu", a)
            ref.upload(b, "mu", a)
        for k in (2, 2, 3):
            m.step(k, check_every=1)
            ref.run(k)
        bad = ref.mismatches(m)
    finally:
        m.close()
    assert not bad, f"fields differ from the oracle: {bad}"


# ---------------------------------------------------------------- advisor regressions (round 4)
def test_multi_barrier_timeout_reports_and_recovers(amd):
    """The multi-step launch's grid barrier is bounded (sw_kernels.hip grid_barrier): forced to give up
    after one poll (OCN_OPT_MULTI_SPIN 1), every workgroup ends, synchronize() reports OCN_ERR_HIP once
    (no hang), and init() starts over: the next run is bitwise the oracle's."""
    n = 100
    m = amd.OceanModel(amd.box_config(n)).init()
    try:
        m.set_multi_spin(1)   # (an option change closes an open sequence: set it first)
        m.step(2, check_every=1).synchronize()   # the verdict reaches the host: the next call is multi
        m.step(12, check_every=1)
        used = m.multi_active
        with pytest.raises(amd.OcnError, match="grid barrier timed out"):
            m.synchronize()
        m.synchronize()   # reported once
        m.set_multi_spin(1 << 20)
        m.init()
        ref = OracleTwin(n)
        m.step(2, check_every=1).synchronize()
        m.step(9, check_every=1)
        used2 = m.multi_active
        m.synchronize()
        ref.run(11)
        bad = ref.mismatches(m)
    finally:
        m.close()
    assert used and used2, (used, used2)
    assert not bad, f"after the timeout and init(): fields differ from the oracle: {bad}"


def test_tracer_step_toggle_revotes_mu_halo(amd):
    """A cached coherence vote taken with tracer steps off does not check mu's halo (only tracer steps
    read it at neighbour-owned points): turning tracer steps on must vote again -- a per-block mu upload
    between them, then every field against the oracle."""
    import numpy as np
    n, blocks = 120, (3, 2)
    m = amd.OceanModel(amd.box_config(n), sw=amd.SWConfig(use_tracers=1, tracer_num=1),
                       par=amd.ParallelConfig(*blocks)).init()
    ref = OracleTwin(n, blocks, 1)
    try:
        m.set_tracer_step(False)
        m.step(2, check_every=1).synchronize()
        ref.run(2)
        for b in m.blocks:
            a = m.download(b.k, "mu")
            i, j = np.meshgrid(np.arange(a.shape[0]), np.arange(a.shape[1]), indexing="ij")
            a = a + 50.0 * np.exp(-((i - a.shape[0] / 2) ** 2 + (j - a.shape[1] / 2) ** 2) / (a.size / 40.0))
            m.upload(b.k, "mu", a)
            ref.upload(b, "mu", a)
        m.step(3, check_every=1).synchronize()   # a vote with tracer steps off (cached)
        ref.run(3)
        m.set_tracer_step(True)
        for k in (3, 2):
            m.step(k, check_every=1)
            ref.run(k)
        bad = ref.mismatches(m)
    finally:
        m.close()
    assert not bad, f"fields differ from the oracle: {bad}"


def test_tracer_steps_with_comm_and_standard_last_step(amd):
    """One block, a (loopback, one-rank) communicator attached and OCN_OPT_ONEPASS_LAST 0: the call's
    last step is a standard step, which does not run a pending tracer step -- so tracer steps are not
    used there, and no step's tracer update is dropped (every field against the oracle)."""
    n = 80
    m = amd.OceanModel(amd.box_config(n), sw=amd.SWConfig(use_tracers=1, tracer_num=1))
    amd.OceanModel.attach_loopback([m])
    m.init()
    ref = OracleTwin(n, (1, 1), 1)
    try:
        m.set_onepass_last(False)
        for k in (3, 4, 1, 2):
            m.step(k, check_every=1)
            ref.run(k)
        m.synchronize()
        bad = ref.mismatches(m)
    finally:
        m.close()
    assert not bad, f"fields differ from the oracle: {bad}"


def test_step_before_init_keeps_the_communicator(amd):
    """A step before init_state is a usage error raised before any collective (OCN_ERR_STATE): it
    must not abort the communicator -- the model still exchanges after init()."""
    n = 64
    ms = [amd.OceanModel(amd.box_config(n), par=amd.ParallelConfig(2, 1), rank=r, nranks=2) for r in range(2)]
    amd.OceanModel.attach_loopback(ms)
    try:
        with pytest.raises(amd.OcnError, match="init_state"):
            ms[0].step(1)

        def body(m):
            m.init()
            m.step(4, check_every=1).synchronize()
        amd.run_ranks(ms, body)
        ref = OracleTwin(n, (2, 1))
        ref.run(4)
        bad = [x for mm in ms for x in ref.mismatches(mm, ["ssh", "ubrtr", "vbrtr", "hhu"])]
    finally:
        for mm in ms:
            mm.close()
    assert not bad, f"fields differ from the oracle: {bad}"
