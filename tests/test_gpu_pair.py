"""GPU parity of the two-step launches (OCN_OPT_PAIR, sw_kernels.hip MarchStep PAIR): two one-pass
steps per launch on one block -- the producer waves' first step kept in LDS, the consumer waves'
second step written where a single step writes -- bitwise against the reference fixtures.

A pair needs the variant chosen on the host -- the known-constant verdict: a synchronising call hands it over (and, without
one, its copy in pinned memory once its event has completed), so the runs below make a first short
call, a synchronize(), then the rest -- the lazy tail keeps the one-pass sequence open across calls,
a call runs two steps per launch while 3 or more are pending and leaves the last 1 or 2 to the next
call (a synchronize() runs them, a read of the fields runs them as the last steps).  Tolerance: none (fp64, the reference's order).
"""
import pytest

from tests.golden import cases
from tests.test_gpu_parity import OracleTwin, bits_equal, build_model, compare_case

pytestmark = pytest.mark.gpu

# single-block cases with every SW term on (the one-pass step's conditions)
PAIR_CASES = ["box70x54_b1x1_s20", "box48x40_cart_s10", "bs_b1x1_s60", "bs_b1x1_s604", "box70x54_topo_b1x1_s20",
              "box1024_b1x1_s10", "box4096_b1x1_s6", "box1521x1111_b1x1_s604"]


@pytest.fixture(scope="module")
def amd():
    import ocean_model_arch_amd as amd
    amd.lib()
    return amd


def _splits(steps, pattern):
    if pattern == "2+rest":
        return [2, steps - 2]
    if pattern == "1,odd,even":   # pairs over odd and even call lengths, calls of 1 between
        a = max(1, (steps - 2) // 2) | 1
        return [1, a, 1, steps - a - 2] if steps - a - 2 > 0 else [1, steps - 1]
    raise ValueError(pattern)


@pytest.mark.parametrize("graph", [False, True], ids=["stream", "graph"])
@pytest.mark.parametrize("pattern", ["2+rest", "1,odd,even"])
@pytest.mark.parametrize("name", PAIR_CASES)
def test_pair_steps_match_reference(amd, name, pattern, graph):
    case = cases.load_e2e(name)
    if graph and case["steps"] > 100:
        pytest.skip("long runs: stream only")
    m = build_model(amd, case, graph=graph).set_pair(2).init()
    used = []
    try:
        for i, n in enumerate(_splits(case["steps"], pattern)):
            m.step(n, tau=1.0, check_every=1)
            if i == 0:
                m.synchronize()   # the known-constant verdict reaches the host
            used.append(m.pair_active)
        m.synchronize()
        bad = compare_case(m, case, name)
        one = m.onepass_active
    finally:
        m.close()
    assert not bad, f"{name} ({pattern}, graph {graph}): fields differ from the reference: {bad}"
    assert one
    # after the verdict a call runs pairs while 3 or more steps are pending (the 1 or 2 it defers
    # from the last call first) and defers the last 1 or 2
    calls, want, d = _splits(case["steps"], pattern), [], 0
    for i, n in enumerate(calls):
        t = d + n
        want.append(i > 0 and t >= 3)
        d = (t - 2 * ((t - 1) // 2)) if i > 0 else 0
    assert used == want, (used, want, calls)


@pytest.mark.parametrize("pattern", ["whole", "1,odd,even"])
@pytest.mark.parametrize("name", ["box70x54_b1x1_s20", "bs_b1x1_s60", "box70x54_topo_b1x1_s20", "box1024_b1x1_s10",
                                  "box1521x1111_b1x1_s604"])
def test_pair_general_variant(amd, name, pattern):
    """Pairs of the general one-pass variant (known constants off: h_r, mu and the forcing read by
    both roles, D's fallback values from memory): no verdict to wait for, so pairs from the first
    call -- bitwise."""
    case = cases.load_e2e(name)
    calls = [case["steps"]] if pattern == "whole" else _splits(case["steps"], pattern)
    m = build_model(amd, case).set_known_constants(False).set_pair(2).init()
    used = []
    try:
        for n in calls:
            m.step(n, tau=1.0, check_every=1)
            used.append(m.pair_active)
        m.synchronize()
        bad = compare_case(m, case, name)
        one, zero = m.onepass_active, m.onepass_zero
    finally:
        m.close()
    assert not bad, f"{name} ({pattern}, general variant): fields differ from the reference: {bad}"
    assert one and not zero
    # as after the verdict, from the first call on (a first call of 1 step runs it: the sequence's
    # first step is not a plain one-pass step)
    want, d = [], 0
    for i, n in enumerate(calls):
        t = d + n
        want.append(t >= 3)
        d = 0 if i == 0 and n == 1 else t - 2 * ((t - 1) // 2)
    assert used == want, (used, want, calls)


@pytest.mark.parametrize("forcing", ["RHSx", "RHSy"])
def test_pair_general_variant_with_forcing(amd, forcing):
    """Pairs of the general variant with a wind forcing on the sea (RHSx / RHSy read by both roles:
    sw_update_uv, vel_ssh.f90:108-195) and a nonuniform mu (uv_diff2, vel_ssh.f90:375-452): bitwise
    against the oracle given the same uploads, the steps split across calls."""
    import numpy as np
    n = 600
    m = amd.OceanModel(amd.box_config(n)).set_known_constants(False).set_pair(2).init()
    ref = OracleTwin(n)
    b = m.blocks[0]
    lu = m.download(0, "lu")
    a = np.zeros(b.shape)
    a[lu > 0.5] = 2e-7 if forcing == "RHSx" else -3e-7
    a[200:260, 100:180] *= 4.0
    m.upload(0, forcing, a)
    ref.upload(b, forcing, a)
    mu = np.full(b.shape, 0.0)
    mu[150:400, 150:400] = 2.0
    m.upload(0, "mu", mu)
    ref.upload(b, "mu", mu)
    used = []
    try:
        for k in (1, 4, 3, 1):
            m.step(k, tau=1.0, check_every=1)
            used.append(m.pair_active)
        m.synchronize()
        ref.run(9)
        bad = ref.mismatches(m)
        one, zero = m.onepass_active, m.onepass_zero
    finally:
        m.close()
    assert not bad, f"general-variant pairs with a {forcing} forcing differ from the oracle: {bad}"
    assert one and not zero and any(used), (one, zero, used)


def test_pair_default_skips_general_variant(amd):
    """OCN_OPT_PAIR 1 (the default) leaves the general variant's steps single (its pair is no
    faster: VALU bound) -- bitwise either way."""
    case = cases.load_e2e("box1024_b1x1_s10")
    m = build_model(amd, case).set_known_constants(False).init()
    try:
        m.step(case["steps"], tau=1.0, check_every=1).synchronize()
        used, one = m.pair_active, m.onepass_active
        bad = compare_case(m, case, "box1024_b1x1_s10")
    finally:
        m.close()
    assert not bad and one and not used, (bad, one, used)


@pytest.mark.parametrize("name", ["box70x54_b1x1_s20", "box1024_b1x1_s10"])
def test_pair_default_threshold(amd, name):
    """OCN_OPT_PAIR 1 (the default): pairs on blocks of at least 512 x 512 interior points only;
    0: never -- both bitwise."""
    case = cases.load_e2e(name)
    for mode in (1, 0):
        m = build_model(amd, case).set_pair(mode).init()
        try:
            m.step(2, tau=1.0, check_every=1).synchronize()
            m.step(case["steps"] - 2, tau=1.0, check_every=1).synchronize()
            used = m.pair_active
            bad = compare_case(m, case, name)
        finally:
            m.close()
        assert not bad, f"{name} (pair {mode}): fields differ from the reference: {bad}"
        assert used == (mode == 1 and name.startswith("box1024")), (mode, used)


@pytest.mark.parametrize("name,calls,want", [("box1024_b1x1_s10", [10], [True]), ("box1024_b1x1_s10", [3, 7], [False, True]),
                                             ("box2048_b2x2_s10", [10], [True]), ("box2048_b2x2_s10", [4, 6], [True, True])])
def test_first_call_waits_for_the_verdict(amd, name, calls, want):
    """A first call of 4 or more steps waits for the known-constant check's verdict (ocn_ctx.hip
    await_kc) and runs pairs (x4 pairs with several blocks in one process) from its second step; a
    first call of 3 leaves the variant to the device -- bitwise against the reference either way."""
    case = cases.load_e2e(name)
    m = build_model(amd, case).init()
    used = []
    try:
        for n in calls:
            m.step(n, tau=1.0, check_every=1)
            used.append(m.x4_active if len(m.blocks) > 1 else m.pair_active)
        m.synchronize()
        bad = compare_case(m, case, name)
    finally:
        m.close()
    assert not bad, f"{name} {calls}: fields differ from the reference: {bad}"
    assert used == want, (used, want)


def test_pair_clock_telemetry(amd):
    """ocn_ctx_clock_info: workgroup 0 of every pair launch counts the shader clock against the
    100 MHz real-time counter -- one sample per pair launch, a clock within the part's range, the
    counters zeroed by a reset; single launches add nothing."""
    m = amd.OceanModel(amd.box_config(1024)).init()
    try:
        m.step(2, check_every=1).synchronize()
        m.clock_info(reset=True)
        m.set_pair(0)
        m.step(4, check_every=1).synchronize()
        assert m.clock_info()["launches"] == 0
        m.set_pair(1)
        m.step(7, check_every=1)
        pairs = m.pair_active
        c = m.clock_info(reset=True)
        again = m.clock_info()
    finally:
        m.close()
    assert pairs and c["launches"] >= 2, c
    assert 0.5 < c["clock_ghz"] < 3.0 and c["sampled_ms"] > 0.0, c
    assert again["launches"] == 0 and again["clock_ghz"] == 0.0, again


def test_pair_counts_blowup_points_once(amd):
    """check_ssh_err_kernel (vel_ssh.f90:40-67) in pair launches: each step counts its points once
    (the producers count only their workgroup's own rows) -- the reported count equals the single
    launches' count."""
    msgs = []
    for mode in (2, 0):
        m = amd.OceanModel(amd.box_config(200)).set_pair(mode).init()
        m.step(2, check_every=1).synchronize()
        s = m.download(0, "ssh")
        s[60:140, 60:140] = 2.0e4   # an 80 x 80 patch: it crosses workgroup row tiles
        for nm in ("ssh", "sshn", "sshp"):
            m.upload(0, nm, s)
        # the upload re-checks the known constants: a one-pass call without counts hands the
        # verdict over (a call of 3: one-pass steps whatever hh_init's state)
        m.step(3, check_every=0).synchronize()
        with pytest.raises(amd.OcnError) as e:
            m.step(4, check_every=1).synchronize()
        used = m.pair_active
        msgs.append(str(e.value))
        m.close()
        assert used == (mode == 2), (mode, used)
    assert msgs[0] == msgs[1], msgs


@pytest.mark.parametrize("name", ["box1024_b1x1_s10", "box1521x1111_b1x1_s604"])
def test_pair_one_step_calls(amd, name):
    """The reference's cadence (model.f90:146: one expl_shallow_water per step) with pairs: 1-step
    calls and no synchronising call -- the verdict arrives through its pinned copy, then every
    second call runs two steps in one launch -- bitwise; the tail formed by the reads."""
    case = cases.load_e2e(name)
    m = build_model(amd, case).init()
    used = []
    try:
        for _ in range(case["steps"]):
            m.step(1, tau=1.0, check_every=1)
            used.append(m.pair_active)
        bad = compare_case(m, case, name)
        m.synchronize()
    finally:
        m.close()
    assert not bad, f"{name} (1-step calls): fields differ from the reference: {bad}"
    assert any(used), "no pair launch"


@pytest.mark.parametrize("how", ["deferred", "redo"])
@pytest.mark.parametrize("name", ["box1024_b1x1_s10", "bs_b1x1_s60"])
def test_pair_last_tail(amd, name, how):
    """The pending tail's last two steps as ONE launch, the second as the call's last step (MarchStep
    PAIR + LAST: the consumer waves also store vort, the stresses and the RHS terms), then a8's copies
    and hh_init -- "deferred": the two steps a call left pending run that way when the fields are read;
    "redo": synchronize() ran them as a pair, so the read re-runs that pair from the state before it as
    the pair + LAST launch.  Bitwise against the reference; the timer shows the launch."""
    case = cases.load_e2e(name)
    m = build_model(amd, case).set_pair(2).init()
    steps = case["steps"]
    try:
        m.step(2, tau=1.0, check_every=1)
        m.synchronize()                       # the verdict reaches the host
        m.set_stage_timing(True)
        m.stage_times()
        m.step(steps - 2, tau=1.0, check_every=1)   # an even count: pairs, the last two pending
        if how == "redo":
            m.synchronize()                   # runs the two pending steps as a plain pair
        bad = compare_case(m, case, name)     # reads: the tail forms
        times = m.stage_times()
    finally:
        m.close()
    assert not bad, f"{name} ({how}): fields differ from the reference: {bad}"
    assert times.get("onepass2_last", (0, 0))[1] == 1, times
    assert "onepass" not in times, times      # no single one-pass launch in the tail


def _ops_run(amd, pair, ops):
    """One context driven through `ops` -- ("step", n, tau) / ("sync",) / ("read", field) /
    ("bump", field): a download, a small change, an upload -- then every field of every block."""
    import numpy as np
    m = amd.OceanModel(amd.box_config(600)).set_pair(pair).init()
    used = False
    try:
        for op in ops:
            if op[0] == "step":
                m.step(op[1], tau=op[2], check_every=1)
                used |= m.pair_active
            elif op[0] == "sync":
                m.synchronize()
            elif op[0] == "read":
                m.download(0, op[1])
            elif op[0] == "bump":
                a = m.download(0, op[1])
                a[300, 280] += 1.0e-3
                m.upload(0, op[1], a)
        m.synchronize()
        out = {nm: m.download(0, nm) for nm in m.field_names}
    finally:
        m.close()
    assert all(np.isfinite(v).all() for v in out.values())
    return out, used


@pytest.mark.parametrize("seq", ["tau", "reads", "upload"])
def test_pair_deferral_matches_single_launches(amd, seq):
    """Pairs across calls under the entries that end or look into an open sequence -- a change of
    tau with a step deferred (it runs as the last step of the old tau), reads of fields between
    calls (the tail formed: after a pair its first step again, a deferred step as the last), an
    upload between calls, synchronize() with a step deferred (it runs alone) -- bitwise the same
    fields as one launch per step."""
    base = [("step", 2, 1.0), ("sync",), ("step", 3, 1.0)]   # the verdict, then a pair + 1 deferred
    more = {"tau": [("step", 1, 0.5), ("step", 3, 0.5), ("step", 1, 1.0)],
            "reads": [("read", "ssh"), ("step", 1, 1.0), ("step", 2, 1.0), ("read", "ubrtr"), ("step", 5, 1.0),
                      ("sync",), ("step", 1, 1.0)],
            "upload": [("bump", "ssh"), ("step", 2, 1.0), ("sync",), ("step", 3, 1.0), ("step", 1, 1.0)]}[seq]
    a, used = _ops_run(amd, 1, base + more)
    b, _ = _ops_run(amd, 0, base + more)
    assert used
    bad = [nm for nm in a if a[nm].tobytes() != b[nm].tobytes()]
    assert not bad, f"{seq}: fields differ between pair and single launches: {bad}"
    # and both against the oracle given the same steps, taus and bumps
    ref = OracleTwin(600)
    f = ref.om.f[0]
    for op in base + more:
        if op[0] == "step":
            ref.run(op[1], op[2])
        elif op[0] == "bump":
            f[op[1]][300, 280] += 1.0e-3
    bad = [nm for nm in a if nm in f and a[nm].tobytes(order="F") != f[nm].tobytes(order="F")]
    assert not bad, f"{seq}: fields differ from the oracle: {bad}"


def test_tail_keeps_n_level_only_while_it_holds(amd):
    """The call tail's hh_init (last_finish) leaves hqn / hun / hvn / hhn as they are while they hold
    hh_init's n level (depth.f90:14-99: formed from h_r alone; ocn_ctx.hip hn_fresh) -- tails after
    pairs, then an upload of h_r (the n level changes: the next tail stores it again), more tails --
    every field against the oracle given the same uploads, after each tail."""
    import numpy as np
    n = 600
    m = amd.OceanModel(amd.box_config(n)).init()
    ref = OracleTwin(n)
    b = m.blocks[0]
    try:
        m.step(3, check_every=1).synchronize()
        ref.run(3)
        bad = []
        for k, calls in enumerate([[6], [6, 1], [5], [6], [2, 3]]):
            if k == 3:   # a non-uniform rest depth from here on (the pair's h_r-reading variant)
                h = m.download(0, "hhq_rest")
                i, j = np.meshgrid(np.arange(h.shape[0]), np.arange(h.shape[1]), indexing="ij")
                bump = 5.0 * np.exp(-((i - 300.0) ** 2 + (j - 250.0) ** 2) / 2.0e3)
                h = h + np.where(h > 0.0, bump, 0.0)
                m.upload(0, "hhq_rest", h)
                ref.upload(b, "hhq_rest", h)
            used = False
            for c in calls:
                m.step(c, check_every=1)
                used = used or m.pair_active
                ref.run(c)
            bad += [f"tail {k}: {x}" for x in ref.mismatches(m)]   # (the reads form the tail)
            assert used or k == 3, k   # (after the upload the first call waits for the variant's verdict)
    finally:
        m.close()
    assert not bad, f"fields differ from the oracle: {bad}"


# (seeds whose sequences reach each path: a known-constant option switched off keeps the pairs off,
# and an h_r upload whose halos do not match the neighbour blocks keeps the x2 steps off -- the
# library's own checks; the fields match the oracle either way)
@pytest.mark.parametrize("layout,seed", [("pair", 3), ("pair", 5), ("pair", 6), ("pair", 8),
                                         ("multi", 2), ("multi", 3), ("x2", 3), ("x2", 5), ("x2", 6),
                                         ("tracer", 2), ("tracer", 3), ("tracer_x2", 3), ("tracer_x2", 5),
                                         ("tracer1_x2", 3), ("tracer1_x2", 5)])
def test_random_call_sequences_match_oracle(amd, layout, seed):
    """Seeded random sequences of the entries that drive or look into an open sequence -- calls of
    1..7 steps, tau changes, synchronize(), field reads (the tail formed), uploads of ssh and of a
    non-uniform h_r (the variant's verdict, the tail's n level), the known-constant option toggled
    -- on a box large enough for pairs ("pair"), a small one (several steps per launch, "multi") and
    a 3x2-block box (x2 steps with exchanges, "x2"), with 2 tracers, 1 tracer (the co-launched tracer
    step, "tracer1_x2") and none: every field against
    the oracle given the same steps, taus and uploads, at every read and at the end (the
    reference's state after each call, model.f90:135-160)."""
    _random_sequence(amd, layout, seed, ["step", "step", "step", "step", "tau", "sync", "sync", "read", "ssh",
                                         "hr", "kc"], need_path=True)


@pytest.mark.parametrize("layout,seed", [(lay, sd) for lay in ("pair", "multi", "x2", "tracer", "tracer_x2", "tracer1_x2")
                                         for sd in (11, 12, 13)] +
                         [(lay, 21) for lay in ("island_pair", "island_multi", "island_x2", "island_tracer",
                                                "island_tracer_x2")])
def test_random_entry_sequences_match_oracle(amd, layout, seed):
    """The same with every entry the library offers between calls: uploads of the velocities, mu
    and the forcing RHSx (the known-constant variant's verdict), of hhq_n, and every step option
    switched at random (one-pass, pairs, several steps per launch, tracer steps, lazy tail, role
    flip, graph replay) -- the fields are the reference's whatever path runs."""
    _random_sequence(amd, layout, seed, ["step", "step", "step", "step", "tau", "sync", "read", "ssh", "hr",
                                         "kc", "uv", "mu", "rhs", "hqn", "opt", "opt", "graph"], need_path=False)


def _random_sequence(amd, layout, seed, ops, need_path, nops=20):
    import numpy as np
    rng = np.random.default_rng(seed)
    base = layout.replace("island_", "")
    n, blocks, active = {"pair": (600, (1, 1), "pair_active"), "multi": (100, (1, 1), "multi_active"),
                         "x2": (120, (3, 2), "x2_active"), "tracer": (100, (1, 1), "tracer_step_active"),
                         "tracer_x2": (120, (3, 2), "tracer_step_active"),
                         "tracer1_x2": (120, (3, 2), "tracer_step_active")}[base]
    tracers = 1 if base.startswith("tracer1") else 2 if base.startswith("tracer") else 0
    sw = amd.SWConfig(use_tracers=1, tracer_num=tracers) if tracers else amd.SWConfig()
    mask = None
    if layout.startswith("island_"):   # land islands (mask 1), some across block boundaries
        mask = np.zeros((n + 4, n + 4), dtype=np.int32, order="F")
        mask[:2, :] = 1; mask[-2:, :] = 1; mask[:, :2] = 1; mask[:, -2:] = 1
        for _ in range(4):
            i0, j0 = int(rng.integers(4, n - 10)), int(rng.integers(4, n - 10))
            mask[i0:i0 + int(rng.integers(1, 9)), j0:j0 + int(rng.integers(1, 9))] = 1
    m = amd.OceanModel(amd.box_config(n, mask=mask), sw=sw, par=amd.ParallelConfig(*blocks)).init()
    ref = OracleTwin(n, blocks, tracers, mask)
    bad, used, log = [], False, []
    reads = ["ssh", "ubrtr", "hhu_n", "hhq", "vort", "sshp", "hhq_n"] + (["ff1_1", f"ff1p_{tracers}"] if tracers else [])

    def bump(nm, f):
        for bl in m.blocks:
            a = m.download(bl.k, nm)
            a = f(a)
            m.upload(bl.k, nm, a)
            ref.upload(bl, nm, a)

    def smooth(a, amp):
        i, j = np.meshgrid(np.arange(a.shape[0]), np.arange(a.shape[1]), indexing="ij")
        return amp * np.exp(-((i - a.shape[0] / 2) ** 2 + (j - a.shape[1] / 2) ** 2) / (a.size / 40.0))

    try:
        m.step(2, check_every=1).synchronize()
        ref.run(2)
        for _ in range(nops):
            op = str(rng.choice(ops))
            log.append(op)
            if op in ("step", "tau"):
                k, tau = int(rng.integers(1, 8)), (0.5 if op == "tau" else 1.0)
                m.step(k, tau=tau, check_every=1)
                on = getattr(m, active)
                used = used or on
                log[-1] += f"{k}{'*' if on else ''}"
                ref.run(k, tau)
            elif op == "sync":
                m.synchronize()
            elif op == "read":
                nm = str(rng.choice(reads))
                for bl in m.blocks:
                    if not bits_equal(m.download(bl.k, nm), ref.om.f[ref.k(bl)][nm]):
                        bad.append(f"read {nm} ({bl.bm},{bl.bn}) after {log}")
            elif op == "ssh":
                def f(a):
                    a[a.shape[0] // 2, a.shape[1] // 3] += 1.0e-3
                    return a
                bump("ssh", f)
            elif op == "hr":
                bump("hhq_rest", lambda a: a + smooth(a, 2.0))
            elif op == "uv":
                bump(str(rng.choice(["ubrtr", "vbrtr"])), lambda a: a + smooth(a, 1.0e-4))
            elif op == "mu":
                bump("mu", lambda a: a + smooth(a, 50.0))
            elif op == "rhs":
                bump("RHSx", lambda a: a + smooth(a, 1.0e-7))
            elif op == "hqn":
                bump("hhq_n", lambda a: a + 1.0)
            elif op == "opt":
                which = str(rng.choice(["onepass", "pair", "multi", "tracer_step", "lazy_tail", "flip", "x4",
                                        "co_launch"]))
                val = int(rng.integers(0, 3 if which in ("pair", "x4") else 2))
                {"onepass": m.set_onepass, "multi": m.set_multi, "tracer_step": m.set_tracer_step,
                 "lazy_tail": m.set_lazy_tail, "flip": m.set_flip, "x4": m.set_x4,
                 "co_launch": m.set_co_launch}.get(which, lambda v: m.set_pair(int(v)))(
                    val if which == "pair" else 3 if (which == "x4" and val == 2) else bool(val))
                log[-1] += f"-{which}{val}"
            elif op == "graph":
                on = bool(rng.integers(0, 2))
                m.set_graph(on)
                log[-1] += str(int(on))
            else:
                on = bool(rng.integers(0, 2))
                m.set_known_constants(on)
                log[-1] += str(int(on))
        bad += ref.mismatches(m)
    finally:
        m.close()
    assert not bad, f"{layout}: fields differ from the oracle: {bad} ({log})"
    if need_path:
        assert used, f"{layout}: the path never ran: {log}"
