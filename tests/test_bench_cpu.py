"""bench.py's host logic without a GPU: the per-launch byte model for the
step kinds a call runs, MPI_Dims_create, and the stamp check that keeps a PMC traffic summary of
another build or workload out of roofline.traffic."""
import json
import os

import pytest

import bench


def test_dims_create_matches_mpi():
    assert [bench.dims_create(n) for n in (1, 2, 4, 8)] == [(1, 1), (2, 1), (2, 2), (4, 2)]


@pytest.mark.parametrize("steps", [2, 3, 6, 20])
def test_onepass_call_launches(steps):
    """One block: K-1 one-pass steps, the one-pass last step, a8's copies, hh_init; the second
    buffers copied back when the number of swaps is odd."""
    kinds = [k for _, k in bench.call_launches(steps, flip=True, one=True)]
    assert kinds[:steps - 1] == ["onepass"] * (steps - 1)
    assert kinds[steps - 1:steps + 2] == ["onepass_last", "copy3", "c2_full"]
    assert kinds.count("copy3") == 1 + steps % 2


def test_step_bytes_orders():
    """Fewer bytes per step the further the fusion goes; the known-constant variant reads less."""
    std = bench.step_bytes(True, [20], flip=False)
    flip = bench.step_bytes(True, [20], flip=True)
    one = bench.step_bytes(True, [20], flip=True, one=True)
    onez = bench.step_bytes(True, [20], flip=True, one=True, zero=True)
    assert std > flip > one > onez
    assert round(one, 2) == 140.25 and round(onez, 2) == 108.25
    # tracer runs: the tracer steps (one-pass steps, a tracer step per step) move far less than the
    # role-flip path with the standard tracer stages
    trs = bench.step_bytes(True, [20], flip=True, one=True, zero=True, tracers=1)
    trf = bench.step_bytes(True, [20], flip=True, tracers=1)
    assert trs < trf / 2, (trs, trf)


def test_lazy_region_launches():
    """An open one-pass sequence (OCN_OPT_LAZY_TAIL): one launch per step whatever the call length,
    and the tail once at the end of the region; 100 steps in 1-step calls move what one 100-step
    call moves plus the one step the tail runs again."""
    one = bench.region_launches([1] * 100, flip=True, one=True, zero=True, lazy=True)
    assert [k for _, k in one[:100]] == ["onepass_z"] * 100
    assert [k for _, k in one[100:]] == ["onepass_last_z", "copy3", "c2_full"]
    lazy = bench.step_bytes(True, [1] * 100, flip=True, one=True, zero=True, lazy=True)
    whole = bench.step_bytes(True, [100], flip=True, one=True, zero=True)
    assert lazy == bench.step_bytes(True, [100], flip=True, one=True, zero=True, lazy=True)
    assert abs(lazy - whole - 97 / 100) < 1e-9
    per_call = bench.step_bytes(True, [1] * 100, flip=False)
    assert per_call > 3 * lazy


class _Amd:
    def __init__(self, bid):
        self._bid = bid

    def build_id(self):
        return self._bid


def test_traffic_needs_matching_stamp(tmp_path, monkeypatch):
    rec = {"build_id": "abc", "box": [64, 64], "blocks": [1, 1],
           "kernels": {"onepass": {"cells": 4096, "compact": True, "hbm_bytes_per_launch": 123.0}}}
    (tmp_path / "profiles").mkdir()
    (tmp_path / "profiles" / "pmc_traffic.json").write_text(json.dumps(rec))
    monkeypatch.setattr(bench, "REPO", str(tmp_path))
    ok = bench.load_traffic(_Amd("abc"), "onepass", 4096, True, [64, 64], [1, 1])
    assert ok == (123.0, "build")
    assert bench.load_traffic(_Amd("other"), "onepass", 4096, True, [64, 64], [1, 1]) == (None, None)
    assert bench.load_traffic(_Amd("abc"), "onepass", 4096, True, [64, 64], [2, 1]) == (None, None)
    assert bench.load_traffic(_Amd("abc"), "onepass", 2048, True, [64, 64], [1, 1]) == (None, None)
    assert bench.load_traffic(_Amd("abc"), "fused_b", 4096, True, [64, 64], [1, 1]) == (None, None)


def test_profile_applies_to_unchanged_kernel_code(tmp_path, monkeypatch):
    """A summary taken on another build applies when the kernel's gfx950 machine code in the loaded
    library is byte for byte the profiled code (code_sha of the record's symbol), not otherwise."""
    import ocean_model_arch_amd as amd
    from ocean_model_arch_amd import _codeobj
    lib = amd._lib.LIB_PATH
    if not os.path.exists(lib):
        pytest.skip("library not built")
    sym = _codeobj.march_step_symbol("true, false, true, false, false, true, false")
    sha = _codeobj.kernel_code_sha(lib, sym)
    assert sha and len(sha) == 16

    class _A(_Amd):
        _lib = amd._lib
    rec = {"build_id": "elsewhere", "box": [64, 64], "blocks": [1, 1],
           "kernels": {"onepass2": {"cells": 4096, "compact": True, "hbm_bytes_per_launch": 7.0, "symbol": sym,
                                    "code_sha": sha}}}
    (tmp_path / "profiles").mkdir()
    (tmp_path / "profiles" / "pmc_traffic.json").write_text(json.dumps(rec))
    monkeypatch.setattr(bench, "REPO", str(tmp_path))
    assert bench.load_traffic(_A("other"), "onepass2", 4096, True, [64, 64], [1, 1]) == (7.0, "kernel code")
    rec["kernels"]["onepass2"]["code_sha"] = "0" * 16
    (tmp_path / "profiles" / "pmc_traffic.json").write_text(json.dumps(rec))
    assert bench.load_traffic(_A("other"), "onepass2", 4096, True, [64, 64], [1, 1]) == (None, None)


def test_valu_needs_matching_stamp(tmp_path, monkeypatch):
    """roofline.valu: the one-pass kernel's VALU issue floor from the committed SQ pass, only on the
    build and workload it was taken on; 1024 SIMDs x 1 wave64 instruction per quad-cycle at 2.4 GHz."""
    per_launch = {"SQ_INSTS_VALU": 1024 * 2.4e6 / 4, "SQ_WAVES": 10}     # 1 ms of issue
    per_wave = {"SQ_WAVE_CYCLES": 100.0, "SQ_ACTIVE_INST_VALU": 60.0, "SQ_WAIT_INST_ANY": 30.0, "SQ_WAIT_ANY": 10.0}
    rec = {"build_id": "abc", "box": [64, 64], "blocks": [1, 1],
           "kernels": {"onepass": {"per_launch": per_launch, "per_wave": per_wave}}}
    (tmp_path / "profiles").mkdir()
    (tmp_path / "profiles" / "sq_valu.json").write_text(json.dumps(rec))
    monkeypatch.setattr(bench, "REPO", str(tmp_path))
    v = bench.load_valu(_Amd("abc"), "onepass", 2.0, [64, 64], [1, 1])
    assert v["issue_floor_ms"] == 1.0 and v["issue_frac"] == 0.5
    assert v["per_wave_frac"] == {"valu_active": 0.6, "wait_inst_any": 0.3, "wait_any": 0.1}
    assert bench.load_valu(_Amd("other"), "onepass", 2.0, [64, 64], [1, 1]) is None
    assert bench.load_valu(_Amd("abc"), "onepass", 2.0, [64, 64], [2, 1]) is None
    assert bench.load_valu(_Amd("abc"), "hh_init", 2.0, [64, 64], [1, 1]) is None


def test_valu_at_live_clock(tmp_path, monkeypatch):
    """roofline.valu at the clock measured in the pair kernel over the timed region
    (ocn_ctx_clock_info): the floor scales with 2.4 GHz / the live clock; only for the pair launch
    and only when pair launches were sampled."""
    per_launch = {"SQ_INSTS_VALU": 1024 * 2.4e6 / 4, "SQ_WAVES": 10}     # 1 ms of issue at 2.4 GHz
    per_wave = {"SQ_WAVE_CYCLES": 100.0, "SQ_ACTIVE_INST_VALU": 60.0, "SQ_WAIT_INST_ANY": 30.0, "SQ_WAIT_ANY": 10.0}
    rec = {"build_id": "abc", "box": [64, 64], "blocks": [1, 1],
           "kernels": {"onepass2": {"per_launch": per_launch, "per_wave": per_wave}}}
    (tmp_path / "profiles").mkdir()
    (tmp_path / "profiles" / "sq_valu.json").write_text(json.dumps(rec))
    monkeypatch.setattr(bench, "REPO", str(tmp_path))
    live = {"launches": 9, "clock_ghz": 1.2, "sampled_ms": 5.0}
    v = bench.load_valu(_Amd("abc"), "onepass2", 4.0, [64, 64], [1, 1], live)
    assert v["live_clock_ghz"] == 1.2 and v["issue_floor_ms_at_live_clock"] == 2.0
    assert v["issue_frac_at_live_clock"] == 0.5 and "9 pair launches" in v["live_clock_source"]
    v = bench.load_valu(_Amd("abc"), "onepass2", 4.0, [64, 64], [1, 1], {"launches": 0, "clock_ghz": 0.0})
    assert "live_clock_ghz" not in v


def test_hr_variant_bytes():
    """The known-constant one-pass variant that reads h_r (a topography) moves 8 B per cell more
    than the one with h_r a constant and 24 B less than the general one (101 one-pass launches in
    100 steps: the tail re-runs one)."""
    z = bench.step_bytes(True, [100], flip=True, one=True, zero=True, lazy=True)
    h = bench.step_bytes(True, [100], flip=True, one=True, zero="h", lazy=True)
    g = bench.step_bytes(True, [100], flip=True, one=True, zero=False, lazy=True)
    assert abs(h - z - 8.0 * 1.01) < 1e-9 and abs(g - h - 24.0 * 1.01) < 1e-9


@pytest.mark.parametrize("calls", [[1], [2], [3], [4], [100], [1] * 100, [1] * 7])
def test_pair_region_launches(calls):
    """Two one-pass steps per launch in an open sequence (OCN_OPT_PAIR, ocn_ctx.hip step_impl):
    pairs across calls while 3 or more steps are pending; the last 1 or 2 are run by the tail (one
    launch whose second step is the last, or the last step) -- no step runs twice."""
    steps = sum(calls)
    one = bench.region_launches(calls, flip=True, one=True, zero=True, lazy=True, pair=True)
    kinds = [k for _, k in one]
    p = (steps - 1) // 2
    assert kinds[:p] == ["onepass2_z"] * p
    tail = ["copy3", "c2_full"]
    assert kinds[p:] == (["onepass_last_z"] + tail if steps % 2 else ["onepass2_last_z"] + tail)
    non_lazy = [k for _, k in bench.call_launches(20, flip=True, one=True, zero=True, pair=True)]
    assert non_lazy[:10] == ["onepass2_z"] * 9 + ["onepass_z"] and non_lazy[10] == "onepass_last_z"


def test_rccl_report_from_rank_records():
    """The N-GPU line's `rccl` object (bench.rccl_report) from per-rank timed-region records: groups per
    step and the exposed time are the worst rank's, the group time's max the largest of any rank,
    hidden_frac = 1 - exposed / group time over all ranks."""
    comm = {"transport": "rccl", "version": "2.27.7", "comm_size": 2, "watchdog_s": 120.0}
    recs = [{"rank": 0, "comm": comm, "groups": 22, "timed_groups": 22, "group_ms_sum": 0.44, "group_ms_max": 0.05,
             "exposed_ms_sum": 0.044, "exposed_n": 19},
            {"rank": 1, "comm": comm, "groups": 22, "timed_groups": 22, "group_ms_sum": 0.66, "group_ms_max": 0.08,
             "exposed_ms_sum": 0.066, "exposed_n": 19}]
    r = bench.rccl_report(recs, 20)
    assert r["version"] == "2.27.7" and r["comm_size"] == 2 and r["transport"] == "rccl"
    assert r["groups_per_step"] == 1.1 and r["group_ms"] == {"mean": 0.025, "max": 0.08}
    assert r["exposed_ms_per_step"] == 0.0033 and r["hidden_frac"] == 0.9
    assert [p["groups"] for p in r["per_rank"]] == [22, 22]
    assert r["overlap"] is None
    ov = {"level": 1, "state": 3, "kind": 2, "seq_ms": 0.11, "overlapped_ms": 0.12}
    r = bench.rccl_report([dict(q, overlap=ov) for q in recs], 20)
    assert r["overlap"] == {"level": 1, "decided": True, "measured_on": "x2 step", "seq_ms": 0.11,
                            "overlapped_ms": 0.12, "per_rank_level": [1, 1]}
