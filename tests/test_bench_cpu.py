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
    assert bench.step_bytes(True, [20], flip=True, one=True, tracers=1) == bench.step_bytes(True, [20], flip=True,
                                                                                             tracers=1)


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
    assert ok == 123.0
    assert bench.load_traffic(_Amd("other"), "onepass", 4096, True, [64, 64], [1, 1]) is None
    assert bench.load_traffic(_Amd("abc"), "onepass", 4096, True, [64, 64], [2, 1]) is None
    assert bench.load_traffic(_Amd("abc"), "onepass", 2048, True, [64, 64], [1, 1]) is None
    assert bench.load_traffic(_Amd("abc"), "fused_b", 4096, True, [64, 64], [1, 1]) is None
