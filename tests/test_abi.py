"""CPU checks of the drop-in boundary: libocn_sw.so loads here (no GPU) and exports every
function include/ocn_sw.h declares; struct layouts agree with the ctypes/Fortran mirrors;
with no device every context call fails loudly (no CPU fallback)."""
import ctypes as C
import os
import re

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "ocn_sw.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(?:int|int64_t|void\s*\*|const\s+char\s*\*)\s*(ocn_\w+)\s*\(", src)))


@pytest.fixture(scope="module")
def lib():
    import ocean_model_arch_amd as amd
    if not os.path.exists(amd._lib.LIB_PATH):
        amd.build()
    return amd.lib()


def test_header_declares_the_stage_entries():
    names = declared_functions()
    for stage in ("sw_update_ssh", "hh_update", "uv_trans_vort", "uv_trans", "stress_components", "uv_diff2",
                  "sw_update_uv", "sw_next_step", "hh_shift", "hh_init", "check_ssh_err"):
        assert f"ocn_{stage}" in names
    assert len(names) >= 30


def test_every_declared_symbol_is_exported(lib):
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, f"declared in include/ocn_sw.h but not exported: {missing}"


def test_python_binding_covers_header(lib):
    from ocean_model_arch_amd import _lib
    assert set(_lib.ALL_SYMBOLS) == set(declared_functions())


STRUCTS = {"ocn_block": "OcnBlock", "ocn_basin": "OcnBasin", "ocn_sw_params": "OcnSwParams",
           "ocn_decomp": "OcnDecomp", "ocn_block_info": "OcnBlockInfo", "ocn_halo_msg": "OcnHaloMsg",
           "ocn_comm_info": "OcnCommInfo"}


def test_struct_layouts(tmp_path):
    """sizeof / offsetof of every ABI struct from the C header (gcc probe) == the ctypes mirror."""
    from ocean_model_arch_amd import _lib
    lines = ['#include <stdio.h>', '#include <stddef.h>', f'#include "{HEADER}"', "int main(void) {"]
    for cs, py in STRUCTS.items():
        lines.append(f'printf("{cs} size %zu\\n", sizeof({cs}));')
        for fname, _ in getattr(_lib, py)._fields_:
            lines.append(f'printf("{cs} {fname} %zu\\n", offsetof({cs}, {fname}));')
    lines += ["return 0; }"]
    src = tmp_path / "probe.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "probe"
    import subprocess
    subprocess.check_call(["gcc", "-std=c11", "-o", str(exe), str(src)])
    got = {}
    for ln in subprocess.check_output([str(exe)], text=True).splitlines():
        cs, what, v = ln.split()
        got[(cs, what)] = int(v)
    for cs, py in STRUCTS.items():
        t = getattr(_lib, py)
        assert C.sizeof(t) == got[(cs, "size")], cs
        for fname, _ in t._fields_:
            assert getattr(t, fname).offset == got[(cs, fname)], f"{cs}.{fname}"


def test_field_ids_match_header():
    from ocean_model_arch_amd import _lib
    src = open(HEADER).read()
    assert _lib.FIELD_ID["lu"] == 0 and _lib.FIELD_ID["r_diss"] == 16 and _lib.FIELD_ID["ssh"] == 32
    assert _lib.FIELD_ID["RHSy_dif"] == 63 and "OCN_FIELD_END" in src
    assert _lib.STAGE_ID["check_ssh_err"] == 10
    # tracer ids (OCN_FLUX_X = OCN_FIELD_END, OCN_FF1(k) = OCN_TRACER_BASE + 3 (k - 1))
    assert _lib.FIELD_ID["flux_x"] == 64 and _lib.FIELD_ID["flux_y"] == 65
    assert [_lib.FIELD_ID[n] for n in ("ff1_1", "ff1p_1", "ff1n_1", "ff1_2")] == [66, 67, 68, 69]
    assert _lib.FIELD_ID.name(71) == "ff1n_2"
    # + fused_ca, onepass, onepass2, onepass2_last, onepass_multi, tracer_step, exchange, exposed
    assert len(_lib.TIMERS) == 11 + 3 + 3 + 8


def test_abi_version_and_loud_failure_without_device(lib):
    import ocean_model_arch_amd as amd
    assert lib.ocn_abi_version() == 5
    bid = amd.build_id()
    assert len(bid) == 16 and int(bid, 16) >= 0, bid   # Makefile: sha256 of sources + flags
    try:
        import torch
        has_gpu = torch.cuda.is_available()
    except Exception:
        has_gpu = False
    if has_gpu:
        pytest.skip("device present")
    with pytest.raises(amd.OcnError):
        amd.OceanModel(amd.box_config(32))


def test_kernel_entry_rejects_bad_block(lib):
    from ocean_model_arch_amd import _lib
    b = _lib.OcnBlock(3, 10, 3, 10, 2, 12, 1, 12, 10)     # pitch 10 < width 11
    p = C.c_void_p(0x1000)
    rc = lib.ocn_sw_update_ssh(C.byref(b), C.c_double(1.0), *([p] * 11), None)
    assert rc == _lib.OCN_ERR_ARG
    b = _lib.OcnBlock(3, 10, 3, 10, 3, 12, 1, 12, 64)     # no halo ring on the left
    assert lib.ocn_sw_update_ssh(C.byref(b), C.c_double(1.0), *([p] * 11), None) == _lib.OCN_ERR_ARG
    b = _lib.OcnBlock(3, 10, 3, 10, 1, 12, 1, 12, 64)
    assert lib.ocn_sw_update_ssh(C.byref(b), C.c_double(1.0), *([p] * 10), None, None) == _lib.OCN_ERR_ARG


def test_par_files_round_trip(tmp_path):
    from ocean_model_arch_amd.config import BasinConfig, ParallelConfig, SWConfig
    (tmp_path / "basin.par").write_text(
        "289 : nx\n163 : ny\n1 : nz\n0 : px\n0 : py\n0.05d0 : dxst\n0.04d0 : dyst\n27.525d0 : rlon\n"
        "40.940d0 : rlat\n0 : x\n0 : y\n1 : curve\n0.0d0 : a\n0.0d0 : b\n90.0d0 :\n60.0d0 :\n90.0d0 :\n"
        "-90.0d0 :\nnone : mask\nnone : topo\n")
    (tmp_path / "sw.par").write_text("1 : a\n0 : b\n1 : c\n0.25d0 : ts\n1.0d+03 : lv\n1 : tr\n2 : n\nnone : f\n")
    (tmp_path / "parallel.par").write_text("0 : m\nnone : f\n4 : bx\n2 : by\n0\n0\nnone\n0\n0\n")
    b = BasinConfig.from_par(str(tmp_path / "basin.par"))
    assert (b.nx, b.ny, b.dxst, b.dyst, b.rlon, b.rlat, b.curve_grid) == (289, 163, 0.05, 0.04, 27.525, 40.94, 1)
    s = SWConfig.from_par(str(tmp_path / "sw.par"))
    assert (s.full_free_surface, s.trans_terms, s.ksw_lat, s.time_smooth, s.lvisc_2) == (1, 0, 1, 0.25, 1000.0)
    assert (s.use_tracers, s.tracer_num) == (1, 2)
    p = ParallelConfig.from_par(str(tmp_path / "parallel.par"))
    assert (p.bppnx, p.bppny) == (4, 2)
