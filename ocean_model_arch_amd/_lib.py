"""ctypes binding of libocn_sw.so (include/ocn_sw.h).

The HIP library is the product: there is no CPU fallback.  If the shared object is missing
or cannot be loaded, every entry point raises ``OcnLibraryError`` -- loudly, on purpose.
"""
from __future__ import annotations

import ctypes as C
import os
import re
import subprocess

_HERE = os.path.dirname(os.path.abspath(__file__))
# OCN_LIB_PATH selects an alternative build (performance variants); default: the in-tree build.
LIB_PATH = os.environ.get("OCN_LIB_PATH") or os.path.join(_HERE, "libocn_sw.so")
_CSRC = os.path.join(_HERE, "csrc")

OCN_OK, OCN_ERR_ARG, OCN_ERR_HIP, OCN_ERR_COMM, OCN_ERR_STATE, OCN_ERR_BLOWUP = range(6)

# field ids (include/ocn_sw.h)
R4_NAMES = ["lu", "luu", "luh", "lcu", "lcv", "llu", "llv", "dx", "dy", "dxt", "dyt", "dxh", "dyh",
            "dxb", "dyb", "rlh_s", "r_diss"]
R8_NAMES = ["ssh", "sshn", "sshp", "ubrtr", "ubrtrn", "ubrtrp", "vbrtr", "vbrtrn", "vbrtrp",
            "hhq", "hhq_p", "hhq_n", "hhu", "hhu_p", "hhu_n", "hhv", "hhv_p", "hhv_n",
            "hhh", "hhh_p", "hhh_n", "hhq_rest", "vort", "str_t", "str_s", "mu",
            "RHSx", "RHSy", "RHSx_adv", "RHSy_adv", "RHSx_dif", "RHSy_dif"]
OCN_FIELD_END = 32 + len(R8_NAMES)
OCN_TRACER_BASE = OCN_FIELD_END + 2        # OCN_FLUX_X, OCN_FLUX_Y, then ff1/ff1p/ff1n per tracer
MAX_TRACERS = 64
_TRACER_RE = re.compile(r"^(ff1|ff1p|ff1n)_([0-9]+)$")


def tracer_names(tracer_num: int) -> list[str]:
    """core/ocean.f90:38-41: flux_x, flux_y, then ff1_k, ff1p_k, ff1n_k for k = 1..tracer_num."""
    return ["flux_x", "flux_y"] + [f"{p}_{k}" for k in range(1, tracer_num + 1) for p in ("ff1", "ff1p", "ff1n")]


class _FieldIds(dict):
    """name -> field id; tracer names (ff1_3, ...) resolve on demand (OCN_FF1(k) etc.)."""
    def __missing__(self, name):
        m = _TRACER_RE.match(name)
        if not m or not 1 <= int(m.group(2)) <= MAX_TRACERS:
            raise KeyError(name)
        return OCN_TRACER_BASE + 3 * (int(m.group(2)) - 1) + ("ff1", "ff1p", "ff1n").index(m.group(1))

    def name(self, fid: int) -> str:
        for k, v in self.items():
            if v == fid:
                return k
        t = fid - OCN_TRACER_BASE
        if 0 <= t < 3 * MAX_TRACERS:
            return f"{('ff1', 'ff1p', 'ff1n')[t % 3]}_{t // 3 + 1}"
        raise KeyError(fid)


FIELD_ID = _FieldIds({n: i for i, n in enumerate(R4_NAMES)})
FIELD_ID.update({n: 32 + i for i, n in enumerate(R8_NAMES)})
FIELD_ID.update({"flux_x": OCN_FIELD_END, "flux_y": OCN_FIELD_END + 1})


def is_r8_name(name: str) -> bool:
    return name not in R4_NAMES

STAGES = ["sw_update_ssh", "hh_update", "uv_trans_vort", "uv_trans", "stress_components", "uv_diff2",
          "sw_update_uv", "sw_next_step", "hh_shift", "hh_init", "check_ssh_err"]
STAGE_ID = {n: i for i, n in enumerate(STAGES)}
TSTAGES = ["tran_diff_fluxes", "tran_diff_tracer", "tracer_next_step"]
TSTAGE_ID = {n: i for i, n in enumerate(TSTAGES)}
TIMERS = STAGES + ["fused_a", "fused_b", "fused_c1"] + TSTAGES + ["fused_ca", "onepass", "onepass2", "onepass2_last", "onepass_multi", "tracer_step",
                                                                       "exchange", "exposed"]    # OCN_NUM_TIMERS slots
OPT_GRAPH = 1
OPT_OVERLAP = 2
OPT_STAGE_TIMING = 3
OPT_FUSED = 4
OPT_COMPACT = 5
OPT_MARCH = 6
OPT_FLIP = 7
OPT_RECOMPUTE = 8
OPT_ONEPASS = 9
OPT_KNOWN_CONSTANTS = 10
OPT_ONEPASS_LAST = 11
OPT_LAZY_TAIL = 12
OPT_X2 = 13
OPT_BATCH = 14
OPT_PAIR = 15
OPT_MULTI = 16
OPT_TRACER_STEP = 17
OPT_MULTI_SPIN = 18
OPT_X4 = 19
OPT_CO_LAUNCH = 20
OPT_XCHG_DELAY = 21

# exported symbols (every one declared in include/ocn_sw.h)
KERNEL_SYMBOLS = ["ocn_sw_update_ssh", "ocn_hh_update", "ocn_uv_trans_vort", "ocn_uv_trans",
                  "ocn_stress_components", "ocn_uv_diff2", "ocn_sw_update_uv", "ocn_sw_next_step",
                  "ocn_hh_shift", "ocn_hh_init", "ocn_check_ssh_err", "ocn_tran_diff_fluxes",
                  "ocn_tran_diff_tracer", "ocn_tracer_next_step"]
CTX_SYMBOLS = ["ocn_decompose", "ocn_halo_schedule", "ocn_ctx_create", "ocn_ctx_destroy", "ocn_ctx_block_count", "ocn_ctx_block_info",
               "ocn_ctx_field", "ocn_ctx_stream", "ocn_comm_unique_id", "ocn_ctx_attach_comm", "ocn_ctx_attach_loopback",
               "ocn_ctx_set_topography", "ocn_ctx_init_state", "ocn_ctx_sync", "ocn_ctx_stage", "ocn_ctx_tracer_stage", "ocn_ctx_step", "ocn_ctx_synchronize",
               "ocn_ctx_download", "ocn_ctx_complete", "ocn_ctx_upload", "ocn_ctx_output_r4", "ocn_ctx_set_option", "ocn_ctx_get_option", "ocn_ctx_stage_times", "ocn_ctx_stage_stats",
               "ocn_ctx_comm_info", "ocn_ctx_overlap_info", "ocn_ctx_clock_info", "ocn_ctx_set_watchdog", "ocn_last_error", "ocn_abi_version",
               "ocn_build_id", "ocn_launch_count"]
ALL_SYMBOLS = KERNEL_SYMBOLS + CTX_SYMBOLS


class OcnLibraryError(RuntimeError):
    pass


class OcnError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"[ocn error {code}] {msg}")
        self.code = code


class OcnBlock(C.Structure):
    _fields_ = [("nx_start", C.c_int32), ("nx_end", C.c_int32), ("ny_start", C.c_int32), ("ny_end", C.c_int32),
                ("bnd_x1", C.c_int32), ("bnd_x2", C.c_int32), ("bnd_y1", C.c_int32), ("bnd_y2", C.c_int32),
                ("pitch", C.c_int64)]


class OcnBasin(C.Structure):
    _fields_ = [("nx", C.c_int32), ("ny", C.c_int32), ("dxst", C.c_double), ("dyst", C.c_double),
                ("rlon", C.c_double), ("rlat", C.c_double), ("curve_grid", C.c_int32),
                ("rotation_on_lon", C.c_double), ("rotation_on_lat", C.c_double)]


class OcnSwParams(C.Structure):
    _fields_ = [("full_free_surface", C.c_int32), ("trans_terms", C.c_int32), ("ksw_lat", C.c_int32),
                ("time_smooth", C.c_double), ("lvisc_2", C.c_double), ("use_tracers", C.c_int32),
                ("tracer_num", C.c_int32)]


class OcnDecomp(C.Structure):
    _fields_ = [("bnx", C.c_int32), ("bny", C.c_int32), ("nranks", C.c_int32), ("rank", C.c_int32),
                ("device", C.c_int32)]


class OcnBlockInfo(C.Structure):
    _fields_ = [("geom", OcnBlock), ("bm", C.c_int32), ("bn", C.c_int32),
                ("nbr_rank", C.c_int32 * 8), ("nbr_k", C.c_int32 * 8)]


class OcnHaloMsg(C.Structure):
    _fields_ = [("kind", C.c_int32), ("peer", C.c_int32), ("k", C.c_int32), ("k_src", C.c_int32),
                ("field", C.c_int32), ("dst_x0", C.c_int32), ("dst_x1", C.c_int32), ("dst_y0", C.c_int32),
                ("dst_y1", C.c_int32), ("src_x0", C.c_int32), ("src_x1", C.c_int32), ("src_y0", C.c_int32),
                ("src_y1", C.c_int32), ("count", C.c_int32), ("offset", C.c_int64)]


class OcnCommInfo(C.Structure):
    _fields_ = [("transport", C.c_int32), ("nccl_version", C.c_int32), ("comm_size", C.c_int32),
                ("comm_rank", C.c_int32), ("exchanges", C.c_int64), ("exchanges_done", C.c_int64),
                ("watchdog_s", C.c_double)]


class OcnOverlapInfo(C.Structure):
    _fields_ = [("level", C.c_int32), ("state", C.c_int32), ("kind", C.c_int32), ("pad", C.c_int32),
                ("seq_ms", C.c_double), ("overlapped_ms", C.c_double)]


class OcnClockInfo(C.Structure):
    _fields_ = [("launches", C.c_int64), ("clock_ghz", C.c_double), ("sampled_ms", C.c_double)]


HALO_LOCAL, HALO_SEND, HALO_RECV = 0, 1, 2

_lib = None


def build(force: bool = False) -> str:
    """Compile libocn_sw.so in-tree for gfx950 (hipcc; no GPU needed)."""
    cmd = ["make", "-s", "-f", os.path.join(_CSRC, "Makefile")]
    if force:
        cmd.insert(2, "-B")
    subprocess.check_call(cmd)
    return LIB_PATH


def lib() -> C.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise OcnLibraryError(f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; "
                              f"g.build()'` (hipcc --offload-arch=gfx950). There is no CPU fallback.")
    try:
        # torch (if used by the host) and this library must share one HIP runtime: import torch first
        # so its libamdhip64.so.7 is the one resolved.
        import torch  # noqa: F401
    except Exception:
        pass
    try:
        L = C.CDLL(LIB_PATH)
    except OSError as e:
        raise OcnLibraryError(f"cannot load {LIB_PATH}: {e}") from e
    for name in ALL_SYMBOLS:
        getattr(L, name)
    L.ocn_last_error.restype = C.c_char_p
    L.ocn_build_id.restype = C.c_char_p
    L.ocn_launch_count.restype = C.c_int64
    L.ocn_ctx_field.restype = C.c_void_p
    L.ocn_ctx_field.argtypes = [C.c_void_p, C.c_int, C.c_int]
    L.ocn_ctx_stream.restype = C.c_void_p
    L.ocn_ctx_stream.argtypes = [C.c_void_p]
    L.ocn_ctx_create.argtypes = [C.POINTER(OcnBasin), C.POINTER(OcnSwParams), C.POINTER(OcnDecomp), C.c_void_p,
                                 C.POINTER(C.c_void_p)]
    for nm in ("ocn_ctx_destroy", "ocn_ctx_init_state", "ocn_ctx_synchronize", "ocn_ctx_block_count",
               "ocn_ctx_complete"):
        getattr(L, nm).argtypes = [C.c_void_p]
    L.ocn_ctx_block_info.argtypes = [C.c_void_p, C.c_int, C.POINTER(OcnBlockInfo)]
    L.ocn_ctx_set_topography.argtypes = [C.c_void_p, C.c_void_p, C.c_int64]
    L.ocn_ctx_sync.argtypes = [C.c_void_p, C.c_int]
    L.ocn_ctx_stage.argtypes = [C.c_void_p, C.c_int, C.c_double]
    L.ocn_ctx_tracer_stage.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_double]
    L.ocn_ctx_step.argtypes = [C.c_void_p, C.c_double, C.c_int32, C.c_int32]
    L.ocn_ctx_download.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p]
    L.ocn_ctx_upload.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p]
    L.ocn_ctx_output_r4.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_float, C.c_void_p]
    L.ocn_ctx_set_option.argtypes = [C.c_void_p, C.c_int32, C.c_int64]
    L.ocn_ctx_get_option.argtypes = [C.c_void_p, C.c_int32, C.POINTER(C.c_int64)]
    L.ocn_ctx_stage_times.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
    L.ocn_ctx_stage_stats.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
    L.ocn_ctx_comm_info.argtypes = [C.c_void_p, C.POINTER(OcnCommInfo)]
    L.ocn_ctx_overlap_info.argtypes = [C.c_void_p, C.POINTER(OcnOverlapInfo)]
    L.ocn_ctx_clock_info.argtypes = [C.c_void_p, C.c_int32, C.POINTER(OcnClockInfo)]
    L.ocn_ctx_set_watchdog.argtypes = [C.c_void_p, C.c_double]
    L.ocn_ctx_attach_comm.argtypes = [C.c_void_p, C.c_void_p, C.c_int32]
    L.ocn_comm_unique_id.argtypes = [C.c_void_p, C.c_int32]
    L.ocn_ctx_attach_loopback.argtypes = [C.POINTER(C.c_void_p), C.c_int32]
    L.ocn_decompose.argtypes = [C.POINTER(OcnBasin), C.POINTER(OcnDecomp), C.c_void_p, C.POINTER(OcnBlockInfo),
                                C.c_int32, C.POINTER(C.c_int32)]
    L.ocn_halo_schedule.argtypes = [C.POINTER(OcnBasin), C.POINTER(OcnDecomp), C.c_void_p, C.POINTER(C.c_int32),
                                    C.c_int32, C.POINTER(OcnHaloMsg), C.c_int32, C.POINTER(C.c_int32)]
    _lib = L
    return L


def build_id() -> str:
    """ocn_build_id(): hash of the loaded library's sources and compile flags."""
    return lib().ocn_build_id().decode()


def launch_count() -> int:
    """ocn_launch_count(): kernel launches issued through the library by this process so far."""
    return int(lib().ocn_launch_count())


def check(rc: int, what: str = ""):
    if rc != OCN_OK:
        msg = lib().ocn_last_error().decode(errors="replace")
        raise OcnError(rc, f"{what}: {msg}" if what else msg)
    return rc
