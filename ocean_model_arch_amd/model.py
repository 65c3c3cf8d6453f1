"""OceanModel: host handle on one process's share of the domain (libocn_sw context).

Mirrors the reference's global model state -- ``domain_data`` (core/decomposition.f90),
``ocean_data`` (core/ocean.f90) and ``grid_data`` (core/grid.f90) -- for the blocks this
process owns.  Device storage lives in the C++ context; this class only holds the handle.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _lib
from ._lib import FIELD_ID, R4_NAMES, R8_NAMES, STAGE_ID, TSTAGE_ID, check, is_r8_name, lib, tracer_names
from .config import BasinConfig, ParallelConfig, SWConfig


@dataclass
class BlockInfo:
    """domain_type's view of local block k (decomposition.f90:40-81, blocks_info :17-32)."""
    k: int
    bm: int
    bn: int
    nx_start: int
    nx_end: int
    ny_start: int
    ny_end: int
    bnd_x1: int
    bnd_x2: int
    bnd_y1: int
    bnd_y2: int
    pitch: int
    nbr_rank: tuple
    nbr_k: tuple

    @property
    def shape(self):
        return (self.bnd_x2 - self.bnd_x1 + 1, self.bnd_y2 - self.bnd_y1 + 1)

    @property
    def cells(self) -> int:
        return (self.nx_end - self.nx_start + 1) * (self.ny_end - self.ny_start + 1)

    def c_block(self) -> _lib.OcnBlock:
        return _lib.OcnBlock(self.nx_start, self.nx_end, self.ny_start, self.ny_end,
                             self.bnd_x1, self.bnd_x2, self.bnd_y1, self.bnd_y2, self.pitch)


class OceanModel:
    """One process's blocks on one GPU.

    ``OceanModel(basin, sw, par, rank=0, nranks=1, device=0)`` decomposes the basin exactly as
    the reference does (uniform blocks, land blocks dropped, blocks dealt to processes), allocates
    every field on the device, and ``init()`` builds the reference's initial state
    (control/init_data.f90).  ``step(n)`` runs expl_shallow_water n times on the device.
    """

    def __init__(self, basin: BasinConfig, sw: SWConfig = SWConfig(), par: ParallelConfig = ParallelConfig(),
                 rank: int = 0, nranks: int = 1, device: int = 0):
        L = lib()
        self.basin, self.sw, self.par = basin, sw, par
        self.rank, self.nranks, self.device = rank, nranks, device
        cb = _lib.OcnBasin(basin.nx, basin.ny, basin.dxst, basin.dyst, basin.rlon, basin.rlat, basin.curve_grid,
                           basin.rotation_on_lon, basin.rotation_on_lat)
        cs = _lib.OcnSwParams(sw.full_free_surface, sw.trans_terms, sw.ksw_lat, sw.time_smooth, sw.lvisc_2,
                              sw.use_tracers, sw.tracer_num)
        # ocean_type / grid_type fields this model holds (core/ocean.f90, core/grid.f90)
        self.field_names = R4_NAMES + R8_NAMES + (tracer_names(sw.tracer_num) if sw.use_tracers > 0 else [])
        cd = _lib.OcnDecomp(par.bppnx, par.bppny, nranks, rank, device)
        self._mask = None
        mptr = None
        if basin.mask is not None:
            self._mask = np.asfortranarray(basin.mask.astype(np.int32))
            if self._mask.shape != (basin.nx, basin.ny):
                raise ValueError(f"mask shape {self._mask.shape} != (nx, ny) = {(basin.nx, basin.ny)}")
            mptr = self._mask.ctypes.data_as(C.c_void_p)
        h = C.c_void_p()
        check(L.ocn_ctx_create(C.byref(cb), C.byref(cs), C.byref(cd), mptr, C.byref(h)), "ocn_ctx_create")
        self.ctx = h
        if basin.topography is not None:   # init_data.f90:115-120 (used by init())
            t = np.asfortranarray(basin.topography, dtype=np.float32)
            if t.shape != (basin.nx - 4, basin.ny - 4):
                raise ValueError(f"topography shape {t.shape} != (nx-4, ny-4) = {(basin.nx - 4, basin.ny - 4)}")
            self._topo = t
            check(L.ocn_ctx_set_topography(self.ctx, t.ctypes.data_as(C.c_void_p), t.size), "ocn_ctx_set_topography")
        self.blocks: list[BlockInfo] = []
        for k in range(L.ocn_ctx_block_count(self.ctx)):
            bi = _lib.OcnBlockInfo()
            check(L.ocn_ctx_block_info(self.ctx, k, C.byref(bi)), "ocn_ctx_block_info")
            g = bi.geom
            self.blocks.append(BlockInfo(k, bi.bm, bi.bn, g.nx_start, g.nx_end, g.ny_start, g.ny_end, g.bnd_x1,
                                         g.bnd_x2, g.bnd_y1, g.bnd_y2, g.pitch, tuple(bi.nbr_rank),
                                         tuple(bi.nbr_k)))

    # ---------------------------------------------------------------- lifecycle
    def close(self):
        if getattr(self, "ctx", None):
            lib().ocn_ctx_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def attach_comm(self, unique_id: bytes):
        """Attach an RCCL communicator (unique id made by ``make_unique_id`` on rank 0)."""
        buf = C.create_string_buffer(bytes(unique_id), len(unique_id))
        check(lib().ocn_ctx_attach_comm(self.ctx, buf, len(unique_id)), "ocn_ctx_attach_comm")

    @staticmethod
    def attach_loopback(models):
        """Test transport (ocn_ctx_attach_loopback): models[i] = rank i of len(models) ranks, all
        on one device, each to be driven from its own thread (run_ranks); only the RCCL calls
        are replaced."""
        arr = (C.c_void_p * len(models))(*[m.ctx.value for m in models])
        check(lib().ocn_ctx_attach_loopback(arr, len(models)), "ocn_ctx_attach_loopback")

    def init(self):
        check(lib().ocn_ctx_init_state(self.ctx), "ocn_ctx_init_state")
        return self

    @property
    def overlap_level(self) -> int:
        """OCN_OPT_OVERLAP in effect (auto resolved)."""
        v = C.c_int64()
        check(lib().ocn_ctx_get_option(self.ctx, _lib.OPT_OVERLAP, C.byref(v)), "ocn_ctx_get_option")
        return int(v.value)

    def set_graph(self, on: bool = True):
        check(lib().ocn_ctx_set_option(self.ctx, _lib.OPT_GRAPH, int(on)), "ocn_ctx_set_option")
        return self

    def set_stage_timing(self, on: bool = True):
        check(lib().ocn_ctx_set_option(self.ctx, _lib.OPT_STAGE_TIMING, int(on)), "ocn_ctx_set_option")
        return self

    def stage_times(self) -> dict:
        """{stage: (total_ms, launches)} from HIP events since the last call (synchronises)."""
        ms = (C.c_double * len(_lib.TIMERS))()
        n = (C.c_int64 * len(_lib.TIMERS))()
        check(lib().ocn_ctx_stage_times(self.ctx, ms, n), "ocn_ctx_stage_times")
        return {s: (ms[i], n[i]) for i, s in enumerate(_lib.TIMERS) if n[i]}

    def stage_stats(self) -> dict:
        """{stage: (total_ms, launches, max_ms)} from HIP events since the last call (synchronises);
        "exchange": the halo exchanges with remote peers, "exposed": per overlapped step, how long the
        exchange chain outlasted the inner march (ocn_ctx_stage_stats)."""
        ms = (C.c_double * len(_lib.TIMERS))()
        mx = (C.c_double * len(_lib.TIMERS))()
        n = (C.c_int64 * len(_lib.TIMERS))()
        check(lib().ocn_ctx_stage_stats(self.ctx, ms, n, mx), "ocn_ctx_stage_stats")
        return {s: (ms[i], n[i], mx[i]) for i, s in enumerate(_lib.TIMERS) if n[i]}

    def set_watchdog(self, seconds: float):
        """Host-side watchdog (ocn_ctx_set_watchdog): a call that may take part in a collective and has
        not returned after `seconds` is ended (RCCL communicator aborted / loopback group failed; the
        call raises OcnError with the rank's last completed exchange id).  0 = off."""
        check(lib().ocn_ctx_set_watchdog(self.ctx, float(seconds)), "ocn_ctx_set_watchdog")
        return self

    def comm_info(self) -> dict:
        """ocn_ctx_comm_info: transport ("none" / "rccl" / "loopback"), RCCL version and communicator
        size / rank, exchanges enqueued and the last completed (-1 without a watchdog)."""
        i = _lib.OcnCommInfo()
        check(lib().ocn_ctx_comm_info(self.ctx, C.byref(i)), "ocn_ctx_comm_info")
        v = int(i.nccl_version)
        return {"transport": ("none", "rccl", "loopback")[i.transport],
                "version": (f"{v // 10000}.{v // 100 % 100}.{v % 100}" if v else None), "version_code": v,
                "comm_size": int(i.comm_size), "comm_rank": int(i.comm_rank),
                "exchanges": int(i.exchanges), "exchanges_done": int(i.exchanges_done),
                "watchdog_s": float(i.watchdog_s)}

    def overlap_info(self) -> dict:
        """ocn_ctx_overlap_info: the overlap level in effect and, with OCN_OPT_OVERLAP auto and peers on
        other ranks, the measured choice (state 3 = decided; seq_ms / overlapped_ms = the two step times
        the vote compared, maxima over the ranks)."""
        i = _lib.OcnOverlapInfo()
        check(lib().ocn_ctx_overlap_info(self.ctx, C.byref(i)), "ocn_ctx_overlap_info")
        return {"level": int(i.level), "state": int(i.state), "kind": int(i.kind),
                "seq_ms": round(float(i.seq_ms), 4), "overlapped_ms": round(float(i.overlapped_ms), 4)}

    def clock_info(self, reset: bool = False) -> dict:
        """ocn_ctx_clock_info: the shader clock the pair launches ran at (measured in the kernel by
        workgroup 0 of each launch; device-wide since the last reset -- reset=True zeroes it after
        reading)."""
        i = _lib.OcnClockInfo()
        check(lib().ocn_ctx_clock_info(self.ctx, int(bool(reset)), C.byref(i)), "ocn_ctx_clock_info")
        return {"launches": int(i.launches), "clock_ghz": round(float(i.clock_ghz), 4),
                "sampled_ms": round(float(i.sampled_ms), 4)}

    def set_exchange_delay(self, us: int):
        """Tests: the device waits `us` microseconds before each exchange with remote peers
        (OCN_OPT_XCHG_DELAY: a slow link)."""
        check(lib().ocn_ctx_set_option(self.ctx, _lib.OPT_XCHG_DELAY, int(us)), "ocn_ctx_set_option")
        return self

    def set_fused(self, on: bool = True):
        """Fused step groups (default) or the reference's 11 envoke stages; same results bit for bit."""
        check(lib().ocn_ctx_set_option(self.ctx, _lib.OPT_FUSED, int(on)), "ocn_ctx_set_option")
        return self

    def set_overlap(self, on: int = -1):
        """Overlap halo exchanges (comm stream) with the inner part of the fused launches: 1 = in
        the standard steps and (frame launches + exchanges as a side chain beside the inner march)
        in the one-pass steps, 2 = in the role-flip steps too, 0 = never, -1 = auto (the default:
        2 with other ranks attached, else 1)."""
        check(lib().ocn_ctx_set_option(self.ctx, _lib.OPT_OVERLAP, int(on)), "ocn_ctx_set_option")
        return self

    def set_compact(self, on: bool = True):
        """Compact static fields for the fused step (bit-packed masks, per-row metrics) when exact
        for the current real(4) fields; re-arms them after raw real(4) pointers were handed out."""
        check(lib().ocn_ctx_set_option(self.ctx, _lib.OPT_COMPACT, int(on)), "ocn_ctx_set_option")
        return self

    def set_march(self, on: bool = True):
        """Register-march form of the stencil launches that have one (default; needs the compact
        static fields); same results bit for bit."""
        check(lib().ocn_ctx_set_option(self.ctx, _lib.OPT_MARCH, int(on)), "ocn_ctx_set_option")
        return self

    def set_flip(self, on: bool = True):
        """Role-flip steps (default; compact + march, no tracers): sw_next_step's copies become
        buffer swaps inside the library and its filters run inside fused B; same results bit for
        bit."""
        check(lib().ocn_ctx_set_option(self.ctx, _lib.OPT_FLIP, int(on)), "ocn_ctx_set_option")
        return self

    def set_recompute(self, on: bool = True):
        """Recompute steps inside role-flip calls (default): fused B forms hhq, hhu_p, hhv_p itself
        instead of re-reading them; same results bit for bit."""
        check(lib().ocn_ctx_set_option(self.ctx, _lib.OPT_RECOMPUTE, int(on)), "ocn_ctx_set_option")
        return self

    def set_onepass(self, on: bool = True):
        """One-pass steps in single-block role-flip calls (default): each middle step of a call is
        one launch that reads the state once and writes the next state once; same results bit
        for bit."""
        check(lib().ocn_ctx_set_option(self.ctx, _lib.OPT_ONEPASS, int(on)), "ocn_ctx_set_option")
        return self

    def set_onepass_last(self, on: bool = True):
        """With halo exchanges or ring work, the call's last step as a one-pass step too (default);
        off: a standard last step there (same results bit for bit)."""
        check(lib().ocn_ctx_set_option(self.ctx, _lib.OPT_ONEPASS_LAST, int(on)), "ocn_ctx_set_option")
        return self

    def set_known_constants(self, on: bool = True):
        """The one-pass steps' known-constant variant (default): forcing and D's fallback values
        zero, h_r and mu uniform, when a check of the arrays finds them so; off: always the
        general variant (same results bit for bit)."""
        check(lib().ocn_ctx_set_option(self.ctx, _lib.OPT_KNOWN_CONSTANTS, int(on)), "ocn_ctx_set_option")
        return self

    def set_lazy_tail(self, on: bool = True):
        """Lazy call tail (default): in one process, one block without halo exchanges, a call whose
        steps are one-pass steps leaves what the reference's last step stores beyond the next state
        pending, so the next step() continues with one-pass steps (1-step calls run as fast as long
        ones); complete(), or anything that looks at the fields, forms it first (same results bit
        for bit)."""
        check(lib().ocn_ctx_set_option(self.ctx, _lib.OPT_LAZY_TAIL, int(on)), "ocn_ctx_set_option")
        return self

    def set_x2(self, on: bool = True):
        """One-pass steps with one 2-deep state exchange each where there are halo exchanges
        (default): every block forms the depths, vort and stresses on its halo itself and marches its
        whole interior; same results bit for bit."""
        check(lib().ocn_ctx_set_option(self.ctx, _lib.OPT_X2, int(on)), "ocn_ctx_set_option")
        return self

    def set_batch(self, on: bool = True):
        """Block batching (default): with several blocks on the device, each launch group of a step
        is issued once for all of them instead of once per block."""
        check(lib().ocn_ctx_set_option(self.ctx, _lib.OPT_BATCH, int(on)), "ocn_ctx_set_option")
        return self

    def set_multi(self, on: bool = True):
        """Small single blocks: the steps of a call (in an open sequence) as one launch
        with a grid-wide barrier between them (default on); same results bit for bit."""
        check(lib().ocn_ctx_set_option(self.ctx, _lib.OPT_MULTI, int(on)), "ocn_ctx_set_option")
        return self

    def set_x4(self, on=True):
        """Blocks with halo exchanges: two x2 steps per launch with one 4-deep state exchange per two
        steps (OCN_OPT_X4: True / 1 = auto, the default -- tracer runs only with peers on other ranks;
        3 = always; False / 0 = off); same results bit for bit."""
        mode = 3 if on == 3 else int(bool(on))
        check(lib().ocn_ctx_set_option(self.ctx, _lib.OPT_X4, mode), "ocn_ctx_set_option")
        return self

    @property
    def x4_active(self) -> bool:
        """Whether the last step() ran pairs of x2 steps (one_step_x4)."""
        return self.option(_lib.OPT_X4) == 2

    def set_co_launch(self, on: bool = True):
        """Tracer runs with x2 steps: each step's march and the previous state's tracer step as one
        launch (default on, OCN_OPT_CO_LAUNCH); same results bit for bit."""
        check(lib().ocn_ctx_set_option(self.ctx, _lib.OPT_CO_LAUNCH, int(on)), "ocn_ctx_set_option")
        return self

    @property
    def co_launched(self) -> bool:
        """Whether the last step() co-launched a march and a tracer step."""
        return self.option(_lib.OPT_CO_LAUNCH) == 2

    def set_multi_spin(self, polls: int):
        """Diagnostics: the multi-step launch's grid barrier gives up after `polls` polls (default
        1 << 20, about 0.5 s); the next synchronize() then raises OCN_ERR_HIP."""
        check(lib().ocn_ctx_set_option(self.ctx, _lib.OPT_MULTI_SPIN, int(polls)), "ocn_ctx_set_option")
        return self

    def set_tracer_step(self, on: bool = True):
        """Tracer runs with one-pass steps: expl_tracer of each step as one launch per tracer (the depths
        it reads formed from the state), run with the next step (default on); same results bit for bit."""
        check(lib().ocn_ctx_set_option(self.ctx, _lib.OPT_TRACER_STEP, int(on)), "ocn_ctx_set_option")
        return self

    @property
    def tracer_step_active(self) -> bool:
        """Whether the last step() ran the tracers as tracer steps with one-pass steps."""
        return self.option(_lib.OPT_TRACER_STEP) == 2

    def set_pair(self, mode: int = 1):
        """Two one-pass steps per launch (default 1: the known-constant variants on single blocks of
        at least 512 x 512 interior points; 2: any variant, any block; 0: never): the first step's
        new state stays on chip; same results bit for bit."""
        check(lib().ocn_ctx_set_option(self.ctx, _lib.OPT_PAIR, int(mode)), "ocn_ctx_set_option")
        return self

    @property
    def multi_active(self) -> bool:
        """Whether the last step() ran its steps as one multi-step launch."""
        return self.option(_lib.OPT_MULTI) == 2

    @property
    def pair_active(self) -> bool:
        """Whether the last step() ran two one-pass steps per launch."""
        return self.option(_lib.OPT_PAIR) == 2

    @property
    def x2_active(self) -> bool:
        """Whether the last step() used one-pass steps with 2-deep state exchanges."""
        return bool(self.option(_lib.OPT_X2))

    @property
    def tail_pending(self) -> bool:
        """Whether the last step() left its call tail pending (OCN_OPT_LAZY_TAIL)."""
        return self.option(_lib.OPT_LAZY_TAIL) == 2

    def complete(self):
        """Form a pending call tail now (ocn_ctx_complete): every array then holds what the
        reference leaves after the last step run.  Asynchronous."""
        check(lib().ocn_ctx_complete(self.ctx), "ocn_ctx_complete")
        return self

    def option(self, key: int) -> int:
        v = C.c_int64(0)
        check(lib().ocn_ctx_get_option(self.ctx, key, C.byref(v)), "ocn_ctx_get_option")
        return v.value

    @property
    def flip_active(self) -> bool:
        """Whether the last step() used role-flip steps."""
        return bool(self.option(_lib.OPT_FLIP))

    @property
    def recompute_active(self) -> bool:
        """Whether the last step() used recompute steps."""
        return bool(self.option(_lib.OPT_RECOMPUTE))

    @property
    def onepass_active(self) -> bool:
        """Whether the last step() used one-pass steps."""
        return bool(self.option(_lib.OPT_ONEPASS))

    @property
    def onepass_zero(self) -> bool:
        """Whether those steps took the forcing, the fallback values (known zeros) and h_r, mu (known
        uniform) as kernel constants instead of reading them."""
        return self.option(_lib.OPT_ONEPASS) == 2

    @property
    def onepass_hr(self) -> bool:
        """Whether those steps took the forcing and the fallback values as known zeros and mu as a
        known uniform value, but read a non-uniform h_r (a topography)."""
        return self.option(_lib.OPT_ONEPASS) == 3

    @property
    def compact_active(self) -> bool:
        """Whether the last step() read the compact static fields."""
        return bool(self.option(_lib.OPT_COMPACT))

    # ---------------------------------------------------------------- execution
    def step(self, nsteps: int = 1, tau: float = 1.0, check_every: int = 1):
        check(lib().ocn_ctx_step(self.ctx, tau, nsteps, check_every), "ocn_ctx_step")
        return self

    def stage(self, name: str, tau: float = 1.0):
        check(lib().ocn_ctx_stage(self.ctx, STAGE_ID[name], tau), f"ocn_ctx_stage({name})")

    def tracer_stage(self, name: str, tracer: int, tau: float = 1.0):
        """envoke of one tracer stage for tracer `tracer` (1-based data_id), with its sync."""
        check(lib().ocn_ctx_tracer_stage(self.ctx, TSTAGE_ID[name], tracer, tau), f"ocn_ctx_tracer_stage({name})")

    def sync(self, field: str):
        check(lib().ocn_ctx_sync(self.ctx, FIELD_ID[field]), f"ocn_ctx_sync({field})")

    def synchronize(self):
        check(lib().ocn_ctx_synchronize(self.ctx), "ocn_ctx_synchronize")
        return self

    @property
    def stream(self) -> int:
        return lib().ocn_ctx_stream(self.ctx)

    # ---------------------------------------------------------------- data access
    def field_ptr(self, k: int, name: str) -> int:
        p = lib().ocn_ctx_field(self.ctx, k, FIELD_ID[name])
        if not p:
            raise _lib.OcnError(_lib.OCN_ERR_ARG, f"no field {name} in block {k}")
        return p

    def download(self, k: int, name: str) -> np.ndarray:
        b = self.blocks[k]
        dt = np.float64 if is_r8_name(name) else np.float32
        a = np.zeros(b.shape, dtype=dt, order="F")
        check(lib().ocn_ctx_download(self.ctx, k, FIELD_ID[name], a.ctypes.data_as(C.c_void_p)), "download")
        return a

    def output_r4(self, k: int, name: str, undef: float) -> np.ndarray:
        """Output record of field `name` on block k's interior: real(4), undef on land
        (output.f90 copy_from_real8 + io.f90:343-349), converted on the device."""
        b = self.blocks[k]
        a = np.zeros((b.nx_end - b.nx_start + 1, b.ny_end - b.ny_start + 1), dtype=np.float32, order="F")
        check(lib().ocn_ctx_output_r4(self.ctx, k, FIELD_ID[name], C.c_float(undef), a.ctypes.data_as(C.c_void_p)),
              "output_r4")
        return a

    def upload(self, k: int, name: str, a: np.ndarray):
        b = self.blocks[k]
        dt = np.float64 if is_r8_name(name) else np.float32
        a = np.asfortranarray(a, dtype=dt)
        if a.shape != b.shape:
            raise ValueError(f"{name}: shape {a.shape} != block shape {b.shape}")
        check(lib().ocn_ctx_upload(self.ctx, k, FIELD_ID[name], a.ctypes.data_as(C.c_void_p)), "upload")

    def state(self, names=None) -> list[dict[str, np.ndarray]]:
        names = names or self.field_names
        return [{n: self.download(b.k, n) for n in names} for b in self.blocks]

    @property
    def interior_cells(self) -> int:
        """(nx-4)(ny-4) share of this process: the cell-updates/s unit of SURVEY.md 8(d)."""
        return sum(b.cells for b in self.blocks)


def run_ranks(models, fn):
    """Drive loopback-attached ranks: fn(model) on one host thread per model (the library calls
    release the GIL), like one process per rank.  Returns the results in rank order; re-raises
    the first rank's exception."""
    import threading
    out, err = [None] * len(models), [None] * len(models)

    def body(i):
        try:
            out[i] = fn(models[i])
        except BaseException as e:  # noqa: BLE001 -- re-raised below
            err[i] = e

    th = [threading.Thread(target=body, args=(i,)) for i in range(len(models))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    for e in err:
        if e is not None:
            raise e
    return out


def make_unique_id() -> bytes:
    buf = C.create_string_buffer(128)
    check(lib().ocn_comm_unique_id(buf, 128), "ocn_comm_unique_id")
    return buf.raw
