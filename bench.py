"""bench.py -- cell-updates/s of the SW barotropic step on the 4096 x 4096 box (BASELINE.json).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--n 4096] [--scaling strong|weak]

One process per GPU (launched by torch.distributed.run for N > 1); the box is split into one
block per GPU with the reference's block grid (2x1, 2x2, 4x2) and halos are
exchanged over RCCL inside libocn_sw.  Rank 0 prints ONE JSON line.

value      = interior cells (nx-4)(ny-4) x K / t_loop, t_loop = max over ranks of the K timed steps
             (barrier + device sync on both sides), inputs resident in HBM.
roofline   = the dominant stage kernel: algorithmic bytes per launch (SURVEY.md 8a B/cell x cells)
             / its mean launch time from HIP events on the context stream, vs 8.0 TB/s.
cpu_baseline = the C restatement (oracle/, 1 core) on a bounded sample of the same workload.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "cell-updates/s, SW barotropic step on 4096x4096 box; %HBM BW at 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E peak (MI355X_MICROARCH.md)
# algorithmic bytes per interior cell per stage (sum = 1136)
STAGE_BYTES = {"sw_update_ssh": 68, "hh_update": 96, "uv_trans_vort": 44, "uv_trans": 84,
               "stress_components": 72, "uv_diff2": 96, "sw_update_uv": 200, "sw_next_step": 132,
               "hh_shift": 176, "hh_init": 168}
B_ALG = sum(STAGE_BYTES.values())
# the same stages over the compact tables (ocn_ctx envoke with OCN_OPT_COMPACT): the real(4) masks
# as one mask byte per point, the metrics as per-row values (bytes per cell: the real(8) arrays + 1)
STAGE_BYTES_COMPACT = {"sw_update_ssh": 49, "hh_update": 49, "uv_trans_vort": 25, "uv_trans": 65,
                       "stress_components": 33, "uv_diff2": 57, "sw_update_uv": 161, "sw_next_step": 121,
                       "hh_shift": 161, "hh_init": 121}
# Distinct arrays read + written once per interior cell by each launch kind, for
# the bench's sw.par (all three flags on), with the compact static fields (index 0) or the 2-D
# real(4) arrays (index 1).  "reuse" = a step that is neither the first nor the last of its
# ocn_ctx_step call (fused A skips hh_update, fused B reads hhu/hhv for hhu_n/hhv_n); "full" =
# the last step (fused B and hh_init also store what only the host reads).
LAUNCH_BYTES = {
    "a": (129, 180), "a_reuse": (89, 128),
    "b": (169, 220), "b_reuse": (153, 204), "b_full": (201, 252),
    "b_flip": (209, 260), "b_flip_reuse": (193, 244),     # + a8's filters: sshn, sshp in; sshp, ubrtrp, vbrtrp out
    "b_flip_rc": (177, 177),                               # hhq, hhu_p, hhv_p formed from h_r, ssh, sshp
    "c1": (121, 132), "c1_ring": (0, 0),                   # role-flip steps: a8 + a9 on the halo ring only
    "c2": (81, 128), "c2_full": (121, 168),
    "ca": (113, 113), "ca_store": (137, 137), "ca_hh": (169, 169),   # hh_init + next step's A (no hhh_p;
    # "ca": next step recomputes -- no interior hhq, hhu_p, hhv_p; "ca_hh": + a2's stores and hhh_p)
    # one-pass step: ssh, sshp, ubrtr, ubrtrp, vbrtr, vbrtrp, h_r, mu, RHSx, RHSy + mask byte in;
    # sshn, ubrtrn, vbrtrn and the filtered sshp, ubrtrp, vbrtrp out
    "onepass": (129, 129),
    "onepass_last": (185, 185),   # + vort, str_t, str_s and the four RHS terms out
    # the same with the forcing RHSx / RHSy known to be zero and h_r, mu known to be uniform
    # (checked once per call chain; taken as kernel constants, not read)
    "onepass_z": (97, 97), "onepass_last_z": (153, 153),
    # ... with h_r read (a non-uniform rest depth: the OCN_KC_KNOWN_HR variant)
    "onepass_h": (105, 105), "onepass_last_h": (161, 161),
    # two one-pass steps in one launch (OCN_OPT_PAIR): one step's reads and writes, the mask byte
    # read by both wave roles (+ h_r by both in the _h variant) -- per launch, i.e. per two steps
    "onepass2_z": (98, 98), "onepass2_h": (114, 114),
    # general variant: h_r, mu and the forcing read by both roles (the consumers' state from LDS)
    "onepass2": (162, 162),
    # the pending tail's last two steps in one launch, the second the call's last step (OCN_TIMER_ONEPASS2_LAST):
    # + vort, str_t, str_s and the four RHS terms out
    "onepass2_last_z": (154, 154), "onepass2_last_h": (170, 170), "onepass2_last": (218, 218),
    "copy3": (48, 48),   # end of a call with an odd number of one-pass steps: 3 fields copied back
    # tracer runs: CA also stores hh_init's hhq_p (read by tran_diff_tracer); per tracer and step:
    # tran_diff_fluxes (lcu, lcv, hhu, hhv, ff, ffp, ubrtr, vbrtr, mu in; flux_x, flux_y out),
    # tran_diff_tracer (lu, hhq_n, hhq_p, flux_x, flux_y, ffp in; ffn out), tracer_next_step (lu,
    # ffn, ffp, ff in; ffp, ff out)
    "hqp": (8, 8),
    # tracer step (one-pass sequences, OCN_OPT_TRACER_STEP), per tracer: ssh, sshp, h_r, ubrtr, vbrtr, mu,
    # ff, ffp + mask byte in (hh_init's depths and the fluxes formed, their fallback values +0.0); ffn, ffp out
    "tr_step": (81, 81),
    "tr_fluxes": (73, 97), "tr_tracer": (57, 69), "tr_next": (41, 44),
}


def _kc(zero) -> str:
    """The one-pass launch kind's suffix: zero = True (the known-constant variant), "h" (known
    constants, h_r read), False (the general variant)."""
    return "_z" if zero is True else "_h" if zero == "h" else ""


def _one_launches(n: int, z: str, pair: bool):
    """n consecutive one-pass steps of a call whose steps after them are not one-pass steps of an
    open sequence: with pairs (ocn_ctx.hip step_impl), steps 1 + 2i and 2 + 2i in one launch while
    the second is not the call's last step run -- (n - 1) // 2 pairs, the rest single."""
    p = (n - 1) // 2 if pair else 0
    return [("onepass2", "onepass2" + z)] * p + [("onepass", "onepass" + z)] * (n - 2 * p)


def call_launches(steps: int, flip: bool, rc: bool = True, ring: bool = False, one: bool = False,
                  tracers: int = 0, full_c2: bool = False, zero: bool = False, lazy: bool = False,
                  pair: bool = False):
    """The launches of one ocn_ctx_step call of `steps` steps, as (timer, launch kind) pairs --
    ocn_ctx.hip ocn_ctx_step / one_step_fused for one block (role-flip calls fuse each step's
    hh_init with the next step's A when full_free_surface = 1, as in sw.par; ring = the ring
    launch runs, i.e. a8 / a9 have work on the halo ring: blocks with neighbours; one = one-pass
    steps 1..K-1 (the first one too: nothing changes the state between the bench's calls); tracers = expl_tracer's three launches per tracer after every step, and
    hh_init's hhq_p stored by every CA / hh_init)."""
    if tracers and one:   # tracer steps: one-pass steps, each step's tracer step run with the next step
        z = _kc(zero)
        out = []
        for s in range(steps if lazy else steps - 1):
            out.append(("onepass", "onepass" + z))
            if s:
                out += [("tracer_step", "tr_step")] * tracers
        if not lazy:   # the last step, after the previous step's tracer step; the standard stages after it
            out += [("tracer_step", "tr_step")] * tracers + [(t, k + (z if t == "onepass" else ""))
                                                             for t, k in TAIL_LAUNCHES] + TRACER_STAGES * tracers
        return out
    if tracers:
        out = []
        for timer, kind in call_launches(steps, flip, rc, ring, False, full_c2=True):
            out.append((timer, kind))
            if timer == "fused_ca":
                out.append((timer, "hqp"))
            if timer in ("fused_ca", "hh_init"):   # the step's last SW launch: then its tracers
                out += [("tran_diff_fluxes", "tr_fluxes"), ("tran_diff_tracer", "tr_tracer"),
                        ("tracer_next_step", "tr_next")] * tracers
        return out
    if one and lazy:   # an open one-pass sequence (OCN_OPT_LAZY_TAIL): every step one launch, no tail
        return _one_launches(steps, _kc(zero), pair)
    if one and flip and steps >= 2:   # steps 1 .. K-1 (the state is unchanged since the last call / init)
        z = _kc(zero)
        out = _one_launches(steps - 1, z, pair and not ring)
        if ring:   # several blocks: CA + the standard last step
            out += [("fused_ca", "ca_hh"), ("fused_b", "b_full"), ("fused_c1", "c1"), ("hh_init", "c2_full")]
            swaps = steps - 1
        else:      # one block: the last step as one march (+ vort, stresses, RHS terms), a8's copies, hh_init
            out += [("onepass", "onepass_last" + z), ("copy", "copy3"), ("hh_init", "c2_full")]
            swaps = steps
        if swaps % 2:
            out.append(("copy", "copy3"))
        return out
    out = []
    for s in range(1, steps + 1):
        first, last = s == 1, s == steps
        reuse = not first and not last
        flip_step = flip and not last and steps >= 2
        if not (flip and steps >= 2 and not first):
            out.append(("fused_a", "a_reuse" if reuse else "a"))
        if flip_step:   # ring launch skipped when no halo-ring point has a8 / a9 work (the box)
            out.append(("fused_b", "b_flip" if first else "b_flip_rc" if rc else "b_flip_reuse"))
            if ring:
                out.append(("fused_c1", "c1_ring"))
            out += [("fused_ca", "ca_hh" if s + 1 >= steps else "ca" if rc else "ca_store")]
        else:
            out += [("fused_b", "b_full" if last else "b_reuse" if reuse else "b"), ("fused_c1", "c1"),
                    ("hh_init", "c2_full" if last or full_c2 else "c2")]
    return out


# the tail of an open one-pass sequence, formed by ocn_ctx_complete: the last step run again as the
# call's last step (+ vort, the stresses, the RHS terms), a8's copies, hh_init with every level
TAIL_LAUNCHES = [("onepass", "onepass_last"), ("copy", "copy3"), ("hh_init", "c2_full")]
TRACER_STAGES = [("tran_diff_fluxes", "tr_fluxes"), ("tran_diff_tracer", "tr_tracer"), ("tracer_next_step", "tr_next")]


def region_launches(calls, flip: bool, rc: bool = True, ring: bool = False, one: bool = False,
                    tracers: int = 0, zero: bool = False, lazy: bool = False, pair: bool = False,
                    multi: bool = False):
    """The launches of a timed region: ocn_ctx_step calls of calls[i] steps each, then (lazy) the
    pending tail formed by ocn_ctx_complete.  multi: each call of an open sequence as one
    launch of its steps (OCN_OPT_MULTI; kind "<one-pass kind>*n" = n steps' bytes in one launch)."""
    out, total = [], sum(calls)
    if lazy and one and multi and not pair:
        z = _kc(zero)
        for n in calls:
            out += [("onepass_multi", f"onepass{z}*{n}")] if n >= 2 else [("onepass", "onepass" + z)]
        return out + [(t, k + (z if t == "onepass" else "")) for t, k in TAIL_LAUNCHES]
    if lazy and one and pair:   # an open sequence with pairs: two steps per launch across calls while
        # 3 or more are pending; the last 1 or 2 run by ocn_ctx_complete
        out += [("onepass2", "onepass2" + _kc(zero))] * ((total - 1) // 2)
        calls = []
    if lazy and one and tracers:   # an open sequence with tracer steps: one tracer step per step but the
        # first; the tail: the last step again, a8's copies, hh_init, the standard tracer stages
        z = _kc(zero)
        out += [("onepass", "onepass" + z)] * total + [("tracer_step", "tr_step")] * ((total - 1) * tracers)
        return out + [(t, k + (z if t == "onepass" else "")) for t, k in TAIL_LAUNCHES] + TRACER_STAGES * tracers
    for n in calls:
        out += call_launches(n, flip, rc, ring, one, tracers, zero=zero, lazy=lazy, pair=pair)
    if lazy and one:
        tail = TAIL_LAUNCHES
        if pair:   # the steps left pending run as the last ones: 1 (the tail) or 2 (one launch: the pair
            # whose second step is the last, + a8's copies and hh_init)
            tail = TAIL_LAUNCHES if total % 2 else [("onepass2_last", "onepass2_last")] + TAIL_LAUNCHES[1:]
        out += [(t, k + (_kc(zero) if t.startswith("onepass") else "")) for t, k in tail]
    return out


def _bytes(kind: str, i: int) -> int:
    """LAUNCH_BYTES of a launch kind; "<kind>*n": n launches' bytes in one (a multi-step launch)."""
    base, _, n = kind.partition("*")
    return LAUNCH_BYTES[base][i] * (int(n) if n else 1)


def fused_bytes(compact: bool, calls, flip: bool = False, rc: bool = True, ring: bool = False,
                one: bool = False, tracers: int = 0, zero: bool = False, lazy: bool = False, pair: bool = False,
                multi: bool = False):
    """Mean bytes per interior cell per launch of each timer over the timed region's calls."""
    i = 0 if compact else 1
    tot, cnt = {}, {}
    for timer, kind in region_launches(calls, flip, rc, ring, one, tracers, zero, lazy, pair, multi):
        tot[timer] = tot.get(timer, 0) + _bytes(kind, i)
        cnt[timer] = cnt.get(timer, 0) + (kind != "hqp")   # "hqp": bytes of the launch before it
    return {t: tot[t] / cnt[t] for t in tot}


def step_bytes(compact: bool, calls, flip: bool = False, rc: bool = True, ring: bool = False,
               one: bool = False, tracers: int = 0, zero: bool = False, lazy: bool = False, pair: bool = False,
               multi: bool = False):
    """Bytes per interior cell per step moved by the timed region's calls."""
    i = 0 if compact else 1
    return sum(_bytes(kind, i) for _, kind in region_launches(calls, flip, rc, ring, one, tracers, zero,
                                                              lazy, pair, multi)) / sum(calls)


def dims_create(n: int):
    """MPI_Dims_create(n, 2) as used by the reference (mpp.f90:89): 2 -> 2x1, 4 -> 2x2, 8 -> 4x2."""
    import math
    for f in range(int(math.isqrt(n)), 0, -1):
        if n % f == 0:
            return n // f, f
    return n, 1


def cpu_cores() -> int:
    """Host cores this process may use (the GPU box exports OMP_NUM_THREADS = its CPU share)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        n = min(n, int(env))
    return max(1, min(n, 64))


def cpu_baseline(n_full: int = 4096):
    """The CPU path on this node's host cores: the C restatement of the reference
    (oracle/, bitwise the reference's results) timed on bounded samples of the bench workload --
      1 core : a 2048^2 box (a quarter of the workload), 1 block, 24 timed steps (~8 s);
      C cores: the 4096^2 box decomposed into C blocks (MPI_Dims_create(C) grid), one block per
               core -- the reference's OpenMP-over-blocks mode (kernel_interface.f90:84-88) --
               30 timed steps (~5 s on 16 cores).
    Each leg runs 1 untimed warm-up step first.  `value` is the C-core rate."""
    from oracle import oracle as O
    cores = cpu_cores()

    def leg(n, bxy, threads, steps):
        om = O.OracleModel(O.BasinConfig(nx=n + 4, ny=n + 4), O.SWConfig(), *bxy, threads=threads).init()
        om.run(1)
        t0 = time.perf_counter()
        om.run(steps)
        dt = time.perf_counter() - t0
        if om.pool is not None:
            om.pool.shutdown()
        return n * n * steps / dt, dt

    s1, sc = 24, 30
    v1, t1 = leg(2048, (1, 1), 1, s1)
    bxy = dims_create(cores)
    vc, tc = leg(n_full, bxy, cores, sc)
    return {"value": vc, "unit": "cell-updates/s", "cores": cores, "kind": "port",
            "1core": {"value": v1, "sample": f"2048x2048 box, 1 block, {s1} timed steps, {t1:.1f} s"},
            "allcores": {"value": vc, "cores": cores,
                         "sample": f"{n_full}x{n_full} box, {bxy[0]}x{bxy[1]} blocks on {cores} threads, {sc} timed steps, "
                                   f"{tc:.1f} s"},
            "sample": "oracle/sw_oracle.c (gcc -O2 -ffp-contract=off, bitwise the reference) on this node's host cores; "
                      "value = the all-cores leg"}


def multi_gpu_parity(amd, dist, rank, world, local_rank, bx, by, uid_for, watchdog=0.0):
    """Run-time check of the N > 1 path: a 512^2 box on the N-GPU block grid (RCCL halos) for
    2 + 6 steps -- a first call, a synchronize (the known-constant verdict reaches every host, so
    the second call's vote lets every rank run the x4 pairs: 4-deep exchanges over RCCL); rank 0
    recomputes the same block grid inside one process on its GPU (device-local halo copies, the path
    tests/test_gpu_x4.py pins to the reference) and compares every rank's block bit for bit.
    Returns True/False on rank 0, None elsewhere."""
    import numpy as np
    n, calls = 512, (2, 6)
    m = amd.OceanModel(amd.box_config(n), amd.SWConfig(), amd.ParallelConfig(bx, by), rank=rank, nranks=world,
                       device=local_rank)
    m.attach_comm(uid_for())
    if watchdog > 0:
        m.set_watchdog(watchdog)
    m.init().step(calls[0]).synchronize()
    m.step(calls[1]).synchronize()
    mine = {(b.bm, b.bn): {f: m.download(b.k, f) for f in ("ssh", "ubrtr", "vbrtr", "hhu", "str_s")}
            for b in m.blocks}
    m.close()
    gathered = [None] * world if rank == 0 else None
    dist.gather_object(mine, gathered, dst=0)
    if rank != 0:
        return None
    ref = amd.OceanModel(amd.box_config(n), amd.SWConfig(), amd.ParallelConfig(bx, by), device=local_rank)
    ref.init().step(calls[0]).synchronize()
    ref.step(calls[1]).synchronize()
    ok = True
    for b in ref.blocks:
        for part in gathered:
            if (b.bm, b.bn) in part:
                for f, a in part[(b.bm, b.bn)].items():
                    ok &= a.tobytes() == ref.download(b.k, f).tobytes()
    ref.close()
    return bool(ok)


def rccl_report(rank_info, steps: int):
    """The multi-GPU line's `rccl` object from every rank's timed-region record: the transport
    (ncclGetVersion, ncclCommCount), halo-exchange groups per step, each group's time on the stream
    it ran on (pack, ncclGroupStart ... ncclGroupEnd, unpack: HIP events), and how much of it the
    inner march hid (exposed = the comm chain's end past the inner march's end, per overlapped step)."""
    r0 = rank_info[0]
    grp = [r["group_ms_sum"] / r["timed_groups"] for r in rank_info if r["timed_groups"]]
    tot_g = sum(r["group_ms_sum"] for r in rank_info)
    tot_e = sum(r["exposed_ms_sum"] for r in rank_info)
    return {"transport": r0["comm"]["transport"], "version": r0["comm"]["version"],
            "comm_size": r0["comm"]["comm_size"],
            "groups_per_step": round(max(r["groups"] for r in rank_info) / steps, 3),
            "group_ms": {"mean": round(sum(grp) / len(grp), 4) if grp else None,
                         "max": round(max(r["group_ms_max"] for r in rank_info), 4)},
            "exposed_ms_per_step": round(max(r["exposed_ms_sum"] for r in rank_info) / steps, 4),
            "hidden_frac": round(1.0 - tot_e / tot_g, 4) if tot_g > 0 else None,
            "watchdog_s": r0["comm"]["watchdog_s"],
            # the x2 / x4 steps' form: measured sequential vs overlapped step (or pair) times, the maxima
            # over the ranks, and the level every rank then runs (ocn_ctx_overlap_info)
            "overlap": ({"level": r0["overlap"]["level"], "decided": r0["overlap"]["state"] == 3,
                         "measured_on": {2: "x2 step", 4: "x4 pair"}.get(r0["overlap"]["kind"]),
                         "seq_ms": r0["overlap"]["seq_ms"], "overlapped_ms": r0["overlap"]["overlapped_ms"],
                         "per_rank_level": [r["overlap"]["level"] for r in rank_info]}
                        if r0.get("overlap") else None),
            "per_rank": [{"rank": r["rank"], "groups": r["groups"],
                          "group_ms_mean": round(r["group_ms_sum"] / r["timed_groups"], 4) if r["timed_groups"] else None,
                          "group_ms_max": round(r["group_ms_max"], 4),
                          "exposed_ms_per_step": round(r["exposed_ms_sum"] / steps, 4)} for r in rank_info],
            "source": "HIP events on the stream of each exchange (OCN_TIMER_EXCHANGE / OCN_TIMER_EXPOSED, "
                      "ocn_ctx_stage_stats); groups = ocn_ctx_comm_info exchanges in the timed region"}


def profile_match(amd, d: dict, rec: dict):
    """How a committed counter summary applies to the loaded library: "build" (taken on this exact
    build, ocn_build_id), "kernel code" (the kernel's gfx950 machine code is byte for byte the profiled
    code: the record's code_sha, ocean_model_arch_amd/_codeobj.py), or None."""
    if d.get("build_id") == amd.build_id():
        return "build"
    try:
        from ocean_model_arch_amd import _codeobj
        if rec.get("code_sha") and rec["code_sha"] == _codeobj.kernel_code_sha(amd._lib.LIB_PATH, rec["symbol"]):
            return "kernel code"
    except Exception:
        pass
    return None


def load_traffic(amd, stage: str, cells: int, compact: bool, box, blocks):
    """HBM bytes per launch of `stage` from the committed rocprofv3 PMC summary
    (profiles/pmc_traffic.json, scripts/pmc_traffic.py), or None unless that summary was taken on
    this workload (box, block grid, cells per block) and on this exact library build or the same
    machine code of the kernel (profile_match).  Returns (bytes, match)."""
    path = os.path.join(REPO, "profiles", "pmc_traffic.json")
    try:
        d = json.load(open(path))
        rec = d["kernels"][stage]
        if (list(d.get("box", [])) != list(box) or list(d.get("blocks", [])) != list(blocks) or
                int(rec["cells"]) != cells or bool(rec.get("compact")) != compact):
            return None, None
        match = profile_match(amd, d, rec)
        return (float(rec["hbm_bytes_per_launch"]), match) if match else (None, None)
    except Exception:
        return None, None


SHADER_CLOCK_GHZ = 2.4          # MI355X peak engine clock (MI355X_MICROARCH.md)
SIMDS = 256 * 4


def load_valu(amd, stage: str, launch_ms: float, box, blocks, live_clock=None):
    """The dominant kernel's VALU issue from the committed SQ counter pass (profiles/sq_valu.json,
    scripts/sq_valu.py) -- only for the one-pass launches (single and pair), and only when that pass was taken on this
    exact library build and workload.  issue_floor_ms: its VALU instructions spread over the
    1024 SIMDs at one wave64 instruction per quad-cycle at the peak clock (the time the launch
    would take if VALU issue were its only limit); issue_frac = that floor / the live launch time."""
    if stage not in ("onepass", "onepass2"):
        return None
    try:
        d = json.load(open(os.path.join(REPO, "profiles", "sq_valu.json")))
        if list(d.get("box", [])) != list(box) or list(d.get("blocks", [])) != list(blocks):
            return None
        match = profile_match(amd, d, d["kernels"][stage])
        if not match:
            return None
        pl, pw = d["kernels"][stage]["per_launch"], d["kernels"][stage]["per_wave"]
        floor_ms = pl["SQ_INSTS_VALU"] * 4.0 / SIMDS / (SHADER_CLOCK_GHZ * 1e9) * 1e3
        wc = pw["SQ_WAVE_CYCLES"]
        out = {"insts_per_launch": int(pl["SQ_INSTS_VALU"]), "issue_floor_ms": round(floor_ms, 4),
               "issue_frac": round(floor_ms / launch_ms, 4),
               "per_wave_frac": {"valu_active": round(pw["SQ_ACTIVE_INST_VALU"] / wc, 4),
                                 "wait_inst_any": round(pw["SQ_WAIT_INST_ANY"] / wc, 4),
                                 "wait_any": round(pw["SQ_WAIT_ANY"] / wc, 4)},
               "source": "profiles/sq_valu.json",
               # the 4 cycles per wave64 VALU instruction the floor charges, measured per class at 2 waves
               # per SIMD (scripts/issuebench.hip, profiles/r06/issuebench.txt; event-timed, launch
               # overhead included): f64 mul / add / fma 4.48-4.54, DPP lane move 4.45, v_frexp 4.40,
               # v_cndmask (SGPR condition) 4.54, int32 alone 2.58 but 3.9 interleaved with f64 (the
               # 10 f64 + 6 int32 mix: 4.29 per instruction) -- the pair launch's mix issues at ~4
               "issue_cost": {"cycles_per_inst": 4.0, "source": "profiles/r06/issuebench.txt"},
               "profile_match": match if match == "build" else
               f"{match}: profiled on build {d.get('build_id')}, the kernel's machine code unchanged"}
        clk = d["kernels"][stage].get("clock")
        if clk:   # the counter pass's effective shader clock (GRBM_GUI_ACTIVE / 8 / launch time) and the
            # VALU issue floor at that clock
            floor_clk = pl["SQ_INSTS_VALU"] * 4.0 / SIMDS / (clk["clock_ghz"] * 1e9) * 1e3
            out["effective_clock_ghz"] = clk["clock_ghz"]
            out["clock_source"] = ("GRBM_GUI_ACTIVE / 8 XCDs / dispatch time, mean over the SQ pass's dispatches of this "
                                   "kernel (rocprofv3 --pmc over bench.py " + d.get("bench_args", "--steps 20 --warmup 5") +
                                   "; counter passes serialize dispatches)")
            out["issue_floor_ms_at_clock"] = round(floor_clk, 4)
            out["issue_frac_at_clock"] = round(floor_clk / launch_ms, 4)
        if live_clock and live_clock.get("launches", 0) > 0 and live_clock.get("clock_ghz", 0) > 0 and stage == "onepass2":
            # the clock the pair launches of THIS timed region ran at (ocn_ctx_clock_info: workgroup 0 of
            # each launch counts s_memtime over 100 MHz s_memrealtime ticks) and the VALU floor at it
            g = live_clock["clock_ghz"]
            floor_live = pl["SQ_INSTS_VALU"] * 4.0 / SIMDS / (g * 1e9) * 1e3
            out["live_clock_ghz"] = g
            out["live_clock_source"] = (f"ocn_ctx_clock_info over the timed region: {live_clock['launches']} pair "
                                        f"launches, {live_clock['sampled_ms']} ms sampled by their workgroup 0")
            out["issue_floor_ms_at_live_clock"] = round(floor_live, 4)
            out["issue_frac_at_live_clock"] = round(floor_live / launch_ms, 4)
        vc = d["kernels"][stage].get("valu_classes")
        if vc:   # by class (SQ_INSTS_VALU_* passes): the reference's f64 arithmetic vs everything else
            tot = pl["SQ_INSTS_VALU"]
            clk_ghz = clk["clock_ghz"] if clk else SHADER_CLOCK_GHZ
            other = tot - vc["f64"]
            out["classes"] = {"f64_frac": vc["f64_frac"], "per_launch": vc["per_launch"],
                              "unclassified_frac": vc["unclassified_frac"],
                              # the non-f64 instructions' share of the issue floor at the pass's clock
                              "non_f64_issue_ms": round(other * 4.0 / SIMDS / (clk_ghz * 1e9) * 1e3, 4),
                              "f64_issue_ms": round(vc["f64"] * 4.0 / SIMDS / (clk_ghz * 1e9) * 1e3, 4)}
        return out
    except Exception:
        return None


def launch_ranks(n: int) -> int:
    """torch.distributed.run with n processes on this node (127.0.0.1 rendezvous), each running
    this script with the same arguments; returns its exit status.  The parent stays GPU-free."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100, help="timed steps (SURVEY.md 8d: >= 100)")
    ap.add_argument("--warmup", type=int, default=10, help="untimed warm-up steps (SURVEY.md 8d: 10)")
    ap.add_argument("--steps-per-call", type=int, default=0,
                    help="steps per ocn_ctx_step call in the timed region (1 = the reference's cadence, one "
                         "expl_shallow_water per time-loop iteration, model.f90:146); 0 = all in one call")
    ap.add_argument("--no-lazy-tail", action="store_true",
                    help="every call forms its own tail (OCN_OPT_LAZY_TAIL off)")
    ap.add_argument("--n", type=int, default=4096, help="box interior size (N x N)")
    ap.add_argument("--box", default=None,
                    help="box interior WxH (overrides --n): e.g. 1024x2048, the per-GPU block of config 4 at 8 GPUs, "
                         "timed as a lone block on one GPU")
    ap.add_argument("--basin", choices=["box", "bs", "bs_tr"], default="box",
                    help="box: the synthetic N x N box; bs / bs_tr: the reference's Black Sea basin (data/BS mask "
                         "and parameters, as stored in tests/golden), without / with the tracer (configs 1 and 5)")
    ap.add_argument("--scaling", choices=["strong", "weak"], default="strong")
    ap.add_argument("--graph", action="store_true", help="replay steps as hipGraphs (single process)")
    ap.add_argument("--no-stage-timing", action="store_true",
                    help="no HIP events around the launches (diagnostic: the roofline's live launch time is then "
                         "not measured)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--stages", action="store_true", help="run the 11 reference stages instead of the fused step")
    ap.add_argument("--no-compact", action="store_true", help="fused step on the 2-D real(4) arrays")
    ap.add_argument("--no-march", action="store_true", help="one thread per point in every launch (no register march)")
    ap.add_argument("--no-flip", action="store_true", help="standard steps only (no role-flip steps)")
    ap.add_argument("--no-recompute", action="store_true", help="role-flip calls without the recompute steps")
    ap.add_argument("--no-onepass", action="store_true", help="role-flip calls without the one-pass steps")
    ap.add_argument("--no-known-constants", action="store_true",
                    help="one-pass steps in their general variant only (no known-constant specialization)")
    ap.add_argument("--overlap", type=int, default=-1, choices=[-1, 0, 1, 2],
                    help="halo exchanges beside inner launches: 0 never, 1 standard steps and the one-pass steps' side "
                         "chain, 2 role-flip steps too, "
                         "-1 the library default (2 with RCCL peers, else 1)")
    ap.add_argument("--topography", action="store_true",
                    help="a non-uniform rest depth (a synthetic smooth basin, 20..180 m) instead of 100 m everywhere: "
                         "the one-pass steps read h_r (what a real-depth basin runs)")
    ap.add_argument("--pair", type=int, default=1, choices=[0, 1, 2],
                    help="two one-pass steps per launch (OCN_OPT_PAIR): 1 = known-constant variants on blocks >= 512^2 "
                         "(default), 2 = always (the general variant too), 0 = never")
    ap.add_argument("--no-multi", action="store_true",
                    help="small single blocks: one launch per step (no multi-step launch, OCN_OPT_MULTI)")
    ap.add_argument("--no-tracer-step", action="store_true",
                    help="tracer runs: the role-flip path with the standard tracer stages (no tracer steps, OCN_OPT_TRACER_STEP)")
    ap.add_argument("--no-x4", action="store_true",
                    help="blocks with halo exchanges: x2 single launches (no pairs with one 4-deep exchange, OCN_OPT_X4)")
    ap.add_argument("--no-co-launch", action="store_true",
                    help="tracer runs with x2 steps: the march and the tracer step as two launches on two streams "
                         "(no co-launch, OCN_OPT_CO_LAUNCH)")
    ap.add_argument("--no-batch", action="store_true",
                    help="several blocks on a GPU: one launch per block and launch group (no block batching)")
    ap.add_argument("--watchdog", type=float, default=120.0,
                    help="N > 1: seconds a library call that may wait on a peer (step, synchronize, ...) may take "
                         "before the rank's watchdog aborts the RCCL communicator and the rank exits non-zero "
                         "(ocn_ctx_set_watchdog; 0 = off)")
    ap.add_argument("--blocks", default=None,
                    help="block grid BXxBY (default: one block per GPU); with one GPU, several blocks on it "
                         "exercise the halo-exchange path without RCCL")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # started directly (`python bench.py --gpus N`): launch the N ranks, one process per GPU,
        # before this process touches torch or HIP; rank 0 prints the JSON line
        sys.exit(launch_ranks(args.gpus))
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")

    import torch
    import torch.distributed as dist
    import ocean_model_arch_amd as amd

    torch.cuda.set_device(local_rank)
    bx, by = dims_create(world)
    if args.blocks:
        bx, by = (int(v) for v in args.blocks.lower().split("x"))
        if world > 1 and bx * by != world:
            raise SystemExit("--blocks with several GPUs must give one block per GPU")
    n = args.n
    if args.basin == "box":
        nw, nh = (int(v) for v in args.box.lower().split("x")) if args.box else (n, n)
        nxbox, nybox = (nw, nh) if args.scaling == "strong" else (nw * bx, nh * by)
        basin, sw = amd.BasinConfig(nx=nxbox + 4, ny=nybox + 4), amd.SWConfig()
        workload = f"{nxbox}x{nybox} box"
        if args.topography:   # float32 (nx-4, ny-4), Fortran order, as a basin.par topography file holds it
            import numpy as np
            x = np.linspace(-1.0, 1.0, nxbox, dtype=np.float64)[:, None]
            y = np.linspace(-1.0, 1.0, nybox, dtype=np.float64)[None, :]
            basin.topography = np.asfortranarray((100.0 + 80.0 * np.cos(np.pi * x) * np.cos(np.pi * y)).astype(np.float32))
            workload += ", topography"
    else:
        # the Black Sea basin: mask bits and basin / sw.par parameters exactly as the reference's
        # run uses them (input data of the golden fixture; nothing of the reference runs here)
        from tests.golden import cases
        case = cases.load_e2e("bs_b1x1_s60" if args.basin == "bs" else "bs_b4x2_tr_s60")
        basin = amd.BasinConfig(**case["basin"], mask=case["mask"])
        sw = amd.SWConfig(**case["sw"])
        nxbox, nybox = case["basin"]["nx"] - 4, case["basin"]["ny"] - 4
        workload = f"Black Sea basin {nxbox}x{nybox}" + (" + tracer" if args.basin == "bs_tr" else "")
    model = amd.OceanModel(basin, sw, amd.ParallelConfig(bx, by), rank=rank, nranks=world,
                           device=local_rank)
    parity = None
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))

        def uid_for():
            uid = [amd.make_unique_id() if rank == 0 else None]
            dist.broadcast_object_list(uid, src=0)
            return uid[0]
        model.attach_comm(uid_for())
        if args.watchdog > 0:   # a rank stuck on a peer ends with a message, not a silent time-out
            model.set_watchdog(args.watchdog)
        parity = multi_gpu_parity(amd, dist, rank, world, local_rank, bx, by, uid_for, args.watchdog)
    model.set_fused(not args.stages)
    model.set_compact(not args.no_compact)
    model.set_march(not args.no_march)
    model.set_flip(not args.no_flip)
    model.set_recompute(not args.no_recompute)
    model.set_onepass(not args.no_onepass)
    model.set_known_constants(not args.no_known_constants)
    model.set_overlap(args.overlap)
    model.set_lazy_tail(not args.no_lazy_tail)
    model.set_batch(not args.no_batch)
    model.set_pair(args.pair)
    model.set_multi(not args.no_multi)
    model.set_tracer_step(not args.no_tracer_step)
    model.set_x4(not args.no_x4)
    model.set_co_launch(not args.no_co_launch)
    if args.graph:
        model.set_graph(True)
    model.init()
    model.step(args.warmup, check_every=1).synchronize()
    model.set_stage_timing(not args.graph and not args.no_stage_timing)
    model.stage_times()
    model.clock_info(reset=True)   # the pair launches' in-kernel clock counters from here on
    xchg0 = model.comm_info()["exchanges"]

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    spc = args.steps_per_call if args.steps_per_call > 0 else args.steps
    calls = [min(spc, args.steps - i) for i in range(0, args.steps, spc)]
    barrier()
    n_launch0 = amd._lib.launch_count()
    t0 = time.perf_counter()
    for n_call in calls:
        model.step(n_call, check_every=1)
    lazy = model.tail_pending
    # the timed region ends with every array as the reference leaves it after the last step: a
    # pending call tail (OCN_OPT_LAZY_TAIL) is formed inside it
    model.complete()
    model.synchronize()
    barrier()
    dt = time.perf_counter() - t0
    launches = amd._lib.launch_count() - n_launch0
    live_clock = model.clock_info()
    stats = model.stage_stats()
    times = {k: (v[0], v[1]) for k, v in stats.items()}
    compact = model.compact_active
    flip = model.flip_active
    rc = model.recompute_active
    one = model.onepass_active
    one_zero = True if model.onepass_zero else "h" if model.onepass_hr else False
    # pair launches ran in the timed region: their timer counted them (graph replays: no timers)
    pair = ("onepass2" in times or "onepass2_last" in times) if times else model.pair_active
    multi = ("onepass_multi" in times) if times else model.multi_active
    # (x4 pairs: the pair launches of blocks with exchanges; 1-step calls run one every second call)
    x4 = (("onepass2" in times) if times else model.x4_active) and bx * by > 1
    co = model.co_launched
    model_overlap = model.overlap_level
    rank_info = None
    if world > 1:
        t = torch.tensor([dt], device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
        # per rank: the exchanges of the timed region (events on the stream each runs on) and the
        # dominant launch's time, for the rccl object and the per-GPU roofline (rank 0 reports)
        ci = model.comm_info()
        ex, exp_ = stats.get("exchange", (0.0, 0, 0.0)), stats.get("exposed", (0.0, 0, 0.0))
        mine = {"rank": rank, "comm": ci, "groups": ci["exchanges"] - xchg0, "timed_groups": ex[1],
                "group_ms_sum": ex[0], "group_ms_max": ex[2], "exposed_ms_sum": exp_[0], "exposed_n": exp_[1],
                "stage_ms": {s: v[0] / v[1] for s, v in stats.items() if v[1]}, "cells": model.interior_cells,
                "overlap": model.overlap_info()}
        rank_info = [None] * world
        dist.all_gather_object(rank_info, mine)

    cells = nxbox * nybox
    value = cells * args.steps / dt
    local_cells = model.interior_cells
    out = None
    if rank == 0:
        ring = bx * by > 1
        ntr = sw.tracer_num if sw.use_tracers > 0 else 0
        stage_tab = STAGE_BYTES_COMPACT if compact else STAGE_BYTES
        kbytes = stage_tab if args.stages else fused_bytes(compact, calls, flip, rc, ring, one, ntr, one_zero, lazy,
                                                           pair, multi)
        b_path = sum(stage_tab.values()) if args.stages else step_bytes(compact, calls, flip, rc, ring, one, ntr,
                                                                          one_zero, lazy, pair, multi)
        stage_ms = {s: ms / cnt for s, (ms, cnt) in times.items() if s in kbytes}
        roof = None
        if stage_ms:   # the dominant kernel: the most device time over the timed steps
            dom = max(stage_ms, key=lambda s: times[s][0])
            alg = kbytes[dom] * local_cells
            achieved = alg / (stage_ms[dom] * 1e-3) / 1e9
            valu = load_valu(amd, dom, stage_ms[dom], [nxbox, nybox], [bx, by], live_clock)
            frac = achieved / HBM_PEAK_GBS
            # the bound: VALU issue when its floor (at the clock the counter pass measured) takes a larger
            # share of the launch than the HBM bytes do; achieved / peak / frac stay the HBM figures
            issue = (valu.get("issue_frac_at_live_clock", valu.get("issue_frac_at_clock", valu.get("issue_frac")))
                     if valu else None)
            traffic, tmatch = load_traffic(amd, dom, local_cells, compact, [nxbox, nybox], [bx, by])
            roof = {"bound": "valu" if issue is not None and issue > frac else "hbm", "kernel": dom,
                    "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                    "unit": "GB/s", "frac": round(frac, 4),
                    "traffic": traffic,
                    **({"traffic_match": tmatch} if tmatch else {}),
                    "valu": valu,
                    "alg_bytes_per_launch": int(alg), "launch_ms": round(stage_ms[dom], 4)}
            if dom in ("onepass2", "onepass2_last") and live_clock.get("launches", 0) > 0:
                # the shader clock the pair launches of this timed region ran at, measured in the kernel
                roof["live_clock"] = {**live_clock, "source": "ocn_ctx_clock_info (workgroup 0 of each pair launch: "
                                                              "s_memtime ticks / 100 MHz s_memrealtime ticks)"}
            if roof["bound"] == "valu":
                roof["bound_note"] = ("VALU issue: issue_frac_at_live_clock (the SQ_INSTS_VALU floor at the clock "
                                      "measured in the kernel over this timed region / the launch time; "
                                      "issue_frac_at_clock without it) exceeds the HBM fraction; frac is the HBM fraction")
        step_gbs = B_ALG * cells * args.steps / dt / 1e9 / world
        moved = b_path * cells * args.steps / dt / 1e9 / world
        out = {"metric": METRIC, "value": value, "unit": "cell-updates/s", "n_gpus": world,
               "steps": args.steps, "warmup": args.warmup, "ms_per_step": dt / args.steps * 1e3,
               "higher_is_better": True, "scaling": args.scaling, "vs_baseline": None, "dtype": "f64",
               "data": (("synthetic (Gaussian SSH hump in a closed box with a smooth synthetic bottom, 20..180 m)"
                         if args.topography else
                         "synthetic (Gaussian SSH hump in a closed flat-bottom box, SURVEY.md 8d)") if args.basin == "box"
                        else "the reference's data/BS mask and basin parameters, its Gaussian initial state"),
               "config": {"workload": f"{workload}, {bx}x{by} blocks ({bx * by // world} per GPU), "
                                      f"{'sw.par defaults' if args.basin == 'box' else 'BS sw.par'}, tau=1s",
                          "basin": args.basin,
                          "box": [nxbox, nybox], "blocks": [bx, by], "graph": bool(args.graph),
                          "step": "reference stages" if args.stages else "fused groups",
                          "static_fields": "compact" if compact else "2-D arrays",
                          "march": bool(compact and not args.stages and not args.no_march),
                          "role_flip_steps": flip, "recompute_steps": rc, "onepass_steps": one,
                          "onepass_known_constants": one_zero is True,
                          "onepass_variant": ("known constants" if one_zero is True else
                                              "known constants, h_r read" if one_zero == "h" else "general")
                                             if one else None,
                          "onepass_pairs": ("two one-pass steps per launch (OCN_OPT_PAIR): the first step's "
                                            "new state kept on chip") if pair else False,
                          "multi_step_launch": ("a call's steps in one launch, a grid barrier between "
                                                "steps (OCN_OPT_MULTI)") if multi else False,
                          "tracer_steps": model.tracer_step_active if sw.use_tracers > 0 else None,
                          "x4_pairs": ("two x2 steps per launch, one 4-deep state exchange per two steps (OCN_OPT_X4)"
                                       if x4 else False) if bx * by > 1 else None,
                          "co_launch": ("each x2 step's march and the previous state's tracer step as one launch "
                                        "(OCN_OPT_CO_LAUNCH)" if co else False) if sw.use_tracers > 0 and bx * by > 1 else None,
                          "steps_per_call": spc, "calls": len(calls),
                          "call_tail": ("pending between calls (OCN_OPT_LAZY_TAIL), formed once by ocn_ctx_complete "
                                        "inside the timed region") if lazy else "formed by every call",
                          "kernel_launches_per_step": round(launches / args.steps, 2),
                          "block_batching": bool(not args.no_batch and bx * by // world > 1),
                          "overlap": model_overlap,
                          "parallelism": (f"block-decomposition {bx}x{by}, RCCL halos" if world > 1 else
                                          "1 block" if bx * by == 1 else f"{bx}x{by} blocks, local halo copies")},
               "build_id": amd.build_id(),
               **({"pair_rows_override": os.environ["OCN_PAIR_ROWS"]} if os.environ.get("OCN_PAIR_ROWS") else {}),
               "roofline": roof,
               # whole-step rates (not the roofline, which is `roofline`: the dominant kernel's bytes
               # over its own time): the bytes this path moves per step, and -- for comparison with
               # SURVEY.md 8d only -- the reference's 11-stage B_alg at this step rate
               "step_moved": {"bytes_per_cell": round(b_path, 1), "GBps_per_gpu": round(moved, 1),
                              "frac_of_peak": round(moved / HBM_PEAK_GBS, 4)},
               "reference_B_alg_equivalent": {"bytes_per_cell": B_ALG, "GBps_per_gpu": round(step_gbs, 1),
                                              "note": "bytes the reference's 11 stages would move at this step "
                                                      "rate; not moved by this path, not a roofline fraction"},
               "stage_ms": {s: round(v, 4) for s, v in stage_ms.items()}}
        if args.stages:   # each stage's rate on the reference's bytes and on the bytes it moves
            out["stage_frac"] = {s: {"survey_B": round(STAGE_BYTES[s] * local_cells / (v * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                                     "moved_B": round(kbytes[s] * local_cells / (v * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}
                                 for s, v in stage_ms.items()}
        if world > 1:
            out["multi_gpu_parity_512"] = parity
            out["rccl"] = rccl_report(rank_info, args.steps)
            if roof:   # the dominant launch on every GPU (its own block's cells, its own launch time)
                roof["per_gpu"] = [
                    {"rank": r["rank"], "launch_ms": round(r["stage_ms"][roof["kernel"]], 4),
                     "frac": round(kbytes[roof["kernel"]] * r["cells"] / (r["stage_ms"][roof["kernel"]] * 1e-3) / 1e9 /
                                   HBM_PEAK_GBS, 4)}
                    for r in rank_info if roof["kernel"] in r["stage_ms"]]
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline()
        elif world > 1:
            out["cpu_baseline"] = {"value": None, "reason": "timed at N=1 only (the same host CPU path; the "
                                                            "N=1 line of the scaling run carries it)"}
    model.close()
    if world > 1:
        dist.destroy_process_group()
    if out is not None:
        if world > 1 and parity is not True:
            # the N-rank path disagrees with the single-process block grid: no number
            print(json.dumps({"error": "multi_gpu_parity_512 failed", "multi_gpu_parity_512": parity}), flush=True)
            sys.exit(3)
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
