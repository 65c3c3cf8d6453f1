/*
 * ocn_sw.h -- C ABI of the MI355X-native shallow-water barotropic step.
 *
 * Drop-in boundary for the reference's kernel and PSy layers
 * (Andrcraft9/ocean_model_arch; citations are path:line in that tree):
 *
 *  - Kernel layer: one entry per SW stage.  Each replaces the Fortran kernel
 *    `S(nx_start,nx_end,ny_start,ny_end,bnd_x1,bnd_x2,bnd_y1,bnd_y2,[scalars],arrays...)`
 *    (every argument by reference, explicit-shape arrays) and its CUDA-Fortran twin
 *    `S_gpu<<<grid,16x16,0,stream(k)>>>` (gpu/kernel/ *_gpu.f90).  Same argument order,
 *    same meaning, same write set, bitwise-identical results.
 *  - PSy layer: a model context that owns the per-block device storage of ocean_type /
 *    grid_type (core/ocean.f90:14-48, core/grid.f90:23-90), runs one stage plus its halo
 *    sync (envoke, core/kernel_interface.f90:48-119) or the whole step
 *    (expl_shallow_water, control/shallow_water/shallow_water.f90:22-94), and exchanges
 *    1-wide 8-direction halos (sync/hybrid_sync, shared/mpp/sync.f90:294-556) between blocks
 *    of this process and, over RCCL, with blocks of other processes (one block per GPU).
 *
 * Conventions
 *  - Indices are the reference's 1-based global Fortran indices.
 *  - Arrays are column-major A(bnd_x1:bnd_x2, bnd_y1:bnd_y2); a pointer is the DEVICE
 *    address of A(bnd_x1,bnd_y1); the leading dimension is ocn_block.pitch elements
 *    (>= bnd_x2-bnd_x1+1; r4 and r8 arrays of one block share the pitch).
 *  - `stream` is a hipStream_t passed as an opaque pointer (NULL = default stream).
 *    Entries are asynchronous on that stream; they never allocate or synchronise.
 *  - Return value: OCN_OK, or an OCN_ERR_* code (ocn_last_error() describes it).
 *    The reference kernels return nothing and ignore CUDA status; here every status is
 *    checked and reported.
 *  - No torch types; plain pointers and sizes only.
 */
#ifndef OCN_SW_H
#define OCN_SW_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OCN_ABI_VERSION 5

enum {
    OCN_OK = 0,
    OCN_ERR_ARG = 1,       /* bad argument (null pointer, bounds, pitch, id) */
    OCN_ERR_HIP = 2,       /* HIP runtime error */
    OCN_ERR_COMM = 3,      /* RCCL error or missing communicator */
    OCN_ERR_STATE = 4,     /* call out of order (e.g. step before init) */
    OCN_ERR_BLOWUP = 5     /* check_ssh_err: |ssh| >= 1e4 on a sea point */
};

/* Block geometry (core/decomposition.f90:40-81, block k of domain_type). */
typedef struct ocn_block {
    int32_t nx_start, nx_end, ny_start, ny_end;   /* interior (bnx_start..) */
    int32_t bnd_x1, bnd_x2, bnd_y1, bnd_y2;       /* array bounds (bbnd_x1..) */
    int64_t pitch;                                 /* leading dimension, elements */
} ocn_block;

/* ---------------------------------------------------------------- kernel layer */
/* kernel/shallow_water/vel_ssh.f90:69  sw_update_ssh_kernel */
int ocn_sw_update_ssh(const ocn_block *b, double tau,
                      const float *lu, const float *dx, const float *dy, const float *dxh, const float *dyh,
                      const double *hhu, const double *hhv, double *sshn, const double *sshp,
                      const double *ubrtr, const double *vbrtr, void *stream);

/* kernel/shallow_water/depth.f90:101  hh_update_kernel */
int ocn_hh_update(const ocn_block *b,
                  const float *lu, const float *llu, const float *llv, const float *luh,
                  const float *dx, const float *dy, const float *dxt, const float *dyt,
                  const float *dxh, const float *dyh, const float *dxb, const float *dyb,
                  double *hqn, double *hun, double *hvn, double *hhn,
                  const double *sh, const double *h_r, void *stream);

/* vel_ssh.f90:247  uv_trans_vort_kernel (nlev = 1) */
int ocn_uv_trans_vort(const ocn_block *b, const float *luu,
                      const float *dxt, const float *dyt, const float *dxb, const float *dyb,
                      const double *u, const double *v, double *vort, void *stream);

/* vel_ssh.f90:283  uv_trans_kernel (nlev = 1; hq accepted and unused, as in the reference) */
int ocn_uv_trans(const ocn_block *b, const float *lcu, const float *lcv, const float *luu,
                 const float *dxh, const float *dyh, const double *u, const double *v,
                 const double *vort, const double *hq, const double *hu, const double *hv,
                 const double *hh, double *RHSx, double *RHSy, void *stream);

/* kernel/shallow_water/mixing.f90:14  stress_components_kernel (nlev = 1) */
int ocn_stress_components(const ocn_block *b, const float *lu, const float *luu,
                          const float *dx, const float *dy, const float *dxt, const float *dyt,
                          const float *dxh, const float *dyh, const float *dxb, const float *dyb,
                          const double *u, const double *v, double *str_t, double *str_s, void *stream);

/* vel_ssh.f90:375  uv_diff2_kernel (nlev = 1; hu/hv accepted and unused, as in the reference) */
int ocn_uv_diff2(const ocn_block *b, const float *lcu, const float *lcv,
                 const float *dx, const float *dy, const float *dxt, const float *dyt,
                 const float *dxh, const float *dyh, const float *dxb, const float *dyb,
                 const double *mu, const double *str_t, const double *str_s,
                 const double *hq, const double *hu, const double *hv, const double *hh,
                 double *RHSx, double *RHSy, void *stream);

/* vel_ssh.f90:108  sw_update_uv */
int ocn_sw_update_uv(const ocn_block *b, double tau, const float *lcu, const float *lcv,
                     const float *dxt, const float *dyt, const float *dxh, const float *dyh,
                     const float *dxb, const float *dyb,
                     const double *hhu, const double *hhun, const double *hhup,
                     const double *hhv, const double *hhvn, const double *hhvp,
                     const double *hhh, const double *ssh,
                     const double *ubrtr, double *ubrtrn, const double *ubrtrp,
                     const double *vbrtr, double *vbrtrn, const double *vbrtrp,
                     const float *rdis, const float *rlh_s,
                     const double *RHSx, const double *RHSy, const double *RHSx_adv,
                     const double *RHSy_adv, const double *RHSx_dif, const double *RHSy_dif,
                     void *stream);

/* vel_ssh.f90:197  sw_next_step (writes interior + halo ring) */
int ocn_sw_next_step(const ocn_block *b, double time_smooth,
                     const float *lu, const float *lcu, const float *lcv,
                     double *ssh, double *sshn, double *sshp,
                     double *ubrtr, double *ubrtrn, double *ubrtrp,
                     double *vbrtr, double *vbrtrn, double *vbrtrp, void *stream);

/* depth.f90:164  hh_shift_kernel (time_smooth is a module variable there; an argument here) */
int ocn_hh_shift(const ocn_block *b, double time_smooth,
                 const float *lu, const float *llu, const float *llv, const float *luh,
                 double *hq, double *hqp, double *hqn, double *hu, double *hup, double *hun,
                 double *hv, double *hvp, double *hvn, double *hh, double *hhp, double *hhn,
                 void *stream);

/* depth.f90:14  hh_init_kernel (full_free_surface is a module variable there; an argument here) */
int ocn_hh_init(const ocn_block *b, int32_t full_free_surface,
                const float *lu, const float *llu, const float *llv, const float *luh,
                const float *dx, const float *dy, const float *dxt, const float *dyt,
                const float *dxh, const float *dyh, const float *dxb, const float *dyb,
                double *hq, double *hqp, double *hqn, double *hu, double *hup, double *hun,
                double *hv, double *hvp, double *hvn, double *hh, double *hhp, double *hhn,
                const double *sh, const double *shp, const double *h_r, void *stream);

/* vel_ssh.f90:40  check_ssh_err_kernel: device reduction; *nbad (device int32) += bad points */
int ocn_check_ssh_err(const ocn_block *b, const float *lu, const double *ssh, int32_t *nbad_device,
                      void *stream);

/* kernel/tracer/leapfrog_tracer.f90:13  tran_diff_fluxes_kernel (flux_x on lcu, flux_y on lcv) */
int ocn_tran_diff_fluxes(const ocn_block *b, const float *lcu, const float *lcv,
                         const float *dxt, const float *dyt, const float *dxh, const float *dyh,
                         const double *hhu, const double *hhv, const double *ff, const double *ffp,
                         const double *uu, const double *vv, const double *mu, double factor_mu,
                         double *flux_x, double *flux_y, void *stream);

/* leapfrog_tracer.f90:94  tran_diff_tracer_kernel */
int ocn_tran_diff_tracer(const ocn_block *b, const float *lu, const float *dx, const float *dy, double tau,
                         const double *hhqn, const double *hhqp, const double *flux_x, const double *flux_y,
                         const double *ffp, double *ffn, void *stream);

/* leapfrog_tracer.f90:138  tracer_next_step_kernel (writes interior + halo ring) */
int ocn_tracer_next_step(const ocn_block *b, double time_smooth, const float *lu, const double *ffn,
                         double *ffp, double *ff, void *stream);

/* ---------------------------------------------------------------- PSy layer: model context */

/* Field ids: storage of ocean_type / grid_type restricted to what the SW step touches. */
enum {
    /* real(4) */
    OCN_LU = 0, OCN_LUU, OCN_LUH, OCN_LCU, OCN_LCV, OCN_LLU, OCN_LLV,
    OCN_DX, OCN_DY, OCN_DXT, OCN_DYT, OCN_DXH, OCN_DYH, OCN_DXB, OCN_DYB, OCN_RLH_S, OCN_R_DISS,
    OCN_NUM_R4,
    /* real(8) */
    OCN_SSH = 32, OCN_SSHN, OCN_SSHP, OCN_UBRTR, OCN_UBRTRN, OCN_UBRTRP, OCN_VBRTR, OCN_VBRTRN, OCN_VBRTRP,
    OCN_HHQ, OCN_HHQ_P, OCN_HHQ_N, OCN_HHU, OCN_HHU_P, OCN_HHU_N, OCN_HHV, OCN_HHV_P, OCN_HHV_N,
    OCN_HHH, OCN_HHH_P, OCN_HHH_N, OCN_HHQ_REST, OCN_VORT, OCN_STR_T, OCN_STR_S, OCN_MU,
    OCN_RHSX, OCN_RHSY, OCN_RHSX_ADV, OCN_RHSY_ADV, OCN_RHSX_DIF, OCN_RHSY_DIF,
    OCN_FIELD_END,
    /* real(8) tracer storage (core/ocean.f90:38-41), present when ocn_sw_params.use_tracers > 0 */
    OCN_FLUX_X = OCN_FIELD_END, OCN_FLUX_Y, OCN_TRACER_BASE
};
#define OCN_NUM_R8 (OCN_FIELD_END - OCN_SSH)
/* ff1(k), ff1p(k), ff1n(k) of tracer k = 1..tracer_num */
#define OCN_FF1(k) (OCN_TRACER_BASE + 3 * ((k) - 1))
#define OCN_FF1P(k) (OCN_TRACER_BASE + 3 * ((k) - 1) + 1)
#define OCN_FF1N(k) (OCN_TRACER_BASE + 3 * ((k) - 1) + 2)

/* Stage ids, in the order of expl_shallow_water (shallow_water.f90:36-92). */
enum {
    OCN_STAGE_SW_UPDATE_SSH = 0, OCN_STAGE_HH_UPDATE, OCN_STAGE_UV_TRANS_VORT, OCN_STAGE_UV_TRANS,
    OCN_STAGE_STRESS_COMPONENTS, OCN_STAGE_UV_DIFF2, OCN_STAGE_SW_UPDATE_UV, OCN_STAGE_SW_NEXT_STEP,
    OCN_STAGE_HH_SHIFT, OCN_STAGE_HH_INIT, OCN_STAGE_CHECK_SSH_ERR, OCN_NUM_STAGES
};
/* Tracer stage ids, in the order of expl_tracer (control/tracer.f90:42-58). */
enum { OCN_TSTAGE_TRAN_DIFF_FLUXES = 0, OCN_TSTAGE_TRAN_DIFF_TRACER, OCN_TSTAGE_TRACER_NEXT_STEP, OCN_NUM_TSTAGES };

/* Basin description (configs/basinpar.f90:53-91, basin.par lines 1-18) */
typedef struct ocn_basin {
    int32_t nx, ny;
    double dxst, dyst, rlon, rlat;
    int32_t curve_grid;                 /* 0 carthesian, 1 undistorted sphere */
    double rotation_on_lon, rotation_on_lat;
} ocn_basin;

/* SW switches (configs/sw.f90:34-41, sw.par lines 1-7) */
typedef struct ocn_sw_params {
    int32_t full_free_surface, trans_terms, ksw_lat;
    double time_smooth, lvisc_2;
    int32_t use_tracers, tracer_num;
} ocn_sw_params;

/* Decomposition request (parallel.par + _DD_MANUAL_BLOCK_GRID_, decomposition.f90:856-858) */
typedef struct ocn_decomp {
    int32_t bnx, bny;        /* block grid (total, not per process) */
    int32_t nranks, rank;    /* processes; blocks are dealt by create_uniform_decomposition */
    int32_t device;          /* HIP device of this process */
} ocn_decomp;

/* Per-block information returned to hosts (block k of this process, k = 0..count-1). */
typedef struct ocn_block_info {
    ocn_block geom;
    int32_t bm, bn;                       /* block coordinates in the block grid (1-based) */
    int32_t nbr_rank[8];                  /* rank of neighbour in dirs 1..8 (kernel_macros.fi:4-12); -1 land, -2 outside */
    int32_t nbr_k[8];                     /* local index on that rank, or -1 */
} ocn_block_info;

typedef struct ocn_ctx ocn_ctx;

/* Host-only (no GPU needed): the blocks rank dec->rank owns, as ocn_ctx_create would make them.
 * Writes min(count, cap) entries; *count = number of blocks. */
int ocn_decompose(const ocn_basin *basin, const ocn_decomp *dec, const int32_t *mask,
                  ocn_block_info *out, int32_t cap, int32_t *count);

/* Host-only schedule of one halo exchange of the real(8) fields `field_ids` for rank dec->rank:
 * the copies/messages ocn_ctx_sync performs (syncborder_block2D_gen_all.fi semantics).
 * LOCAL: strip src of local block k_src -> strip dst of local block k.
 * SEND : strip src of local block k_src -> message to `peer` at element `offset`.
 * RECV : message from `peer` at element `offset` -> strip dst of local block k.
 * Rects are inclusive global 1-based indices; strips are walked column-major. */
enum { OCN_HALO_LOCAL = 0, OCN_HALO_SEND = 1, OCN_HALO_RECV = 2 };
typedef struct ocn_halo_msg {
    int32_t kind, peer, k, k_src, field;
    int32_t dst_x0, dst_x1, dst_y0, dst_y1;
    int32_t src_x0, src_x1, src_y0, src_y1;
    int32_t count;
    int64_t offset;
} ocn_halo_msg;
int ocn_halo_schedule(const ocn_basin *basin, const ocn_decomp *dec, const int32_t *mask,
                      const int32_t *field_ids, int32_t nfields, ocn_halo_msg *out, int32_t cap,
                      int32_t *count);

/* Create a context: decomposes the basin (mask = int32 global (nx,ny) column-major, 0 = sea,
 * 1 = land, or NULL for the closed box of tools/io.f90:49-59), allocates every field of every
 * local block on `device` (zero-filled, as data_types.f90:517-533). */
int ocn_ctx_create(const ocn_basin *basin, const ocn_sw_params *sw, const ocn_decomp *dec,
                   const int32_t *mask, ocn_ctx **out);
int ocn_ctx_destroy(ocn_ctx *ctx);

int ocn_ctx_block_count(const ocn_ctx *ctx);
int ocn_ctx_block_info(const ocn_ctx *ctx, int k, ocn_block_info *out);
/* Device pointer of field `id` of local block k (element (bnd_x1,bnd_y1)); NULL on error. */
void *ocn_ctx_field(const ocn_ctx *ctx, int k, int id);
/* Compute stream of the context (hipStream_t). */
void *ocn_ctx_stream(const ocn_ctx *ctx);

/* RCCL: unique id (128 bytes) made on rank 0, broadcast by the host, then attached. */
int ocn_comm_unique_id(void *out_id, int32_t nbytes);
int ocn_ctx_attach_comm(ocn_ctx *ctx, const void *unique_id, int32_t nbytes);
/* Test transport: the n ranks of one decomposition as n contexts of ONE process on one device (n >= 1)
 * (ctxs[i] = rank i of nranks = n), each then driven by its own host thread.  Replaces only the
 * RCCL calls (the per-peer ncclRecv/ncclSend of an exchange become device copies between the
 * contexts' message buffers behind event handshakes; the role-flip vote's ncclAllReduce a device
 * max over the contexts); every other part of the multi-rank path is the production one.  Call
 * before ocn_ctx_init_state; the contexts may be destroyed in any order. */
int ocn_ctx_attach_loopback(ocn_ctx *const *ctxs, int32_t n);

/* What a multi-rank run reports about its transport (bench.py's `rccl` object): transport 0 = none,
 * 1 = RCCL (nccl_version = ncclGetVersion, comm_size / comm_rank = ncclCommCount /
 * ncclCommUserRank), 2 = loopback; exchanges = halo exchanges with remote peers enqueued so far (one
 * ncclGroupStart ... ncclGroupEnd group each), exchanges_done = the id of the last of them whose end
 * the device has reached (polled from events while a watchdog is set, else -1). */
typedef struct ocn_comm_info {
    int32_t transport, nccl_version, comm_size, comm_rank;
    int64_t exchanges, exchanges_done;
    double watchdog_s;
} ocn_comm_info;
int ocn_ctx_comm_info(ocn_ctx *ctx, ocn_comm_info *out);
/* The x2 / x4 steps' overlap with OCN_OPT_OVERLAP auto (-1) and peers on other ranks: the first step
 * of a sequence's kind (not the one that opens it) runs exchange-then-march, the next the inner part
 * beside the exchange, each timed with events; the next vote max-reduces both times over the ranks
 * and every rank keeps the faster form.  level = the OCN_OPT_OVERLAP level in effect; state 0 =
 * nothing measured, 1 = the sequential step measured, 2 = both (not yet voted), 3 = decided; kind =
 * the form measured (2: x2 steps, 4: x4 pairs); seq_ms / overlapped_ms = the times (after the
 * decision: the maxima over the ranks it used).  The reference's hybrid overlap mode
 * (core/kernel_interface.f90:105-117) has no such choice. */
typedef struct ocn_overlap_info {
    int32_t level, state, kind, pad;
    double seq_ms, overlapped_ms;
} ocn_overlap_info;
int ocn_ctx_overlap_info(ocn_ctx *ctx, ocn_overlap_info *out);
/* The shader clock the two-step launches (the dominant kernel: MarchStep pairs) ran at, measured in
 * the kernel: workgroup 0 of every pair launch counts the s_memtime ticks and the 100 MHz
 * s_memrealtime ticks over its tiles.  launches = pair launches sampled, clock_ghz = the ticks'
 * ratio (0 with none), sampled_ms = the real time sampled.  Device-wide (every context on the
 * context's device) since the last reset; reset != 0 zeroes the counters after reading them.
 * Synchronises the context's stream.  Telemetry only: no counterpart in the reference. */
typedef struct ocn_clock_info {
    int64_t launches;
    double clock_ghz, sampled_ms;
} ocn_clock_info;
int ocn_ctx_clock_info(ocn_ctx *ctx, int32_t reset, ocn_clock_info *out);
/* Host-side watchdog (seconds > 0; 0 = off): a thread of the context watches every call that may
 * take part in a collective (init_state, step, complete, synchronize, sync, stage, tracer_stage,
 * download, upload, output_r4).  One that has not returned after `seconds` is ended: the watchdog
 * prints "ocn watchdog: rank R of N: <call> ... last completed exchange id D of E" to stderr, aborts
 * the RCCL communicator (ncclCommAbort: RCCL's kernels waiting on a peer exit) or fails the loopback
 * group, and the call returns OCN_ERR_COMM with that message; if it still has not returned 10 s
 * later, the watchdog ends the process with exit status 3 (no exec).  The reference's analogue is
 * abort_model -> mpi_abort (shared/errors.f90:30-37), which has no timeout of its own. */
int ocn_ctx_set_watchdog(ocn_ctx *ctx, double seconds);

/* Bottom topography (basin.par line 20, control/init_data.f90:111-121): the real(4) file's values,
 * the (nx-4) x (ny-4) interior points in Fortran order (tools/io.f90:84-176 read_data2D_real4);
 * h = NULL: none (100 m everywhere).  Used by the next ocn_ctx_init_state. */
int ocn_ctx_set_topography(ocn_ctx *ctx, const float *h, int64_t count);
/* Initial state: init_grid_data + init_ocean_data (control/init_data.f90:29-125). */
int ocn_ctx_init_state(ocn_ctx *ctx);

/* sync(domain, field) for one field over all local blocks (+ remote neighbours). */
int ocn_ctx_sync(ocn_ctx *ctx, int field_id);
/* envoke(stage): the stage on every local block, then its sync list (sw_interface.f90). */
int ocn_ctx_stage(ocn_ctx *ctx, int stage_id, double tau);
/* envoke of tracer stage `stage_id` (OCN_TSTAGE_*) for tracer k (1-based, data_id), then its
 * sync list (interface/tracer/tracer_interface.f90). */
int ocn_ctx_tracer_stage(ocn_ctx *ctx, int stage_id, int tracer, double tau);
/* nsteps model steps (model.f90:146-160): expl_shallow_water(tau), then expl_tracer(tau) when
 * use_tracers > 0.  check_every: run check_ssh_err every N steps (0 = never). */
int ocn_ctx_step(ocn_ctx *ctx, double tau, int32_t nsteps, int32_t check_every);
/* Wait for the context's stream; returns OCN_ERR_BLOWUP if a check found |ssh| >= 1e4, and
 * OCN_ERR_HIP if a multi-step launch's grid barrier timed out since the last synchronize (the
 * results are invalid; ocn_ctx_init_state starts over).  With a communicator attached (RCCL or
 * loopback) this is a COLLECTIVE: the blow-up counts are max-reduced over the ranks
 * (check_ssh_err_kernel -> abort_model stops every rank, shared/errors.f90:30-37), so every rank
 * must call it, in the same order relative to its steps; a rank that skips it leaves the others
 * waiting in the reduction. */
int ocn_ctx_synchronize(ocn_ctx *ctx);
/* Form a pending call tail now (OCN_OPT_LAZY_TAIL): afterwards every array holds what the
 * reference leaves after the last step run.  Every entry that reads or writes fields, hands out a
 * pointer, runs a stage or a sync, or sets an option does this first; a host that reads device
 * memory by other means calls it itself.  Asynchronous on the context stream. */
int ocn_ctx_complete(ocn_ctx *ctx);

/* Host <-> device copies of a whole field of local block k (host array: Fortran order,
 * leading dim bnd_x2-bnd_x1+1, 4 or 8 bytes per element by field kind). Synchronous. */
int ocn_ctx_download(ocn_ctx *ctx, int k, int field_id, void *host);
int ocn_ctx_upload(ocn_ctx *ctx, int k, int field_id, const void *host);
/* Output record of one field of local block k (control/output.f90:32-174 bufwp4%copy_from_real8
 * + tools/io.f90:276-386 write_data2D_real4): the interior nx_start..nx_end x ny_start..ny_end,
 * Fortran order, as real(4) (round to nearest from real(8)), with `undef` where |lu| < 0.5.
 * Converted on the device; host receives (nx_end-nx_start+1)*(ny_end-ny_start+1) floats. Synchronous. */
int ocn_ctx_output_r4(ocn_ctx *ctx, int k, int field_id, float undef, float *host);

/* Execution options.
 *  OCN_OPT_GRAPH: replay each step as one hipGraph (single-process runs).
 *  OCN_OPT_OVERLAP (default -1 = auto): with halo exchanges, run each exchange on a second stream
 *  beside the launches' inner parts (points that neither read halos nor feed the exchange): 1 = in
 *  the standard steps and in the one-pass steps (there the frame launches and both exchanges as one
 *  chain on the second stream beside the whole inner march), 2 = in the role-flip steps too,
 *  0 = never (same results bit for bit); auto
 *  is 2 when the context exchanges with other ranks (RCCL or loopback attached, nranks > 1), else
 *  1.  ocn_ctx_get_option returns the level in effect.
 *  OCN_OPT_STAGE_TIMING: bracket every launch group with HIP events on the context stream.
 *  OCN_OPT_FUSED (default 1): ocn_ctx_step runs the step as 4 fused launch groups and 3 halo
 *  syncs (same results and final state bit for bit); 0 = the 11 envoke stages of the reference.
 *  OCN_OPT_COMPACT (default 1): the fused step -- and the reference stages run by ocn_ctx_step
 *  with OCN_OPT_FUSED 0 or by ocn_ctx_stage -- read the real(4) masks as one bit-packed byte
 *  per point and the grid metrics as one value per row, when that is exact for the current
 *  real(4) fields (checked when they were last set; same results bit for bit).  Handing out a
 *  real(4) pointer with ocn_ctx_field disables this until it is set to 1 again, which also
 *  rebuilds the tables from the fields at the next ocn_ctx_step.
 *  OCN_OPT_MARCH (default 1): with the compact tables, the stencil launches that have a
 *  register-march form (fused A, fused B, hh_init) run as one (same results bit for bit);
 *  0 = one thread per point.
 *  OCN_OPT_FLIP (default 1): with compact tables and march, no tracers: every step of an
 *  ocn_ctx_step call but the last replaces sw_next_step's copies (ssh := sshn, ubrtr := ubrtrn,
 *  vbrtr := vbrtrn) by swapping the two buffers of each pair inside the library, and runs its
 *  time filters inside fused B (same results bit for bit; the pointers of ocn_ctx_field are the
 *  same after the call).  Needs the pairs to agree outside their write sets and, with halo
 *  exchanges, the halo ring of ssh, ubrtr, vbrtr, hhu, hhv, hhq_rest to hold the neighbours'
 *  values; both hold from ocn_ctx_init_state on and are checked on the device whenever fields
 *  were uploaded or handed out (with an RCCL communicator: at every call, all ranks deciding
 *  together); otherwise the standard step runs.
 *  OCN_OPT_RECOMPUTE (default 1): in such calls (full_free_surface = 1, no a8 / a9 work on the
 *  halo ring, so one block without halo exchanges), steps 2..K-1 form hhq, hhu_p, hhv_p inside
 *  fused B instead of storing and re-reading them (same results bit for bit).
 *  OCN_OPT_ONEPASS (default 1): in such calls with trans_terms and ksw_lat on and no tracers,
 *  steps 2..K-1 run as one launch each: the state is read once and the next state written once,
 *  hh_init's depths, vort and the stresses formed in registers (same results bit for bit; takes
 *  precedence over OCN_OPT_RECOMPUTE).  Step 1 too when nothing changed the state since the
 *  last hh_init; on one block without halo exchanges and a8 / a9 work on the halo ring, the last
 *  step as well; with halo exchanges, the bands along the exchanged sides run the role-flip path.
 *  OCN_OPT_KNOWN_CONSTANTS (default 1): the one-pass steps take the forcing and D's fallback
 *  values as zero and h_r, mu as uniform constants when a check of the arrays (at the first
 *  one-pass call, and after any field is handed in) finds them so; 0: always the general variant.
 *  OCN_OPT_ONEPASS_LAST (default 1): with halo exchanges or a8 / a9 work on the halo ring, the
 *  call's last step as a one-pass step too (the inner march storing what the reference's last
 *  step leaves, then a8's copies and hh_init with every level); 0: a standard last step there.
 *  OCN_OPT_LAZY_TAIL (default 1): in one process (one block without halo exchanges, or the blocks of
 *  OCN_OPT_X2 steps), no tracers and no raw real(8) pointer handed out, a call whose steps are one-pass steps leaves its tail (what
 *  the reference's last step stores beyond the next state: vort, the stresses, the RHS terms,
 *  sw_next_step's copies, hh_init with every level) pending: the next ocn_ctx_step continues with
 *  one-pass steps -- so 1-step calls (the reference's own cadence, model.f90:146) run as fast as
 *  long ones -- and ocn_ctx_complete, or any entry that looks at the fields, forms it first (the
 *  last step run again from the previous state, which is still in the library's second buffers:
 *  the same results bit for bit).  ocn_ctx_get_option returns 2 while a tail is pending.
 *  OCN_OPT_X2 (default 1): with halo exchanges (several blocks or ranks), the one-pass steps
 *  exchange the state (ssh, sshp, ubrtr, ubrtrp, vbrtr, vbrtrp) two points deep, once per step, and
 *  form the depths, vort and stresses on the halo themselves, so the march covers the whole
 *  interior (one exchange per step instead of two, no frame launches); needs the real(4) fields
 *  from ocn_ctx_init_state, blocks of at least 2 x 2 points, no a8 / a9 work on a halo ring no
 *  neighbour fills, and OCN_OPT_ONEPASS_LAST; the second halo ring, which the reference never
 *  writes, is restored before the call's last step (same results bit for bit).  ocn_ctx_get_option:
 *  whether the last ocn_ctx_step used such steps.  Lazy call tails (OCN_OPT_LAZY_TAIL) apply to them
 *  too when the context exchanges only with blocks of its own process.
 *  OCN_OPT_BATCH (default 1): with several blocks on the device, each launch group of a step is
 *  issued once for all of them (the blocks' tiles in one grid) instead of once per block.
 *  OCN_OPT_PAIR (default 1): two one-pass steps in one launch where both are plain one-pass steps
 *  of a single-block context without exchanges, the one-pass variant is chosen on the host (a
 *  known-constant verdict the host read, or the general variant), and the second is not the call's
 *  last step run -- the first step's new state stays on chip (98 B per cell for two steps in the
 *  known-constant variant); 1: the known-constant variants on blocks of at least 512 x 512 interior
 *  points, 2: any variant on any block, 0: never.  Same results bit for bit.  ocn_ctx_get_option: 2 if the last
 *  ocn_ctx_step ran such launches, else whether the option is on.
 *  OCN_OPT_MULTI (default 1): in an open sequence (OCN_OPT_LAZY_TAIL) without pairs, all steps of a
 *  call in ONE launch with a grid-wide barrier between the steps, where the block is small
 *  enough for its whole grid to be resident (the launch-latency-bound case: the Black Sea basin as one
 *  block), single block without exchanges, the variant chosen on the host, check_every 0 or 1, no
 *  graph replay.  Same results bit for bit.  ocn_ctx_get_option: 2 if the last ocn_ctx_step ran one.
 *  OCN_OPT_TRACER_STEP (default 1): tracer runs (use_tracers) with one-pass steps -- each step's
 *  expl_tracer as one launch per tracer that forms hh_init's depths it reads from the state, run with
 *  the next step (after its exchange, which carries the tracers one point deep); the call's last step
 *  runs the standard tracer stages.  Needs the call's first step to be a one-pass step, and with
 *  exchanges the x2 steps; no graph replay.  Same results bit for bit.  ocn_ctx_get_option: 2 if the
 *  last ocn_ctx_step used them.
 *  OCN_OPT_X4 (default 1): with halo exchanges, x2 steps run two per launch with ONE exchange of the
 *  state four points deep per two steps (the launch's first step also updates the two halo rings
 *  neighbour blocks own, as they do) -- the pair launch of single blocks (OCN_OPT_PAIR) for blocks with
 *  neighbours; the known-constant variant, every block at least 4 x 4; two more halo rings outside the
 *  reference's arrays hold the exchanged state.  Tracer runs (tracer steps): the tracers exchanged two
 *  deep, two tracer steps per exchange -- with 1 only where exchanges go to other ranks, with 3 always.
 *  0 = off.  Same results bit for bit.  ocn_ctx_get_option: 2 if the last ocn_ctx_step used such
 *  launches.
 *  OCN_OPT_CO_LAUNCH (default 1): tracer runs with x2 steps (one tracer, block batching on): each
 *  step's march -- with OCN_OPT_OVERLAP 2 the part after the exchange -- and the previous state's
 *  tracer step go as ONE launch (their workgroups in one grid) instead of two.  Same results bit for
 *  bit.  ocn_ctx_get_option: 2 if the last ocn_ctx_step co-launched.
 *  OCN_OPT_MULTI_SPIN (diagnostics; default 1 << 20, about 0.5 s): the multi-step launch's grid
 *  barrier gives up after this many polls -- the launch's workgroups end and ocn_ctx_synchronize
 *  returns OCN_ERR_HIP instead of the device hanging if the grid was not co-resident.  Tests set it
 *  to 1 to exercise that path.
 *  OCN_OPT_XCHG_DELAY (tests; default 0): microseconds the device waits before each exchange with
 *  remote peers (a slow link, for the measured overlap choice: ocn_ctx_overlap_info).
 * ocn_ctx_get_option: current value; for OCN_OPT_COMPACT whether the last ocn_ctx_step used
 * the compact tables, for OCN_OPT_FLIP whether it used role-flip steps, for OCN_OPT_RECOMPUTE
 * whether it used recompute steps, for OCN_OPT_ONEPASS whether it used one-pass steps (2: with
 * the forcing and fallback values known to be zero and h_r, mu known to be uniform, taken as
 * kernel constants instead of being read; 3: the same with h_r read -- a non-uniform rest depth,
 * e.g. a topography file). */
int ocn_ctx_set_option(ocn_ctx *ctx, int32_t key, int64_t value);
int ocn_ctx_get_option(const ocn_ctx *ctx, int32_t key, int64_t *value);
enum { OCN_OPT_GRAPH = 1, OCN_OPT_OVERLAP = 2, OCN_OPT_STAGE_TIMING = 3, OCN_OPT_FUSED = 4, OCN_OPT_COMPACT = 5,
       OCN_OPT_MARCH = 6, OCN_OPT_FLIP = 7, OCN_OPT_RECOMPUTE = 8, OCN_OPT_ONEPASS = 9,
       OCN_OPT_KNOWN_CONSTANTS = 10, OCN_OPT_ONEPASS_LAST = 11, OCN_OPT_LAZY_TAIL = 12, OCN_OPT_X2 = 13,
       OCN_OPT_BATCH = 14, OCN_OPT_PAIR = 15, OCN_OPT_MULTI = 16, OCN_OPT_TRACER_STEP = 17,
       OCN_OPT_MULTI_SPIN = 18, OCN_OPT_X4 = 19, OCN_OPT_CO_LAUNCH = 20, OCN_OPT_XCHG_DELAY = 21 };

/* Timer slots: the stage ids, then the fused groups (fused C2 is OCN_STAGE_HH_INIT), then the
 * three tracer stages (summed over tracers), then the role-flip steps' fused hh_init + next A,
 * then the one-pass steps: one step, two steps per launch, two steps the second of which is the
 * call's last (the tail of an open sequence, ocn_ctx_complete), several steps in one launch
 * (OCN_OPT_MULTI), the tracer step of one-pass sequences (OCN_OPT_TRACER_STEP), then the halo
 * exchanges with remote peers and the exposed part of the overlapped ones (ocn_ctx_stage_stats). */
enum { OCN_TIMER_FUSED_A = OCN_NUM_STAGES, OCN_TIMER_FUSED_B, OCN_TIMER_FUSED_C1, OCN_TIMER_TRACER,
       OCN_TIMER_FUSED_CA = OCN_TIMER_TRACER + OCN_NUM_TSTAGES, OCN_TIMER_ONEPASS, OCN_TIMER_ONEPASS2,
       OCN_TIMER_ONEPASS2_LAST, OCN_TIMER_ONEPASS_MULTI, OCN_TIMER_TRACER_STEP, OCN_TIMER_EXCHANGE,
       OCN_TIMER_EXPOSED, OCN_NUM_TIMERS };

/* Per-timer device time (ms, summed) and launch counts since the last call, from the HIP
 * events of OCN_OPT_STAGE_TIMING; arrays of OCN_NUM_TIMERS entries.  Synchronises. */
int ocn_ctx_stage_times(ocn_ctx *ctx, double *ms, int64_t *counts);
/* The same, plus the longest single record per timer (ms_max; may be NULL).  OCN_TIMER_EXCHANGE:
 * one halo exchange with remote peers (pack, the RCCL group / loopback copies, unpack) on the
 * stream that runs it; OCN_TIMER_EXPOSED: per overlapped step, how long the comm stream's chain
 * (exchange + frame march) outlasted the compute stream's inner march -- the part of the exchange
 * not hidden (0 when hidden). */
int ocn_ctx_stage_stats(ocn_ctx *ctx, double *ms, int64_t *counts, double *ms_max);

const char *ocn_last_error(void);
int ocn_abi_version(void);
/* Build id: a hash of the library's sources and compile flags (Makefile), e.g. to tie a
 * profile taken on one build to the library that is loaded. */
const char *ocn_build_id(void);
/* Kernel launches this process has issued through the library so far (every context, copies
 * between buffers not included): a host takes differences around a region to count launches. */
int64_t ocn_launch_count(void);

#ifdef __cplusplus
}
#endif
#endif /* OCN_SW_H */
