// ocn_internal.h -- shared internals of libocn_sw (not part of the C ABI).
#pragma once
#include <hip/hip_runtime.h>

#include <initializer_list>
#include <string>
#include <vector>

#include "../../include/ocn_sw.h"

// Stencil tile of one 256-thread workgroup (sw_kernels.hip k_range): OCN_TW columns (a
// multiple of 64) x OCN_ROWS rows; OCN_XCD_REMAP = XCD-banded tile order.
#ifndef OCN_TW
#define OCN_TW 64
#endif
#ifndef OCN_ROWS
#define OCN_ROWS 8
#endif
#ifndef OCN_XCD_REMAP
#define OCN_XCD_REMAP 1
#endif
#define OCN_WY (256 / OCN_TW)
static_assert(OCN_TW % 64 == 0 && 256 % OCN_TW == 0, "OCN_TW must be 64, 128 or 256");

#ifndef OCN_FIELD_SKEW
#define OCN_FIELD_SKEW 0
#endif
static_assert(OCN_FIELD_SKEW % 256 == 0, "OCN_FIELD_SKEW must keep fields 256-B aligned");

// Minimum waves per SIMD requested from the register allocator for the stencil kernels.
#ifndef OCN_LB_WAVES
#define OCN_LB_WAVES 1
#endif

// shared/constants.f90:23  FreeFallAcc = 9.8 (real(4))
#define OCN_FREE_FALL_ACC 9.8f

namespace ocn {

int set_error(int code, const std::string &msg);

inline bool is_r8(int id) { return id >= OCN_SSH && id < OCN_FIELD_END; }   // SW fields (tracers: ctx_has_field)
inline bool is_r4(int id) { return id >= 0 && id < OCN_NUM_R4; }
inline int field_slot(int id) { return is_r4(id) ? id : OCN_NUM_R4 + (id - OCN_SSH); }
constexpr int kNumSlots = OCN_NUM_R4 + OCN_NUM_R8;   // without tracer fields
constexpr int kMaxTracers = 64;

#ifndef OCN_RANGE_DEFINED   // also in sw_stencils.h
#define OCN_RANGE_DEFINED
struct Range { int m0, m1, n0, n1; };   // [m0, m1] x [n0, n1], 1-based global indices
#endif

// A block's compact static fields (sw_stencils.h): mask bytes (pitch x rows) and metric rows;
// march: run the stencil launches that have one as register marches (sw_kernels.hip k_march).
struct Compact {
    const uint8_t *bits;
    const float *rows;
    bool march;
};

// Fused step groups (sw_kernels.hip); `ptr` = the block's field table indexed by field_slot(),
// `cp` = its compact tables or nullptr for the 2-D real(4) arrays, `part` = which part of the
// launch range (sw_stencils.h frame_rects: the halo-overlap split).
enum { OCN_PART_ALL = 0, OCN_PART_FRAME = 1, OCN_PART_INNER = 2 };
int launch_fused_a(const ocn_block *b, void *const *ptr, int nptr, const Compact *cp, int part,
                   const ocn_sw_params &sw, double tau, bool reuse, hipStream_t s);
// flip: the role-flip form (sw_kernels.hip MarchFusedB<true>: + a8's filters and check_ssh_err
// into flip_nbad on the interior; needs cp->march); rc: hhq / hhu_p / hhv_p recomputed from
// h_r, ssh, sshp (after a MarchCA<false>, which does not store them)
// up_out / vp_out / inner (one-pass calls with halo exchanges): the role-flip B on the interior
// outside *inner, a8's filtered sshp / ubrtrp / vbrtrp into sshp_out / up_out / vp_out
int launch_fused_b(const ocn_block *b, void *const *ptr, int nptr, const Compact *cp, int part,
                   const ocn_sw_params &sw, double tau, bool full, bool reuse, hipStream_t s,
                   int32_t *flip_nbad = nullptr, bool flip = false, bool rc = false, double *sshp_out = nullptr,
                   double *up_out = nullptr, double *vp_out = nullptr, const Range *inner = nullptr);
// sshp_in: a8 reads sshp there and writes the table's sshp (recompute steps), nullptr = in place
int launch_fused_c1(const ocn_block *b, void *const *ptr, int nptr, const Compact *cp, int part,
                    const ocn_sw_params &sw, int32_t *nbad, hipStream_t s, const double *sshp_in = nullptr,
                    const double *up_in = nullptr, const double *vp_in = nullptr);
// keep_n (march path, full): hqn / hun / hvn / hhn already hold hh_init's n level (from h_r) and
// are not stored again.  copy (march path, whole bnd range): also dst[k] := src[k] (the call tail's
// a8 copies sshn := ssh, ubrtrn := ubrtr, vbrtrn := vbrtr; src[0] the ssh hh_init reads)
struct TailCopy { const double *src[3]; double *dst[3]; };
int launch_fused_c2(const ocn_block *b, void *const *ptr, int nptr, const Compact *cp, int part,
                    const ocn_sw_params &sw, bool full, hipStream_t s, bool keep_n = false,
                    const TailCopy *copy = nullptr);
// Role-flip calls: step k's hh_init (non-final) and step k+1's fused A in one launch
// (sw_kernels.hip MarchCA); next_reuse = step k+1 is a reuse step (else A's a2 stores too);
// skip_rc = step k+1 is a recompute step (hhq on the interior, hhu_p, hhv_p not stored).
// inner: only the bnd range outside *inner (the frame of a one-pass step with halo exchanges)
int launch_fused_ca(const ocn_block *b, void *const *ptr, int nptr, const Compact *cp, int part,
                    const ocn_sw_params &sw, double tau_next, bool next_reuse, bool skip_rc, hipStream_t s,
                    const Range *inner = nullptr);
// floats of a block's compact row table for nrows rows: metric rows, ratios, reciprocals
// (sw_stencils.h kRowTable, recip_offset)
size_t row_table_size(unsigned nrows);

// Initial state on the device (init_kernels.hip; ocn_ctx.hip init_state).  GridInit: one block's
// real(4) static fields from the basin mask (device copy, nx x ny int32, 1-based (m, n) at
// (m-1) + (n-1) nx) and the grid's row / column factors from the host's libm.
struct GridInit {
    ocn_block g;
    const int32_t *mask;
    int nx;
    float *r4[OCN_NUM_R4];
    const float *cos_t, *cos_v;                    // per row (n - bnd_y1): (float) dcosd(lat_mod(yt / yv))
    const double *sin_v, *cosy_v, *cos_xu;         // dsind(yv), dcosd(yv) per row; dcosd(xu) per column
    double cos_rot, sin_rot, sin_extr;             // dcosd / dsind(rotation_on_lat), dsind(lat_extr)
    float sx, sy, cor, sqrt2;                      // base steps (m), 2 * EarthAngVel, sqrt(2.0)
    int curve;
    // rows outside the metric range: their factors and where their metric values go (kExtRows x
    // (OCN_NUM_R4 - OCN_DX) floats: OCN_DX .. OCN_R_DISS of each; nullptr: not formed) -- rows
    // bnd_y1, bnd_y2 (the x2 steps' second ring), then bnd_y1 - 1, bnd_y1 - 2, bnd_y2 + 1, bnd_y2 + 2
    // (the x4 pairs' third and fourth rings, outside the reference's arrays)
    static constexpr int kExt = 6;
    float ext_ct[kExt], ext_cv[kExt];
    double ext_sin_v[kExt], ext_cosy_v[kExt];
    float *ext;
};
constexpr int kExtRows = GridInit::kExt;
constexpr int kExtRowFloats = kExtRows * (OCN_NUM_R4 - OCN_DX);
// Extra halo rings of every real(8) field and of the x4 mask bytes beyond the reference's 2
// (bnd_x1 - kXRing .. bnd_x2 + kXRing, bnd_y1 - kXRing .. bnd_y2 + kXRing addressable): the pair
// launches with halo exchanges read the state 4 points out (ocn_ctx.hip one_step_x4)
constexpr int kXRing = 2;
int launch_init_grid(const GridInit &q, hipStream_t s);
// gaussian_elimination_kernel (vel_ssh.f90:15-38) into p (zero outside the sea interior)
int launch_gaussian(const ocn_block &g, double *p, const float *lu, int nx0, int ny0, double sigma, hipStream_t s);
// v at every point of the block array (not the row padding)
int launch_fill_field(const ocn_block &g, double *p, double v, hipStream_t s);
// One-pass role-flip step (sw_kernels.hip MarchStep): a1 + fused B + a8's filters + check_ssh_err
// with hh_init's depths, vort and the stresses formed in registers from the state; single block,
// no a8 / a9 work on the halo ring; a8's filtered sshp / ubrtrp / vbrtrp go to the given buffers.
// range: the points it computes (default: the interior) -- with halo exchanges, the part of the
// interior whose stencils stay off the halos the exchanges fill.
// kc: which variant -- OCN_KC_GENERAL reads h_r, mu, the forcing and D's fallback values;
// OCN_KC_KNOWN takes them as +0.0 / the uniform values kc[0], kc[1] (device memory, written by
// launch_fallback_check); OCN_KC_KNOWN_HR the same but reads h_r (a non-uniform rest depth:
// topography); OCN_KC_DEVICE launches all three, each running only if the device verdict *flag
// (launch_fallback_check's: bit 0 h_r varies, bit 1 anything else) is its own -- no host wait.
enum { OCN_KC_GENERAL = 0, OCN_KC_KNOWN = 1, OCN_KC_DEVICE = 2, OCN_KC_KNOWN_HR = 3 };
struct OnepassKC { int mode; const int32_t *flag; const double *kc; };
// own (sw_stencils.h own_class bits, not with last): the halo points neighbour blocks own hold the
// neighbours' state two points deep -- D there is formed as on their interior (MarchStep X2).
// frame_of: only the part of the range outside *frame_of, as up to 4 bands in one launch
int launch_onepass(const ocn_block *b, void *const *ptr, int nptr, const Compact *cp, const ocn_sw_params &sw,
                   double tau, int32_t *nbad, double *sshp_out, double *up_out, double *vp_out, hipStream_t s,
                   const Range *range, bool last, const OnepassKC &kc, unsigned own = 0,
                   const Range *frame_of = nullptr);
// Two one-pass steps in one launch (sw_kernels.hip MarchStep PAIR): single block, no exchange,
// a variant chosen on the host (kc.mode OCN_KC_KNOWN / OCN_KC_KNOWN_HR / OCN_KC_GENERAL); reads the state where a single step reads it and writes the second step's new state where
// a single step writes (one role flip); nbad1 / nbad2: the steps' check_ssh_err counts (null: none)
// last: the second step is the call's last step (MarchStep LAST: the consumers also store vort, the
// stresses and the RHS terms the reference's last step leaves)
// the pair launches' shader-clock counters (sw_kernels.hip g_clk: ticks, 100 MHz ticks, launches)
int clock_read(bool reset, unsigned long long out[3]);
int launch_onepass_pair(const ocn_block *b, void *const *ptr, int nptr, const Compact *cp, const ocn_sw_params &sw,
                        double tau, int32_t *nbad1, int32_t *nbad2, double *sshp_out, double *up_out, double *vp_out,
                        hipStream_t s, const OnepassKC &kc, bool last = false);
// Two one-pass steps per launch with halo exchanges (sw_kernels.hip MarchStep PAIR + X2; ocn_ctx.hip
// one_step_x4): bx = the block widened by kXRing rings, ptr / cp over that geometry (launch_x4_tables),
// the state exchanged 4 deep; the known-constant variant (kc.mode OCN_KC_KNOWN); own: the halo points
// neighbour blocks own; range: the consumers' points (nullptr: the interior), frame_of: only the bands
// of it outside *frame_of (one launch of up to 4 rects); nblk: blocks of this size batched into the
// launch (the tile height's cost model); trs (tracer runs): four arrays (based like the fields) that get the
// first step's new ssh, sshp, ubrtr, vbrtr on the producers' points -- the second tracer step's state
int launch_onepass_pair_x4(const ocn_block *bx, void *const *ptr, int nptr, const Compact *cp, const ocn_sw_params &sw,
                           double tau, int32_t *nbad1, int32_t *nbad2, double *sshp_out, double *up_out, double *vp_out,
                           hipStream_t s, const OnepassKC &kc, unsigned own, const Range *range = nullptr,
                           int nblk = 1, const Range *frame_of = nullptr, double *const *trs = nullptr);
// one_step_x4's tables of block g: mask bytes over g widened by kXRing (bits4, its base at
// A(bnd_x1 - kXRing, bnd_y1 - kXRing), pitch g->pitch) and the row table of those rows (rows4,
// row_table_size(rows + 2 kXRing)) from the block's own tables, its ext rows and the basin mask
// (device, nx x ny); ORs OCN_COMPACT_DIVISOR_RANGE into *flags
int launch_x4_tables(const ocn_block *g, const uint8_t *bits, const float *rows, const float *ext, uint8_t *bits4,
                     float *rows4, const int32_t *mask, int nx, int ny, unsigned own, int32_t *flags, hipStream_t s);
// nsteps one-pass steps in one launch (sw_kernels.hip k_march_multi): single small block, no
// exchange, a variant chosen on the host; step 1 reads the table's buffers, each step the buffers
// the previous one wrote (the role pairs and sshp / ubrtrp / vbrtrp against *_alt, alternating);
// ctr: kMultiBarBytes of device words for the grid barrier, at the start of their own allocation
// (zeroed on the stream first); err: ORed 1 if a barrier timed out.  onepass_multi_fits: the block's
// grid is small enough for one resident launch on the current device (its tile count against every
// variant's occupancy x the device's CUs, queried once per device).  spin: the barrier's bound on
// polls before it gives up (kMultiSpin; tests force it low to exercise the timeout path).
constexpr size_t kMultiBarBytes = 17 * 128;   // the top counter, 8 group counters, 8 group generations
constexpr int kMultiSpin = 1 << 20;           // ~0.5 s of s_sleep(1) polls
int onepass_multi_fits(const ocn_block *b);
int launch_onepass_multi(const ocn_block *b, void *const *ptr, int nptr, const Compact *cp, const ocn_sw_params &sw,
                         double tau, int nsteps, int32_t *nbad, double *sshp_alt, double *up_alt, double *vp_alt,
                         unsigned *ctr, int32_t *err, hipStream_t s, const OnepassKC &kc, int spin = kMultiSpin);
// the known-constant precondition of launch_onepass over r (sw_kernels.hip FallbackCheck: the
// fallback points and the forcing hold +0.0, h_r and mu are uniform): ORs 1 into *flag where it
// does not hold; writes h_r and mu at (r.m0, r.n0) to kc[0], kc[1]
int launch_fallback_check(const ocn_block *b, void *const *ptr, const uint8_t *bits, const Range &r, int32_t *flag,
                          double *kc, hipStream_t s, unsigned own = 0);
// Builds the compact tables of a block from its real(4) arrays; ORs OCN_COMPACT_* reasons
// they cannot be used into *flags (device int); own: the halo points neighbour blocks own
// (sw_stencils.h own_class bits; OCN_COMPACT_EDGE_RING_SEA tests the others)
int launch_prepare(const ocn_block *b, void *const *ptr, uint8_t *bits, float *rows, int32_t *flags, hipStream_t s,
                   unsigned own = 0);
// rows_x = the row table `rows` with rows 0 and nrows - 1 formed from ext (init_kernels.hip k_ext_rows:
// the metric values of rows bnd_y1 / bnd_y2 as the neighbours form them); ORs
// OCN_COMPACT_DIVISOR_RANGE into *flags if a divisor there is out of udiv's range
int launch_rows_ext(const ocn_block *b, const float *rows, float *rows_x, const float *ext, int32_t *flags,
                    hipStream_t s);
constexpr int kCompactEdgeRingSea = 16;   // sw_stencils.h OCN_COMPACT_EDGE_RING_SEA
// Tracer stage `stage` (OCN_TSTAGE_*) of tracer k (1-based) on one block.
// one reference stage (OCN_STAGE_*) over the compact tables: the ocn_<stage> entry's write set
// and results (sw_kernels.hip KStage; hh_init as the register march with cp->march)
int launch_stage(const ocn_block *b, void *const *ptr, int nptr, const Compact *cp, int stage, const ocn_sw_params &sw,
                 double tau, int32_t *nbad, hipStream_t s);
int launch_tracer(const ocn_block *b, void *const *ptr, int nptr, const Compact *cp, int stage, int k, double tau,
                  double ts, hipStream_t s);
// the three tracer stages of tracer k as one launch in a one-pass sequence (sw_stencils.h TracerStep:
// hh_init's hhu / hhv / hhq_p formed from the state): ffn into ffn_out, the filtered ffp into ffp_out;
// own: the halo points neighbour blocks own (their fluxes formed here, as the exchange delivers them);
// ext: also the first halo ring's points neighbours own, updated as those neighbours update them (x4
// pairs with tracers: the state 4 and the tracers 2 points deep exchanged)
int launch_tracer_step(const ocn_block *b, void *const *ptr, int nptr, const Compact *cp, int k, double tau,
                       double ts, double *ffn_out, double *ffp_out, unsigned own, hipStream_t s, bool ext = false);
// ORs 1 into *flags (device int) if a buffer pair of the role-flip step differs outside the
// pair's write set (sw_stencils.h Coherence).
int launch_coherence(const ocn_block *b, void *const *ptr, const uint8_t *bits, int32_t *flags, hipStream_t s);
// the same for tracer k's ff1 / ff1n (the tracer steps' role pair) outside the ring range's lu points
int launch_tracer_coherence(const ocn_block *b, void *const *ptr, const uint8_t *bits, int k, int32_t *flags,
                            hipStream_t s);
// Prepare's flag bit reporting mask bits on the halo ring (sw_stencils.h OCN_COMPACT_RING_SEA)
constexpr int kCompactRingSea = 4;
constexpr int kCompactDivisorRange = 8;   // sw_stencils.h OCN_COMPACT_DIVISOR_RANGE

// Block batching (sw_kernels.hip): while a Batcher is active on this thread, the launches of the
// march / range / frame kernels are collected per kernel type instead of issued, and batch_end
// issues each kind for all the blocks that added one together (their tiles in one grid, up to
// kPack launch bodies by value in the kernel arguments).  A block loop of a stage launches one
// kernel per block: with several small blocks per device those launches are latency-bound.
//   batch_begin(bt, s); for each block { batch_next(bt); launches on s } batch_end(bt);
// Each block's launches keep their order (a block that adds a kind out of the batch's kind order,
// or one kind twice, flushes the batch first); launches of different blocks may be reordered, so
// a batched loop must not let one block's launch read what another block's writes.  Any other
// launch while a batch is open (another kernel, another stream) is an error (check_launch).
// co_launch: the caller states that no launch of the batch reads what another writes (a one-pass
// x2 step and the previous state's tracer step: both read the exchanged state, each writes its own
// buffers), so an entry may issue itself and the next one as ONE launch (co_flush: the x2 march's
// and the tracer step's workgroups in one grid) instead of two in order.
struct BatchEntry {
    virtual ~BatchEntry() {}
    virtual int flush(hipStream_t s) = 0;
    // issue this entry and `next` as one launch; false: not possible (each flushes on its own)
    virtual bool co_flush(BatchEntry *next, hipStream_t s, int &rc) { (void)next; (void)s; (void)rc; return false; }
    const void *kind = nullptr;   // the kernel type (its host stub's address)
};
struct Batcher {
    bool active = false;
    bool co_launch = false;              // see BatchEntry::co_flush (cleared by batch_begin)
    int co_launched = 0;                 // launches that issued two entries (the last flush)
    hipStream_t s = nullptr;
    int cur = -1;                        // position of the current block's last entry
    std::vector<BatchEntry *> entries;   // in first-added order
    int flush();                         // issue and clear the collected launches
    ~Batcher();
};
extern thread_local Batcher *g_batcher;
void batch_begin(Batcher *bt, hipStream_t s);
inline void batch_next(Batcher *bt) { if (bt) bt->cur = -1; }
int batch_end(Batcher *bt);

int check_hip(hipError_t e, const char *what);
// every kernel launch of the library is followed by check_launch(): it also counts them
// (ocn_launch_count, for the launches-per-step figure of bench.py)
void count_launch();
int batch_violation();
inline int check_launch()
{
    count_launch();
    if (g_batcher && g_batcher->active) return batch_violation();
    return check_hip(hipGetLastError(), "kernel launch");
}

}  // namespace ocn
