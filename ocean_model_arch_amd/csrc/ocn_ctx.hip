// ocn_ctx.hip -- PSy layer of the MI355X shallow-water step: model context, decomposition,
// device storage, initial state, halo exchange (intra-device copies + RCCL), step driver.
//
// Reference counterparts (Andrcraft9/ocean_model_arch):
//   storage        core/data_types.f90:44-144, core/ocean.f90:14-48, core/grid.f90:23-90
//   decomposition  core/decomposition.f90:427-503 (uniform blocks), :614-669 (block -> rank),
//                  :672-760 (local numbering, _MPP_SORTED_BLOCKS_), :950-1062 (neighbour maps)
//   dispatcher     core/kernel_interface.f90:48-119 (envoke) + interface/shallow_water/sw_interface.f90
//   algorithm      control/shallow_water/shallow_water.f90:22-94 (expl_shallow_water)
//   halo           shared/mpp/sync.f90:294-556 + syncborder_block2D_gen_all.fi
//   init           control/init_data.f90:29-125, kernel/service/grid_kernels.f90,
//                  kernel/service/grid_parameters.f90:80-181, kernel/shallow_water/vel_ssh.f90:15-38
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "ocn_internal.h"

namespace ocn {

static thread_local std::string g_last_error;

int set_error(int code, const std::string &msg)
{
    g_last_error = msg;
    return code;
}

static std::atomic<long long> g_launches{0};
void count_launch() { g_launches.fetch_add(1, std::memory_order_relaxed); }

int check_hip(hipError_t e, const char *what)
{
    if (e == hipSuccess) return OCN_OK;
    return set_error(OCN_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

#define HIPCHK(call)                                          \
    do {                                                      \
        int _rc = check_hip((call), #call);                   \
        if (_rc) return _rc;                                  \
    } while (0)
#define RC(call)                                              \
    do {                                                      \
        int _rc = (call);                                     \
        if (_rc) return _rc;                                  \
    } while (0)


// ------------------------------------------------------------------ halo segments
// w strided 1-D runs of doubles side by side: dst[i*dst_stride + j*dst_jstride] =
// src[i*src_stride + j*src_jstride], i < count, j < w.  A column strip several layers deep is one
// such segment (merge_columns: w adjacent columns), so a wave's loads take the layers of 64 / w rows
// from shared cache lines instead of one line per element and layer.
struct Seg {
    const double *src;
    double *dst;
    long src_stride, dst_stride;
    int count;
    int w = 1;
    long src_jstride = 0, dst_jstride = 0;
};

// Grid: one workgroup per 64-element chunk of a segment (SegChunk: the chunk table of the list, so
// no workgroup of a short segment idles as in a segments x longest-chunks grid); element e of a
// segment: run j = e % w, row i = e / w -- one element per thread and one wave per workgroup, so
// every load of a strip is in flight at once, spread over many CUs (a loop per workgroup would pay
// one memory round trip per pass).
constexpr int kSegChunk = 64;
struct SegChunk { int seg, e0; };
__device__ __forceinline__ bool seg_at(const Seg &g, int e, long &si, long &di)
{
    if (e >= g.count * g.w) return false;
    const int i = e / g.w, j = e - i * g.w;
    si = (long)i * g.src_stride + (long)j * g.src_jstride;
    di = (long)i * g.dst_stride + (long)j * g.dst_jstride;
    return true;
}
__global__ __launch_bounds__(kSegChunk) void k_segments(const Seg *__restrict__ segs, const SegChunk *__restrict__ ch,
                                                        int nch)
{
    const int b = blockIdx.x;
    if (b >= nch) return;
    const SegChunk q = ch[b];
    const Seg g = segs[q.seg];
    long si, di;
    if (!seg_at(g, q.e0 + (int)threadIdx.x, si, di)) return;
    g.dst[di] = g.src[si];
}

// The same runs compared instead of copied: ORs 1 into *flags where dst differs from src (bits).
__global__ __launch_bounds__(kSegChunk) void k_segments_cmp(const Seg *__restrict__ segs, const SegChunk *__restrict__ ch,
                                                            int nch, int32_t *flags)
{
    const int k = blockIdx.x;
    if (k >= nch) return;
    const SegChunk q = ch[k];
    const Seg g = segs[q.seg];
    long si, di;
    if (!seg_at(g, q.e0 + (int)threadIdx.x, si, di)) return;
    const double a = g.dst[di], b = g.src[si];
    unsigned long long x, y;
    __builtin_memcpy(&x, &a, 8);
    __builtin_memcpy(&y, &b, 8);
    if (x != y) atomicOr(flags, 1);
}

// A segment list on the device with its chunk table (make_seglist)
struct SegList {
    Seg *d = nullptr;
    SegChunk *ch = nullptr;
    int n = 0, nch = 0;
};

// init_grid_data's bottom topography (control/init_data.f90:115-120): read_data2D_real4 fills the
// block's interior from the file (tools/io.f90:130-147; the file holds the (nx-4) x (ny-4) interior,
// Fortran order) and zeroes every point with |lu| < 0.5 (:158-171), the rest of the zero-initialised
// array stays 0, then copy_from_real4 promotes it (core/data_types.f90:638-652); the sync follows.
__global__ void k_topography(ocn_block g, double *h, const float *lu, const float *topo, int nxi)
{
    const int w = g.bnd_x2 - g.bnd_x1 + 1, rows = g.bnd_y2 - g.bnd_y1 + 1;
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (long)w * rows) return;
    const int m = g.bnd_x1 + (int)(i % w), n = g.bnd_y1 + (int)(i / w);
    const long at = (long)(m - g.bnd_x1) + (long)(n - g.bnd_y1) * g.pitch;
    float v = 0.0f;
    if (m >= g.nx_start && m <= g.nx_end && n >= g.ny_start && n <= g.ny_end) v = topo[(long)(m - 3) + (long)(n - 3) * nxi];
    if (fabsf(lu[at]) < 0.5f) v = 0.0f;
    h[at] = (double)v;
}

__global__ void k_fill_r8(double *p, long n, double v)
{
    long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = v;
}

// One output record of a field (output.f90:101-106 copy_from_real8 + io.f90:343-349): real(4) of
// the interior value, undef where |lu| < 0.5; dst is the packed interior, Fortran order.
template <typename T>
__global__ void k_output_r4(const T *src, const float *lu, long pitch, int w, int h, float undef, float *dst)
{
    const int i = (int)(blockIdx.x * blockDim.x + threadIdx.x), j = (int)blockIdx.y;
    if (i >= w || j >= h) return;
    const long s = (long)j * pitch + i;
    dst[(long)j * w + i] = fabsf(lu[s]) < 0.5f ? undef : (float)src[s];
}

// ------------------------------------------------------------------ geometry helpers
// decomposition.f90:94-290, directions macros/kernel_macros.fi:4-12
struct Rect { int x0, x1, y0, y1; };
static const int kDirDm[9] = {0, 1, -1, 0, 0, 1, 1, -1, -1};
static const int kDirDn[9] = {0, 0, 0, 1, -1, 1, -1, 1, -1};

// Strip of a Rect inside a block array as (offset, count, stride): a 1-wide rect is a row
// (stride 1) or a column (stride pitch).
static void strip(const ocn_block &b, const Rect &r, long &off, int &count, long &stride)
{
    off = (long)(r.x0 - b.bnd_x1) + (long)(r.y0 - b.bnd_y1) * (long)b.pitch;
    if (r.y0 == r.y1) { count = r.x1 - r.x0 + 1; stride = 1; }
    else { count = r.y1 - r.y0 + 1; stride = (long)b.pitch; }
}

}  // namespace ocn

using namespace ocn;

// ------------------------------------------------------------------ context
struct GBlock {            // one block of the global block grid
    int bm, bn;
    ocn_block g;           // pitch filled for local blocks only
    int rank;              // -1 land block (bglob_proc = -1)
    int k;                 // local index on its rank
    double weight;         // sea points (bglob_weight)
};

struct LBlock {
    ocn_block g;
    int bm, bn, gid;
    int nbr_rank[8], nbr_k[8], nbr_gid[8];
    void *slab = nullptr;
    std::vector<void *> ptr;           // field table, indexed by field_slot(id)
    uint8_t *bits = nullptr;           // compact static fields (sw_stencils.h): mask bytes
    float *rows = nullptr;             // and metric row tables
    void *sshp_alt = nullptr;          // second sshp buffer of the recompute steps (one_step_fused)
    void *up_alt = nullptr, *vp_alt = nullptr;   // second ubrtrp / vbrtrp buffers of the one-pass steps
    std::vector<void *> ffp_alt;       // second ff1p buffer of every tracer (one-pass steps' tracer step)
    double *kc = nullptr;              // device: h_r, mu of the one-pass step's known-constant variant
    // one_step_x2 (one 2-deep state exchange per one-pass step, the march over the whole interior):
    unsigned own = 0;                  // halo points neighbour blocks own (sw_stencils.h own_class bits)
    float *ext = nullptr;              // metric values of rows bnd_y1 / bnd_y2 as the neighbours form them
    float *rows_x = nullptr;           // the row table with those two rows (launch_rows_ext)
    double *hr_x = nullptr;            // h_r with its second halo ring from the neighbours
    double *ring2 = nullptr;           // the state's second halo ring as the reference leaves it (saved)
    // one_step_x4 (two one-pass steps per launch, one 4-deep state exchange per pair): mask bytes and the
    // row table over the block widened by kXRing rings (launch_x4_tables; bits_x4 based at
    // A(bnd_x1 - kXRing, bnd_y1 - kXRing), pitch g.pitch)
    uint8_t *bits_x4 = nullptr;
    float *rows_x4 = nullptr;
    SegList save, restore;   // its save / restore runs (k_segments)
    // x4 pairs with tracers: the first step's new ssh, sshp, ubrtr, vbrtr (based like the fields: kXRing
    // extra rows; MarchStep::trs), the state the second tracer step reads
    double *trs[4] = {nullptr, nullptr, nullptr, nullptr};
    template <typename T> T *f(int id) const { return (T *)ptr[field_slot(id)]; }
};

// Loopback transport (ocn_ctx_attach_loopback): the N ranks of a decomposition as N contexts of
// ONE process on one device, each driven by its own host thread.  It replaces exactly two RCCL
// calls and nothing else -- the ncclRecv / ncclSend pair of an exchange (run_sync) and the
// ncclAllReduce of the role-flip vote (check_coherence) -- so the remote branch of the halo plans
// (device pack / unpack, per-peer messages, per-role plans, sync_ca, overlap forks) runs as in
// production.  An exchange is two host rendezvous with the peers:
//   A: each rank has enqueued its pack and recorded lb_ev_a, and publishes its plan; then every
//      rank copies each peer's send buffer (for it) into its own receive buffer, on its stream,
//      after the peer's lb_ev_a, and records lb_ev_b;
//   B: every rank's stream waits for its peers' lb_ev_b, so no send buffer is repacked before the
//      peer's copy out of it has run (the completion guarantee of ncclGroupEnd).
// The counters make the rendezvous of the k-th exchange of every rank meet (all ranks run the
// same sequence of exchanges, as with RCCL); a peer cannot pass phase A of exchange k+1 before
// this rank passed phase B of exchange k, so a published plan / recorded event is never replaced
// before it was consumed.
struct HaloPlan;
struct Loopback {
    int n = 0;
    std::vector<ocn_ctx *> ctx;
    std::mutex mu;
    std::condition_variable cv;
    std::vector<uint64_t> cnt[4];              // per rank: exchange A/B, reduce A/B phases passed
    std::vector<const HaloPlan *> plan;        // plan of the rank's current exchange (phase A)
    std::vector<int32_t *> vote;               // the rank's flag word (reduce phase A)
    bool failed = false;
    int refs = 0;
};

struct HaloPlan {
    SegList local;                    // intra-process copies
    // remote: per peer rank, pack segments (into send buffer) and unpack segments (from recv)
    struct Peer { int rank; long count; double *send, *recv; };
    std::vector<Peer> peers;
    SegList pack, unpack;
};

namespace ocn {
// What one step of an ocn_ctx_step call runs: check = check_ssh_err; first / last step of the
// call; flip = role-flip step; a_done = its fused A already ran (fused into the previous step's
// hh_init launch); next_a = fuse the next step's fused A into this step's hh_init (MarchCA),
// next_reuse = the next step is a reuse step; rc = recompute steps (fused B forms hhq, hhu_p,
// hhv_p itself and writes sshp's filter into the second sshp buffer), rc_next = the next step is
// one (this step's hh_init + A launch then does not store hhq on the interior, hhu_p, hhv_p).
// one = one-pass step (sw_kernels.hip MarchStep), next_one = the next step is one (this step
// then runs no hh_init: the one-pass step forms hh_init's values itself).
// x2 = the one-pass step as one_step_x2 (2-deep state exchange, whole-interior march); x2_save = the
// first of a sequence (the reference's second halo ring of the state is saved first); x2_end = a
// last step after such a sequence (that ring restored and the state's first ring exchanged first).
// pair = this one-pass step and the next as one launch (one_step_pair), check2 = the next one's check.
// multi = this many one-pass steps in one launch (one_step_multi), each checked if check.
struct StepKind {
    bool check, first, last, flip, a_done, next_a, next_reuse, rc, rc_next, one, next_one, one_last;
    bool x2, x2_save, x2_end;
    bool pair = false, check2 = false;
    int multi = 0;
    bool operator==(const StepKind &o) const
    {
        return check == o.check && first == o.first && last == o.last && flip == o.flip && a_done == o.a_done &&
               next_a == o.next_a && next_reuse == o.next_reuse && rc == o.rc && rc_next == o.rc_next &&
               one == o.one && next_one == o.next_one && one_last == o.one_last && x2 == o.x2 &&
               x2_save == o.x2_save && x2_end == o.x2_end && pair == o.pair && check2 == o.check2 && multi == o.multi;
    }
};

}  // namespace ocn

// ocn_ctx::fb_state
enum { kFbUnchecked = 0, kFbDevice = 1, kFbZero = 2, kFbGeneral = 3, kFbHr = 4 };

#ifndef OCN_COMM_PRIO
#define OCN_COMM_PRIO 1   // the comm stream at the device's highest stream priority
#endif
struct ocn_ctx {
    ocn_basin basin;
    ocn_sw_params sw;
    ocn_decomp dec;
    std::vector<int32_t> mask;         // global (nx, ny) column-major
    std::vector<float> topo;           // bottom topography, (nx-4) x (ny-4) interior points (empty: none)
    int bnx = 1, bny = 1;
    std::vector<GBlock> gblocks;       // (bm-1) + (bn-1)*bnx
    std::vector<LBlock> blocks;
    hipStream_t stream = nullptr;
    hipStream_t comm_stream = nullptr;  // halo exchanges overlapped with interior compute
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
    // the known-constant check's verdict copied to pinned host memory behind an event: a later call
    // reads it once the event has completed (hipEventQuery: no wait), learn_fb_async
    hipEvent_t ev_fb = nullptr;
    int32_t *h_fbz = nullptr;
    bool fb_copy = false;
    int overlap = -1;            // OCN_OPT_OVERLAP: 0 none, 1 standard steps, 2 + role-flip steps, -1 auto
    // OCN_OPT_OVERLAP auto with peers on other ranks: the x2 / x4 steps' form (inner part beside the
    // exchange, or exchange then march) chosen from a measurement (ov_begin): ov_state 0 = nothing
    // measured, 1 = a sequential step's events recorded, 2 = an overlapped one's too (the next vote
    // reduces them), 3 = decided (ov_level); ov_kind = the step form measured (2: x2 steps, 4: x4 pairs);
    // ov_ms = the two step times (this rank's, then the maxima over the ranks the decision used)
    int ov_state = 0, ov_kind = 0, ov_level = 2;
    hipEvent_t ov_ev[4] = {nullptr, nullptr, nullptr, nullptr};
    double ov_ms[2] = {0.0, 0.0};
    int xdelay_us = 0;           // OCN_OPT_XCHG_DELAY (tests): a device wait before each exchange with remote peers
    int32_t *d_nbad = nullptr;
    unsigned *d_bar = nullptr;   // the multi-step launch's grid-barrier words (kMultiBarBytes)
    ncclComm_t comm = nullptr;
    bool comm_aborted = false;         // fail_fatal aborted the communicator: calls with exchanges fail
    Loopback *lb = nullptr;            // test transport between contexts of one process (ocn_ctx_attach_loopback)
    hipEvent_t lb_ev_a = nullptr, lb_ev_b = nullptr;
    std::map<std::vector<int>, HaloPlan> plans;
    bool initialized = false;
    bool use_graph = false;
    // the launches a captured step replays depend on everything in its key (march and ring_sea
    // select launch forms and the ring launch; options that change them also drop the cache)
    struct Graph { hipGraphExec_t exec; double tau; ocn::StepKind kind; bool compact, march, ring_sea; int role, kc_mode; };
    std::vector<Graph> graphs;         // one captured step per key
    std::vector<void *> allocs;
    // per-stage HIP-event timing (OCN_OPT_STAGE_TIMING): pending (stage, start, stop) records
    bool stage_timing = false;
    struct Rec { int stage; hipEvent_t a, b; };
    std::vector<Rec> recs;
    std::vector<hipEvent_t> event_pool;
    double stage_ms[OCN_NUM_TIMERS] = {0};
    int64_t stage_n[OCN_NUM_TIMERS] = {0};
    bool fused = true;
    std::vector<int> sync_a, sync_a_reuse, sync_b, sync_ca, sync_ca_reuse;
    // compact static fields: requested (OCN_OPT_COMPACT), in use, stale (real(4) fields
    // changed since they were built), or unusable because raw real(4) pointers were handed out
    bool compact_req = true, compact = false, static_dirty = true;
    bool march = true;   // OCN_OPT_MARCH
    mutable bool r4_escaped = false;
    // role-flip steps (one_step_fused): role = 1 while the ssh/sshn, ubrtr/ubrtrn, vbrtr/vbrtrn
    // buffers of every block are swapped (only inside an ocn_ctx_step call); coherent = the pairs
    // agree outside their write sets (sw_stencils.h Coherence), coherent_known = that was checked
    // after the state last changed outside ocn_ctx_step; r8_escaped = raw pointers of a pair were
    // handed out (check at every call); flip = OCN_OPT_FLIP
    bool flip = true, coherent = false, flip_used = false, rc_used = false;
    bool capturing = false;      // a step is being captured into a hipGraph
    bool sync_pending = false;   // an exchange on comm_stream not yet joined (fork_sync)
    bool ring_sea = true;   // some halo-ring point has a mask set (Prepare); else no ring launch
    bool udiv_ok = true;    // every row divisor of the one-pass step in [2^-60, 2^60] (Prepare)
    bool recompute = true;  // OCN_OPT_RECOMPUTE: recompute steps in role-flip calls
    bool onepass = true;    // OCN_OPT_ONEPASS: one-pass steps in single-block role-flip calls
    // OCN_OPT_PAIR: two one-pass steps per launch (one_step_pair) -- 0 never, 1 on blocks of at least
    // kPairMinCells interior points, 2 on any block; pair_used: a call ran one
    int pair = 1;
    bool pair_used = false;
    // OCN_OPT_MULTI: the one-pass steps of a small single block as one launch per call
    // (one_step_multi); multi_used: the last call ran one
    bool multi = true, multi_used = false;
    // OCN_OPT_TRACER_STEP: tracer runs with one-pass steps -- expl_tracer of each step as one launch per
    // tracer (run_tracer_step), run with the next step, after its exchange; tr_call: this call does;
    // tr_pending: the current state's tracer step has not run yet; tr_alt_ok: the second ff1p
    // buffers agree with the fields outside the tracer step's write set.  Role bits 8 (ff1 / ff1n
    // traded) and 16 (ff1p / its second buffer traded), for every tracer at once.
    bool tr_step = true, tr_call = false, tr_pending = false;
    bool tr_forked = false;   // a tracer step runs on the comm stream beside the march (joined by run_step)
    mutable bool tr_alt_ok = false;
    bool known_const = true;   // OCN_OPT_KNOWN_CONSTANTS: the one-pass step's known-constant variant
    bool last_hybrid = true;   // OCN_OPT_ONEPASS_LAST: one-pass last steps with exchanges / ring work too
    bool one_used = false;
    // the one-pass steps' second sshp / ubrtrp / vbrtrp buffers agree with the fields outside a8's
    // write set (else they are copied at the start of the next such call)
    mutable bool alt_ok = false;
    // hh_init's stored depths were formed from the current state (the last step of the previous
    // call or init_state ran it and nothing has changed the state since): the first step of a
    // call may then be a one-pass step too, as a reuse step.  Never again once an r8 field's
    // device pointer was handed out (it may be written behind our back).
    mutable bool hh_consistent = false, r8_handed = false;
    // hh_init's n level -- hqn = h_r and its interpolations hun / hvn / hhn (depth.f90:14-99 with
    // ffs; no ssh in it) -- is what those arrays hold: a full hh_init wrote them from the current
    // h_r, masks and metrics, and nothing has written them since (the one-pass, pair and
    // multi-step launches never do).  last_finish's hh_init then leaves them as they are (32 B
    // per cell of its 96 B of stores).  Cleared by every other step kind, by any upload, stage,
    // sync or init, and never trusted once a raw pointer was handed out.
    mutable bool hn_fresh = false;
    // hhq_n may differ from h_r (an upload of either, or a raw pointer): every hh_init stores
    // hhq_n = h_r, but the role-flip steps' fused hh_init + A (CA) does not, so the standard tracer
    // stages after such a step copy it first (expl_tracer)
    mutable bool hqn_stale = false;
    // the one-pass step's known-constant precondition (sw_kernels.hip FallbackCheck: fallback points
    // and forcing +0.0, h_r and mu uniform): kFbUnchecked until a check ran after the arrays last
    // changed from outside the step; kFbDevice = its verdict is in device memory (d_fbz; both
    // variants are launched and the device picks, ocn_ctx.hip never waits for it) until a host
    // sync the caller makes anyway reads it (learn_fb): kFbZero / kFbHr (all but h_r: a
    // non-uniform rest depth, read by the OCN_KC_KNOWN_HR variant) / kFbGeneral
    mutable int fb_state = 0;
    int kc_mode = 0;             // OCN_KC_* of the current call's one-pass launches
    int32_t *d_fbz = nullptr;    // the check's verdict word
    // lazy call tail (OCN_OPT_LAZY_TAIL): the last step run was a one-pass step; what the reference's
    // last step leaves beyond the state (vort, stresses, RHS terms, hh_init's levels, a8's copies) is
    // formed when the host next looks (complete_open: the step redone from the previous state, still
    // intact in the other buffers, as the call's last step), so 1-step calls run one-pass steps
    bool lazy = true, open = false, open_x2 = false;
    double open_tau = 0.0;
    // pairs in an open sequence (one_step_pair): open_pair = its last launch was a pair (the state
    // before it is two steps back: complete_open redoes the pair's first step single, then the tail);
    // deferred = the last 1 or 2 steps of the sequence, not yet run: a call runs pairs while 3 or
    // more steps are pending and leaves the rest to the next call -- the 1-step cadence runs a pair
    // every second call -- or to complete_open, which runs them as the last steps (a single + the
    // last step, or the last step: no step run twice); synchronize runs them (as a pair or alone)
    bool open_pair = false;
    int deferred = 0;
    bool deferred_check[2] = {false, false};
    // one_step_x2 (OCN_OPT_X2): its static conditions (ext_ok: the real(4) fields are init_state's,
    // so the ext rows are the neighbours' metric rows; rows_x_ok: their divisors in udiv's range;
    // edge_ring_sea: a8 / a9 work on a halo ring no neighbour fills), the device checks of the last
    // check_coherence (x2_dev_ok: the state's first halo ring holds the neighbours' values and its
    // halo points no exchange fills hold +0.0), whether the h_r copy is current, and whether the
    // state's second halo ring is saved (a sequence of x2 steps is under way)
    bool x2 = true, rows_x_ok = false, edge_ring_sea = true, x2_dev_ok = false;
    mutable bool ext_ok = false, hrx_ok = false;
    bool ring2_saved = false, x2_used = false;
    // one_step_x4 (OCN_OPT_X4): pairs of x2 steps with one 4-deep exchange each; x4_tab_ok: its tables
    // were built from init_state's real(4) fields with every divisor in udiv's range; x4_dev_ok: the
    // last vote found every rank able to run them (a communicator attached); x4_used: the last call did
    // x4: 0 off, 1 auto (tracer runs: only with peers on other ranks), 3 always
    int x4 = 1;
    bool x4_tab_ok = false, x4_dev_ok = false, x4_used = false;
    bool fb_x2 = false;          // the known-constant check's verdict is for the x2 range / tables
    mutable bool coherent_known = false, r8_escaped = false;
    int multi_spin = kMultiSpin;   // OCN_OPT_MULTI_SPIN (the multi-step launch's barrier bound)
    // OCN_OPT_CO_LAUNCH: an x2 step's march and the previous state's tracer step as one launch;
    // co_used: the last call did
    bool co_launch = true, co_used = false;
    double stage_max[OCN_NUM_TIMERS] = {0};   // longest record per timer (ocn_ctx_stage_stats)
    // halo exchanges with remote peers (run_sync): how many were enqueued; while a watchdog is set an
    // event after each (xq, under xmu) tells it the id of the last one the device completed (xdone)
    int64_t xchg = 0, xdone = -1;
    std::mutex xmu;
    std::deque<std::pair<int64_t, hipEvent_t>> xq;
    std::vector<hipEvent_t> xpool;
    // host-side watchdog (ocn_ctx_set_watchdog): the thread, the call it watches (call_depth > 0: a
    // guarded entry is running since call_t0), and whether it fired (wd_msg: what the calls return)
    double wd_s = 0;
    std::thread wd;
    std::mutex wd_mu;
    std::condition_variable wd_cv;
    bool wd_stop = false;
    int call_depth = 0;
    std::chrono::steady_clock::time_point call_t0;
    const char *call_name = "";
    std::atomic<bool> wd_fired{false};
    std::string wd_msg;
    std::mutex comm_mu;          // the communicator is aborted once: by the watchdog or by fail_fatal
    bool comm_abort_done = false;
    int role = 0;
    int steps_run = 0;           // launches statistics of the last call (ocn_ctx_get_option OCN_OPT_LAUNCHES)
    int64_t launches = 0;
    int32_t *d_flags = nullptr;
    bool batch = true;           // OCN_OPT_BATCH
    ocn::Batcher batcher;
};

// v on the device with its chunk table (one entry per kSegChunk elements of each segment), in one
// allocation freed with the context
static int make_seglist(ocn_ctx *c, const std::vector<Seg> &v, SegList &out)
{
    out = SegList{};
    std::vector<SegChunk> ch;
    for (size_t i = 0; i < v.size(); ++i)
        for (long e = 0; e < (long)v[i].count * v[i].w; e += kSegChunk) ch.push_back(SegChunk{(int)i, (int)e});
    if (v.empty() || ch.empty()) return OCN_OK;
    const size_t sb = sizeof(Seg) * v.size(), cb = sizeof(SegChunk) * ch.size();
    char *d = nullptr;
    HIPCHK(hipMalloc(&d, sb + cb));
    c->allocs.push_back(d);
    HIPCHK(hipMemcpy(d, v.data(), sb, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(d + sb, ch.data(), cb, hipMemcpyHostToDevice));
    out.d = (Seg *)d;
    out.ch = (SegChunk *)(d + sb);
    out.n = (int)v.size();
    out.nch = (int)ch.size();
    return OCN_OK;
}
// the list's copies on s (cmp: compared instead, 1 ORed into *cmp where they differ)
static int launch_segs(const SegList &l, hipStream_t s, int32_t *cmp = nullptr)
{
    if (!l.nch) return OCN_OK;
    if (cmp) hipLaunchKernelGGL(k_segments_cmp, dim3((unsigned)l.nch), dim3(kSegChunk), 0, s, l.d, l.ch, l.nch, cmp);
    else hipLaunchKernelGGL(k_segments, dim3((unsigned)l.nch), dim3(kSegChunk), 0, s, l.d, l.ch, l.nch);
    return check_launch();
}

namespace ocn {

// real(8) fields of a context: the SW set, then flux_x, flux_y and ff1/ff1p/ff1n per tracer
static int num_r8(const ocn_ctx *c)
{
    return OCN_NUM_R8 + (c->sw.use_tracers > 0 ? 2 + 3 * c->sw.tracer_num : 0);
}
static bool has_r8(const ocn_ctx *c, int id) { return id >= OCN_SSH && id < OCN_SSH + num_r8(c); }
static bool has_field(const ocn_ctx *c, int id) { return is_r4(id) || has_r8(c, id); }

// ------------------------------------------------------------------ decomposition
// decomposition.f90:448-482: floor(real(remaining)/real(parts_left)) in default real(4)
static std::vector<int> uniform_sizes(int total, int parts, std::string &err)
{
    std::vector<int> s;
    int acc = 0;
    for (int i = 1; i <= parts; ++i) {
        int v = (i == parts) ? total - acc : (int)std::floor((float)(total - acc) / (float)(parts - i + 1));
        if (v <= 0) { err = "Error in decomposition to uniform blocks: size <= 0"; return {}; }
        s.push_back(v);
        acc += v;
    }
    return s;
}

// MPI_Dims_create(n, 2): balanced, non-increasing factors (mpp.f90:89).
static void dims_create(int n, int &d1, int &d2)
{
    d1 = n; d2 = 1;
    for (int f = (int)std::floor(std::sqrt((double)n)); f >= 1; --f)
        if (n % f == 0) { d1 = n / f; d2 = f; break; }
}

static int decompose(ocn_ctx *c)
{
    const int nx = c->basin.nx, ny = c->basin.ny;
    std::string err;
    auto xs = uniform_sizes(nx - 4, c->bnx, err);
    auto ys = uniform_sizes(ny - 4, c->bny, err);
    if (!err.empty()) return set_error(OCN_ERR_ARG, err);
    int p1, p2;
    dims_create(c->dec.nranks, p1, p2);
    if (c->bnx % p1 || c->bny % p2)
        return set_error(OCN_ERR_ARG, "mod(bnx, p_size(1)) or mod(bny, p_size(2)) not equal 0 (decomposition.f90:628)");
    const int lbx = c->bnx / p1, lby = c->bny / p2;
    c->gblocks.assign((size_t)c->bnx * c->bny, GBlock{});
    int x0 = 0;
    for (int bm = 1; bm <= c->bnx; ++bm) {
        int y0 = 0;
        for (int bn = 1; bn <= c->bny; ++bn) {
            GBlock &g = c->gblocks[(size_t)(bm - 1) + (size_t)(bn - 1) * c->bnx];
            g.bm = bm; g.bn = bn;
            g.g.nx_start = 3 + x0; g.g.nx_end = g.g.nx_start + xs[bm - 1] - 1;
            g.g.ny_start = 3 + y0; g.g.ny_end = g.g.ny_start + ys[bn - 1] - 1;
            g.g.bnd_x1 = g.g.nx_start - 2; g.g.bnd_x2 = g.g.nx_end + 2;
            g.g.bnd_y1 = g.g.ny_start - 2; g.g.bnd_y2 = g.g.ny_end + 2;
            g.g.pitch = 0;
            double w = 0.0;
            for (int i = g.g.nx_start; i <= g.g.nx_end; ++i)
                for (int j = g.g.ny_start; j <= g.g.ny_end; ++j)
                    w += 1.0 - (double)c->mask[(size_t)(i - 1) + (size_t)(j - 1) * nx];
            g.weight = w;
            // create_uniform_decomposition: process coords (row-major cart), land blocks -> -1
            const int c1 = (bm - 1) / lbx, c2 = (bn - 1) / lby;
            g.rank = (w == 0.0) ? -1 : c1 * p2 + c2;
            g.k = -1;
            y0 += ys[bn - 1];
        }
        x0 += xs[bm - 1];
    }
    // local numbering per rank: _MPP_SORTED_BLOCKS_ = MINLOC over weight (column-major order)
    std::vector<int> next(c->dec.nranks, 0);
    std::vector<int> order(c->gblocks.size());
    for (size_t i = 0; i < order.size(); ++i) order[i] = (int)i;
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) {
        return c->gblocks[a].weight < c->gblocks[b].weight;
    });
    for (int gid : order) {
        GBlock &g = c->gblocks[gid];
        if (g.rank >= 0) g.k = next[g.rank]++;
    }
    // local blocks of this rank, k order
    std::vector<int> mine;
    for (int gid : order)
        if (c->gblocks[gid].rank == c->dec.rank) mine.push_back(gid);
    c->blocks.clear();
    for (int gid : mine) {
        const GBlock &g = c->gblocks[gid];
        LBlock lb;
        lb.g = g.g;
        lb.bm = g.bm; lb.bn = g.bn; lb.gid = gid;
        const int w = g.g.bnd_x2 - g.g.bnd_x1 + 1;
        // 512-B aligned rows for r8, with room for 2 * kXRing more columns (the extra halo rings of
        // one_step_x4 live in the row padding: column bnd_x1 - j is the previous row's tail)
        lb.g.pitch = (int64_t)((w + 2 * kXRing + 63) / 64 * 64);
        for (int d = 1; d <= 8; ++d) {
            const int m = g.bm + kDirDm[d], n = g.bn + kDirDn[d];
            if (m < 1 || m > c->bnx || n < 1 || n > c->bny) {
                lb.nbr_rank[d - 1] = -2; lb.nbr_k[d - 1] = -1; lb.nbr_gid[d - 1] = -1;
            } else {
                const int ng = (m - 1) + (n - 1) * c->bnx;
                lb.nbr_rank[d - 1] = c->gblocks[ng].rank;
                lb.nbr_k[d - 1] = c->gblocks[ng].k;
                lb.nbr_gid[d - 1] = c->gblocks[ng].rank >= 0 ? ng : -1;
            }
            if (lb.nbr_rank[d - 1] >= 0)   // own_class(m) * 3 + own_class(n) of direction d's halo points
                lb.own |= 1u << ((unsigned)(kDirDm[d] + 1) * 3u + (unsigned)(kDirDn[d] + 1));
        }
        c->blocks.push_back(lb);
    }
    return OCN_OK;
}

// ------------------------------------------------------------------ storage
// The state arrays of the one-pass step as groups of physical buffers that agree on the second
// halo ring (the reference never writes it; the pairs are coherent, the second buffers copies):
// the field's own buffer first.
static const int kStateIds[6] = {OCN_SSH, OCN_SSHP, OCN_UBRTR, OCN_UBRTRP, OCN_VBRTR, OCN_VBRTRP};
static void state_group(const LBlock &b, int g, void *out[2])
{
    const int id = kStateIds[g];
    out[0] = b.ptr[field_slot(id)];
    switch (id) {
    case OCN_SSH: out[1] = b.ptr[field_slot(OCN_SSHN)]; break;
    case OCN_UBRTR: out[1] = b.ptr[field_slot(OCN_UBRTRN)]; break;
    case OCN_VBRTR: out[1] = b.ptr[field_slot(OCN_VBRTRN)]; break;
    case OCN_SSHP: out[1] = b.sshp_alt; break;
    case OCN_UBRTRP: out[1] = b.up_alt; break;
    default: out[1] = b.vp_alt; break;
    }
}

// one_step_x2's per-block storage: the ext metric rows, the row table with them, the h_r copy, the
// save area of the state's second halo ring and the runs that save / restore it (pointers of the
// physical buffers: role independent)
static int allocate_x2(ocn_ctx *c, LBlock &b)
{
    const int w = b.g.bnd_x2 - b.g.bnd_x1 + 1, h = b.g.bnd_y2 - b.g.bnd_y1 + 1;
    const size_t nrow = row_table_size((unsigned)h);
    HIPCHK(hipMalloc(&b.ext, kExtRowFloats * sizeof(float)));
    c->allocs.push_back(b.ext);
    HIPCHK(hipMalloc(&b.rows_x, nrow * sizeof(float)));
    c->allocs.push_back(b.rows_x);
    {   // based like the real(8) fields (kXRing more rows each side): x4 pairs of the h_r-read variant
        // read it 4 rings deep
        char *d = nullptr;
        const size_t nb = sizeof(double) * (size_t)(b.g.pitch * (h + 2 * kXRing)) + 512;
        HIPCHK(hipMalloc(&d, nb));
        c->allocs.push_back(d);
        HIPCHK(hipMemsetAsync(d, 0, nb, c->stream));   // (rings no exchange fills: +0.0)
        b.hr_x = (double *)(d + 256) + (long)kXRing * b.g.pitch;
    }
    const long per = 2L * w + 2L * (h - 2);   // rows bnd_y1, bnd_y2; columns bnd_x1, bnd_x2 between them
    // the state's six groups, then two per tracer (ff1 / ff1n, ff1p / its second buffer: x4 pairs
    // exchange the tracers 2 deep)
    const int ntr = c->sw.use_tracers > 0 ? c->sw.tracer_num : 0, ngroups = 6 + 2 * ntr;
    HIPCHK(hipMalloc(&b.ring2, sizeof(double) * (size_t)(ngroups * per)));
    c->allocs.push_back(b.ring2);
    HIPCHK(hipMalloc(&b.bits_x4, (size_t)b.g.pitch * (h + 2 * kXRing)));
    c->allocs.push_back(b.bits_x4);
    HIPCHK(hipMalloc(&b.rows_x4, row_table_size((unsigned)(h + 2 * kXRing)) * sizeof(float)));
    c->allocs.push_back(b.rows_x4);
    if (ntr) {
        const long xr = (long)kXRing * b.g.pitch;
        for (double *&q : b.trs) {
            char *d = nullptr;
            HIPCHK(hipMalloc(&d, sizeof(double) * (size_t)(b.g.pitch * (h + 2 * kXRing)) + 512));
            c->allocs.push_back(d);
            q = (double *)(d + 256) + xr;
        }
    }
    std::vector<Seg> save, restore;
    const long p = (long)b.g.pitch;
    for (int g = 0; g < ngroups; ++g) {
        void *buf[2];
        if (g < 6) {
            state_group(b, g, buf);
        } else {
            const int t = 1 + (g - 6) / 2;
            buf[0] = b.ptr[field_slot((g - 6) % 2 ? OCN_FF1P(t) : OCN_FF1(t))];
            buf[1] = (g - 6) % 2 ? b.ffp_alt[(size_t)t - 1] : b.ptr[field_slot(OCN_FF1N(t))];
        }
        double *area = b.ring2 + g * per;
        // (offset in the array, stride, count, offset in the area)
        const long runs[4][4] = {{0, 1, w, 0}, {(long)(h - 1) * p, 1, w, w}, {p, p, h - 2, 2L * w},
                                 {p + w - 1, p, h - 2, 2L * w + h - 2}};
        for (const auto &r : runs) {
            if (r[2] <= 0) continue;
            save.push_back(Seg{(const double *)buf[0] + r[0], area + r[3], r[1], 1, (int)r[2]});
            for (void *q : buf) restore.push_back(Seg{area + r[3], (double *)q + r[0], 1, r[1], (int)r[2]});
        }
    }
    RC(make_seglist(c, save, b.save));
    RC(make_seglist(c, restore, b.restore));
    return OCN_OK;
}

static int allocate(ocn_ctx *c)
{
    for (LBlock &b : c->blocks) {
        const long rows = b.g.bnd_y2 - b.g.bnd_y1 + 1;
        const long n = (long)b.g.pitch * rows;
        // every field padded to a 256-B multiple, based so that A(nx_start, :) rows are
        // 256-B aligned: base offset shifted by (nx_start - bnd_x1) = 2 elements.
        // OCN_FIELD_SKEW (bytes, multiple of 256): extra gap between consecutive fields.
        // real(8) fields: kXRing more rows above and below the array (one_step_x4's extra rings)
        const long xr = (long)kXRing * b.g.pitch * 8;
        const long r8b = ((n * 8 + 16 + 255) / 256) * 256 + 256 + OCN_FIELD_SKEW + 2 * xr;
        const long r4b = ((n * 4 + 8 + 255) / 256) * 256 + 256 + OCN_FIELD_SKEW;
        const int nr8 = num_r8(c), ntr = c->sw.use_tracers > 0 ? c->sw.tracer_num : 0;
        // + the three second buffers of the role-flip / one-pass steps, one per tracer (ff1p)
        const size_t total = (size_t)(nr8 + 3 + ntr) * r8b + (size_t)OCN_NUM_R4 * r4b + 256;
        HIPCHK(hipMalloc(&b.slab, total));
        c->allocs.push_back(b.slab);
        HIPCHK(hipMemsetAsync(b.slab, 0, total, c->stream));
        char *base = (char *)b.slab;
        size_t off = 0;
        b.ptr.assign((size_t)(OCN_NUM_R4 + nr8), nullptr);
        // r8 order in the slab: the one-pass step's state fields and their second buffers first,
        // next to each other (the arrays one march streams through share DRAM pages and TLB
        // entries), then the other SW fields, then the tracers'.  (Kernels address every field
        // through its own pointer; only byte offsets within one field are 32-bit.)
        std::vector<int> order = {OCN_SSH, OCN_SSHN, OCN_SSHP, OCN_UBRTR, OCN_UBRTRN, OCN_UBRTRP, OCN_VBRTR,
                                  OCN_VBRTRN, OCN_VBRTRP, -1, -2, -3, OCN_HHU, OCN_HHU_P, OCN_HHV, OCN_HHV_P, OCN_HHH,
                                  OCN_HHQ_REST, OCN_VORT, OCN_STR_T, OCN_STR_S, OCN_MU, OCN_RHSX, OCN_RHSY};
        for (int id = OCN_SSH; id < OCN_SSH + nr8; ++id)
            if (std::find(order.begin(), order.end(), id) == order.end()) order.push_back(id);
        for (int k = 1; k <= ntr; ++k) order.push_back(-3 - k);
        b.ffp_alt.assign((size_t)ntr, nullptr);
        for (int id : order) {
            char *p = base + off + 256 - 16 + xr;
            off += r8b;
            if (id == -1) b.sshp_alt = p;
            else if (id == -2) b.up_alt = p;
            else if (id == -3) b.vp_alt = p;
            else if (id < -3) b.ffp_alt[(size_t)(-4 - id)] = p;
            else b.ptr[field_slot(id)] = p;
        }
        for (int id = 0; id < OCN_NUM_R4; ++id) {
            b.ptr[field_slot(id)] = base + off + 256 - 8;
            off += r4b;
        }
    }
    for (LBlock &b : c->blocks) {
        const size_t n = (size_t)b.g.pitch * (b.g.bnd_y2 - b.g.bnd_y1 + 1);
        // metric row tables + ratios + reciprocals (sw_stencils.h kRowTable, recip_offset)
        const size_t nrow = row_table_size((unsigned)(b.g.bnd_y2 - b.g.bnd_y1 + 1));
        HIPCHK(hipMalloc(&b.bits, n));
        c->allocs.push_back(b.bits);
        HIPCHK(hipMalloc(&b.rows, nrow * sizeof(float)));
        c->allocs.push_back(b.rows);
        RC(allocate_x2(c, b));
    }
    // d_nbad words: 0 check_ssh_err's count, 16 the fallback check's verdict (d_fbz), 32..47 flags and
    // the vote (d_flags), 48..55 the loopback vote's reduction, 56 the count's maximum over the ranks
    // (sync_impl), 61 the multi-step launch's barrier timeout flag; then per block h_r, mu (LBlock::kc)
    const size_t kcb = 16 * c->blocks.size();
    HIPCHK(hipMalloc(&c->d_nbad, 256 + kcb));
    c->allocs.push_back(c->d_nbad);
    HIPCHK(hipMalloc(&c->d_bar, kMultiBarBytes));
    c->allocs.push_back(c->d_bar);
    HIPCHK(hipMemsetAsync(c->d_nbad, 0, 256 + kcb, c->stream));
    c->d_fbz = c->d_nbad + 16;
    c->d_flags = c->d_nbad + 32;
    for (size_t i = 0; i < c->blocks.size(); ++i) c->blocks[i].kc = (double *)((char *)c->d_nbad + 256) + 2 * i;
    return OCN_OK;
}

// ------------------------------------------------------------------ halo plans
// syncborder_block2D_gen_all.fi: halo of block k in dir d <- boundary of neighbour in inverse(d).
// Messages between two processes carry, for every (sending block, dir) pair in global block
// order and every field of the sync group, the boundary strip in column-major order.
// Host-only schedule of one halo exchange (no device pointers): every entry copies the
// 1-wide strip `src` of local block ks (local copy or send) into the strip `dst` of local block
// k (local copy or receive).  Message layout between two processes: for every (receiving
// block, dir) in global block order, every field of the group, the sender's boundary strip in
// column-major order -- enumerated identically on both sides from global knowledge.
struct PlanEntry {
    int kind;          // OCN_HALO_LOCAL / OCN_HALO_SEND / OCN_HALO_RECV
    int peer;          // rank (send/recv), own rank for local
    int k, ks;         // destination / source local block (-1 where not applicable)
    int field;
    Rect dst, src;
    long buf_off;      // element offset in the peer's message (send/recv)
    int count;
};

// Layer j (1 .. depth) of the halo of block `rcv` in direction d and the boundary of its
// neighbour `src` it receives: layer 1 is the reference's 1-wide exchange (syncborder_block2D_gen_all.fi);
// layer 2 (depth 2, the one-pass steps' state exchange, one_step_x2) the next row / column out
// (and depth x depth corner patches).  Corner layers are rows of `depth` points.
static void halo_layer(const ocn_block &rcv, const ocn_block &src, int d, int j, int depth, Rect &hr, Rect &br)
{
    const int dm = kDirDm[d], dn = kDirDn[d];
    // x: halo columns / source columns of this direction
    int hx0, hx1, sx0, sx1;
    if (dm > 0) { hx0 = rcv.nx_end + 1; hx1 = rcv.nx_end + (dn ? depth : 1); sx0 = src.nx_start; sx1 = sx0 + (hx1 - hx0); }
    else if (dm < 0) { hx1 = rcv.nx_start - 1; hx0 = rcv.nx_start - (dn ? depth : 1); sx1 = src.nx_end; sx0 = sx1 - (hx1 - hx0); }
    else { hx0 = rcv.nx_start; hx1 = rcv.nx_end; sx0 = src.nx_start; sx1 = src.nx_end; }
    if (dm && !dn) {   // E / W edge: layer j is one column
        hx0 = hx1 = dm > 0 ? rcv.nx_end + j : rcv.nx_start - j;
        sx0 = sx1 = dm > 0 ? src.nx_start + j - 1 : src.nx_end - j + 1;
    }
    int hy, sy;
    if (dn > 0) { hy = rcv.ny_end + j; sy = src.ny_start + j - 1; }
    else if (dn < 0) { hy = rcv.ny_start - j; sy = src.ny_end - j + 1; }
    else { hy = -1; sy = -1; }
    if (dn) { hr = {hx0, hx1, hy, hy}; br = {sx0, sx1, sy, sy}; }
    else { hr = {hx0, hx1, rcv.ny_start, rcv.ny_end}; br = {sx0, sx1, src.ny_start, src.ny_end}; }
}

// a tracer field (ff1 / ff1p / ff1n of some tracer)
static bool is_tracer_field(int id) { return id >= OCN_TRACER_BASE; }
// Depth of field id in an exchange of `depth`: the tracer fields are exchanged one point deep in
// every exchange (one_step_x2 sends them with the state's two-deep strips: one message per peer)
// tracers: 1 deep, 2 with the x4 pairs' 4-deep state (one_step_x4's first tracer step covers the halo
// ring neighbours own)
static int field_depth(int id, int depth) { return is_tracer_field(id) ? (depth >= 4 ? 2 : 1) : depth; }

static int plan_entries(const ocn_ctx *c, const std::vector<int> &fields, std::vector<PlanEntry> &out,
                        int depth = 1)
{
    out.clear();
    std::map<int, int> k_of_gid;
    for (size_t k = 0; k < c->blocks.size(); ++k) k_of_gid[c->blocks[k].gid] = (int)k;
    std::map<int, long> send_count, recv_count;
    // receiving side: my halos in gid order, dirs 1..8, layers 1..depth
    for (auto &kv : k_of_gid) {
        const int k = kv.second;
        const LBlock &b = c->blocks[k];
        for (int d = 1; d <= 8; ++d) {
            const int r = b.nbr_rank[d - 1];
            if (r < 0) continue;
            const GBlock &src = c->gblocks[b.nbr_gid[d - 1]];
            for (int j = 1; j <= depth; ++j) {
                for (int id : fields) {
                    const int fd = field_depth(id, depth);
                    if (j > fd) continue;
                    Rect hr, br;
                    halo_layer(b.g, src.g, d, j, fd, hr, br);
                    const int cnt = (hr.x1 - hr.x0 + 1) * (hr.y1 - hr.y0 + 1);
                    if (r == c->dec.rank)
                        out.push_back(PlanEntry{OCN_HALO_LOCAL, r, k, k_of_gid.at(b.nbr_gid[d - 1]), id, hr, br, 0, cnt});
                    else {
                        out.push_back(PlanEntry{OCN_HALO_RECV, r, k, -1, id, hr, br, recv_count[r], cnt});
                        recv_count[r] += cnt;
                    }
                }
            }
        }
    }
    // sending side: remote receivers in gid order, dirs 1..8, layers 1..depth, whose source block is mine
    for (size_t gid = 0; gid < c->gblocks.size(); ++gid) {
        const GBlock &rb = c->gblocks[gid];
        if (rb.rank < 0 || rb.rank == c->dec.rank) continue;
        for (int d = 1; d <= 8; ++d) {
            const int m = rb.bm + kDirDm[d], n = rb.bn + kDirDn[d];
            if (m < 1 || m > c->bnx || n < 1 || n > c->bny) continue;
            const int sg = (m - 1) + (n - 1) * c->bnx;
            if (c->gblocks[sg].rank != c->dec.rank) continue;
            const int ks = k_of_gid.at(sg);
            for (int j = 1; j <= depth; ++j) {
                for (int id : fields) {
                    const int fd = field_depth(id, depth);
                    if (j > fd) continue;
                    Rect hr, br;
                    halo_layer(rb.g, c->blocks[ks].g, d, j, fd, hr, br);
                    const int cnt = (br.x1 - br.x0 + 1) * (br.y1 - br.y0 + 1);
                    out.push_back(PlanEntry{OCN_HALO_SEND, rb.rank, -1, ks, id, hr, br, send_count[rb.rank], cnt});
                    send_count[rb.rank] += cnt;
                }
            }
        }
    }
    for (auto &kv : recv_count)
        if (send_count[kv.first] != kv.second) return set_error(OCN_ERR_STATE, "halo plan: asymmetric message sizes");
    for (auto &kv : send_count)
        if (recv_count[kv.first] != kv.second) return set_error(OCN_ERR_STATE, "halo plan: asymmetric message sizes");
    return OCN_OK;
}

// Column strips (a side with a stride) of the same length whose runs are adjacent columns on a strided
// side (step +1 or -1), the other side's runs equally spaced -- as the layers of one field's E / W strip
// are: one segment of w runs (up to kSegMaxW) instead of w, copying the same elements.
constexpr int kSegMaxW = 8;
static std::vector<Seg> merge_columns(const std::vector<Seg> &in)
{
    std::vector<Seg> out;
    std::vector<char> used(in.size(), 0);
    std::map<const double *, size_t> by_src, by_dst;   // the column strips by their strided side
    for (size_t i = 0; i < in.size(); ++i) {
        if (in[i].w != 1) continue;
        if (in[i].src_stride > 1) by_src[in[i].src] = i;
        else if (in[i].dst_stride > 1) by_dst[in[i].dst] = i;
    }
    for (size_t i = 0; i < in.size(); ++i) {
        if (used[i]) continue;
        used[i] = 1;
        Seg g = in[i];
        const bool sc = g.src_stride > 1, dc = !sc && g.dst_stride > 1;
        if (g.w == 1 && (sc || dc)) {
            for (const long step : {1L, -1L}) {
                if (g.w > 1) break;
                while (g.w < kSegMaxW) {
                    auto &idx = sc ? by_src : by_dst;
                    auto it = idx.find((sc ? (const double *)g.src : (const double *)g.dst) + (long)g.w * step);
                    if (it == idx.end() || used[it->second]) break;
                    const Seg &b = in[it->second];
                    if (b.count != g.count || b.src_stride != g.src_stride || b.dst_stride != g.dst_stride) break;
                    // the other side's spacing: set by the second run, kept by the rest
                    const long other = sc ? (long)(b.dst - g.dst) : (long)(b.src - g.src);
                    if (g.w == 1) {
                        if (sc) { g.src_jstride = step; g.dst_jstride = other; }
                        else { g.dst_jstride = step; g.src_jstride = other; }
                    } else if (other != (long)g.w * (sc ? g.dst_jstride : g.src_jstride)) {
                        break;
                    }
                    used[it->second] = 1;
                    ++g.w;
                }
            }
        }
        out.push_back(g);
    }
    return out;
}

static int build_plan(ocn_ctx *c, const std::vector<int> &fields, HaloPlan &plan, int depth = 1)
{
    std::vector<PlanEntry> entries;
    RC(plan_entries(c, fields, entries, depth));
    std::map<int, long> msg;                       // peer -> message length
    for (const PlanEntry &e : entries)
        if (e.kind == OCN_HALO_RECV) msg[e.peer] = std::max(msg[e.peer], e.buf_off + e.count);
    std::map<int, HaloPlan::Peer> peers;
    for (auto &kv : msg) {
        HaloPlan::Peer p{kv.first, kv.second, nullptr, nullptr};
        HIPCHK(hipMalloc(&p.send, sizeof(double) * std::max(1L, p.count)));
        HIPCHK(hipMalloc(&p.recv, sizeof(double) * std::max(1L, p.count)));
        c->allocs.push_back(p.send); c->allocs.push_back(p.recv);
        peers[kv.first] = p;
        plan.peers.push_back(p);
    }
    std::vector<Seg> local, pack, unpack;
    for (const PlanEntry &e : entries) {
        long doff, soff, dstr, sstr; int dcnt, scnt;
        if (e.kind == OCN_HALO_LOCAL) {
            const LBlock &db = c->blocks[e.k], &sb = c->blocks[e.ks];
            strip(db.g, e.dst, doff, dcnt, dstr);
            strip(sb.g, e.src, soff, scnt, sstr);
            local.push_back(Seg{sb.f<double>(e.field) + soff, db.f<double>(e.field) + doff, sstr, dstr, dcnt});
        } else if (e.kind == OCN_HALO_RECV) {
            const LBlock &db = c->blocks[e.k];
            strip(db.g, e.dst, doff, dcnt, dstr);
            unpack.push_back(Seg{peers.at(e.peer).recv + e.buf_off, db.f<double>(e.field) + doff, 1, dstr, dcnt});
        } else {
            const LBlock &sb = c->blocks[e.ks];
            strip(sb.g, e.src, soff, scnt, sstr);
            pack.push_back(Seg{sb.f<double>(e.field) + soff, peers.at(e.peer).send + e.buf_off, sstr, 1, scnt});
        }
    }
    RC(make_seglist(c, merge_columns(local), plan.local));
    RC(make_seglist(c, merge_columns(pack), plan.pack));
    RC(make_seglist(c, merge_columns(unpack), plan.unpack));
    return OCN_OK;
}

// Plans hold raw field pointers, so a plan is kept per role of the buffers its fields swap
// between (the key is the field list followed by -1 - the relevant role bits).
static bool is_alt_field(int id);
// depth 2: the one-pass steps' 2-deep state exchange (halo_layer); priv: a plan over a private
// buffer swapped into the field table while it is built and run (one_step_x2's h_r copy)
static int get_plan(ocn_ctx *c, const std::vector<int> &fields, HaloPlan *&out, int depth = 1, int priv = 0)
{
    std::vector<int> key = fields;
    // a plan holds the buffers its fields had when it was built: the pair roles (bit 1), and for
    // sshp / ubrtrp / vbrtrp the second buffers' roles (bit 4: they persist between one-pass calls)
    const bool alt = std::any_of(fields.begin(), fields.end(), [](int id) { return is_alt_field(id); });
    // (tracer fields: the tracer steps' role bits 8 -- ff1 / ff1n -- and 16 -- ff1p's second buffer)
    const bool tr = std::any_of(fields.begin(), fields.end(), [](int id) { return is_tracer_field(id); });
    key.push_back(-1 - (c->role & 1) - (alt ? (c->role & 4) : 0) - (tr ? (c->role & 24) : 0));
    if (depth != 1 || priv) key.push_back(-100 - depth - 10 * priv);
    auto it = c->plans.find(key);
    if (it == c->plans.end()) {
        if (c->capturing) return set_error(OCN_ERR_STATE, "halo plan built while a step is captured");
        HaloPlan p;
        RC(build_plan(c, fields, p, depth));
        it = c->plans.emplace(key, p).first;
    }
    out = &it->second;
    return OCN_OK;
}

static int nccl_rc(ncclResult_t r, const char *what)
{
    if (r == ncclSuccess) return OCN_OK;
    return set_error(OCN_ERR_COMM, std::string(what) + ": " + ncclGetErrorString(r));
}

static bool has_comm(const ocn_ctx *c) { return c->comm || c->lb || c->comm_aborted; }
static int comm_gone(const ocn_ctx *c)
{
    return set_error(OCN_ERR_COMM, "the RCCL communicator was aborted after an earlier fatal error");
}
// OCN_OPT_OVERLAP in effect: by default (-1) the role-flip steps' exchanges overlap their inner
// launches (2) when exchanges go to other ranks (RCCL: latency, not copy bandwidth), and run
// between the launches (1) when every exchange is a local device copy -- there the frame bands
// cost as much as the copies they hide (HISTORY.md section 5)
static int overlap_level(const ocn_ctx *c)
{
    if (c->overlap >= 0) return c->overlap;
    if (!(has_comm(c) && c->dec.nranks > 1)) return 1;
    return c->ov_state == 3 ? c->ov_level : 2;   // (measured: ov_begin, check_coherence)
}

// The form of an x2 step (kind 2) or an x4 pair (kind 4) under OCN_OPT_OVERLAP auto with peers on
// other ranks.  Until the vote has decided, the first such step (not one that opens a sequence: its
// ring save would be timed too) runs in sequence and the next of the same kind overlapped, each
// between two events on the context stream (probe 1 / 2: ov_mark at its start and end); the next
// check_coherence max-reduces both times over the ranks and keeps the faster form (ov_level) --
// every rank the same.  Either form runs the same exchange (one group per step or pair), so ranks
// may differ in form meanwhile; the results are the same bit for bit.
static int ov_begin(ocn_ctx *c, int kind, bool allow, int &probe)
{
    probe = 0;
    const int lv = overlap_level(c);
    if (c->overlap >= 0 || !(has_comm(c) && c->dec.nranks > 1) || c->capturing || !allow || c->ov_state >= 2)
        return lv;
    for (hipEvent_t &e : c->ov_ev)
        if (!e && hipEventCreate(&e) != hipSuccess) return lv;
    if (c->ov_state == 0 || c->ov_kind != kind) {
        c->ov_state = 0;
        c->ov_kind = kind;
        probe = 1;
        return 1;
    }
    probe = 2;
    return 2;
}
// probe's start (end = false) or end event on the context stream; the end advances ov_state
static int ov_mark(ocn_ctx *c, int probe, bool end)
{
    if (!probe) return OCN_OK;
    HIPCHK(hipEventRecord(c->ov_ev[2 * (probe - 1) + (end ? 1 : 0)], c->stream));
    if (end) c->ov_state = probe;
    return OCN_OK;
}

// a rank of a loopback group that fails releases its peers' waits at once
static int lb_fail_on_error(ocn_ctx *c, int rc)
{
    if (rc && c->lb) {
        std::lock_guard<std::mutex> g(c->lb->mu);
        c->lb->failed = true;
        c->lb->cv.notify_all();
    }
    return rc;
}

// An error inside a call that takes part in collectives (step, init_state, synchronize): the
// loopback group's waits are released (lb_fail_on_error), and a fatal one (HIP, RCCL, state) aborts
// the RCCL communicator -- its queued sends / receives are cancelled and nothing of this rank waits
// on a peer that will not come; the host then ends the job, as abort_model's mpi_abort does
// (shared/errors.f90:30-37).  OCN_ERR_BLOWUP is not fatal here: every rank returns it from the same
// synchronize (sync_impl reduces the counts), and OCN_ERR_ARG is raised before any collective.
static int fail_fatal(ocn_ctx *c, int rc)
{
    rc = lb_fail_on_error(c, rc);
    if ((rc && rc != OCN_ERR_BLOWUP && rc != OCN_ERR_ARG) || c->wd_fired.load()) {
        std::lock_guard<std::mutex> g(c->comm_mu);
        if (c->comm) {
            if (!c->comm_abort_done) (void)ncclCommAbort(c->comm);   // (the watchdog may have)
            c->comm_abort_done = true;
            c->comm = nullptr;
            c->comm_aborted = true;
        }
    }
    return rc;
}

// ------------------------------------------------------------------ host-side watchdog
// ocn_ctx_set_watchdog: a thread per context watches the entries that may take part in a collective
// (guarded below).  One that has not returned after wd_s is ended: the message names the call and the
// last exchange with remote peers the device completed (polled from c->xq), the RCCL communicator is
// aborted (RCCL's kernels waiting on a peer exit, so the call's stream wait returns) or the loopback
// group failed (its rendezvous return), and the call returns OCN_ERR_COMM with the message.  A call
// still stuck 10 s later ends the process (exit status 3).
static int64_t poll_xdone(ocn_ctx *c)
{
    std::lock_guard<std::mutex> g(c->xmu);
    while (!c->xq.empty() && hipEventQuery(c->xq.front().second) == hipSuccess) {
        c->xdone = c->xq.front().first;
        c->xpool.push_back(c->xq.front().second);
        c->xq.pop_front();
    }
    return c->xdone;
}

static void wd_fire(ocn_ctx *c, const char *call, double waited)
{
    const int64_t done = poll_xdone(c);
    char buf[512];
    std::snprintf(buf, sizeof buf,
                  "ocn watchdog: rank %d of %d: %s has not returned after %.1f s (limit %.1f s); last completed "
                  "exchange id %lld of %lld enqueued; %s",
                  c->dec.rank, c->dec.nranks, call, waited, c->wd_s, (long long)done, (long long)c->xchg,
                  c->lb ? "failing the loopback group" : c->comm ? "aborting the RCCL communicator" : "no communicator");
    c->wd_msg = buf;
    c->wd_fired.store(true);
    std::fprintf(stderr, "%s\n", buf);
    std::fflush(stderr);
    if (c->lb) {
        std::lock_guard<std::mutex> g(c->lb->mu);
        c->lb->failed = true;
        c->lb->cv.notify_all();
    }
    std::lock_guard<std::mutex> g(c->comm_mu);
    if (c->comm && !c->comm_abort_done) {
        (void)ncclCommAbort(c->comm);
        c->comm_abort_done = true;
    }
}

static void wd_loop(ocn_ctx *c)
{
    (void)hipSetDevice(c->dec.device);
    std::unique_lock<std::mutex> g(c->wd_mu);
    while (!c->wd_stop) {
        c->wd_cv.wait_for(g, std::chrono::milliseconds(100));
        if (c->wd_stop || c->call_depth == 0 || c->wd_fired.load() || c->wd_s <= 0) continue;
        const double waited = std::chrono::duration<double>(std::chrono::steady_clock::now() - c->call_t0).count();
        if (waited < c->wd_s) continue;
        const char *call = c->call_name;
        g.unlock();
        wd_fire(c, call, waited);
        g.lock();
        if (!c->wd_cv.wait_for(g, std::chrono::seconds(10), [c] { return c->wd_stop || c->call_depth == 0; })) {
            std::fprintf(stderr, "ocn watchdog: rank %d: %s still blocked 10 s after the abort; exiting (status 3)\n",
                         c->dec.rank, call);
            std::fflush(stderr);
            std::_Exit(3);
        }
    }
}

// An entry that may take part in a collective, watched while a watchdog is set
struct CallGuard {
    ocn_ctx *c;
    CallGuard(ocn_ctx *ctx, const char *name) : c(ctx)
    {
        std::lock_guard<std::mutex> g(c->wd_mu);
        if (c->call_depth++ == 0) {
            c->call_t0 = std::chrono::steady_clock::now();
            c->call_name = name;
        }
    }
    ~CallGuard()
    {
        std::lock_guard<std::mutex> g(c->wd_mu);
        --c->call_depth;
        c->wd_cv.notify_all();
    }
};
template <class F> static int guarded(ocn_ctx *c, const char *name, F &&f)
{
    if (c->wd_fired.load()) return set_error(OCN_ERR_COMM, c->wd_msg);
    int rc;
    {
        CallGuard g(c, name);
        rc = f();
    }
    if (c->wd_fired.load()) {   // (the call returned because the watchdog ended it)
        std::lock_guard<std::mutex> g(c->comm_mu);
        if (c->comm) { c->comm = nullptr; c->comm_aborted = true; }
        return set_error(OCN_ERR_COMM, c->wd_msg);
    }
    return rc;
}

// One loopback rendezvous: this rank passes phase `ph`, then waits until every rank in `peers`
// has passed it as often (bounded wait: a rank that failed or never comes ends it with an error).
static int lb_meet(ocn_ctx *c, int ph, const std::vector<int> &peers)
{
    Loopback &L = *c->lb;
    const int r = c->dec.rank;
    std::unique_lock<std::mutex> g(L.mu);
    const uint64_t mine = ++L.cnt[ph][r];
    L.cv.notify_all();
    bool lost = false;   // a peer still needed failed or was destroyed
    const bool ok = L.cv.wait_for(g, std::chrono::seconds(120), [&] {
        bool all = true;
        for (int p : peers)
            if (L.cnt[ph][p] < mine) {
                all = false;
                lost = lost || L.failed || !L.ctx[p];
            }
        return all || lost;
    });
    if (!ok || lost) {
        L.failed = true;
        L.cv.notify_all();
        return set_error(OCN_ERR_COMM, "loopback transport: a peer rank did not reach the exchange");
    }
    return OCN_OK;
}

// The ncclRecv / ncclSend pairs of one exchange over the loopback transport (see Loopback).
static int lb_exchange(ocn_ctx *c, const HaloPlan *p, hipStream_t stream)
{
    Loopback &L = *c->lb;
    const int r = c->dec.rank;
    std::vector<int> peers;
    for (const auto &q : p->peers) peers.push_back(q.rank);
    HIPCHK(hipEventRecord(c->lb_ev_a, stream));
    {
        std::lock_guard<std::mutex> g(L.mu);
        L.plan[r] = p;
    }
    RC(lb_meet(c, 0, peers));
    for (const auto &q : p->peers) {
        const HaloPlan *pp;
        hipEvent_t ev;
        {   // a peer destroyed after the rendezvous has left its slot empty: fail, do not dereference
            std::lock_guard<std::mutex> g(L.mu);
            if (!L.ctx[q.rank]) return set_error(OCN_ERR_COMM, "loopback transport: a peer rank was destroyed");
            pp = L.plan[q.rank];
            ev = L.ctx[q.rank]->lb_ev_a;
        }
        const HaloPlan::Peer *src = nullptr;
        for (const auto &e : pp->peers)
            if (e.rank == r) src = &e;
        if (!src || src->count != q.count) return set_error(OCN_ERR_STATE, "loopback transport: message sizes disagree");
        HIPCHK(hipStreamWaitEvent(stream, ev, 0));
        HIPCHK(hipMemcpyAsync(q.recv, src->send, sizeof(double) * (size_t)q.count, hipMemcpyDeviceToDevice, stream));
    }
    HIPCHK(hipEventRecord(c->lb_ev_b, stream));
    RC(lb_meet(c, 1, peers));
    std::vector<hipEvent_t> evs;
    {
        std::lock_guard<std::mutex> g(L.mu);
        for (const auto &q : p->peers) {
            if (!L.ctx[q.rank]) return set_error(OCN_ERR_COMM, "loopback transport: a peer rank was destroyed");
            evs.push_back(L.ctx[q.rank]->lb_ev_b);
        }
    }
    for (hipEvent_t e : evs) HIPCHK(hipStreamWaitEvent(stream, e, 0));
    return OCN_OK;
}

// max over the ranks of one device int32 (the role-flip vote): ncclAllReduce, or over the
// loopback transport every rank reads every rank's word (after its lb_ev_a) into d_red and copies
// it back after all ranks have read (lb_ev_b).
struct VotePtrs { const int32_t *p[64]; int n, words; };
__global__ void k_vote_max(VotePtrs v, int32_t *out)
{
    const int w = (int)threadIdx.x;
    if (w >= v.words) return;
    int32_t m = v.p[0][w];
    for (int i = 1; i < v.n; ++i) m = max(m, v.p[i][w]);
    out[w] = m;
}
constexpr int kVoteWords = 8;   // the role-flip vote (check_coherence): one 0/1 word per condition
static int allreduce_max(ocn_ctx *c, int32_t *word, hipStream_t s, int words = 1)
{
    if (c->comm_aborted) return comm_gone(c);
    if (c->wd_fired.load()) return set_error(OCN_ERR_COMM, c->wd_msg);
    if (c->comm)
        return nccl_rc(ncclAllReduce(word, word, (size_t)words, ncclInt32, ncclMax, c->comm, s), "ncclAllReduce");
    if (!c->lb) return OCN_OK;
    Loopback &L = *c->lb;
    std::vector<int> all(L.n);
    for (int i = 0; i < L.n; ++i) all[i] = i;
    HIPCHK(hipEventRecord(c->lb_ev_a, s));
    {
        std::lock_guard<std::mutex> g(L.mu);
        L.vote[c->dec.rank] = word;
    }
    RC(lb_meet(c, 2, all));
    VotePtrs v{};
    v.n = L.n;
    v.words = words;
    std::vector<hipEvent_t> evs;
    {   // snapshot under the lock: a peer destroyed after the rendezvous fails the vote
        std::lock_guard<std::mutex> g(L.mu);
        for (int i = 0; i < L.n; ++i) {
            if (!L.ctx[i]) return set_error(OCN_ERR_COMM, "loopback transport: a peer rank was destroyed");
            v.p[i] = L.vote[i];
            evs.push_back(L.ctx[i]->lb_ev_a);
        }
    }
    for (hipEvent_t e : evs) HIPCHK(hipStreamWaitEvent(s, e, 0));
    int32_t *red = c->d_nbad + 48;
    hipLaunchKernelGGL(k_vote_max, dim3(1), dim3(64), 0, s, v, red);
    RC(check_launch());
    HIPCHK(hipEventRecord(c->lb_ev_b, s));
    RC(lb_meet(c, 3, all));
    evs.clear();
    {
        std::lock_guard<std::mutex> g(L.mu);
        for (int i = 0; i < L.n; ++i) {
            if (!L.ctx[i]) return set_error(OCN_ERR_COMM, "loopback transport: a peer rank was destroyed");
            evs.push_back(L.ctx[i]->lb_ev_b);
        }
    }
    for (hipEvent_t e : evs) HIPCHK(hipStreamWaitEvent(s, e, 0));
    HIPCHK(hipMemcpyAsync(word, red, sizeof(int32_t) * (size_t)words, hipMemcpyDeviceToDevice, s));
    return OCN_OK;
}

static int get_event(ocn_ctx *c, hipEvent_t &e);

// The end of an exchange with remote peers on `stream`: its timer record, and while a watchdog is set
// an event the watchdog polls for the last completed exchange (c->xq; completed events are recycled)
static int exchange_done(ocn_ctx *c, ocn_ctx::Rec &xrec, hipStream_t stream)
{
    if (c->capturing) return OCN_OK;
    if (xrec.b) {
        HIPCHK(hipEventRecord(xrec.b, stream));
        c->recs.push_back(xrec);
    }
    if (c->wd_s <= 0) return OCN_OK;
    std::lock_guard<std::mutex> g(c->xmu);
    while (!c->xq.empty() && (c->xq.size() > 256 || hipEventQuery(c->xq.front().second) == hipSuccess)) {
        if (hipEventQuery(c->xq.front().second) == hipSuccess) c->xdone = c->xq.front().first;
        else HIPCHK(hipEventSynchronize(c->xq.front().second));   // (256 in flight: the oldest has to finish)
        c->xpool.push_back(c->xq.front().second);
        c->xq.pop_front();
    }
    hipEvent_t e;
    if (!c->xpool.empty()) { e = c->xpool.back(); c->xpool.pop_back(); }
    else HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming | hipEventDisableSystemFence));
    HIPCHK(hipEventRecord(e, stream));
    c->xq.emplace_back(c->xchg, e);
    return OCN_OK;
}

// cmp != nullptr: compare the halos with what the exchange would deliver instead of writing them
// (ORs 1 into *cmp where they differ); same messages, so every rank must take part.
// OCN_OPT_XCHG_DELAY (tests): one wave waits c->xdelay_us on the device clock (a slow link's latency,
// in front of an exchange with remote peers); the loop always ends
__global__ void k_delay(unsigned long long ticks)
{
    const unsigned long long t0 = wall_clock64();
    while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
}
static int launch_delay(ocn_ctx *c, hipStream_t s)
{
    int khz = 0;
    HIPCHK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, c->dec.device));
    const unsigned long long ticks = (unsigned long long)c->xdelay_us * (unsigned long long)(khz > 0 ? khz : 100000) / 1000ull;
    hipLaunchKernelGGL(k_delay, dim3(1), dim3(64), 0, s, ticks);
    return check_launch();
}

static int run_sync(ocn_ctx *c, const std::vector<int> &fields, hipStream_t stream = nullptr, int32_t *cmp = nullptr,
                    int depth = 1, int priv = 0)
{
    HaloPlan *p;
    RC(get_plan(c, fields, p, depth, priv));
    if (!stream) stream = c->stream;
    ocn_ctx::Rec xrec{OCN_TIMER_EXCHANGE, nullptr, nullptr};
    const bool remote = !p->peers.empty();
    if (remote) {
        if (!has_comm(c)) return set_error(OCN_ERR_COMM, "remote neighbours but no RCCL communicator attached");
        if (c->comm_aborted) return comm_gone(c);
        if (c->wd_fired.load()) return set_error(OCN_ERR_COMM, c->wd_msg);
        if (c->stage_timing && !c->capturing) {   // the exchange on its stream: pack, group, unpack
            RC(get_event(c, xrec.a)); RC(get_event(c, xrec.b));
            HIPCHK(hipEventRecord(xrec.a, stream));
        }
        ++c->xchg;
        if (c->xdelay_us > 0) RC(launch_delay(c, stream));
        RC(launch_segs(p->pack, stream));
        if (c->lb) {
            RC(lb_exchange(c, p, stream));
        } else {
            RC(nccl_rc(ncclGroupStart(), "ncclGroupStart"));
            for (auto &peer : p->peers) {
                RC(nccl_rc(ncclRecv(peer.recv, (size_t)peer.count, ncclDouble, peer.rank, c->comm, stream), "ncclRecv"));
                RC(nccl_rc(ncclSend(peer.send, (size_t)peer.count, ncclDouble, peer.rank, c->comm, stream), "ncclSend"));
            }
            RC(nccl_rc(ncclGroupEnd(), "ncclGroupEnd"));
        }
    }
    if (cmp) {
        RC(launch_segs(p->local, stream, cmp));
        RC(launch_segs(p->unpack, stream, cmp));
        return remote ? exchange_done(c, xrec, stream) : OCN_OK;
    }
    RC(launch_segs(p->local, stream));
    RC(launch_segs(p->unpack, stream));
    if (remote) RC(exchange_done(c, xrec, stream));
    return OCN_OK;
}

// ------------------------------------------------------------------ stages (envoke)
// sync lists: interface/shallow_water/sw_interface.f90 envoke_*_sync
static const std::vector<int> kSyncSsh = {OCN_SSHN};
static const std::vector<int> kSyncHhUpdate = {OCN_HHU_N, OCN_HHV_N, OCN_HHH_N};
static const std::vector<int> kSyncVort = {OCN_VORT};
static const std::vector<int> kSyncUvTrans = {OCN_HHU_P, OCN_HHV_P, OCN_HHH_P};
static const std::vector<int> kSyncStress = {OCN_STR_T, OCN_STR_S};
static const std::vector<int> kSyncUv = {OCN_VBRTRN, OCN_UBRTRN};
static const std::vector<int> kSyncHhInit = {OCN_HHU, OCN_HHV, OCN_HHH};
// role-flip steps with halo exchanges: halo values that must equal the neighbours' (ocn_ctx.hip
// check_coherence)
static const std::vector<int> kHaloCheck = {OCN_SSH, OCN_UBRTR, OCN_VBRTR, OCN_HHU, OCN_HHV, OCN_HHQ_REST};

// f(b) for every block of the context.  With OCN_OPT_BATCH and several blocks the launches f makes
// on stream s are batched (ocn_internal.h Batcher): each kernel of the loop is launched once for all
// the blocks (up to kPack of them per launch) instead of once per block.  Only for loops whose
// launches read and write their own block's arrays, with nothing but batchable launches on s.
// co: the loop's launches read nothing another writes -- a march batch and the tracer-step batch
// after it may go as one launch (Batcher::co_launch; batched for one block too)
template <class F> static int each_block(ocn_ctx *c, hipStream_t s, F &&f, bool co = false)
{
    const bool on = c->batch && (c->blocks.size() > 1 || co);
    if (on) {
        batch_begin(&c->batcher, s);
        c->batcher.co_launch = co;
    }
    int rc = OCN_OK;
    for (size_t i = 0; i < c->blocks.size() && rc == OCN_OK; ++i) {
        if (on) batch_next(&c->batcher);
        rc = f(c->blocks[i]);
    }
    if (on) {
        const int r2 = batch_end(&c->batcher);
        if (rc == OCN_OK) rc = r2;
        if (co && c->batcher.co_launched) c->co_used = true;
    }
    return rc;
}

static int stage_kernel(ocn_ctx *c, const LBlock &b, int stage, double tau)
{
    const ocn_block *g = &b.g;
    void *s = c->stream;
    if (c->compact) {   // the compact tables (prepare_static): mask bytes and row metrics
        const Compact t{b.bits, b.rows, c->march};
        return launch_stage(g, b.ptr.data(), (int)b.ptr.size(), &t, stage, c->sw, tau, c->d_nbad, c->stream);
    }
#define R4(id) b.f<const float>(id)
#define R8(id) b.f<double>(id)
    switch (stage) {
    case OCN_STAGE_SW_UPDATE_SSH:
        return ocn_sw_update_ssh(g, tau, R4(OCN_LU), R4(OCN_DX), R4(OCN_DY), R4(OCN_DXH), R4(OCN_DYH),
                                 R8(OCN_HHU), R8(OCN_HHV), R8(OCN_SSHN), R8(OCN_SSHP), R8(OCN_UBRTR),
                                 R8(OCN_VBRTR), s);
    case OCN_STAGE_HH_UPDATE:
        return ocn_hh_update(g, R4(OCN_LU), R4(OCN_LLU), R4(OCN_LLV), R4(OCN_LUH), R4(OCN_DX), R4(OCN_DY),
                             R4(OCN_DXT), R4(OCN_DYT), R4(OCN_DXH), R4(OCN_DYH), R4(OCN_DXB), R4(OCN_DYB),
                             R8(OCN_HHQ_N), R8(OCN_HHU_N), R8(OCN_HHV_N), R8(OCN_HHH_N), R8(OCN_SSH),
                             R8(OCN_HHQ_REST), s);
    case OCN_STAGE_UV_TRANS_VORT:
        return ocn_uv_trans_vort(g, R4(OCN_LUU), R4(OCN_DXT), R4(OCN_DYT), R4(OCN_DXB), R4(OCN_DYB),
                                 R8(OCN_UBRTR), R8(OCN_VBRTR), R8(OCN_VORT), s);
    case OCN_STAGE_UV_TRANS:
        return ocn_uv_trans(g, R4(OCN_LCU), R4(OCN_LCV), R4(OCN_LUU), R4(OCN_DXH), R4(OCN_DYH), R8(OCN_UBRTR),
                            R8(OCN_VBRTR), R8(OCN_VORT), R8(OCN_HHQ), R8(OCN_HHU), R8(OCN_HHV), R8(OCN_HHH),
                            R8(OCN_RHSX_ADV), R8(OCN_RHSY_ADV), s);
    case OCN_STAGE_STRESS_COMPONENTS:
        return ocn_stress_components(g, R4(OCN_LU), R4(OCN_LUU), R4(OCN_DX), R4(OCN_DY), R4(OCN_DXT),
                                     R4(OCN_DYT), R4(OCN_DXH), R4(OCN_DYH), R4(OCN_DXB), R4(OCN_DYB),
                                     R8(OCN_UBRTRP), R8(OCN_VBRTRP), R8(OCN_STR_T), R8(OCN_STR_S), s);
    case OCN_STAGE_UV_DIFF2:
        return ocn_uv_diff2(g, R4(OCN_LCU), R4(OCN_LCV), R4(OCN_DX), R4(OCN_DY), R4(OCN_DXT), R4(OCN_DYT),
                            R4(OCN_DXH), R4(OCN_DYH), R4(OCN_DXB), R4(OCN_DYB), R8(OCN_MU), R8(OCN_STR_T),
                            R8(OCN_STR_S), R8(OCN_HHQ), R8(OCN_HHU), R8(OCN_HHV), R8(OCN_HHH), R8(OCN_RHSX_DIF),
                            R8(OCN_RHSY_DIF), s);
    case OCN_STAGE_SW_UPDATE_UV:
        return ocn_sw_update_uv(g, tau, R4(OCN_LCU), R4(OCN_LCV), R4(OCN_DXT), R4(OCN_DYT), R4(OCN_DXH),
                                R4(OCN_DYH), R4(OCN_DXB), R4(OCN_DYB), R8(OCN_HHU), R8(OCN_HHU_N), R8(OCN_HHU_P),
                                R8(OCN_HHV), R8(OCN_HHV_N), R8(OCN_HHV_P), R8(OCN_HHH), R8(OCN_SSH),
                                R8(OCN_UBRTR), R8(OCN_UBRTRN), R8(OCN_UBRTRP), R8(OCN_VBRTR), R8(OCN_VBRTRN),
                                R8(OCN_VBRTRP), R4(OCN_R_DISS), R4(OCN_RLH_S), R8(OCN_RHSX), R8(OCN_RHSY),
                                R8(OCN_RHSX_ADV), R8(OCN_RHSY_ADV), R8(OCN_RHSX_DIF), R8(OCN_RHSY_DIF), s);
    case OCN_STAGE_SW_NEXT_STEP:
        return ocn_sw_next_step(g, c->sw.time_smooth, R4(OCN_LU), R4(OCN_LCU), R4(OCN_LCV), R8(OCN_SSH),
                                R8(OCN_SSHN), R8(OCN_SSHP), R8(OCN_UBRTR), R8(OCN_UBRTRN), R8(OCN_UBRTRP),
                                R8(OCN_VBRTR), R8(OCN_VBRTRN), R8(OCN_VBRTRP), s);
    case OCN_STAGE_HH_SHIFT:
        return ocn_hh_shift(g, c->sw.time_smooth, R4(OCN_LU), R4(OCN_LLU), R4(OCN_LLV), R4(OCN_LUH),
                            R8(OCN_HHQ), R8(OCN_HHQ_P), R8(OCN_HHQ_N), R8(OCN_HHU), R8(OCN_HHU_P), R8(OCN_HHU_N),
                            R8(OCN_HHV), R8(OCN_HHV_P), R8(OCN_HHV_N), R8(OCN_HHH), R8(OCN_HHH_P), R8(OCN_HHH_N), s);
    case OCN_STAGE_HH_INIT:
        return ocn_hh_init(g, c->sw.full_free_surface, R4(OCN_LU), R4(OCN_LLU), R4(OCN_LLV), R4(OCN_LUH),
                           R4(OCN_DX), R4(OCN_DY), R4(OCN_DXT), R4(OCN_DYT), R4(OCN_DXH), R4(OCN_DYH), R4(OCN_DXB),
                           R4(OCN_DYB), R8(OCN_HHQ), R8(OCN_HHQ_P), R8(OCN_HHQ_N), R8(OCN_HHU), R8(OCN_HHU_P),
                           R8(OCN_HHU_N), R8(OCN_HHV), R8(OCN_HHV_P), R8(OCN_HHV_N), R8(OCN_HHH), R8(OCN_HHH_P),
                           R8(OCN_HHH_N), R8(OCN_SSH), R8(OCN_SSHP), R8(OCN_HHQ_REST), s);
    case OCN_STAGE_CHECK_SSH_ERR:
        return ocn_check_ssh_err(g, R4(OCN_LU), R8(OCN_SSH), c->d_nbad, s);
    default:
        return set_error(OCN_ERR_ARG, "unknown stage id");
    }
#undef R4
#undef R8
}

static const std::vector<int> *stage_sync(int stage)
{
    switch (stage) {
    case OCN_STAGE_SW_UPDATE_SSH: return &kSyncSsh;
    case OCN_STAGE_HH_UPDATE: return &kSyncHhUpdate;
    case OCN_STAGE_UV_TRANS_VORT: return &kSyncVort;
    case OCN_STAGE_UV_TRANS: return &kSyncUvTrans;
    case OCN_STAGE_STRESS_COMPONENTS: return &kSyncStress;
    case OCN_STAGE_SW_UPDATE_UV: return &kSyncUv;
    case OCN_STAGE_HH_INIT: return &kSyncHhInit;
    default: return nullptr;   // uv_diff2, sw_next_step, hh_shift, check: empty sync
    }
}

static void swap_roles(ocn_ctx *c);

// every plan a step can use, built before any graph capture (no hipMalloc while capturing)
static int prebuild_plans(ocn_ctx *c)
{
    // fused-step sync groups (shallow_water.f90 syncs regrouped, see one_step_fused)
    const ocn_sw_params &sw = c->sw;
    c->sync_a = {OCN_SSHN};
    if (sw.full_free_surface > 0) c->sync_a.insert(c->sync_a.end(), {OCN_HHU_N, OCN_HHV_N, OCN_HHH_N});
    if (sw.trans_terms > 0) c->sync_a.push_back(OCN_VORT);
    if (sw.ksw_lat > 0) c->sync_a.insert(c->sync_a.end(), {OCN_STR_T, OCN_STR_S});
    c->sync_a_reuse.clear();
    for (int id : c->sync_a)
        if (id != OCN_HHU_N && id != OCN_HHV_N && id != OCN_HHH_N) c->sync_a_reuse.push_back(id);
    c->sync_b = {};
    if (sw.trans_terms > 0) c->sync_b = {OCN_HHU_P, OCN_HHV_P, OCN_HHH_P};
    c->sync_b.insert(c->sync_b.end(), {OCN_VBRTRN, OCN_UBRTRN});
    HaloPlan *p;
    RC(get_plan(c, c->sync_a, p));
    RC(get_plan(c, c->sync_a_reuse, p));
    RC(get_plan(c, c->sync_b, p));
    if (sw.use_tracers > 0) {
        RC(get_plan(c, {OCN_FLUX_X, OCN_FLUX_Y}, p));
        for (int k = 1; k <= sw.tracer_num; ++k) {
            RC(get_plan(c, {OCN_FF1N(k)}, p));
            RC(get_plan(c, {OCN_FF1(k)}, p));
        }
    }
    for (const std::vector<int> *l : {&kSyncSsh, &kSyncHhUpdate, &kSyncVort, &kSyncUvTrans, &kSyncStress, &kSyncUv,
                                      &kSyncHhInit, &kHaloCheck})
        RC(get_plan(c, *l, p));
    // role-flip steps: after hh_init + the next step's A, one exchange of both launches' fields
    c->sync_ca = kSyncHhInit;
    c->sync_ca.insert(c->sync_ca.end(), c->sync_a.begin(), c->sync_a.end());
    c->sync_ca_reuse = kSyncHhInit;
    c->sync_ca_reuse.insert(c->sync_ca_reuse.end(), c->sync_a_reuse.begin(), c->sync_a_reuse.end());
    RC(get_plan(c, c->sync_ca, p));
    RC(get_plan(c, c->sync_ca_reuse, p));
    // the same plans with the pairs' buffers swapped (role 1)
    if (c->role == 0) {
        swap_roles(c);
        const int rc = prebuild_plans(c);
        swap_roles(c);
        RC(rc);
    }
    return OCN_OK;
}

// Timer events (OCN_OPT_STAGE_TIMING) only measure: no system-scope fence when they are recorded --
// the default record writes back and invalidates the caches, which showed as a ~10 us gap before
// every timed launch (rocprofv3 kernel trace) and slowed the launch after it.  A pool is made when
// timing is switched on, so no event is created inside a timed region.
static int make_timer_event(hipEvent_t &e)
{
    HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableSystemFence));
    return OCN_OK;
}
static int get_event(ocn_ctx *c, hipEvent_t &e)
{
    if (!c->event_pool.empty()) { e = c->event_pool.back(); c->event_pool.pop_back(); return OCN_OK; }
    return make_timer_event(e);
}

static int timer_begin(ocn_ctx *c, int id, ocn_ctx::Rec &rec)
{
    rec = ocn_ctx::Rec{id, nullptr, nullptr};
    if (!c->stage_timing) return OCN_OK;
    RC(get_event(c, rec.a)); RC(get_event(c, rec.b));
    HIPCHK(hipEventRecord(rec.a, c->stream));
    return OCN_OK;
}
static int timer_end(ocn_ctx *c, ocn_ctx::Rec &rec)
{
    if (!c->stage_timing) return OCN_OK;
    HIPCHK(hipEventRecord(rec.b, c->stream));
    c->recs.push_back(rec);
    return OCN_OK;
}

static int envoke(ocn_ctx *c, int stage, double tau)
{
    ocn_ctx::Rec rec;
    RC(timer_begin(c, stage, rec));
    RC(each_block(c, c->stream, [&](const LBlock &b) { return stage_kernel(c, b, stage, tau); }));
    RC(timer_end(c, rec));
    const std::vector<int> *sl = stage_sync(stage);
    if (sl) RC(run_sync(c, *sl));
    return OCN_OK;
}

// expl_shallow_water (shallow_water.f90:22-94) with the flag gates
static int one_step(ocn_ctx *c, double tau, bool check)
{
    const ocn_sw_params &sw = c->sw;
    RC(envoke(c, OCN_STAGE_SW_UPDATE_SSH, tau));
    if (sw.full_free_surface > 0) RC(envoke(c, OCN_STAGE_HH_UPDATE, tau));
    if (sw.trans_terms > 0) {
        RC(envoke(c, OCN_STAGE_UV_TRANS_VORT, tau));
        RC(envoke(c, OCN_STAGE_UV_TRANS, tau));
    }
    if (sw.ksw_lat > 0) {
        RC(envoke(c, OCN_STAGE_STRESS_COMPONENTS, tau));
        RC(envoke(c, OCN_STAGE_UV_DIFF2, tau));
    }
    RC(envoke(c, OCN_STAGE_SW_UPDATE_UV, tau));
    RC(envoke(c, OCN_STAGE_SW_NEXT_STEP, tau));
    if (sw.full_free_surface > 0) {
        RC(envoke(c, OCN_STAGE_HH_SHIFT, tau));
        RC(envoke(c, OCN_STAGE_HH_INIT, tau));
    }
    if (check) RC(envoke(c, OCN_STAGE_CHECK_SSH_ERR, tau));
    return OCN_OK;
}

static bool has_exchange(const ocn_ctx *c);

// (Re)builds the compact static fields when the real(4) fields may have changed, and decides
// whether the fused step reads them (sw_stencils.h "compact static fields").  Synchronises
// only when a rebuild was needed (once after init / an upload of a real(4) field).
static int prepare_static(ocn_ctx *c)
{
    if (!c->compact_req || c->r4_escaped) { c->compact = false; return OCN_OK; }
    if (!c->static_dirty) return OCN_OK;
    HIPCHK(hipMemsetAsync(c->d_flags, 0, 3 * sizeof(int32_t), c->stream));
    RC(each_block(c, c->stream, [&](const LBlock &b) { return launch_prepare(&b.g, b.ptr.data(), b.bits, b.rows, c->d_flags, c->stream, b.own); }));
    if (c->ext_ok)   // one_step_x2's row tables: the ext rows' divisor range into the second word
        for (const LBlock &b : c->blocks) RC(launch_rows_ext(&b.g, b.rows, b.rows_x, b.ext, c->d_flags + 1, c->stream));
    const bool x4_tabs = c->ext_ok && has_exchange(c);
    int32_t *d_mask = nullptr;
    if (x4_tabs) {   // one_step_x4's tables (the neighbours' mask bytes from the basin mask): the third word
        const size_t nxy = (size_t)c->basin.nx * c->basin.ny;
        HIPCHK(hipMallocAsync((void **)&d_mask, nxy * sizeof(int32_t), c->stream));
        HIPCHK(hipMemcpyAsync(d_mask, c->mask.data(), nxy * sizeof(int32_t), hipMemcpyHostToDevice, c->stream));
        for (const LBlock &b : c->blocks)
            RC(launch_x4_tables(&b.g, b.bits, b.rows, b.ext, b.bits_x4, b.rows_x4, d_mask, c->basin.nx, c->basin.ny, b.own,
                                c->d_flags + 2, c->stream));
        HIPCHK(hipFreeAsync(d_mask, c->stream));
    }
    int32_t flags[3] = {0, 0, 0};
    HIPCHK(hipMemcpyAsync(flags, c->d_flags, sizeof(flags), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    c->ring_sea = (flags[0] & kCompactRingSea) != 0;
    c->edge_ring_sea = (flags[0] & kCompactEdgeRingSea) != 0;
    c->udiv_ok = (flags[0] & kCompactDivisorRange) == 0;
    c->rows_x_ok = c->ext_ok && flags[1] == 0;
    c->x4_tab_ok = x4_tabs && flags[2] == 0;
    c->compact = (flags[0] & ~(kCompactRingSea | kCompactDivisorRange | kCompactEdgeRingSea)) == 0;
    c->static_dirty = false;
    return OCN_OK;
}

// Fused step (sw_kernels.hip "fused step groups"): 4 launches and 3 halo syncs per step,
// bitwise the same state as one_step.  last = false skips stores no later kernel reads
// (sw_stencils.h FusedB / HhInit `full`); the last step of every ocn_ctx_step call leaves the
// full state.
//
// With halo exchanges to do (several blocks or ranks) and OCN_OPT_OVERLAP, each exchange runs
// on the comm stream while the compute stream works on points that neither feed it nor read
// its halos (sw_stencils.h frame_rects):
//   A.frame | fork: sync A || A.inner, B.inner | join | B.frame | fork: sync B || C1.inner |
//   join | C1.frame | C2.frame | fork: sync C2 || C2.inner | join
// Every halo write of an exchange lands on points the concurrent inner launches neither read
// nor write, and every value it sends was produced by the frame launch before the fork.
// Whether any exchange has strips: some local block has a neighbour block (local or on another
// rank) in one of the 8 directions -- exactly when plan_entries enumerates an entry.  Decided from
// the decomposition alone (no plan is built, so nothing can fail inside a graph capture).
static bool has_exchange(const ocn_ctx *c)
{
    for (const LBlock &b : c->blocks)
        for (int d = 0; d < 8; ++d)
            if (b.nbr_rank[d] >= 0) return true;
    return false;
}

// An exchange forked onto the comm stream stays pending until join_sync (a no-op without one);
// a role-flip step may leave its last exchange pending for the next step's inner launch.
static int fork_sync(ocn_ctx *c, const std::vector<int> &fields)
{
    HIPCHK(hipEventRecord(c->ev_fork, c->stream));
    HIPCHK(hipStreamWaitEvent(c->comm_stream, c->ev_fork, 0));
    RC(run_sync(c, fields, c->comm_stream));
    HIPCHK(hipEventRecord(c->ev_join, c->comm_stream));
    c->sync_pending = true;
    return OCN_OK;
}
static int join_sync(ocn_ctx *c)
{
    if (!c->sync_pending) return OCN_OK;
    HIPCHK(hipStreamWaitEvent(c->stream, c->ev_join, 0));
    c->sync_pending = false;
    return OCN_OK;
}

// block b's launch arguments: geometry, field table, compact tables (or nullptr)
#define FT(b) &(b).g, (b).ptr.data(), (int)(b).ptr.size(), cp(b, t)
// The buffer pairs whose roles a role-flip step swaps (a8's copies ssh := sshn etc.)
static const int kFlipPairs[3][2] = {{OCN_SSH, OCN_SSHN}, {OCN_UBRTR, OCN_UBRTRN}, {OCN_VBRTR, OCN_VBRTRN}};
static void swap_roles(ocn_ctx *c)
{
    for (LBlock &b : c->blocks)
        for (const auto &pr : kFlipPairs) std::swap(b.ptr[field_slot(pr[0])], b.ptr[field_slot(pr[1])]);
    c->role ^= 1;
}
// recompute steps: sshp and its second buffer trade places (role bit 2)
static void swap_sshp(ocn_ctx *c)
{
    for (LBlock &b : c->blocks) std::swap(b.ptr[field_slot(OCN_SSHP)], b.sshp_alt);
    c->role ^= 2;
}
// one-pass steps: sshp, ubrtrp, vbrtrp and their second buffers trade places (role bit 4)
static void swap_alt3(ocn_ctx *c)
{
    for (LBlock &b : c->blocks) {
        std::swap(b.ptr[field_slot(OCN_SSHP)], b.sshp_alt);
        std::swap(b.ptr[field_slot(OCN_UBRTRP)], b.up_alt);
        std::swap(b.ptr[field_slot(OCN_VBRTRP)], b.vp_alt);
    }
    c->role ^= 4;
}
// tracer steps (run_tracer_step): every tracer's ff1 and ff1n trade places (role bit 8, the role-flip
// form of tracer_next_step's ff := ffn), and ff1p with its second buffer (role bit 16)
static void swap_tracer_roles(ocn_ctx *c)
{
    for (LBlock &b : c->blocks)
        for (int k = 1; k <= c->sw.tracer_num; ++k)
            std::swap(b.ptr[field_slot(OCN_FF1(k))], b.ptr[field_slot(OCN_FF1N(k))]);
    c->role ^= 8;
}
static void swap_tracer_alt(ocn_ctx *c)
{
    for (LBlock &b : c->blocks)
        for (int k = 1; k <= c->sw.tracer_num; ++k) std::swap(b.ptr[field_slot(OCN_FF1P(k))], b.ffp_alt[(size_t)k - 1]);
    c->role ^= 16;
}
static size_t field_bytes(const LBlock &b) { return (size_t)b.g.pitch * (b.g.bnd_y2 - b.g.bnd_y1 + 1) * 8; }
static bool is_alt_field(int id) { return id == OCN_SSHP || id == OCN_UBRTRP || id == OCN_VBRTRP; }
static bool is_flip_field(int id)
{
    for (const auto &pr : kFlipPairs)
        if (id == pr[0] || id == pr[1]) return true;
    return id >= OCN_TRACER_BASE && (id - OCN_TRACER_BASE) % 3 != 1;   // a tracer's ff1 / ff1n (tracer steps)
}

// Whether role-flip steps are exact for the current state (synchronises):
//  - the pairs agree outside their write sets (sw_stencils.h Coherence);
//  - with halo exchanges, the halo ring of ssh / ubrtr / vbrtr, hhu / hhv and hhq_rest holds the
//    neighbours' values (what an exchange would deliver; compared, not written).  After a swap
//    the new ssh holds the exchanged sshn on the whole ring, where a8 copies only under lu (so the
//    land points of the ring must already agree), and the fused hh_init + A launch takes hh_init's
//    own ring values where the standard step takes the exchanged ones.
// Every rank must run the same kind of step (the exchanges differ), so with RCCL the verdicts
// are max-reduced over the ranks; eligible = false: this rank cannot run role-flip steps at all.
// The vote also carries the other per-rank conditions that decide which launches and exchanges a
// call runs (one 0/1 word each, max-reduced = OR over the ranks): every rank then takes the same
// one-pass / hybrid decisions, so the exchange sequences of all ranks match.
// kVoteX4: this rank cannot run one_step_x4's pairs (its tables, or the known-constant verdict its host
// has read for the x2 range) -- every rank then runs the same steps and exchanges
// kVoteOvSeq / kVoteOvOv: the measured sequential / overlapped step times in us (ov_begin; INT32_MAX
// from a rank that has not measured both: no decision)
enum { kVoteIncoherent = 0, kVoteIneligible, kVoteUdiv, kVoteHhStale, kVoteX2, kVoteX4, kVoteOvSeq, kVoteOvOv,
       kVoteUsed };
static_assert(kVoteUsed <= kVoteWords, "vote words");
struct VoteIn { bool eligible, udiv_ok, hh_consistent, x2_ok, x4_ok; };
struct VoteOut { bool udiv_ok, hh_consistent, x2_ok, x4_ok; };

// one_step_x2's condition on the state's halo points that no exchange fills (the rings 1 and 2 of a
// side, or corner, without a neighbour block): +0.0 in the six state arrays.  The reference never
// writes them (no a8 / a9 work on such a ring: ocn_ctx::edge_ring_sea) and init leaves +0.0 there;
// a neighbour's D formed next to such a point reads the neighbour's own copy of it, which then
// holds +0.0 as well (every rank checks and the verdicts are reduced).  ORs 1 into *flag otherwise.
// The same at the points of the outer halo ring (nx_end + 1, ny_end + 1) no neighbour fills for the
// nine depth arrays of hh_shift's u / v / h triples (a9's own arrays there: hh_init and hh_update
// stop at nx_end / ny_end): +0.0 makes a9 there an exact no-op (0 + ts (0 - 0 + 0) / 2 = +0), which
// the x2 steps then skip; the hybrid last step runs it as the reference does.
struct HaloZero {
    const double *a[6], *d[9];
    int w, h, nxs, nxe, nys, nye, bx1, by1;
    long pitch;
    unsigned own;
};
__global__ void k_halo_zero(HaloZero q, int32_t *flag)
{
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (long)q.w * q.h) return;
    const int m = q.bx1 + (int)(i % q.w), n = q.by1 + (int)(i / q.w);
    const unsigned cx = m < q.nxs ? 0u : m > q.nxe ? 2u : 1u, cy = n < q.nys ? 0u : n > q.nye ? 2u : 1u;
    if ((cx == 1u && cy == 1u) || ((q.own >> (cx * 3u + cy)) & 1u)) return;   // interior, or a neighbour's
    const long at = (i % q.w) + (i / q.w) * q.pitch;
    auto nz = [&](const double *p) {
        unsigned long long x;
        const double v = p[at];
        __builtin_memcpy(&x, &v, 8);
        return x != 0ull;
    };
    bool bad = false;
    for (int k = 0; k < 6; ++k) bad |= nz(q.a[k]);
    const bool outer = (m == q.nxe + 1 && n >= q.nys - 1 && n <= q.nye + 1) ||
                       (n == q.nye + 1 && m >= q.nxs - 1 && m <= q.nxe + 1);
    if (outer)
        for (int k = 0; k < 9; ++k) bad |= nz(q.d[k]);
    if (bad) atomicOr(flag, 1);
}
static int launch_halo_zero(ocn_ctx *c, int32_t *flag)
{
    static const int ids[6] = {OCN_SSH, OCN_SSHP, OCN_UBRTR, OCN_UBRTRP, OCN_VBRTR, OCN_VBRTRP};
    static const int dids[9] = {OCN_HHU, OCN_HHU_P, OCN_HHU_N, OCN_HHV, OCN_HHV_P, OCN_HHV_N, OCN_HHH, OCN_HHH_P, OCN_HHH_N};
    for (const LBlock &b : c->blocks) {
        HaloZero q{};
        for (int k = 0; k < 6; ++k) q.a[k] = b.f<double>(ids[k]);
        for (int k = 0; k < 9; ++k) q.d[k] = b.f<double>(dids[k]);
        q.w = b.g.bnd_x2 - b.g.bnd_x1 + 1; q.h = b.g.bnd_y2 - b.g.bnd_y1 + 1;
        q.nxs = b.g.nx_start; q.nxe = b.g.nx_end; q.nys = b.g.ny_start; q.nye = b.g.ny_end;
        q.bx1 = b.g.bnd_x1; q.by1 = b.g.bnd_y1; q.pitch = (long)b.g.pitch; q.own = b.own;
        const long pts = (long)q.w * q.h;
        hipLaunchKernelGGL(k_halo_zero, dim3((unsigned)((pts + 255) / 256)), dim3(256), 0, c->stream, q, flag);
        RC(check_launch());
    }
    return OCN_OK;
}

static int check_coherence(ocn_ctx *c, const VoteIn &in, VoteOut &out)
{
    int32_t host[kVoteWords] = {0};
    host[kVoteIneligible] = !in.eligible;
    host[kVoteUdiv] = !in.udiv_ok;
    host[kVoteHhStale] = !in.hh_consistent;
    host[kVoteX2] = !in.x2_ok;
    host[kVoteX4] = !in.x4_ok;
    host[kVoteOvSeq] = host[kVoteOvOv] = INT32_MAX;
    if (c->ov_state == 2) {   // both probe steps recorded (ov_begin): their times, in us
        float ms[2] = {0.f, 0.f};
        HIPCHK(hipEventSynchronize(c->ov_ev[3]));
        HIPCHK(hipEventElapsedTime(&ms[0], c->ov_ev[0], c->ov_ev[1]));
        HIPCHK(hipEventElapsedTime(&ms[1], c->ov_ev[2], c->ov_ev[3]));
        for (int i = 0; i < 2; ++i) {
            c->ov_ms[i] = ms[i];
            host[kVoteOvSeq + i] = (int32_t)std::min(1.0e9, std::max(1.0, std::round(1000.0 * ms[i])));
        }
    }
    HIPCHK(hipMemcpyAsync(c->d_flags, host, sizeof(host), hipMemcpyHostToDevice, c->stream));
    if (in.eligible)
        RC(each_block(c, c->stream, [&](const LBlock &b) { return launch_coherence(&b.g, b.ptr.data(), b.bits, c->d_flags, c->stream); }));
    if (in.eligible && c->sw.use_tracers > 0 && c->tr_step)   // the tracer steps' ff1 / ff1n pairs too
        for (int t = 1; t <= c->sw.tracer_num; ++t)
            RC(each_block(c, c->stream, [&](const LBlock &b) {
                return launch_tracer_coherence(&b.g, b.ptr.data(), b.bits, t, c->d_flags, c->stream);
            }));
    const bool exch = has_exchange(c);
    if (exch) RC(run_sync(c, kHaloCheck, c->stream, c->d_flags));
    if (exch && c->x2) {   // one_step_x2: the rest of the state's first halo ring, and the unexchanged halos
        RC(run_sync(c, {OCN_SSHP, OCN_UBRTRP, OCN_VBRTRP}, c->stream, c->d_flags + kVoteX2));
        // tracer steps form tran_diff_fluxes' fluxes at the halo points neighbours own (the reference
        // exchanges them) from mu there: its first halo ring must hold the neighbours' values too
        if (c->sw.use_tracers > 0 && c->tr_step) RC(run_sync(c, {OCN_MU}, c->stream, c->d_flags + kVoteX2));
        RC(launch_halo_zero(c, c->d_flags + kVoteX2));
    }
    RC(allreduce_max(c, c->d_flags, c->stream, kVoteUsed));
    int32_t w[kVoteWords] = {0};
    HIPCHK(hipMemcpyAsync(w, c->d_flags, sizeof(int32_t) * kVoteUsed, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    c->coherent = w[kVoteIncoherent] == 0 && w[kVoteIneligible] == 0;
    c->coherent_known = !c->r8_escaped && !has_comm(c);
    out.udiv_ok = w[kVoteUdiv] == 0;
    out.hh_consistent = w[kVoteHhStale] == 0;
    out.x2_ok = w[kVoteX2] == 0 && exch && c->x2;
    c->x2_dev_ok = out.x2_ok;
    out.x4_ok = out.x2_ok && w[kVoteX4] == 0;
    if (w[kVoteOvSeq] != INT32_MAX && w[kVoteOvOv] != INT32_MAX) {   // every rank measured: the faster form
        c->ov_ms[0] = 1.0e-3 * w[kVoteOvSeq];
        c->ov_ms[1] = 1.0e-3 * w[kVoteOvOv];
        c->ov_level = w[kVoteOvOv] < w[kVoteOvSeq] ? 2 : 1;
        c->ov_state = 3;
    } else if (c->ov_state == 2) {   // another rank has not: measure again, together
        c->ov_state = 0;
    }
    c->x4_dev_ok = out.x4_ok;
    return OCN_OK;
}

// Role-flip steps: the step's a8 copies (ssh := sshn, ubrtr := ubrtrn, vbrtr := vbrtrn on the
// interior and the ring, under the masks) become a swap of the two buffers of each pair, and
// a8's time filters and check_ssh_err move into fused B (sw_kernels.hip MarchFusedB<true>), so
// the step is A | B+a8 | a8+a9 on the ring | swap | hh_init -- one full pass (C1) fewer.  Exact
// when the pairs are coherent (sw_stencils.h Coherence): inside the write sets the reference
// leaves both buffers of a pair equal to the new value, and the buffer that becomes "sshn" /
// "ubrtrn" / "vbrtrn" after the swap holds the old value there instead -- which no kernel
// reads before a1 / a7 of the next step rewrite it.  The last step of every call is a standard
// step; it leaves both buffers of each pair equal everywhere, so the swap is undone at the end
// of the call by swapping the pointers back, with no copy.  Used with the compact tables + march,
// tracer runs included (CA then also stores hh_init's hhq_p, which expl_tracer reads after every
// step).  With halo exchanges the swapped buffers are exchanged through plans built for the
// swapped roles (get_plan), the ring launch (a8 + a9 on the halo ring) runs after sync B, and
// each hh_init's sync and the next step's sync A are one exchange (sync_ca); the exchanges do
// not overlap computation in these steps.
static bool flip_eligible(ocn_ctx *c)
{
    return c->flip && c->fused && c->compact && c->march;
}

// tracer steps (run_tracer_step, below): the pending one of the current state, and the tracer fields
// the exchanges of a one-pass call carry with the state
static int run_tracer_step(ocn_ctx *c, double tau);
static int run_tracer_step(ocn_ctx *c, double tau, hipStream_t st);
static int tracer_step_block(ocn_ctx *c, const LBlock &b, int k, double tau, hipStream_t st);
static std::vector<int> with_tracers(const ocn_ctx *c, const std::vector<int> &fields);

// block b's one-pass variant for the current call (ctx kc_mode, the device verdict, its constants)
static OnepassKC kc_of(const ocn_ctx *c, const LBlock &b) { return OnepassKC{c->kc_mode, c->d_fbz, b.kc}; }

// The part of block b's interior the one-pass step covers when halos are exchanged: the interior
// less w points on each side that has a neighbour block (E, W, N, S; diagonal neighbours only
// feed the state at the halo corners, which the stencils read as the reference does).
static Range onepass_inner(const LBlock &b, int w)
{
    Range r{b.g.nx_start, b.g.nx_end, b.g.ny_start, b.g.ny_end};
    if (b.nbr_rank[1] >= 0) r.m0 += w;   // kDirDm / kDirDn: d = 2 W, 1 E, 4 S, 3 N
    if (b.nbr_rank[0] >= 0) r.m1 -= w;
    if (b.nbr_rank[3] >= 0) r.n0 += w;
    if (b.nbr_rank[2] >= 0) r.n1 -= w;
    return r;
}

// A one-pass step with halo exchanges (several blocks or ranks), or with a8 / a9 work on the
// halo ring.  The one-pass march needs D (hh_init's depths, vort, stresses) at the points next to
// the ones it updates, formed from the state one point further out; at a halo the reference holds
// D as exchanged from the neighbour, which would need the neighbour's state TWO points out -- the
// reference never exchanges that.  So the points one away from an exchanged side take the
// role-flip path (D stored by CA, exchanged, read back by B) and the rest the one-pass march:
//   CA frame (hh_init of the previous step + this step's A, on the bands two points deep along
//   the exchanged sides and their halos) | sync CA | B on the one-point bands | sync B, as a side
//   chain on the comm stream beside the one-pass march of the inner part on the compute stream |
//   join | swap | ring launch (a8 + a9 on the halo ring).  With OCN_OPT_OVERLAP 0 (or while
//   capturing a graph) the same launches run in that order on one stream, the inner march
//   between sync CA and B.  (The side chain is the overlap of every level >= 1: with local copies
//   too it hides the latency-bound frame launches -- one GPU, 4x2 blocks of a 4096^2 box: 0.947
//   -> 0.856 ms per step, 2x2 of 2048^2: 0.334 -> 0.294; the earlier split of the inner march
//   into two halves beside the two exchanges took 1.065 / 0.398.)
// All of a8's filtered sshp / ubrtrp / vbrtrp go to the second buffers (the inner part reads the
// current ones at neighbours); the ring launch reads the current ones and writes the new ones on
// the ring after the swap, as the recompute steps do with sshp.
static int hybrid_tail(ocn_ctx *c, double tau, const StepKind &k, bool last);
// last: the call's last step (StepKind::one_last with exchanges or ring work): the CA frames' A
// stores hh_update's levels and sync CA exchanges them (the halo values the reference's a2 sync
// leaves and its a9 on the halo ring reads), the inner march also stores vort, the stresses and
// the RHS terms (MarchStep<.., true>), B on the bands keeps the RHS terms (fused B `full`), and the
// tail adds a8's copies and hh_init with every level + its sync
static int one_step_hybrid(ocn_ctx *c, double tau, const StepKind &k, bool last = false)
{
    const ocn_sw_params &sw = c->sw;
    ocn_ctx::Rec rec;
    Compact t;
    auto cp = [c](const LBlock &b, Compact &tt) -> const Compact * {
        tt = Compact{b.bits, b.rows, c->march};
        return &tt;
    };
    int32_t *nbad = k.check ? c->d_nbad : nullptr;
    hipStream_t s = c->stream;
    const bool xch = has_exchange(c);
    // the previous step's hh_init and this step's A on the frames (bnd range outside inner_ca)
    auto ca_frames = [&](hipStream_t st) -> int {
        RC(each_block(c, st, [&](const LBlock &b) -> int {
            Range in = onepass_inner(b, 2);
            if (b.nbr_rank[1] < 0) in.m0 = b.g.bnd_x1;   // no frame on the sides without a neighbour
            if (b.nbr_rank[0] < 0) in.m1 = b.g.bnd_x2;
            if (b.nbr_rank[3] < 0) in.n0 = b.g.bnd_y1;
            if (b.nbr_rank[2] < 0) in.n1 = b.g.bnd_y2;
            RC(launch_fused_ca(&b.g, b.ptr.data(), (int)b.ptr.size(), cp(b, t), OCN_PART_FRAME, sw, tau, !last, false,
                               st, &in));
            return OCN_OK;
        }));
        return OCN_OK;
    };
    // B on the one-point bands along the exchanged sides
    auto b_bands = [&](hipStream_t st) -> int {
        RC(each_block(c, st, [&](const LBlock &b) -> int {
            const Range in = onepass_inner(b, 1);
            const Range all{b.g.nx_start, b.g.nx_end, b.g.ny_start, b.g.ny_end};
            if (in.m0 == all.m0 && in.m1 == all.m1 && in.n0 == all.n0 && in.n1 == all.n1) return OCN_OK;
            RC(launch_fused_b(FT(b), OCN_PART_ALL, sw, tau, last, true, st, nbad, true, false, (double *)b.sshp_alt,
                              (double *)b.up_alt, (double *)b.vp_alt, &in));
            return OCN_OK;
        }));
        return OCN_OK;
    };
    if (xch && overlap_level(c) >= 1 && !c->capturing) {
        // side chain (OCN_OPT_OVERLAP >= 1): CA frames | sync CA | B bands | sync B on the comm stream,
        // beside the whole inner march on the compute stream -- the two read nothing the other
        // writes (disjoint points; the inner march forms its D from the state, the bands read
        // CA's stored D and the exchanged halos), so the frame launches and both exchanges hide
        // behind it
        // The inner march is enqueued first (the fork event recorded before it): with several
        // blocks the host's enqueueing of the side chain's ~3 launches per block took longer than
        // the GPU's previous work, and the compute stream sat idle until it was done
        HIPCHK(hipEventRecord(c->ev_fork, s));
        RC(timer_begin(c, OCN_TIMER_ONEPASS, rec));
        RC(each_block(c, s, [&](const LBlock &b) -> int {
            const Range in = onepass_inner(b, 1);
            RC(launch_onepass(&b.g, b.ptr.data(), (int)b.ptr.size(), cp(b, t), sw, tau, nbad, (double *)b.sshp_alt,
                              (double *)b.up_alt, (double *)b.vp_alt, s, &in, last, kc_of(c, b)));
            return OCN_OK;
        }));
        RC(timer_end(c, rec));
        HIPCHK(hipStreamWaitEvent(c->comm_stream, c->ev_fork, 0));
        RC(ca_frames(c->comm_stream));
        RC(run_sync(c, last ? c->sync_ca : c->sync_ca_reuse, c->comm_stream));
        RC(b_bands(c->comm_stream));
        RC(run_sync(c, c->sync_b, c->comm_stream));
        HIPCHK(hipEventRecord(c->ev_join, c->comm_stream));
        c->sync_pending = true;
        RC(join_sync(c));
        return hybrid_tail(c, tau, k, last);
    }
    // without overlap (or while capturing a graph): CA frames | sync CA | inner | B bands | sync B
    RC(timer_begin(c, OCN_TIMER_FUSED_CA, rec));
    RC(ca_frames(s));
    RC(timer_end(c, rec));
    if (xch) RC(run_sync(c, last ? c->sync_ca : c->sync_ca_reuse));
    RC(timer_begin(c, OCN_TIMER_ONEPASS, rec));
    RC(each_block(c, s, [&](const LBlock &b) -> int {
        const Range in = onepass_inner(b, 1);
        RC(launch_onepass(&b.g, b.ptr.data(), (int)b.ptr.size(), cp(b, t), sw, tau, nbad, (double *)b.sshp_alt,
                          (double *)b.up_alt, (double *)b.vp_alt, s, &in, last, kc_of(c, b)));
        return OCN_OK;
    }));
    RC(timer_end(c, rec));
    if (xch) {
        RC(timer_begin(c, OCN_TIMER_FUSED_B, rec));
        RC(b_bands(s));
        RC(timer_end(c, rec));
        RC(run_sync(c, c->sync_b));
    }
    return hybrid_tail(c, tau, k, last);
}

// the end of a hybrid one-pass step (one_step_hybrid): the role swaps, the ring launch, and the
// next step's CA + sync before a standard last step -- or, on the call's last step, a8's copies
// (both buffers of each pair end equal, as one_step_last leaves them) and hh_init with every level
// (a10; the levels a9 and hh_update leave are rewritten by it on the same ranges) and its sync
static int hybrid_tail(ocn_ctx *c, double tau, const StepKind &k, bool last)
{
    const ocn_sw_params &sw = c->sw;
    ocn_ctx::Rec rec;
    Compact t;
    auto cp = [c](const LBlock &b, Compact &tt) -> const Compact * {
        tt = Compact{b.bits, b.rows, c->march};
        return &tt;
    };
    hipStream_t s = c->stream;
    const bool xch = has_exchange(c);
    swap_alt3(c);
    std::vector<std::vector<void *>> pre;   // the ring launch's field tables (pair roles before the swap)
    for (const LBlock &b : c->blocks) pre.push_back(b.ptr);
    swap_roles(c);
    if (c->ring_sea) {   // a8 + a9 on the ring: the previous sshp / ubrtrp / vbrtrp in, the new ones out
        RC(timer_begin(c, OCN_TIMER_FUSED_C1, rec));
        for (size_t i = 0; i < c->blocks.size(); ++i) {
            const LBlock &b = c->blocks[i];
            RC(launch_fused_c1(&b.g, pre[i].data(), (int)pre[i].size(), cp(b, t), OCN_PART_FRAME, sw, nullptr, s,
                               (const double *)b.sshp_alt, (const double *)b.up_alt, (const double *)b.vp_alt));
        }
        RC(timer_end(c, rec));
    }
    if (last) {
        for (const LBlock &b : c->blocks)
            for (const auto &pr : kFlipPairs)
                HIPCHK(hipMemcpyAsync(b.ptr[field_slot(pr[1])], b.ptr[field_slot(pr[0])], field_bytes(b),
                                      hipMemcpyDeviceToDevice, s));
        RC(timer_begin(c, OCN_STAGE_HH_INIT, rec));
        RC(each_block(c, s, [&](const LBlock &b) { return launch_fused_c2(FT(b), OCN_PART_ALL, sw, true, s); }));
        RC(timer_end(c, rec));
        if (xch) RC(run_sync(c, *stage_sync(OCN_STAGE_HH_INIT)));
        return OCN_OK;
    }
    if (k.next_a) {   // the next step is the last, standard one: hh_init + its fused A, then their sync
        RC(timer_begin(c, OCN_TIMER_FUSED_CA, rec));
        RC(each_block(c, s, [&](const LBlock &b) { return launch_fused_ca(&b.g, b.ptr.data(), (int)b.ptr.size(), cp(b, t), OCN_PART_ALL, sw, tau, k.next_reuse,
                               false, s); }));
        RC(timer_end(c, rec));
        if (xch) RC(run_sync(c, k.next_reuse ? c->sync_ca_reuse : c->sync_ca));
    }
    return OCN_OK;
}

// The last step of a single-block one-pass call (no exchange, no a8 / a9 work on the halo ring):
// the one-pass march that also stores vort, the stresses and the RHS terms (sw_kernels.hip
// MarchStep<.., true>), the role swaps, a8's copies (ssh := sshn, ubrtr := ubrtrn, vbrtr := vbrtrn:
// both buffers of each pair end equal, as the reference leaves them), then hh_init with every
// level (a10; a9's results on its range are rewritten by it).  Replaces CA + fused B + C1 +
// hh_init of the standard last step.
// what follows the last step's march (one block, no exchange; the roles swapped): a8's copies
// (ssh := sshn, ubrtr := ubrtrn, vbrtr := vbrtrn, whole arrays: both buffers of each pair end equal,
// as the reference leaves them) and hh_init with every level (a10, depth.f90:14-99)
static int last_finish(ocn_ctx *c)
{
    hipStream_t s = c->stream;
    ocn_ctx::Rec rec;
    Compact t;
    auto cp = [c](const LBlock &b, Compact &tt) -> const Compact * {
        tt = Compact{b.bits, b.rows, c->march};
        return &tt;
    };
    // a8's copies sshn := ssh, ubrtrn := ubrtr, vbrtrn := vbrtr (the new state is in the first
    // buffers): in the hh_init march, which reads ssh anyway (one pass instead of three copies)
    auto copy_of = [](const LBlock &b) {
        auto p = [&](int id) { return (double *)b.ptr[field_slot(id)]; };
        return TailCopy{{p(OCN_SSH), p(OCN_UBRTR), p(OCN_VBRTR)}, {p(OCN_SSHN), p(OCN_UBRTRN), p(OCN_VBRTRN)}};
    };
    if (!c->march)
        for (const LBlock &b : c->blocks)
            for (const auto &pr : {std::make_pair(OCN_SSH, OCN_SSHN), std::make_pair(OCN_UBRTR, OCN_UBRTRN),
                                   std::make_pair(OCN_VBRTR, OCN_VBRTRN)})
                HIPCHK(hipMemcpyAsync(b.ptr[field_slot(pr.second)], b.ptr[field_slot(pr.first)], field_bytes(b),
                                      hipMemcpyDeviceToDevice, s));
    // (not while capturing a graph: the replays would not see hn_fresh)
    const bool keep_n = c->hn_fresh && !c->capturing && !c->r8_handed && !c->r4_escaped;
    RC(timer_begin(c, OCN_STAGE_HH_INIT, rec));
    RC(each_block(c, s, [&](const LBlock &b) {
        const TailCopy tc = copy_of(b);
        return launch_fused_c2(FT(b), OCN_PART_ALL, c->sw, true, s, keep_n, c->march ? &tc : nullptr);
    }));
    RC(timer_end(c, rec));
    c->hn_fresh = !c->capturing;
    return OCN_OK;
}

static int one_step_last(ocn_ctx *c, double tau, const StepKind &k)
{
    const ocn_sw_params &sw = c->sw;
    ocn_ctx::Rec rec;
    Compact t;
    auto cp = [c](const LBlock &b, Compact &tt) -> const Compact * {
        tt = Compact{b.bits, b.rows, c->march};
        return &tt;
    };
    hipStream_t s = c->stream;
    RC(timer_begin(c, OCN_TIMER_ONEPASS, rec));
    RC(each_block(c, s, [&](const LBlock &b) { return launch_onepass(&b.g, b.ptr.data(), (int)b.ptr.size(), cp(b, t), sw, tau, k.check ? c->d_nbad : nullptr,
                          (double *)b.sshp_alt, (double *)b.up_alt, (double *)b.vp_alt, s, nullptr, true,
                          kc_of(c, b)); }));
    RC(timer_end(c, rec));
    swap_alt3(c);
    swap_roles(c);
    return last_finish(c);
}

// ------------------------------------------------------------------ one-pass steps with one exchange
// With halo exchanges the reference holds D (hh_init's depths, vort, the stresses) at a halo as the
// neighbour formed it on its interior, from the neighbour's state one point further out -- two
// points into our halo.  one_step_x2 exchanges the state (ssh, sshp, ubrtr, ubrtrp, vbrtr, vbrtrp)
// two points deep once per step, so every block forms D on its halo itself (the same operands, the
// same arithmetic: sw_kernels.hip MarchStep X2, with the metric rows of the second ring from
// ext / rows_x and h_r's second ring from the h_r copy hr_x) and the one-pass march covers the whole
// interior: no CA / B frame launches and one exchange per step instead of two.  The state's first
// halo ring then holds the neighbours' values as the reference's a8 on the ring leaves it (checked
// in check_coherence); its second ring, which the reference never writes, is saved when a sequence
// of such steps starts and restored when it ends (x2_end, before the call's last step).
static const std::vector<int> kStateX2 = {OCN_SSH, OCN_SSHP, OCN_UBRTR, OCN_UBRTRP, OCN_VBRTR, OCN_VBRTRP};

static int ring2_run(ocn_ctx *c, bool save, hipStream_t s)
{
    for (const LBlock &b : c->blocks) RC(launch_segs(save ? b.save : b.restore, s));
    return OCN_OK;
}

// the end of a sequence of x2 steps: the second ring as the reference leaves it, the first ring of
// the current state exchanged (what the reference's exchanges and a8 on the ring leave there)
static int x2_end(ocn_ctx *c, hipStream_t s)
{
    RC(ring2_run(c, false, s));
    return run_sync(c, with_tracers(c, kStateX2), s);
}

// hr_x = h_r with the neighbours' second ring (the general variant of one_step_x2 reads it there) --
// four rings deep where x4 pairs may run (their h_r-read variant reads it on the block widened by
// kXRing rings, as the neighbours' own h_r); x4_tables: x4 pairs may run (their tables and the option)
static bool x4_tables(const ocn_ctx *c) { return c->x4 && c->x4_tab_ok; }
static int refresh_hrx(ocn_ctx *c)
{
    for (const LBlock &b : c->blocks)
        HIPCHK(hipMemcpyAsync(b.hr_x, b.ptr[field_slot(OCN_HHQ_REST)], field_bytes(b), hipMemcpyDeviceToDevice,
                              c->stream));
    auto swap_hr = [c] {
        for (LBlock &b : c->blocks) {
            void *t = b.ptr[field_slot(OCN_HHQ_REST)];
            b.ptr[field_slot(OCN_HHQ_REST)] = b.hr_x;
            b.hr_x = (double *)t;
        }
    };
    swap_hr();
    const int rc = run_sync(c, {OCN_HHQ_REST}, c->stream, nullptr, x4_tables(c) ? 4 : 2, 1);
    swap_hr();
    RC(rc);
    c->hrx_ok = true;
    return OCN_OK;
}

// every plan one_step_x2 and x2_end use, for the pair / second-buffer roles a call passes through
// (built before any graph capture)
static int prebuild_x2(ocn_ctx *c)
{
    int rc = OCN_OK;
    for (int i = 0; i < 4 && rc == OCN_OK; ++i) {
        if (i & 1) swap_roles(c);
        if (i & 2) swap_alt3(c);
        HaloPlan *p;
        rc = get_plan(c, kStateX2, p, 2);
        if (rc == OCN_OK) rc = get_plan(c, kStateX2, p, 1);
        if (rc == OCN_OK && c->x4 && c->x4_tab_ok) rc = get_plan(c, kStateX2, p, 4);   // (one_step_x4)
        if (i & 2) swap_alt3(c);
        if (i & 1) swap_roles(c);
    }
    return rc;
}

// The part of the interior an x2 step computes without the exchange: the interior less 2 points
// on every side a neighbour (diagonals included) fills halos of -- a point's stencil reaches the
// state 2 points away (D at +-1, formed from the state at +-1).
constexpr int kX2BandCols = 60;   // a one-pass wave's output columns (sw_kernels.hip MarchStep, kHalo 2)
static Range x2_inner(const LBlock &b)
{
    auto any = [&](int a, int d1, int d2) { return b.nbr_rank[a - 1] >= 0 || b.nbr_rank[d1 - 1] >= 0 || b.nbr_rank[d2 - 1] >= 0; };
    Range r{b.g.nx_start, b.g.nx_end, b.g.ny_start, b.g.ny_end};
    // (the E / W bands a whole wave wide where the block is wide enough: a band's waves march 60
    // columns whatever its width, so the wider band takes them off the inner launch for nothing)
    const int ew = b.g.nx_end - b.g.nx_start + 1 >= 3 * kX2BandCols ? kX2BandCols : 2;
    if (any(1, 5, 6)) r.m1 -= ew;   // E, NE, SE
    if (any(2, 7, 8)) r.m0 += ew;   // W, NW, SW
    if (any(3, 5, 7)) r.n1 -= 2;   // N, NE, NW
    if (any(4, 6, 8)) r.n0 += 2;   // S, SE, SW
    return r;
}

// One x2 step.  With OCN_OPT_OVERLAP 2 (the default when the context exchanges with other ranks;
// not while capturing a graph): the inner part (x2_inner) on the compute stream beside the exchange
// and then the frame bands on the comm stream (which runs at the device's highest priority) -- the
// exchange's latency hides behind the inner march.  The two parts write disjoint points of the new
// state (other buffers than the ones read), the exchange writes halos only the frame reads; the join
// orders the next step after both.  With only local copies (one GPU) the exchange costs less than
// the extra frame launch: one GPU, 4x2 blocks of 4096^2, 0.482 ms per step in sequence against
// 0.521 overlapped; 2x2 of 2048^2 0.154 against 0.170.
static int one_step_x2(ocn_ctx *c, double tau, const StepKind &k)
{
    const ocn_sw_params &sw = c->sw;
    hipStream_t s = c->stream;
    ocn_ctx::Rec rec;
    int32_t *nbad = k.check ? c->d_nbad : nullptr;
    auto march = [&](const LBlock &b, hipStream_t st, const Range *range, const Range *frame_of) -> int {
        std::vector<void *> tab = b.ptr;
        tab[field_slot(OCN_HHQ_REST)] = b.hr_x;
        const Compact t{b.bits, b.rows_x, c->march};
        return launch_onepass(&b.g, tab.data(), (int)tab.size(), &t, sw, tau, nbad, (double *)b.sshp_alt,
                              (double *)b.up_alt, (double *)b.vp_alt, st, range, false, kc_of(c, b), b.own, frame_of);
    };
    // OCN_OPT_CO_LAUNCH: the previous state's tracer step in a march launch after the exchange (one
    // tracer, block batching: sw_kernels.hip k_march_tracer_b) -- both read the state just exchanged,
    // the march writes the other buffers, the tracer step only the tracers'.  One block per rank too
    // (the C5 layout over 8 GPUs: two launches per step become one)
    const bool co = c->tr_pending && c->co_launch && c->sw.tracer_num == 1 && c->batch;
    auto co_done = [c] {
        c->tr_pending = false;
        swap_tracer_roles(c);
        swap_tracer_alt(c);
    };
    int probe = 0;
    const int lv = ov_begin(c, 2, !k.x2_save, probe);
    RC(ov_mark(c, probe, false));
    if (lv >= 2 && !c->capturing) {
        HIPCHK(hipEventRecord(c->ev_fork, s));
        RC(timer_begin(c, OCN_TIMER_ONEPASS, rec));
        RC(each_block(c, s, [&](const LBlock &b) -> int {
            const Range in = x2_inner(b);
            RC(march(b, s, &in, nullptr));
            return OCN_OK;
        }));
        RC(timer_end(c, rec));
        ocn_ctx::Rec xrec{OCN_TIMER_EXPOSED, nullptr, nullptr};   // inner march end -> comm chain end
        if (c->stage_timing) {
            RC(get_event(c, xrec.a)); RC(get_event(c, xrec.b));
            HIPCHK(hipEventRecord(xrec.a, s));
        }
        HIPCHK(hipStreamWaitEvent(c->comm_stream, c->ev_fork, 0));
        if (k.x2_save) RC(ring2_run(c, true, c->comm_stream));
        RC(run_sync(c, with_tracers(c, kStateX2), c->comm_stream, nullptr, 2));   // the state two points deep
        RC(each_block(c, c->comm_stream, [&](const LBlock &b) -> int {   // the bands (+ the tracer step)
            const Range in = x2_inner(b);
            RC(march(b, c->comm_stream, nullptr, &in));
            return co ? tracer_step_block(c, b, 1, tau, c->comm_stream) : OCN_OK;
        }, co));
        if (co) co_done();
        if (xrec.b) {
            HIPCHK(hipEventRecord(xrec.b, c->comm_stream));
            c->recs.push_back(xrec);
        }
        HIPCHK(hipEventRecord(c->ev_join, c->comm_stream));
        c->sync_pending = true;
        RC(join_sync(c));
    } else {
        if (k.x2_save) RC(ring2_run(c, true, s));
        RC(run_sync(c, with_tracers(c, kStateX2), s, nullptr, 2));   // the state two points deep
        if (c->tr_pending && !co && !c->capturing && c->comm_stream) {
            // the previous state's tracer step beside this step's march (on the comm stream: both read
            // the state just exchanged, the march writes the other buffers, the tracer step only the
            // tracers'); joined by the next step (run_step) or the call's end (finish_call)
            HIPCHK(hipEventRecord(c->ev_fork, s));
            HIPCHK(hipStreamWaitEvent(c->comm_stream, c->ev_fork, 0));
            RC(run_tracer_step(c, tau, c->comm_stream));
            HIPCHK(hipEventRecord(c->ev_join, c->comm_stream));
            c->sync_pending = true;
            c->tr_forked = true;
        }
        RC(timer_begin(c, OCN_TIMER_ONEPASS, rec));
        if (co) {   // (a variant that cannot co-launch flushes the two batches in order: the same results)
            RC(each_block(c, s, [&](const LBlock &b) -> int {
                RC(march(b, s, nullptr, nullptr));
                return tracer_step_block(c, b, 1, tau, s);
            }, true));
            co_done();
        } else {
            RC(each_block(c, s, [&](const LBlock &b) { return march(b, s, nullptr, nullptr); }));
        }
        RC(timer_end(c, rec));
    }
    RC(ov_mark(c, probe, true));
    // the previous state's tracer step: it reads that state (untouched by the march) and the tracers
    // with their first halo ring, both just exchanged
    RC(run_tracer_step(c, tau));
    swap_alt3(c);
    swap_roles(c);
    return OCN_OK;
}

// Two one-pass steps as one launch per block (sw_kernels.hip MarchStep PAIR): the first step's new
// state stays in LDS, the second's is written where a single step writes -- so the pair is one role
// flip of the pairs and of the second buffers, as a single one-pass step is.  Single block, no
// exchange, a variant chosen on the host (pair_ok); 98 B per cell for two steps in the known-constant
// variant, 162 in the general one.  k.one_last: the second step is the call's last (the pending tail's
// last two steps in one launch, complete_open): its consumer waves also store vort, the stresses and
// the RHS terms (MarchStep PAIR + LAST), then last_finish -- in place of a single one-pass step + the
// last step's own march.
static int one_step_pair(ocn_ctx *c, double tau, const StepKind &k)
{
    ocn_ctx::Rec rec;
    hipStream_t s = c->stream;
    RC(timer_begin(c, k.one_last ? OCN_TIMER_ONEPASS2_LAST : OCN_TIMER_ONEPASS2, rec));
    RC(each_block(c, s, [&](const LBlock &b) {
        const Compact t{b.bits, b.rows, c->march};
        return launch_onepass_pair(&b.g, b.ptr.data(), (int)b.ptr.size(), &t, c->sw, tau, k.check ? c->d_nbad : nullptr,
                                   k.check2 ? c->d_nbad : nullptr, (double *)b.sshp_alt, (double *)b.up_alt,
                                   (double *)b.vp_alt, s, kc_of(c, b), k.one_last);
    }));
    RC(timer_end(c, rec));
    swap_alt3(c);
    swap_roles(c);
    return k.one_last ? last_finish(c) : OCN_OK;
}

// Two x2 steps as one launch per block (sw_kernels.hip MarchStep PAIR + X2): the state exchanged FOUR
// points deep once (the pair's producers form the first step on the interior and the 2 halo rings
// neighbours own -- their D 3 deep, from the state 4 deep -- the consumers the second step on the
// interior), so a block with neighbours runs pairs as a single block does: one exchange and one
// launch per two steps instead of one each per step.  The extra rings live outside the reference's
// arrays (allocate: kXRing more rows, the row padding); the second ring is saved / restored around
// the sequence as for the x2 steps (ring2_run, x2_end).  The known-constant variant (x4_now).
// (shared/mpp/syncborder_block2D_gen_all.fi:100-129 per stage in the reference: 7 per step)
// The part of the interior a pair of x2 steps computes without the exchange: the interior less 4
// points on every side a neighbour (diagonals included) fills halos of (the pair reads the state 4
// points out: the producers' D 3 out, from the state 4 out).
// The E / W bands are a whole pair tile wide (kX4BandCols, where the block is wide enough): a band's
// tiles cost the same whatever its width up to that (a pair workgroup marches 116 columns), so the
// wider band takes that many columns off the inner launch for nothing -- one GPU, 2x1 blocks of
// 4096^2 overlapped: see DESIGN.md 4.4
constexpr int kX4BandCols = 116;   // sw_kernels.hip MarchStep::kPairCols
static Range x4_inner(const LBlock &b)
{
    auto any = [&](int a, int d1, int d2) { return b.nbr_rank[a - 1] >= 0 || b.nbr_rank[d1 - 1] >= 0 || b.nbr_rank[d2 - 1] >= 0; };
    Range r{b.g.nx_start, b.g.nx_end, b.g.ny_start, b.g.ny_end};
    const int ew = b.g.nx_end - b.g.nx_start + 1 >= 3 * kX4BandCols ? kX4BandCols : 4;
    if (any(1, 5, 6)) r.m1 -= ew;   // E, NE, SE
    if (any(2, 7, 8)) r.m0 += ew;   // W, NW, SW
    if (any(3, 5, 7)) r.n1 -= 4;   // N, NE, NW
    if (any(4, 6, 8)) r.n0 += 4;   // S, SE, SW
    return r;
}

// With OCN_OPT_OVERLAP 2 (the default with remote peers; not while capturing): the inner part
// (x4_inner) on the compute stream beside the exchange on the comm stream (the device's highest
// priority), then the bands around it there -- the RCCL group's latency hides behind the inner
// pair; the two launches write disjoint points of the new state (other buffers than the ones read),
// the exchange writes halos only the bands read.
// Tracer runs (tracer steps, c->tr_call): the exchange carries the tracers 2 deep; the pending tracer
// step of the state before the pair (A) runs over the interior and the first halo ring neighbours own
// (launch_tracer_step ext: as those neighbours update it), co-launched with the pair where it can be;
// the producers also write the first step's new state (LBlock::trs), and the tracer step of that state
// (B) runs after the pair from there -- two tracer steps per exchange, as the reference runs one per
// step after its exchanges; the second tracer ring is saved / restored with the state's (ring2_run).
static int one_step_x4(ocn_ctx *c, double tau, const StepKind &k)
{
    hipStream_t s = c->stream;
    ocn_ctx::Rec rec;
    c->hn_fresh = false;
    const bool tr = c->tr_call, trA = tr && c->tr_pending;
    const bool co = trA && c->co_launch && c->sw.tracer_num == 1 && c->batch;
    auto tr_a = [&](const LBlock &b, int t, hipStream_t st) -> int {
        std::vector<void *> tab = b.ptr;
        tab[field_slot(OCN_HHQ_REST)] = b.hr_x;   // (h_r with the neighbours' second ring)
        const Compact ct{b.bits, b.rows_x, c->march};
        return launch_tracer_step(&b.g, tab.data(), (int)tab.size(), &ct, t, tau, c->sw.time_smooth,
                                  (double *)b.ptr[field_slot(OCN_FF1N(t))], (double *)b.ffp_alt[(size_t)t - 1], b.own,
                                  st, true);
    };
    auto tr_b = [&](const LBlock &b, int t, hipStream_t st) -> int {
        std::vector<void *> tab = b.ptr;   // the state the pair's first step formed
        tab[field_slot(OCN_SSH)] = b.trs[0]; tab[field_slot(OCN_SSHP)] = b.trs[1];
        tab[field_slot(OCN_UBRTR)] = b.trs[2]; tab[field_slot(OCN_VBRTR)] = b.trs[3];
        const Compact ct{b.bits, b.rows_x, c->march};
        return launch_tracer_step(&b.g, tab.data(), (int)tab.size(), &ct, t, tau, c->sw.time_smooth,
                                  (double *)b.ptr[field_slot(OCN_FF1N(t))], (double *)b.ffp_alt[(size_t)t - 1], b.own,
                                  st, false);
    };
    auto tr_done = [c] {
        swap_tracer_roles(c);
        swap_tracer_alt(c);
    };
    auto pair = [&](const LBlock &b, hipStream_t st, const Range *range, const Range *frame_of) -> int {
        ocn_block bx = b.g;   // the block widened by kXRing rings, the bases moved to A(bnd_x1 - kXRing, bnd_y1 - kXRing)
        bx.bnd_x1 -= kXRing; bx.bnd_x2 += kXRing; bx.bnd_y1 -= kXRing; bx.bnd_y2 += kXRing;
        const long sh = (long)kXRing * b.g.pitch + kXRing;
        std::vector<void *> tab(b.ptr.size(), nullptr);
        for (int id = OCN_SSH; id < OCN_SSH + num_r8(c); ++id) tab[field_slot(id)] = b.f<double>(id) - sh;
        tab[field_slot(OCN_HHQ_REST)] = b.hr_x - sh;   // (the h_r-read variant: h_r with the neighbours' 4 rings)
        const Compact t{b.bits_x4, b.rows_x4, c->march};
        double *trs_x[4];
        for (int i = 0; i < 4; ++i) trs_x[i] = b.trs[i] ? b.trs[i] - sh : nullptr;
        return launch_onepass_pair_x4(&bx, tab.data(), (int)tab.size(), &t, c->sw, tau, k.check ? c->d_nbad : nullptr,
                                      k.check2 ? c->d_nbad : nullptr, (double *)b.sshp_alt - sh, (double *)b.up_alt - sh,
                                      (double *)b.vp_alt - sh, st, kc_of(c, b), b.own, range, (int)c->blocks.size(),
                                      frame_of, tr ? trs_x : nullptr);
    };
    bool inner_ok = true;   // (every block keeps an inner part: the bands around it are disjoint)
    for (const LBlock &b : c->blocks) {
        const Range in = x4_inner(b);
        inner_ok = inner_ok && in.m0 <= in.m1 && in.n0 <= in.n1;
    }
    int probe = 0;
    const int lv = ov_begin(c, 4, !k.x2_save && inner_ok, probe);
    RC(ov_mark(c, probe, false));
    if (lv >= 2 && !c->capturing && inner_ok) {
        HIPCHK(hipEventRecord(c->ev_fork, s));
        RC(timer_begin(c, OCN_TIMER_ONEPASS2, rec));
        RC(each_block(c, s, [&](const LBlock &b) -> int {
            const Range in = x4_inner(b);
            return pair(b, s, &in, nullptr);
        }));
        RC(timer_end(c, rec));
        ocn_ctx::Rec xrec{OCN_TIMER_EXPOSED, nullptr, nullptr};   // inner pair end -> comm chain end
        if (c->stage_timing) {
            RC(get_event(c, xrec.a)); RC(get_event(c, xrec.b));
            HIPCHK(hipEventRecord(xrec.a, s));
        }
        HIPCHK(hipStreamWaitEvent(c->comm_stream, c->ev_fork, 0));
        if (k.x2_save) RC(ring2_run(c, true, c->comm_stream));
        RC(run_sync(c, tr ? with_tracers(c, kStateX2) : kStateX2, c->comm_stream, nullptr, 4));   // the state 4 deep
        RC(each_block(c, c->comm_stream, [&](const LBlock &b) -> int {   // the bands (+ tracer step A)
            const Range in = x4_inner(b);
            RC(pair(b, c->comm_stream, nullptr, &in));
            return co ? tr_a(b, 1, c->comm_stream) : OCN_OK;
        }, co));
        if (xrec.b) {
            HIPCHK(hipEventRecord(xrec.b, c->comm_stream));
            c->recs.push_back(xrec);
        }
        HIPCHK(hipEventRecord(c->ev_join, c->comm_stream));
        c->sync_pending = true;
        RC(join_sync(c));
    } else {
        if (k.x2_save) RC(ring2_run(c, true, s));
        RC(run_sync(c, tr ? with_tracers(c, kStateX2) : kStateX2, s, nullptr, 4));   // the state four points deep
        RC(timer_begin(c, OCN_TIMER_ONEPASS2, rec));
        RC(each_block(c, s, [&](const LBlock &b) -> int {
            RC(pair(b, s, nullptr, nullptr));
            return co ? tr_a(b, 1, s) : OCN_OK;
        }, co));
        RC(timer_end(c, rec));
    }
    RC(ov_mark(c, probe, true));
    if (trA) {   // tracer step A (here when not co-launched: after the join, it reads the exchanged halos)
        c->tr_pending = false;
        for (int t = co ? 2 : 1; t <= c->sw.tracer_num; ++t)
            RC(each_block(c, s, [&](const LBlock &b) { return tr_a(b, t, s); }));
        tr_done();
    }
    if (tr) {   // tracer step B: the state of the pair's first step
        for (int t = 1; t <= c->sw.tracer_num; ++t)
            RC(each_block(c, s, [&](const LBlock &b) { return tr_b(b, t, s); }));
        tr_done();
    }
    swap_alt3(c);
    swap_roles(c);
    return OCN_OK;
}

// Several one-pass steps as one launch (sw_kernels.hip k_march_multi: a grid barrier
// between the steps; the block's tiles resident together): single small block, no exchange, a
// variant chosen on the host (multi_ok).  Step parity alternates the buffers as the role flips of
// single launches do, so the host flips the roles k.multi times.
static int one_step_multi(ocn_ctx *c, double tau, const StepKind &k)
{
    ocn_ctx::Rec rec;
    hipStream_t s = c->stream;
    const LBlock &b = c->blocks[0];
    const Compact t{b.bits, b.rows, c->march};
    RC(timer_begin(c, OCN_TIMER_ONEPASS_MULTI, rec));
    RC(launch_onepass_multi(&b.g, b.ptr.data(), (int)b.ptr.size(), &t, c->sw, tau, k.multi, k.check ? c->d_nbad : nullptr,
                            (double *)b.sshp_alt, (double *)b.up_alt, (double *)b.vp_alt, c->d_bar,
                            c->d_nbad + 61, s, kc_of(c, b), c->multi_spin));
    RC(timer_end(c, rec));
    if (k.multi & 1) {
        swap_alt3(c);
        swap_roles(c);
    }
    return OCN_OK;
}

// one_step_pair possible in this call: one block without exchanges or ring work, the compact tables
// and the march, the one-pass variant chosen by the host (kc_mode not OCN_KC_DEVICE; OCN_OPT_PAIR 1:
// a known-constant one on blocks of 512^2 or more, 2: any)
#ifndef OCN_PAIR_MIN_CELLS
#define OCN_PAIR_MIN_CELLS (512L * 512L)
#endif
static bool pair_ok(ocn_ctx *c)
{
    if (!c->pair || c->blocks.size() != 1 || has_exchange(c) || has_comm(c) || c->ring_sea || !c->compact || !c->march ||
        c->sw.use_tracers > 0)
        return false;
    if (c->kc_mode == OCN_KC_DEVICE) return false;   // (the variant the launches run is chosen on the device)
    if (c->pair >= 2) return true;
    // the default: the known-constant variants only -- the general variant's pair is VALU bound at
    // twice its single launch (4096^2: 1.09 vs 0.54 ms), no faster
    if (c->kc_mode == OCN_KC_GENERAL) return false;
    const ocn_block &g = c->blocks[0].g;
    return (long)(g.nx_end - g.nx_start + 1) * (g.ny_end - g.ny_start + 1) >= OCN_PAIR_MIN_CELLS;
}

// one_step_multi possible in this call (an open sequence, pairs not used): one block without exchanges or
// ring work, the compact tables and the march, the variant chosen on the host, every step checked or
// none, and a block small enough that its grid is resident at once -- the launch-latency-bound case
static bool multi_ok(ocn_ctx *c, int32_t check_every)
{
    return c->multi && c->sw.use_tracers <= 0 && c->blocks.size() == 1 && !has_exchange(c) && !has_comm(c) &&
           !c->ring_sea && c->compact &&
           c->march && c->kc_mode != OCN_KC_DEVICE && (check_every == 0 || check_every == 1) &&
           onepass_multi_fits(&c->blocks[0].g);
}

static int one_step_fused(ocn_ctx *c, double tau, const StepKind &k)
{
    if (k.multi) return one_step_multi(c, tau, k);
    if (k.pair && k.x2) return one_step_x4(c, tau, k);
    if (k.pair) return one_step_pair(c, tau, k);
    // every other step kind may write the n-level depths (hh_update, hh_shift, hh_init), except a
    // single-block one-pass step (not followed by the fused hh_init + A) and the last step's march
    if (!((k.one || k.one_last) && !k.x2 && !k.next_a && !has_exchange(c) && !c->ring_sea)) c->hn_fresh = false;
    if (k.x2) return one_step_x2(c, tau, k);
    if (k.one_last && k.x2_end) RC(x2_end(c, c->stream));
    if (k.one_last && c->tr_pending) {   // the previous state's tracer step, then its tracers' halos
        RC(run_tracer_step(c, tau));
        if (has_exchange(c)) RC(run_sync(c, with_tracers(c, {})));
    }
    if (k.one_last) return has_exchange(c) || c->ring_sea ? one_step_hybrid(c, tau, k, true) : one_step_last(c, tau, k);
    const bool check = k.check, first = k.first, last = k.last, flip = k.flip;
    const ocn_sw_params &sw = c->sw;
    ocn_ctx::Rec rec;
    auto cp = [c](const LBlock &b, Compact &t) -> const Compact * {
        t = Compact{b.bits, b.rows, c->march};
        return c->compact ? &t : nullptr;
    };
    Compact t;
    int32_t *nbad = check ? c->d_nbad : nullptr;
    hipStream_t s = c->stream;
    const bool ffs = sw.full_free_surface > 0;
    const bool full_c2 = last || sw.use_tracers > 0;   // tracers read hh_init's hhq_p every step
    // sw_stencils.h "reuse" steps: hun/hvn/hhn are hh_init's hu/hv/hh of the previous step.  Not
    // on the first step of a call (the host may have changed ssh since) nor on the last one.
    const bool reuse = sw.full_free_surface == 1 && !first && !last;
    const std::vector<int> &sync_a = reuse ? c->sync_a_reuse : c->sync_a;
    if (flip) {
        if (last) return set_error(OCN_ERR_STATE, "role-flip step on a last step");
        if (k.one && (has_exchange(c) || c->ring_sea)) return one_step_hybrid(c, tau, k);
        if (k.one) {   // the whole step in one launch (single block: no exchange, no ring launch)
            RC(timer_begin(c, OCN_TIMER_ONEPASS, rec));
            RC(each_block(c, s, [&](const LBlock &b) { return launch_onepass(&b.g, b.ptr.data(), (int)b.ptr.size(), cp(b, t), sw, tau, nbad,
                                  (double *)b.sshp_alt, (double *)b.up_alt, (double *)b.vp_alt, s, nullptr, false,
                                  kc_of(c, b)); }));
            RC(timer_end(c, rec));
            swap_alt3(c);
            swap_roles(c);
            if (k.next_a) {   // the next step is the last, standard one: hh_init + its fused A
                RC(timer_begin(c, OCN_TIMER_FUSED_CA, rec));
                RC(each_block(c, s, [&](const LBlock &b) { return launch_fused_ca(&b.g, b.ptr.data(), (int)b.ptr.size(), cp(b, t), OCN_PART_ALL, sw, tau,
                                       k.next_reuse, false, s); }));
                RC(timer_end(c, rec));
            }
            return OCN_OK;
        }
        // With halo exchanges and OCN_OPT_OVERLAP = 2 (not while capturing a graph: the last
        // exchange stays pending into the next step), each exchange runs on the comm stream beside
        // the inner part (launch_march_part) of the next launch:
        //   [A.frame | fork: sync A || A.inner] B.inner | join | B.frame | fork: sync B || swap,
        //   CA.inner | join | ring launch (the roles before the swap) | CA.frame | fork: sync CA
        //   || the next step's B.inner ...
        // The default (overlap_level) with remote peers; off with only local copies, whose cost
        // the frame bands match (one GPU, 2x2 / 4x2 blocks: 1.61 vs 1.47, 1.89 vs 1.69 ms per step).
        const bool ov = overlap_level(c) >= 2 && has_exchange(c) && !c->capturing;
        if (!k.a_done) {
            RC(timer_begin(c, OCN_TIMER_FUSED_A, rec));
            if (ov) {
                RC(each_block(c, s, [&](const LBlock &b) { return launch_fused_a(FT(b), OCN_PART_FRAME, sw, tau, reuse, s); }));
                RC(fork_sync(c, sync_a));
                RC(each_block(c, s, [&](const LBlock &b) { return launch_fused_a(FT(b), OCN_PART_INNER, sw, tau, reuse, s); }));
            } else {
                RC(each_block(c, s, [&](const LBlock &b) { return launch_fused_a(FT(b), OCN_PART_ALL, sw, tau, reuse, s); }));
            }
            RC(timer_end(c, rec));
            if (!ov) RC(run_sync(c, sync_a));
        }
        RC(timer_begin(c, OCN_TIMER_FUSED_B, rec));
        for (int part : ov ? std::initializer_list<int>{OCN_PART_INNER, OCN_PART_FRAME}
                           : std::initializer_list<int>{OCN_PART_ALL}) {
            if (part == OCN_PART_FRAME) RC(join_sync(c));
            RC(each_block(c, s, [&](const LBlock &b) { return launch_fused_b(FT(b), part, sw, tau, false, reuse, s, nbad, true, k.rc, (double *)b.sshp_alt); }));
        }
        RC(timer_end(c, rec));
        // the current roles' ubrtrn / vbrtrn (+ hhu_p / hhv_p / hhh_p)
        if (ov) RC(fork_sync(c, c->sync_b));
        else RC(run_sync(c, c->sync_b));
        if (k.rc) swap_sshp(c);
        std::vector<std::vector<void *>> pre;   // the ring launch's field tables (roles before the swap)
        for (const LBlock &b : c->blocks) pre.push_back(b.ptr);
        swap_roles(c);
        // hh_init + the next step's fused A (full_free_surface = 1), else hh_init alone
        auto hh_init = [&](int part) -> int {
            RC(each_block(c, s, [&](const LBlock &b) -> int {
                if (k.next_a)
                    RC(launch_fused_ca(&b.g, b.ptr.data(), (int)b.ptr.size(), cp(b, t), part, sw, tau, k.next_reuse,
                                       k.next_reuse && k.rc_next, s));
                else
                    RC(launch_fused_c2(FT(b), part, sw, full_c2, s));
                return OCN_OK;
            }));
            return OCN_OK;
        };
        const int hh_timer = k.next_a ? OCN_TIMER_FUSED_CA : OCN_STAGE_HH_INIT;
        const bool hh = !k.next_one && (k.next_a || ffs);   // a one-pass step forms hh_init's values itself
        if (ov && hh) {
            RC(timer_begin(c, hh_timer, rec));
            RC(hh_init(OCN_PART_INNER));
            RC(timer_end(c, rec));
        }
        RC(join_sync(c));
        if (c->ring_sea) {   // a8 + a9 on the ring (no interior points); nothing to do on an all-land ring
            RC(timer_begin(c, OCN_TIMER_FUSED_C1, rec));
            for (size_t i = 0; i < c->blocks.size(); ++i) {
                const LBlock &b = c->blocks[i];
                // recompute steps: B filtered sshp into the other buffer, now the current one; a8
                // on the ring reads the previous one (sshp_alt after the swap) and completes it
                RC(launch_fused_c1(&b.g, pre[i].data(), (int)pre[i].size(), cp(b, t), OCN_PART_FRAME, sw, nullptr, s,
                                   k.rc ? (const double *)b.sshp_alt : nullptr));
            }
            RC(timer_end(c, rec));
        }
        if (hh) {
            RC(timer_begin(c, hh_timer, rec));
            RC(hh_init(ov ? OCN_PART_FRAME : OCN_PART_ALL));
            RC(timer_end(c, rec));
            // with CA, hh_init's sync and the next step's sync A in one exchange: A's a1 took
            // hhu / hhv on the low halo ring from hh_init's registers, the values it delivers there
            const std::vector<int> &l = !k.next_a ? *stage_sync(OCN_STAGE_HH_INIT)
                                        : k.next_reuse ? c->sync_ca_reuse : c->sync_ca;
            if (ov) RC(fork_sync(c, l));
            else RC(run_sync(c, l));
        }
        return OCN_OK;
    }
    if (!(overlap_level(c) && has_exchange(c))) {
        RC(join_sync(c));
        if (!k.a_done) {   // else fused A and its sync ran with the previous step's hh_init
            RC(timer_begin(c, OCN_TIMER_FUSED_A, rec));
            RC(each_block(c, s, [&](const LBlock &b) { return launch_fused_a(FT(b), OCN_PART_ALL, sw, tau, reuse, s); }));
            RC(timer_end(c, rec));
            RC(run_sync(c, sync_a));
        }
        RC(timer_begin(c, OCN_TIMER_FUSED_B, rec));
        RC(each_block(c, s, [&](const LBlock &b) { return launch_fused_b(FT(b), OCN_PART_ALL, sw, tau, last, reuse, s); }));
        RC(timer_end(c, rec));
        RC(run_sync(c, c->sync_b));
        RC(timer_begin(c, OCN_TIMER_FUSED_C1, rec));
        RC(each_block(c, s, [&](const LBlock &b) { return launch_fused_c1(FT(b), OCN_PART_ALL, sw, nbad, s); }));
        RC(timer_end(c, rec));
        if (ffs) {
            RC(timer_begin(c, OCN_STAGE_HH_INIT, rec));
            RC(each_block(c, s, [&](const LBlock &b) { return launch_fused_c2(FT(b), OCN_PART_ALL, sw, full_c2, s); }));
            RC(timer_end(c, rec));
            RC(run_sync(c, *stage_sync(OCN_STAGE_HH_INIT)));
        }
        return OCN_OK;
    }
    if (!k.a_done) {   // else fused A and its sync ran with the previous step's hh_init
        RC(timer_begin(c, OCN_TIMER_FUSED_A, rec));
        RC(each_block(c, s, [&](const LBlock &b) { return launch_fused_a(FT(b), OCN_PART_FRAME, sw, tau, reuse, s); }));
        RC(fork_sync(c, sync_a));
        RC(each_block(c, s, [&](const LBlock &b) { return launch_fused_a(FT(b), OCN_PART_INNER, sw, tau, reuse, s); }));
        RC(timer_end(c, rec));
    }
    RC(timer_begin(c, OCN_TIMER_FUSED_B, rec));
    RC(each_block(c, s, [&](const LBlock &b) { return launch_fused_b(FT(b), OCN_PART_INNER, sw, tau, last, reuse, s); }));
    RC(join_sync(c));   // sync A, or the previous role-flip step's last exchange
    RC(each_block(c, s, [&](const LBlock &b) { return launch_fused_b(FT(b), OCN_PART_FRAME, sw, tau, last, reuse, s); }));
    RC(fork_sync(c, c->sync_b));
    RC(timer_end(c, rec));
    RC(timer_begin(c, OCN_TIMER_FUSED_C1, rec));
    RC(each_block(c, s, [&](const LBlock &b) { return launch_fused_c1(FT(b), OCN_PART_INNER, sw, nbad, s); }));
    RC(join_sync(c));
    RC(each_block(c, s, [&](const LBlock &b) { return launch_fused_c1(FT(b), OCN_PART_FRAME, sw, nbad, s); }));
    RC(timer_end(c, rec));
    if (ffs) {
        RC(timer_begin(c, OCN_STAGE_HH_INIT, rec));
        RC(each_block(c, s, [&](const LBlock &b) { return launch_fused_c2(FT(b), OCN_PART_FRAME, sw, full_c2, s); }));
        RC(fork_sync(c, *stage_sync(OCN_STAGE_HH_INIT)));
        RC(each_block(c, s, [&](const LBlock &b) { return launch_fused_c2(FT(b), OCN_PART_INNER, sw, full_c2, s); }));
        RC(join_sync(c));
        RC(timer_end(c, rec));
    }
    return OCN_OK;
}
#undef FT

// ------------------------------------------------------------------ tracers
// expl_tracer (control/tracer.f90:33-62): for every tracer, envoke of the three tracer stages
// with the syncs of interface/tracer/tracer_interface.f90 (flux_x, flux_y; ff1n; none).
static const std::vector<int> kSyncFlux = {OCN_FLUX_X, OCN_FLUX_Y};

static int tracer_stage(ocn_ctx *c, int stage, int k, double tau, bool compact)
{
    ocn_ctx::Rec rec;
    RC(timer_begin(c, OCN_TIMER_TRACER + stage, rec));
    RC(each_block(c, c->stream, [&](const LBlock &b) -> int {
        const Compact t{b.bits, b.rows};
        RC(launch_tracer(&b.g, b.ptr.data(), (int)b.ptr.size(), compact ? &t : nullptr, stage, k, tau, c->sw.time_smooth,
                          c->stream));
        return OCN_OK;
    }));
    RC(timer_end(c, rec));
    if (stage == OCN_TSTAGE_TRAN_DIFF_FLUXES) RC(run_sync(c, kSyncFlux));
    if (stage == OCN_TSTAGE_TRAN_DIFF_TRACER) RC(run_sync(c, {OCN_FF1N(k)}));
    return OCN_OK;
}

static int expl_tracer(ocn_ctx *c, double tau, bool compact)
{
    if (c->sw.use_tracers <= 0) return OCN_OK;
    RC(join_sync(c));   // an exchange a role-flip step left in flight (hh_init's hhu / hhv halos)
    // tran_diff_tracer reads hhq_n, which the step's hh_init set to h_r (depth.f90:14-99, whole
    // array) -- the role-flip steps' CA leaves it as it was, which is h_r unless one of them was
    // uploaded or written through a raw pointer since the last hh_init that stored it
    if (c->hqn_stale || c->r8_handed || c->capturing) {
        for (const LBlock &b : c->blocks)
            HIPCHK(hipMemcpyAsync(b.ptr[field_slot(OCN_HHQ_N)], b.ptr[field_slot(OCN_HHQ_REST)], field_bytes(b),
                                  hipMemcpyDeviceToDevice, c->stream));
        if (!c->capturing) c->hqn_stale = false;
    }
    for (int k = 1; k <= c->sw.tracer_num; ++k)
        for (int stage = 0; stage < OCN_NUM_TSTAGES; ++stage) RC(tracer_stage(c, stage, k, tau, compact));
    return OCN_OK;
}

// Tracer runs with one-pass steps (OCN_OPT_TRACER_STEP): a one-pass step keeps hh_init's depths in
// registers, so expl_tracer after it (control/tracer.f90:33-62, model.f90:156) runs later, as ONE
// launch per tracer (sw_kernels.hip launch_tracer_step, sw_stencils.h TracerStep) that forms the
// depths it reads from the state with hh_init's own functions -- with the next step, after that
// step's exchange (which carries the tracers' ff1 / ff1p one point deep with the state: with_tracers)
// and before anything writes the state it reads.  Its ffn goes to the ff1n buffer and the roles of
// ff1 / ff1n trade (tracer_next_step's ff := ffn); the filtered ff1p to the second buffer.  The call's
// last step (standard hh_init with every level) runs the standard stages after it.
// st: the stream it runs on (one_step_x2 forks it onto the comm stream beside the next step's march:
// the march reads the state the tracer step reads and writes the other buffers; the next step's
// exchange and march wait for it -- run_step joins first)
// tracer k's tracer step on block b
static int tracer_step_block(ocn_ctx *c, const LBlock &b, int k, double tau, hipStream_t st)
{
    const Compact t{b.bits, b.rows, c->march};
    return launch_tracer_step(&b.g, b.ptr.data(), (int)b.ptr.size(), c->compact ? &t : nullptr, k, tau, c->sw.time_smooth,
                              (double *)b.ptr[field_slot(OCN_FF1N(k))], (double *)b.ffp_alt[(size_t)k - 1], b.own, st);
}
static int run_tracer_step(ocn_ctx *c, double tau, hipStream_t st)
{
    if (!c->tr_pending) return OCN_OK;
    c->tr_pending = false;
    ocn_ctx::Rec rec{OCN_TIMER_TRACER_STEP, nullptr, nullptr};
    if (c->stage_timing) {
        RC(get_event(c, rec.a)); RC(get_event(c, rec.b));
        HIPCHK(hipEventRecord(rec.a, st));
    }
    for (int k = 1; k <= c->sw.tracer_num; ++k)
        RC(each_block(c, st, [&](const LBlock &b) { return tracer_step_block(c, b, k, tau, st); }));
    if (rec.b) {
        HIPCHK(hipEventRecord(rec.b, st));
        c->recs.push_back(rec);
    }
    swap_tracer_roles(c);
    swap_tracer_alt(c);
    return OCN_OK;
}
static int run_tracer_step(ocn_ctx *c, double tau) { return run_tracer_step(c, tau, c->stream); }

static std::vector<int> with_tracers(const ocn_ctx *c, const std::vector<int> &fields)
{
    if (!c->tr_call) return fields;
    std::vector<int> out = fields;
    for (int k = 1; k <= c->sw.tracer_num; ++k) { out.push_back(OCN_FF1(k)); out.push_back(OCN_FF1P(k)); }
    return out;
}

// ------------------------------------------------------------------ initial state
// init_grid_data + init_ocean_data (control/init_data.f90:29-125) with every 2-D field formed on
// the device (init_kernels.hip); the host supplies the basin mask and the grid's O(nx + ny)
// trigonometric row / column factors from its libm, as the reference computes them.
static const float kPi = 3.1415926f;              // constants.f90:14
static const double kDPi = 3.14159265358979;      // constants.f90:17
static const double kLatExtr = 89.99999;          // constants.f90:20
static const float kRadEarth = 6371000.0f;        // constants.f90:22
static const float kEarthAngVel = 7.2921159e-5f;  // constants.f90:22
static double dsind(double x) { return std::sin((x / 180.0) * kDPi); }   // core/math_tools.f90
static double dcosd(double x) { return std::cos((x / 180.0) * kDPi); }

// One block's grid tables in one device allocation (freed by the caller after the launch ran):
// grid_base_init's coordinates xt / xu (columns) and yt / yv (rows) (grid_kernels.f90:94-202),
// then grid_geo_init's factors of them (grid_parameters.f90:80-181).
struct GridTables {
    std::vector<float> cos_t, cos_v;                   // (float) dcosd(lat_mod(yt)), of yv, per row
    std::vector<double> sin_v, cosy_v, cos_xu;         // dsind(yv), dcosd(yv) per row; dcosd(xu) per column
    // the same factors of rows bnd_y1 and bnd_y2 (outside the metric range) from the global row
    // formulas, as the neighbour blocks form them (GridInit ext)
    float ext_ct[kExtRows], ext_cv[kExtRows];
    double ext_sin_v[kExtRows], ext_cosy_v[kExtRows];
};
static void grid_tables(const ocn_ctx *c, const ocn_block &g, GridTables &t)
{
    const ocn_basin &bs = c->basin;
    const int w = g.bnd_x2 - g.bnd_x1 + 1, h = g.bnd_y2 - g.bnd_y1 + 1, mmm = 3, nnn = 3;
    std::vector<double> xt(w), xu(w, 0.0), yt(h), yv(h, 0.0);
    for (int m = g.bnd_x1; m <= g.bnd_x2; ++m) xt[m - g.bnd_x1] = bs.rlon + (double)(m - mmm) * bs.dxst;
    for (int n = g.bnd_y1; n <= g.bnd_y2; ++n) yt[n - g.bnd_y1] = bs.rlat + (double)(n - nnn) * bs.dyst;
    for (int i = 0; i + 1 < w; ++i) xu[i] = (xt[i] + xt[i + 1]) / 2.0;
    for (int i = 0; i + 1 < h; ++i) yv[i] = (yt[i] + yt[i + 1]) / 2.0;
    auto lat_mod = [](double y) { return std::max(std::min(y, kLatExtr), -kLatExtr); };
    t.cos_t.assign(h, 0.0f); t.cos_v.assign(h, 0.0f); t.sin_v.assign(h, 0.0); t.cosy_v.assign(h, 0.0);
    t.cos_xu.assign(w, 0.0);
    for (int n = g.ny_start - 1; n <= g.ny_end + 1; ++n) {   // the metric range's rows and columns
        const int r = n - g.bnd_y1;
        t.cos_t[r] = (float)dcosd(lat_mod(yt[r]));
        t.cos_v[r] = (float)dcosd(lat_mod(yv[r]));
        t.sin_v[r] = dsind(yv[r]);
        t.cosy_v[r] = dcosd(yv[r]);
    }
    for (int m = g.nx_start - 1; m <= g.nx_end + 1; ++m) t.cos_xu[m - g.bnd_x1] = dcosd(xu[m - g.bnd_x1]);
    // grid_base_init on the neighbour: yt(n), yv(n) = (yt(n) + yt(n + 1)) / 2 (GridInit ext's rows)
    const int ext_row[kExtRows] = {g.bnd_y1, g.bnd_y2, g.bnd_y1 - 1, g.bnd_y1 - 2, g.bnd_y2 + 1, g.bnd_y2 + 2};
    for (int i = 0; i < kExtRows; ++i) {
        const int n = ext_row[i];
        const double yt_n = bs.rlat + (double)(n - nnn) * bs.dyst, yt_n1 = bs.rlat + (double)(n + 1 - nnn) * bs.dyst;
        const double yv_n = (yt_n + yt_n1) / 2.0;
        t.ext_ct[i] = (float)dcosd(lat_mod(yt_n));
        t.ext_cv[i] = (float)dcosd(lat_mod(yv_n));
        t.ext_sin_v[i] = dsind(yv_n);
        t.ext_cosy_v[i] = dcosd(yv_n);
    }
}

static int upload_field(ocn_ctx *c, const LBlock &b, int id, const void *host, bool async)
{
    const size_t es = is_r4(id) ? 4 : 8;
    const size_t w = (size_t)(b.g.bnd_x2 - b.g.bnd_x1 + 1), rows = (size_t)(b.g.bnd_y2 - b.g.bnd_y1 + 1);
    if (async)
        HIPCHK(hipMemcpy2DAsync(b.ptr[field_slot(id)], (size_t)b.g.pitch * es, host, w * es, w * es, rows,
                                hipMemcpyHostToDevice, c->stream));
    else
        HIPCHK(hipMemcpy2D(b.ptr[field_slot(id)], (size_t)b.g.pitch * es, host, w * es, w * es, rows,
                           hipMemcpyHostToDevice));
    return OCN_OK;
}

static int init_state(ocn_ctx *c)
{
    HIPCHK(hipStreamSynchronize(c->stream));
    const ocn_basin &bs = c->basin;
    const size_t nxy = (size_t)bs.nx * bs.ny;
    // device scratch of this call: the basin mask, then per block its grid tables
    std::vector<GridTables> tabs(c->blocks.size());
    const size_t topo_at = (nxy * sizeof(int32_t) + 255) / 256 * 256;
    size_t bytes = topo_at + c->topo.size() * sizeof(float);
    std::vector<size_t> at(c->blocks.size());
    for (size_t i = 0; i < c->blocks.size(); ++i) {
        grid_tables(c, c->blocks[i].g, tabs[i]);
        at[i] = (bytes + 255) / 256 * 256;
        bytes = at[i] + tabs[i].cos_t.size() * 2 * 4 + 256 + (tabs[i].sin_v.size() * 2 + tabs[i].cos_xu.size()) * 8;
    }
    char *scratch = nullptr;
    HIPCHK(hipMalloc(&scratch, bytes));
    struct Free { char *p; ~Free() { if (p) (void)hipFree(p); } } free_scratch{scratch};
    HIPCHK(hipMemcpy(scratch, c->mask.data(), nxy * sizeof(int32_t), hipMemcpyHostToDevice));
    if (!c->topo.empty())
        HIPCHK(hipMemcpy(scratch + topo_at, c->topo.data(), c->topo.size() * sizeof(float), hipMemcpyHostToDevice));
    const float pip180 = kPi / 180.0f;
    for (size_t i = 0; i < c->blocks.size(); ++i) {
        const LBlock &b = c->blocks[i];
        const GridTables &t = tabs[i];
        const size_t h = t.cos_t.size(), w = t.cos_xu.size();
        char *p = scratch + at[i];
        GridInit q{};
        q.g = b.g;
        q.mask = (const int32_t *)scratch;
        q.nx = bs.nx;
        for (int id = 0; id < OCN_NUM_R4; ++id) q.r4[id] = b.f<float>(id);
        q.cos_t = (const float *)p; q.cos_v = q.cos_t + h;
        p += (h * 2 * 4 + 255) / 256 * 256;
        q.sin_v = (const double *)p; q.cosy_v = q.sin_v + h; q.cos_xu = q.cosy_v + h;
        HIPCHK(hipMemcpy((void *)q.cos_t, t.cos_t.data(), h * 4, hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy((void *)q.cos_v, t.cos_v.data(), h * 4, hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy((void *)q.sin_v, t.sin_v.data(), h * 8, hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy((void *)q.cosy_v, t.cosy_v.data(), h * 8, hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy((void *)q.cos_xu, t.cos_xu.data(), w * 8, hipMemcpyHostToDevice));
        q.cos_rot = dcosd(bs.rotation_on_lat);
        q.sin_rot = dsind(bs.rotation_on_lat);
        q.sin_extr = dsind(kLatExtr);
        q.sx = (float)bs.dxst * pip180 * kRadEarth;
        q.sy = (float)bs.dyst * pip180 * kRadEarth;
        q.cor = 2.0f * kEarthAngVel;
        q.sqrt2 = std::sqrt(2.0f);
        q.curve = bs.curve_grid != 0;
        for (int j = 0; j < kExtRows; ++j) {
            q.ext_ct[j] = t.ext_ct[j]; q.ext_cv[j] = t.ext_cv[j];
            q.ext_sin_v[j] = t.ext_sin_v[j]; q.ext_cosy_v[j] = t.ext_cosy_v[j];
        }
        q.ext = b.ext;
        RC(launch_init_grid(q, c->stream));
        c->static_dirty = true;
        if (c->topo.empty()) {
            RC(launch_fill_field(b.g, b.f<double>(OCN_HHQ_REST), 100.0, c->stream));   // init_data.f90:112-114
        } else {
            const long pts = (long)(b.g.bnd_x2 - b.g.bnd_x1 + 1) * (b.g.bnd_y2 - b.g.bnd_y1 + 1);
            hipLaunchKernelGGL(k_topography, dim3((unsigned)((pts + 255) / 256)), dim3(256), 0, c->stream, b.g,
                               b.f<double>(OCN_HHQ_REST), b.f<float>(OCN_LU), (const float *)(scratch + topo_at), bs.nx - 4);
            RC(check_launch());
        }
        RC(launch_gaussian(b.g, b.f<double>(OCN_SSH), b.f<float>(OCN_LU), bs.nx / 2, bs.ny / 2, 1.0, c->stream));
    }
    if (!c->topo.empty()) RC(run_sync(c, {OCN_HHQ_REST}));   // init_data.f90:119
    RC(run_sync(c, {OCN_SSH}));                               // envoke_gaussian_elimination's sync
    for (const LBlock &b : c->blocks) {                       // sshn = ssh, sshp = ssh (whole arrays)
        const size_t bytes = (size_t)b.g.pitch * (b.g.bnd_y2 - b.g.bnd_y1 + 1) * 8;
        HIPCHK(hipMemcpyAsync(b.ptr[field_slot(OCN_SSHN)], b.ptr[field_slot(OCN_SSH)], bytes,
                              hipMemcpyDeviceToDevice, c->stream));
        HIPCHK(hipMemcpyAsync(b.ptr[field_slot(OCN_SSHP)], b.ptr[field_slot(OCN_SSH)], bytes,
                              hipMemcpyDeviceToDevice, c->stream));
    }
    RC(envoke(c, OCN_STAGE_HH_INIT, 0.0));                    // init_data.f90:60-63
    for (const LBlock &b : c->blocks) {                       // u = v = 0, mu = lvisc_2 then 0 (:67-77)
        const long n = (long)b.g.pitch * (b.g.bnd_y2 - b.g.bnd_y1 + 1);
        for (int id : {OCN_UBRTR, OCN_UBRTRN, OCN_UBRTRP, OCN_VBRTR, OCN_VBRTRN, OCN_VBRTRP, OCN_MU}) {
            hipLaunchKernelGGL(k_fill_r8, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, c->stream,
                               b.f<double>(id), n, 0.0);
            RC(check_launch());
        }
    }
    if (c->sw.use_tracers > 0) {                              // init_data.f90:80-90
        for (int k = 1; k <= c->sw.tracer_num; ++k) {
            for (const LBlock &b : c->blocks)
                RC(launch_gaussian(b.g, b.f<double>(OCN_FF1(k)), b.f<float>(OCN_LU), bs.nx / 2, bs.ny / 2, 0.5,
                                   c->stream));
            RC(run_sync(c, {OCN_FF1(k)}));
            for (const LBlock &b : c->blocks) {
                const size_t bytes = (size_t)b.g.pitch * (b.g.bnd_y2 - b.g.bnd_y1 + 1) * 8;
                HIPCHK(hipMemcpyAsync(b.ptr[field_slot(OCN_FF1N(k))], b.ptr[field_slot(OCN_FF1(k))], bytes,
                                      hipMemcpyDeviceToDevice, c->stream));
                HIPCHK(hipMemcpyAsync(b.ptr[field_slot(OCN_FF1P(k))], b.ptr[field_slot(OCN_FF1(k))], bytes,
                                      hipMemcpyDeviceToDevice, c->stream));
            }
        }
        for (const LBlock &b : c->blocks) {
            const long n = (long)b.g.pitch * (b.g.bnd_y2 - b.g.bnd_y1 + 1);
            for (int id : {OCN_FLUX_X, OCN_FLUX_Y}) {
                hipLaunchKernelGGL(k_fill_r8, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, c->stream,
                                   b.f<double>(id), n, 0.0);
                RC(check_launch());
            }
        }
    }
    HIPCHK(hipStreamSynchronize(c->stream));
    c->initialized = true;
    c->ext_ok = true;   // the real(4) fields are init_state's: the ext rows are the neighbours' metric rows
    c->hrx_ok = false;
    return OCN_OK;
}

}  // namespace ocn

static void set_mask(ocn_ctx *c, const int32_t *mask)
{
    const ocn_basin *basin = &c->basin;
    const size_t nxy = (size_t)basin->nx * basin->ny;
    c->mask.assign(nxy, 0);
    if (mask) {
        std::memcpy(c->mask.data(), mask, nxy * sizeof(int32_t));
    } else {   // tools/io.f90:49-59: closed box with a 2-cell land frame
        for (int n = 1; n <= basin->ny; ++n)
            for (int m = 1; m <= basin->nx; ++m)
                c->mask[(size_t)(m - 1) + (size_t)(n - 1) * basin->nx] =
                    (m < 3 || m > basin->nx - 2 || n < 3 || n > basin->ny - 2) ? 1 : 0;
    }
}

// ================================================================== C ABI (PSy layer)
extern "C" {

const char *ocn_last_error(void) { return g_last_error.c_str(); }
int ocn_abi_version(void) { return OCN_ABI_VERSION; }
#ifndef OCN_BUILD_ID
#define OCN_BUILD_ID "unknown"
#endif
const char *ocn_build_id(void) { return OCN_BUILD_ID; }
int64_t ocn_launch_count(void) { return (int64_t)g_launches.load(std::memory_order_relaxed); }

int ocn_ctx_create(const ocn_basin *basin, const ocn_sw_params *sw, const ocn_decomp *dec, const int32_t *mask,
                   ocn_ctx **out)
{
    if (!basin || !sw || !dec || !out) return set_error(OCN_ERR_ARG, "null argument");
    if (basin->nx < 5 || basin->ny < 5) return set_error(OCN_ERR_ARG, "nx, ny must be >= 5");
    if (dec->bnx < 1 || dec->bny < 1 || dec->nranks < 1 || dec->rank < 0 || dec->rank >= dec->nranks)
        return set_error(OCN_ERR_ARG, "bad decomposition request");
    if (sw->use_tracers > 0 && (sw->tracer_num < 1 || sw->tracer_num > kMaxTracers))
        return set_error(OCN_ERR_ARG, "tracer_num must be 1.." + std::to_string(kMaxTracers));
    ocn_ctx *c = new ocn_ctx();
    c->basin = *basin; c->sw = *sw; c->dec = *dec;
    c->bnx = dec->bnx; c->bny = dec->bny;
    set_mask(c, mask);
    int rc = check_hip(hipSetDevice(dec->device), "hipSetDevice");
    if (!rc) rc = check_hip(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking), "hipStreamCreate");
    // the comm stream at the highest priority: the side chains' short frame launches and the
    // exchanges take wave slots as they free up instead of queueing behind the inner marches
    if (!rc) {
        int lo = 0, hi = 0;
        rc = check_hip(hipDeviceGetStreamPriorityRange(&lo, &hi), "hipDeviceGetStreamPriorityRange");
        if (!rc)
            rc = check_hip(hipStreamCreateWithPriority(&c->comm_stream, hipStreamNonBlocking, OCN_COMM_PRIO ? hi : lo),
                           "hipStreamCreateWithPriority");
    }
    if (!rc) rc = check_hip(hipEventCreateWithFlags(&c->ev_fork, hipEventDisableTiming), "hipEventCreate");
    if (!rc) rc = check_hip(hipEventCreateWithFlags(&c->ev_join, hipEventDisableTiming), "hipEventCreate");
    if (!rc) rc = check_hip(hipEventCreateWithFlags(&c->ev_fb, hipEventDisableTiming), "hipEventCreate");
    if (!rc) rc = check_hip(hipHostMalloc((void **)&c->h_fbz, sizeof(int32_t), hipHostMallocDefault), "hipHostMalloc");
    if (!rc) rc = decompose(c);
    if (!rc) rc = allocate(c);
    if (!rc) rc = prebuild_plans(c);
    if (!rc) rc = check_hip(hipStreamSynchronize(c->stream), "hipStreamSynchronize");
    if (rc) { ocn_ctx_destroy(c); return rc; }
    *out = c;
    return OCN_OK;
}

// host-only context (decomposition only, no device) for the query entry points
static int host_ctx(const ocn_basin *basin, const ocn_decomp *dec, const int32_t *mask, ocn_ctx *&c)
{
    if (!basin || !dec) return set_error(OCN_ERR_ARG, "null argument");
    if (basin->nx < 5 || basin->ny < 5) return set_error(OCN_ERR_ARG, "nx, ny must be >= 5");
    if (dec->bnx < 1 || dec->bny < 1 || dec->nranks < 1 || dec->rank < 0 || dec->rank >= dec->nranks)
        return set_error(OCN_ERR_ARG, "bad decomposition request");
    c = new ocn_ctx();
    c->basin = *basin; c->dec = *dec; c->bnx = dec->bnx; c->bny = dec->bny;
    set_mask(c, mask);
    const int rc = decompose(c);
    if (rc) { delete c; c = nullptr; }
    return rc;
}

int ocn_decompose(const ocn_basin *basin, const ocn_decomp *dec, const int32_t *mask, ocn_block_info *out,
                  int32_t cap, int32_t *count)
{
    ocn_ctx *c = nullptr;
    RC(host_ctx(basin, dec, mask, c));
    const int n = (int)c->blocks.size();
    if (count) *count = n;
    for (int k = 0; k < n && k < cap && out; ++k) {
        const LBlock &b = c->blocks[k];
        out[k].geom = b.g; out[k].bm = b.bm; out[k].bn = b.bn;
        for (int d = 0; d < 8; ++d) { out[k].nbr_rank[d] = b.nbr_rank[d]; out[k].nbr_k[d] = b.nbr_k[d]; }
    }
    delete c;
    return OCN_OK;
}

int ocn_halo_schedule(const ocn_basin *basin, const ocn_decomp *dec, const int32_t *mask, const int32_t *field_ids,
                      int32_t nfields, ocn_halo_msg *out, int32_t cap, int32_t *count)
{
    if (!field_ids || nfields < 1) return set_error(OCN_ERR_ARG, "no fields");
    std::vector<int> fields(field_ids, field_ids + nfields);
    for (int id : fields)
        if (id < OCN_SSH || id >= OCN_TRACER_BASE + 3 * kMaxTracers)
            return set_error(OCN_ERR_ARG, "halo exchange is defined for real(8) fields");
    ocn_ctx *c = nullptr;
    RC(host_ctx(basin, dec, mask, c));
    std::vector<PlanEntry> es;
    const int rc = plan_entries(c, fields, es);
    delete c;
    RC(rc);
    if (count) *count = (int32_t)es.size();
    for (size_t i = 0; i < es.size() && (int32_t)i < cap && out; ++i) {
        const PlanEntry &e = es[i];
        ocn_halo_msg &o = out[i];
        o.kind = e.kind; o.peer = e.peer; o.k = e.k; o.k_src = e.ks; o.field = e.field;
        o.dst_x0 = e.dst.x0; o.dst_x1 = e.dst.x1; o.dst_y0 = e.dst.y0; o.dst_y1 = e.dst.y1;
        o.src_x0 = e.src.x0; o.src_x1 = e.src.x1; o.src_y0 = e.src.y0; o.src_y1 = e.src.y1;
        o.offset = e.buf_off; o.count = e.count;
    }
    return OCN_OK;
}

int ocn_ctx_destroy(ocn_ctx *c)
{
    if (!c) return OCN_OK;
    if (c->wd.joinable()) {   // the watchdog first: nothing is watched from here on
        {
            std::lock_guard<std::mutex> g(c->wd_mu);
            c->wd_stop = true;
            c->wd_cv.notify_all();
        }
        c->wd.join();
    }
    (void)hipSetDevice(c->dec.device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    for (auto &g : c->graphs) (void)hipGraphExecDestroy(g.exec);
    for (auto &r : c->recs) { (void)hipEventDestroy(r.a); (void)hipEventDestroy(r.b); }
    for (hipEvent_t e : c->event_pool) (void)hipEventDestroy(e);
    if (c->comm && !c->comm_abort_done) ncclCommDestroy(c->comm);
    for (auto &x : c->xq) (void)hipEventDestroy(x.second);
    for (hipEvent_t e : c->xpool) (void)hipEventDestroy(e);
    if (c->lb) {
        Loopback *L = c->lb;
        bool last;
        {
            std::lock_guard<std::mutex> g(L->mu);
            L->ctx[c->dec.rank] = nullptr;   // a rank still waiting for this one fails (lb_meet)
            last = --L->refs == 0;
            L->cv.notify_all();
        }
        if (last) delete L;
    }
    if (c->lb_ev_a) (void)hipEventDestroy(c->lb_ev_a);
    if (c->lb_ev_b) (void)hipEventDestroy(c->lb_ev_b);
    for (void *p : c->allocs) (void)hipFree(p);
    if (c->comm_stream) (void)hipStreamSynchronize(c->comm_stream);
    if (c->ev_fork) (void)hipEventDestroy(c->ev_fork);
    for (hipEvent_t e : c->ov_ev)
        if (e) (void)hipEventDestroy(e);
    if (c->ev_join) (void)hipEventDestroy(c->ev_join);
    if (c->ev_fb) (void)hipEventDestroy(c->ev_fb);
    if (c->h_fbz) (void)hipHostFree(c->h_fbz);
    if (c->comm_stream) (void)hipStreamDestroy(c->comm_stream);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
    return OCN_OK;
}

int ocn_ctx_block_count(const ocn_ctx *c) { return c ? (int)c->blocks.size() : -1; }

int ocn_ctx_block_info(const ocn_ctx *c, int k, ocn_block_info *out)
{
    if (!c || !out || k < 0 || k >= (int)c->blocks.size()) return set_error(OCN_ERR_ARG, "bad block index");
    const LBlock &b = c->blocks[k];
    out->geom = b.g;
    out->bm = b.bm; out->bn = b.bn;
    for (int d = 0; d < 8; ++d) { out->nbr_rank[d] = b.nbr_rank[d]; out->nbr_k[d] = b.nbr_k[d]; }
    return OCN_OK;
}

static int alt_home(ocn_ctx *c);
static int complete_open(ocn_ctx *c);
void *ocn_ctx_field(const ocn_ctx *c, int k, int id)
{
    if (!c || k < 0 || k >= (int)c->blocks.size() || !has_field(c, id)) {
        set_error(OCN_ERR_ARG, "bad block index or field id");
        return nullptr;
    }
    ocn_ctx *w = const_cast<ocn_ctx *>(c);
    if (complete_open(w) != OCN_OK) return nullptr;   // the arrays hold what the reference leaves
    if (is_r4(id)) { c->r4_escaped = true; c->ext_ok = false; }   // may be written behind our back: no compact tables
    // a raw r8 pointer names the field's own buffer from now on (step_impl returns the current
    // values there at the end of every call)
    if (!is_r4(id) && alt_home(w) != OCN_OK) return nullptr;
    if (is_flip_field(id)) { c->r8_escaped = true; c->coherent_known = false; }
    if (is_alt_field(id)) c->alt_ok = false;
    if (is_tracer_field(id)) c->tr_alt_ok = false;
    if (!is_r4(id)) { c->r8_handed = true; c->hh_consistent = false; c->fb_state = kFbUnchecked; c->hrx_ok = false; }
    c->hn_fresh = false;
    if (is_alt_field(id) || id == OCN_HHQ_REST || id == OCN_MU) { c->r8_escaped = true; c->coherent_known = false; }
    return c->blocks[k].ptr[field_slot(id)];
}

void *ocn_ctx_stream(const ocn_ctx *c) { return c ? (void *)c->stream : nullptr; }

int ocn_comm_unique_id(void *out_id, int32_t nbytes)
{
    if (!out_id || nbytes < (int32_t)sizeof(ncclUniqueId)) return set_error(OCN_ERR_ARG, "buffer < 128 bytes");
    ncclUniqueId id;
    RC(nccl_rc(ncclGetUniqueId(&id), "ncclGetUniqueId"));
    std::memcpy(out_id, &id, sizeof(id));
    return OCN_OK;
}

int ocn_ctx_attach_comm(ocn_ctx *c, const void *unique_id, int32_t nbytes)
{
    if (!c || !unique_id || nbytes < (int32_t)sizeof(ncclUniqueId)) return set_error(OCN_ERR_ARG, "bad unique id");
    HIPCHK(hipSetDevice(c->dec.device));
    ncclUniqueId id;
    std::memcpy(&id, unique_id, sizeof(id));
    if (c->comm) return set_error(OCN_ERR_STATE, "a communicator is attached already");
    RC(nccl_rc(ncclCommInitRank(&c->comm, c->dec.nranks, id, c->dec.rank), "ncclCommInitRank"));
    c->comm_aborted = false;
    return OCN_OK;
}

int ocn_ctx_attach_loopback(ocn_ctx *const *ctxs, int32_t n)
{
    if (!ctxs || n < 1 || n > 64) return set_error(OCN_ERR_ARG, "loopback: 1..64 contexts");
    for (int i = 0; i < n; ++i) {
        const ocn_ctx *c = ctxs[i];
        if (!c || c->dec.nranks != n || c->dec.rank != i || c->dec.device != ctxs[0]->dec.device)
            return set_error(OCN_ERR_ARG, "loopback: context i must be rank i of nranks = n, all on one device");
        if (c->comm || c->lb || c->initialized)
            return set_error(OCN_ERR_STATE, "loopback: attach before ocn_ctx_init_state, once, without RCCL");
    }
    Loopback *L = new Loopback();
    L->n = n;
    L->ctx.assign(ctxs, ctxs + n);
    for (auto &v : L->cnt) v.assign((size_t)n, 0);
    L->plan.assign((size_t)n, nullptr);
    L->vote.assign((size_t)n, nullptr);
    L->refs = n;
    int rc = OCN_OK;
    for (int i = 0; i < n && !rc; ++i) {
        ocn_ctx *c = ctxs[i];
        rc = check_hip(hipSetDevice(c->dec.device), "hipSetDevice");
        if (!rc) rc = check_hip(hipEventCreateWithFlags(&c->lb_ev_a, hipEventDisableTiming), "hipEventCreate");
        if (!rc) rc = check_hip(hipEventCreateWithFlags(&c->lb_ev_b, hipEventDisableTiming), "hipEventCreate");
    }
    if (rc) { delete L; return rc; }
    for (int i = 0; i < n; ++i) ctxs[i]->lb = L;
    return OCN_OK;
}

int ocn_ctx_overlap_info(ocn_ctx *c, ocn_overlap_info *out)
{
    if (!c || !out) return set_error(OCN_ERR_ARG, "null argument");
    *out = ocn_overlap_info{};
    out->level = overlap_level(c);
    out->state = c->ov_state;
    out->kind = c->ov_kind;
    out->seq_ms = c->ov_ms[0];
    out->overlapped_ms = c->ov_ms[1];
    return OCN_OK;
}

int ocn_ctx_clock_info(ocn_ctx *c, int32_t reset, ocn_clock_info *out)
{
    if (!c || !out) return set_error(OCN_ERR_ARG, "null argument");
    *out = ocn_clock_info{};
    HIPCHK(hipSetDevice(c->dec.device));
    HIPCHK(hipStreamSynchronize(c->stream));
    unsigned long long v[3] = {0, 0, 0};
    RC(clock_read(reset != 0, v));
    out->launches = (int64_t)v[2];
    out->clock_ghz = v[1] ? (double)v[0] / ((double)v[1] * 10.0) : 0.0;
    out->sampled_ms = (double)v[1] * 1e-5;
    return OCN_OK;
}

int ocn_ctx_comm_info(ocn_ctx *c, ocn_comm_info *out)
{
    if (!c || !out) return set_error(OCN_ERR_ARG, "null argument");
    *out = ocn_comm_info{};
    out->comm_size = 1;
    if (c->lb) {
        out->transport = 2;
        out->comm_size = c->lb->n;
        out->comm_rank = c->dec.rank;
    } else if (c->comm || c->comm_aborted) {
        out->transport = 1;
        int v = 0, n = 0, r = 0;
        if (ncclGetVersion(&v) == ncclSuccess) out->nccl_version = v;
        std::lock_guard<std::mutex> g(c->comm_mu);
        if (c->comm && !c->comm_abort_done && ncclCommCount(c->comm, &n) == ncclSuccess &&
            ncclCommUserRank(c->comm, &r) == ncclSuccess) {
            out->comm_size = n;
            out->comm_rank = r;
        } else {
            out->comm_size = c->dec.nranks;
            out->comm_rank = c->dec.rank;
        }
    }
    out->exchanges = c->xchg;
    out->exchanges_done = c->wd_s > 0 ? poll_xdone(c) : -1;
    out->watchdog_s = c->wd_s;
    return OCN_OK;
}

int ocn_ctx_set_watchdog(ocn_ctx *c, double seconds)
{
    if (!c || !(seconds >= 0)) return set_error(OCN_ERR_ARG, "watchdog: null ctx or seconds < 0");
    {
        std::lock_guard<std::mutex> g(c->wd_mu);
        c->wd_s = seconds;
        c->call_t0 = std::chrono::steady_clock::now();   // (a call under way is timed from now)
    }
    if (seconds > 0 && !c->wd.joinable()) c->wd = std::thread(wd_loop, c);
    return OCN_OK;
}

int ocn_ctx_set_topography(ocn_ctx *c, const float *h, int64_t count)
{
    if (!c) return set_error(OCN_ERR_ARG, "null ctx");
    if (!h) { c->topo.clear(); return OCN_OK; }
    const int64_t n = (int64_t)(c->basin.nx - 4) * (c->basin.ny - 4);
    if (count != n) return set_error(OCN_ERR_ARG, "topography: (nx-4)*(ny-4) values expected");
    c->topo.assign(h, h + n);
    return OCN_OK;
}

static int init_state_entry(ocn_ctx *c)
{
    if (!c) return set_error(OCN_ERR_ARG, "null ctx");
    HIPCHK(hipSetDevice(c->dec.device));
    c->open = false;   // a pending call tail is void: every field is formed again
    c->open_pair = false;
    c->deferred = 0;
    c->ring2_saved = false;   // (a saved second ring of an x2 sequence is void: init forms it again)
    c->tr_pending = false;
    c->coherent_known = false;
    c->alt_ok = false; c->tr_alt_ok = false;
    c->hn_fresh = false;
    c->fb_state = kFbUnchecked;
    // a multi-step launch's barrier timeout not yet reported is void too: the state is formed again
    if (c->d_nbad) HIPCHK(hipMemsetAsync(c->d_nbad + 61, 0, sizeof(int32_t), c->stream));
    const int rc = fail_fatal(c, init_state(c));
    c->hh_consistent = rc == OCN_OK && !c->r8_handed;   // init_data.f90:60-63 ran hh_init last
    c->hn_fresh = c->hh_consistent && !c->r4_escaped;    // (every level: the n one from h_r)
    return rc;
}

int ocn_ctx_init_state(ocn_ctx *c)
{
    if (!c) return set_error(OCN_ERR_ARG, "null ctx");
    return guarded(c, "ocn_ctx_init_state", [&] { return init_state_entry(c); });
}

static int sync_entry(ocn_ctx *c, int field_id)
{
    if (!c || !has_r8(c, field_id)) return set_error(OCN_ERR_ARG, "sync: bad ctx or non-real(8) field");
    HIPCHK(hipSetDevice(c->dec.device));
    HaloPlan *p;
    RC(get_plan(c, {field_id}, p));
    // no neighbour block anywhere (one block, no other rank): the exchange writes nothing, so
    // nothing the step decisions rest on changes and a pending call tail may stay pending -- a
    // PSy-style caller syncing between 1-step calls pays no re-check, host wait or tail for it
    if (!p->local.n && p->peers.empty()) return OCN_OK;
    RC(complete_open(c));
    c->coherent_known = false;
    c->hh_consistent = false;
    c->hn_fresh = false;
    c->fb_state = kFbUnchecked;
    if (field_id == OCN_HHQ_REST) c->hrx_ok = false;
    // the current buffer's halos change; the one-pass steps' second buffer must be copied again
    if (is_alt_field(field_id)) c->alt_ok = false;
    if (is_tracer_field(field_id)) c->tr_alt_ok = false;
    return run_sync(c, {field_id});
}

int ocn_ctx_sync(ocn_ctx *c, int field_id)
{
    if (!c) return set_error(OCN_ERR_ARG, "null ctx");
    return guarded(c, "ocn_ctx_sync", [&] { return sync_entry(c, field_id); });
}

static int stage_entry(ocn_ctx *c, int stage_id, double tau)
{
    if (!c) return set_error(OCN_ERR_ARG, "null ctx");
    HIPCHK(hipSetDevice(c->dec.device));
    if (stage_id < 0 || stage_id >= OCN_NUM_STAGES) return set_error(OCN_ERR_ARG, "bad stage id");
    RC(complete_open(c));
    c->coherent_known = false;
    c->alt_ok = false; c->tr_alt_ok = false;
    c->hh_consistent = false;
    c->hn_fresh = false;
    c->fb_state = kFbUnchecked;
    RC(prepare_static(c));
    return envoke(c, stage_id, tau);
}

int ocn_ctx_stage(ocn_ctx *c, int stage_id, double tau)
{
    if (!c) return set_error(OCN_ERR_ARG, "null ctx");
    return guarded(c, "ocn_ctx_stage", [&] { return stage_entry(c, stage_id, tau); });
}

static void drop_graphs(ocn_ctx *c)
{
    for (auto &g : c->graphs) (void)hipGraphExecDestroy(g.exec);
    c->graphs.clear();
}

// one model step (model.f90:146-160): expl_shallow_water, then expl_tracer
static int run_step(ocn_ctx *c, double tau, const StepKind &k)
{
    if (c->tr_forked) {   // a tracer step forked beside the previous step's march (one_step_x2)
        RC(join_sync(c));
        c->tr_forked = false;
    }
    // tracer steps (OCN_OPT_TRACER_STEP): a one-pass step's tracer step runs with the next step; the
    // pending one of the state a single-block one-pass step reads runs before its march (x2 steps
    // and the last step: after their exchanges, one_step_x2 / one_step_fused)
    if (c->tr_call && k.one && !k.x2) RC(run_tracer_step(c, tau));
    if (!c->fused) c->hn_fresh = false;   // (the reference's stages)
    RC(c->fused ? one_step_fused(c, tau, k) : one_step(c, tau, k.check));
    if (c->tr_call && k.one) {
        c->tr_pending = true;
        return OCN_OK;
    }
    return expl_tracer(c, tau, c->compact);
}

// one step as a replayed hipGraph, captured once per (tau, step kind, compact, role, one-pass
// variant); a role-flip step swaps the host's pointer roles as the captured launches did.  The
// known-constant variant's constants and the device check's verdict are read from device memory
// by the launches, so a replay sees their current values.
static int graph_step(ocn_ctx *c, double tau, const StepKind &k)
{
    c->hn_fresh = false;   // (a replay runs whatever the captured step ran)
    for (const auto &g : c->graphs)
        if (g.tau == tau && g.kind == k && g.compact == c->compact && g.march == c->march && g.ring_sea == c->ring_sea &&
            g.role == c->role && g.kc_mode == c->kc_mode) {
            HIPCHK(hipGraphLaunch(g.exec, c->stream));
            if (k.rc) swap_sshp(c);
            if (k.one || k.one_last) swap_alt3(c);
            if (k.flip || k.one_last) swap_roles(c);
            return OCN_OK;
        }
    if (c->graphs.size() >= 16) drop_graphs(c);
    const int role = c->role;
    hipGraph_t graph;
    HIPCHK(hipStreamBeginCapture(c->stream, hipStreamCaptureModeThreadLocal));
    c->capturing = true;
    int rc = run_step(c, tau, k);
    c->capturing = false;
    hipError_t e = hipStreamEndCapture(c->stream, &graph);
    if (rc) return rc;
    HIPCHK(e);
    hipGraphExec_t exec;
    e = hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0);
    (void)hipGraphDestroy(graph);
    HIPCHK(e);
    c->graphs.push_back(ocn_ctx::Graph{exec, tau, k, c->compact, c->march, c->ring_sea, role, c->kc_mode});
    HIPCHK(hipGraphLaunch(exec, c->stream));
    return OCN_OK;
}

static int tracer_stage_entry(ocn_ctx *c, int stage_id, int tracer, double tau)
{
    if (!c) return set_error(OCN_ERR_ARG, "null ctx");
    HIPCHK(hipSetDevice(c->dec.device));
    if (c->sw.use_tracers <= 0 || tracer < 1 || tracer > c->sw.tracer_num)
        return set_error(OCN_ERR_ARG, "no such tracer (use_tracers / tracer_num)");
    if (stage_id < 0 || stage_id >= OCN_NUM_TSTAGES) return set_error(OCN_ERR_ARG, "bad tracer stage id");
    RC(complete_open(c));
    return tracer_stage(c, stage_id, tracer, tau, false);
}

int ocn_ctx_tracer_stage(ocn_ctx *c, int stage_id, int tracer, double tau)
{
    if (!c) return set_error(OCN_ERR_ARG, "null ctx");
    return guarded(c, "ocn_ctx_tracer_stage", [&] { return tracer_stage_entry(c, stage_id, tracer, tau); });
}

// the current sshp / ubrtrp / vbrtrp (in the second buffers after one-pass steps: role bit 4)
// back into the fields' own buffers, stream-ordered
static int alt_home(ocn_ctx *c)
{
    if (!(c->role & 4)) return OCN_OK;
    for (LBlock &b : c->blocks)
        for (const auto &pr : {std::make_pair(&b.sshp_alt, OCN_SSHP), std::make_pair(&b.up_alt, OCN_UBRTRP),
                               std::make_pair(&b.vp_alt, OCN_VBRTRP)})
            HIPCHK(hipMemcpyAsync(*pr.first, b.ptr[field_slot(pr.second)], field_bytes(b), hipMemcpyDeviceToDevice,
                                  c->stream));
    swap_alt3(c);
    return OCN_OK;
}

// The stream has been synchronised by the caller: read a pending device verdict of the
// known-constant check, so that later calls launch only the variant it selected.
static void learn_fb(ocn_ctx *c)
{
    if (c->fb_state != kFbDevice) return;
    int32_t f = 0;
    if (hipMemcpy(&f, c->d_fbz, sizeof(f), hipMemcpyDeviceToHost) != hipSuccess) return;
    c->fb_state = f == 0 ? kFbZero : f == 1 ? kFbHr : kFbGeneral;
    c->fb_copy = false;
}

// Without a synchronising call: the verdict's copy (prepare_kc) has arrived if its event has
// completed -- a query, never a wait -- so a caller of 1-step calls gets the host-chosen variant
// (and pair launches) a few calls after the check.
static void learn_fb_async(ocn_ctx *c)
{
    if (c->fb_state != kFbDevice || !c->fb_copy || hipEventQuery(c->ev_fb) != hipSuccess) return;
    const int32_t f = *(volatile int32_t *)c->h_fbz;
    c->fb_state = f == 0 ? kFbZero : f == 1 ? kFbHr : kFbGeneral;
    c->fb_copy = false;
}

// The one-pass variant of this call (OCN_KC_*): the known-constant one only when its precondition
// is known to hold; a raw r8 pointer in the caller's hands (r8_handed) may change the arrays at any
// time, so then always the general one (a check per call would cost a pass over 12 arrays);
// unchecked: the check runs on the stream and both variants are launched (the device picks) --
// no host wait inside a step.
// x2: for one_step_x2 (the whole interior; the halo points neighbours own are no fallback points;
// h_r with the neighbours' second ring).  A verdict for that range also holds for the hybrid
// steps' inner range (its points and their +-2 neighbourhood lie inside what it covered, with the
// same values there), not the other way round.
static int kc_of_fb(const ocn_ctx *c)
{
    return c->fb_state == kFbZero ? OCN_KC_KNOWN : c->fb_state == kFbHr ? OCN_KC_KNOWN_HR
         : c->fb_state == kFbGeneral ? OCN_KC_GENERAL : OCN_KC_DEVICE;
}
static int prepare_kc(ocn_ctx *c, bool x2 = false)
{
    if (!c->known_const || c->r8_handed) { c->kc_mode = OCN_KC_GENERAL; return OCN_OK; }
    learn_fb_async(c);
    if (c->fb_state != kFbUnchecked && x2 && !c->fb_x2) c->fb_state = kFbUnchecked;
    if (c->fb_state == kFbUnchecked) {
        HIPCHK(hipMemsetAsync(c->d_fbz, 0, sizeof(int32_t), c->stream));
        for (const LBlock &b : c->blocks) {
            std::vector<void *> tab = b.ptr;
            if (x2) tab[field_slot(OCN_HHQ_REST)] = b.hr_x;
            const Range r = x2 ? Range{b.g.nx_start, b.g.nx_end, b.g.ny_start, b.g.ny_end} : onepass_inner(b, 1);
            RC(launch_fallback_check(&b.g, tab.data(), b.bits, r, c->d_fbz, b.kc, c->stream, x2 ? b.own : 0u));
        }
        if (!c->capturing) {   // the verdict to pinned host memory, learn_fb_async
            HIPCHK(hipMemcpyAsync(c->h_fbz, c->d_fbz, sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
            HIPCHK(hipEventRecord(c->ev_fb, c->stream));
            c->fb_copy = true;
        }
        c->fb_state = kFbDevice;
        c->fb_x2 = x2;
    }
    c->kc_mode = kc_of_fb(c);
    return OCN_OK;
}

// The end of a call that leaves no step pending: nothing stays in flight, the pairs' roles return
// (the last step left both buffers of each pair equal), the recompute steps' sshp comes home
static int finish_call(ocn_ctx *c, int rc)
{
    if (const int rj = join_sync(c); rc == OCN_OK) rc = rj;
    // a failed call drops its sequence: a saved second halo ring (x2 steps) must not be restored
    // over what the host uploads or init_state forms next
    if (rc != OCN_OK) c->ring2_saved = false;
    if (c->role & 1) swap_roles(c);
    if (c->role & 2) {   // sshp's buffers are not equal: the current one is copied into the field's own buffer
        for (LBlock &b : c->blocks)
            HIPCHK(hipMemcpyAsync(b.sshp_alt, b.ptr[field_slot(OCN_SSHP)], field_bytes(b), hipMemcpyDeviceToDevice,
                                  c->stream));
        swap_sshp(c);
    }
    // one-pass steps: sshp / ubrtrp / vbrtrp stay in the second buffers (every access goes through
    // the field table) unless a raw r8 pointer was handed out: then back into the fields' buffers
    if ((c->role & 4) && c->r8_handed) RC(alt_home(c));
    // tracer steps: the last step's standard tracer stages leave ff1 = ff1n everywhere (tracer_next_step's
    // ff := ffn where tran_diff_tracer wrote ffn and its exchange delivered it, both untouched elsewhere):
    // the roles return with no copy; the current ff1p is copied into the field's own buffer
    if (c->role & 8) swap_tracer_roles(c);
    if (c->role & 16) {
        for (LBlock &b : c->blocks)
            for (int t = 1; t <= c->sw.tracer_num; ++t)
                HIPCHK(hipMemcpyAsync(b.ffp_alt[(size_t)t - 1], b.ptr[field_slot(OCN_FF1P(t))], field_bytes(b),
                                      hipMemcpyDeviceToDevice, c->stream));
        swap_tracer_alt(c);
    }
    c->tr_pending = false;
    c->hh_consistent = rc == OCN_OK && !c->r8_handed;   // the last step ran a full hh_init
    return rc;
}

// Lazy call tail possible: single process (a tail formed on one rank only would unbalance the
// exchanges), no raw r8 pointers handed out, no tracers (expl_tracer reads hh_init's arrays after
// every step), and the one-pass step as one launch per block (no exchange, no a8 / a9 work on the
// halo ring: the redone step must find the previous state intact).
static bool lazy_allowed(const ocn_ctx *c, bool x2)
{
    return c->lazy && !has_comm(c) && !c->r8_handed && (c->sw.use_tracers <= 0 || c->tr_step) &&
           (x2 || (!c->ring_sea && !has_exchange(c)));
}

// one_step_x2's static conditions on this rank (the device checks come from check_coherence):
// halo exchanges to do, the compact tables with the ext rows, no a8 / a9 work on a ring no neighbour
// fills, every block of the grid at least 2 x 2 (its 2-deep strips lie in its interior)
static bool x2_local(const ocn_ctx *c)
{
    if (!c->x2 || !c->compact || !c->rows_x_ok || c->edge_ring_sea || !has_exchange(c))
        return false;
    for (const GBlock &g : c->gblocks)
        if (g.rank >= 0 && (g.g.nx_end - g.g.nx_start < 1 || g.g.ny_end - g.g.ny_start < 1)) return false;
    return true;
}

// one_step_x4's static conditions on this rank (with x2_local's): its tables, no tracers (expl_tracer
// after every step), the known-constant variant allowed, every block of the grid at least 4 x 4 (its
// 4-deep strips lie in its interior) and row padding for the extra rings
static bool x4_local(const ocn_ctx *c)
{
    // (tracer runs: with the tracer steps, one_step_x4 runs them -- by default only where exchanges go to
    // other ranks: a pair's second tracer step is one more launch after it, which with only local copies
    // costs more than the exchange it saves -- C5 layout on one GPU 0.0281 (x2) vs 0.0338 ms per step,
    // profiles/r06a; over RCCL each exchange is a group's latency)
    if (!c->x4 || !c->x4_tab_ok || !c->known_const || c->r8_handed || (c->sw.use_tracers > 0 && !c->tr_step) ||
        !c->march)
        return false;
    if (c->sw.use_tracers > 0 && c->x4 < 3 && !(has_comm(c) && c->dec.nranks > 1)) return false;
    for (const GBlock &g : c->gblocks)
        if (g.rank >= 0 && (g.g.nx_end - g.g.nx_start < 3 || g.g.ny_end - g.g.ny_start < 3)) return false;
    for (const LBlock &b : c->blocks)
        if (b.g.pitch < (int64_t)(b.g.bnd_x2 - b.g.bnd_x1 + 1 + 2 * kXRing)) return false;
    return true;
}
// pairs of x2 steps in this call (after prepare_kc): x4_local on every rank (the vote) or this one
// (one process), the known-constant variant chosen on the host
static bool x4_now(const ocn_ctx *c)
{
    return (c->kc_mode == OCN_KC_KNOWN || c->kc_mode == OCN_KC_KNOWN_HR) &&
           (has_comm(c) ? c->x4_dev_ok : x4_local(c) && c->fb_x2);
}

// The first call of a sequence long enough for pairs, right after prepare_kc issued the known-
// constant check: wait for the check's verdict (one host wait per check -- the check's pass over
// the fields and a 4-byte copy, behind whatever the stream holds) so that the call's steps run as
// pairs of the host-chosen variant instead of single launches of both variants with the device
// picking (4096^2: 0.39 ms per single step against 0.28-0.30 ms per step in pairs; the single
// steps' HBM traffic also pulls the shader clock down, 2.25 -> 1.55 GHz over 5 ms, and the pairs'
// clock climbs back over ~30 ms: profiles/r06/clock_*.txt).  Not while a graph is captured (no
// host wait there), not with a communicator (the ranks' votes carry the verdicts), not for calls
// of 1-3 steps (no pair before their deferred last steps).
static int await_kc(ocn_ctx *c, bool x2, int nsteps)
{
    if (c->kc_mode != OCN_KC_DEVICE || !c->fb_copy || c->capturing || has_comm(c) || nsteps < 4) return OCN_OK;
    c->kc_mode = OCN_KC_KNOWN;   // would the call run pairs with a host-chosen known-constant variant?
    const bool pairs = x2 ? x4_now(c) : pair_ok(c);
    c->kc_mode = OCN_KC_DEVICE;
    if (!pairs) return OCN_OK;
    HIPCHK(hipEventSynchronize(c->ev_fb));
    learn_fb_async(c);
    c->kc_mode = kc_of_fb(c);
    return OCN_OK;
}

// The pending tail of an open sequence: the last step run (a one-pass step) is run again from the
// previous state -- untouched in the other buffer of each pair and the other sshp / ubrtrp / vbrtrp
// buffers -- as the call's last step (one_step_last: the same new state bit for bit, plus vort,
// the stresses, the RHS terms, a8's copies and hh_init with every level).  Its check_ssh_err
// count was taken the first time.
static int complete_open(ocn_ctx *c)
{
    if (!c->open) return OCN_OK;
    c->open = false;
    HIPCHK(hipSetDevice(c->dec.device));
    if (c->deferred) {   // steps not yet run: the last ones, from the current state
        const int d = c->deferred;
        c->deferred = 0;
        c->open_pair = false;
        if (d == 2 && pair_ok(c)) {   // both in one launch, the second as the last step (pair + LAST)
            StepKind k{};
            k.last = k.one_last = k.pair = true;
            k.check = c->deferred_check[0];
            k.check2 = c->deferred_check[1];
            return finish_call(c, run_step(c, c->open_tau, k));
        }
        if (d == 2) {
            StepKind k1{};
            k1.check = c->deferred_check[0];
            k1.flip = k1.one = k1.next_one = k1.a_done = true;
            k1.x2 = c->open_x2;   // (x2 sequences with pairs of x2 steps: one_step_x4 deferred it)
            if (const int rc = run_step(c, c->open_tau, k1)) return finish_call(c, rc);
        }
        StepKind k{};
        k.last = k.one_last = true;
        k.check = c->deferred_check[d - 1];
        k.x2_end = c->ring2_saved;
        c->ring2_saved = false;
        return finish_call(c, run_step(c, c->open_tau, k));
    }
    swap_roles(c);
    swap_alt3(c);
    c->tr_pending = false;   // (the tracer step of the state before the last step has run)
    if (c->open_pair) {   // the last launch was a pair (one flip, two steps): both again, from the state
        c->open_pair = false;   // before it, the second as the last step (counted the first time: no checks)
        if (pair_ok(c)) {
            StepKind k{};
            k.last = k.one_last = k.pair = true;
            return finish_call(c, run_step(c, c->open_tau, k));
        }
        StepKind k1{};
        k1.flip = k1.one = k1.next_one = k1.a_done = true;
        k1.x2 = c->open_x2;   // (a pair of x2 steps: its first step again, one_step_x2)
        if (const int rc = run_step(c, c->open_tau, k1)) return finish_call(c, rc);
        c->tr_pending = false;   // (tracer runs: the pair ran the tracer step of that state too)
    }
    StepKind k{};
    k.last = k.one_last = true;
    k.x2_end = c->ring2_saved;   // x2 steps: the second ring restored, the first exchanged (x2_end)
    c->ring2_saved = false;
    return finish_call(c, run_step(c, c->open_tau, k));
}

static int step_impl(ocn_ctx *c, double tau, int32_t nsteps, int32_t check_every)
{
    HIPCHK(hipSetDevice(c->dec.device));
    if (nsteps < 0) return set_error(OCN_ERR_ARG, "nsteps < 0");
    if (nsteps == 0) return OCN_OK;
    // (RCCL / events stay outside graphs; so do the tracer steps' calls: their launches follow pending state)
    const bool graph_ok = c->use_graph && !has_comm(c) && !c->stage_timing && !(c->sw.use_tracers > 0 && c->tr_step);
    c->pair_used = false;
    c->co_used = false;
    c->multi_used = false;
    if (c->open) {
        if (tau == c->open_tau && c->onepass && lazy_allowed(c, c->open_x2)) {
            // the open sequence goes on: every step of this call is a one-pass step (the state and
            // the constants are what its last step left), and the tail stays pending; a device
            // verdict the host has read since selects one variant
            RC(prepare_kc(c, c->open_x2));
            // (x2 sequences: pairs of x2 steps, one_step_x4)
            const bool pairs = c->open_x2 ? x4_now(c) : pair_ok(c);
            c->x4_used = c->open_x2 && pairs;
            int rc = OCN_OK;
            if (pairs) {   // two steps per launch -- the steps deferred by the last call first -- while
                           // 3 or more are pending; the last 1 or 2 deferred (next call, complete_open)
                std::vector<char> chk(c->deferred_check, c->deferred_check + c->deferred);
                for (int s = 1; s <= nsteps; ++s) chk.push_back(check_every > 0 && (s % check_every == 0));
                c->deferred = 0;
                size_t i = 0;
                for (; i + 2 < chk.size() && rc == OCN_OK; i += 2) {
                    StepKind k{};
                    k.check = chk[i];
                    k.check2 = chk[i + 1];
                    k.flip = k.one = k.next_one = k.a_done = k.pair = true;
                    k.x2 = c->open_x2;
                    rc = graph_ok ? graph_step(c, tau, k) : run_step(c, tau, k);
                    c->open_pair = c->pair_used = true;
                }
                if (rc == OCN_OK) {
                    c->deferred = (int)(chk.size() - i);   // 1 or 2
                    for (int j = 0; j < c->deferred; ++j) c->deferred_check[j] = chk[i + j];
                }
            } else {
                for (int j = 0; j < c->deferred && rc == OCN_OK; ++j) {   // (no pairs now: deferred steps first)
                    StepKind k{};
                    k.check = c->deferred_check[j];
                    k.flip = k.one = k.next_one = k.a_done = true;
                    k.x2 = c->open_x2;
                    rc = run_step(c, tau, k);
                }
                c->deferred = 0;
                if (!c->open_x2 && !graph_ok && nsteps >= 2 && rc == OCN_OK && multi_ok(c, check_every)) {
                    StepKind k{};   // all the call's steps in one launch
                    k.check = check_every == 1;
                    k.flip = k.one = k.next_one = k.a_done = true;
                    k.multi = nsteps;
                    rc = run_step(c, tau, k);
                    c->open_pair = false;
                    c->multi_used = true;
                } else {
                    for (int s = 1; s <= nsteps && rc == OCN_OK; ++s) {
                        StepKind k{};
                        k.check = check_every > 0 && (s % check_every == 0);
                        k.flip = k.one = k.next_one = k.a_done = true;
                        k.x2 = c->open_x2;
                        rc = graph_ok ? graph_step(c, tau, k) : run_step(c, tau, k);
                        c->open_pair = false;
                    }
                }
            }
            if (rc) { c->open = false; c->deferred = 0; c->open_pair = false; return finish_call(c, rc); }
            return OCN_OK;
        }
        RC(complete_open(c));
    }
    RC(prepare_static(c));   // (the stage path reads the compact tables too)
    // with RCCL every rank takes part in the decisions (check_coherence reduces the verdicts)
    const bool eligible = flip_eligible(c);
    const bool x2_here = x2_local(c);
    // one_step_x4 possible on this rank: its static conditions and a known-constant verdict for the x2
    // range its host has read (the variant the pairs run; kFbZero stays put through prepare_kc(x2))
    const bool x4_here = x2_here && x4_local(c) && (c->fb_state == kFbZero || c->fb_state == kFbHr) && c->fb_x2;
    // a lazy call is planned as the first nsteps steps of a call of nsteps + 1 (the last deferred)
    const bool lazy_cand = eligible && c->onepass && lazy_allowed(c, x2_here);
    bool udiv_ok = c->udiv_ok, first_one = c->hh_consistent, x2_ok = x2_here && c->x2_dev_ok;
    int N = lazy_cand ? nsteps + 1 : nsteps;
    if (N >= 2 && (eligible || (has_comm(c) && c->flip)) && !c->coherent_known) {
        VoteOut v;
        RC(check_coherence(c, VoteIn{eligible, c->udiv_ok, c->hh_consistent, x2_here, x4_here}, v));
        udiv_ok = v.udiv_ok;
        first_one = v.hh_consistent;
        x2_ok = x2_here && v.x2_ok;
    }
    bool flip_call = false, ca = false, one_call = false;
    // tracer runs with one-pass steps (tracer steps): the call's first step a one-pass step too, and
    // with exchanges the x2 steps (their exchange carries the tracers); one block: no ring work
    // and the last step a one-pass step (last_one below: it runs the pending tracer step)
    const bool tr_ok = c->sw.use_tracers <= 0 ||
                       (c->tr_step && first_one &&
                        (has_exchange(c) ? x2_ok && c->last_hybrid
                                         : !c->ring_sea && (c->last_hybrid || (c->blocks.size() == 1 && !has_comm(c)))));
    auto decide = [&](int n) {
        flip_call = n >= 2 && eligible && c->coherent;
        // role-flip calls with full_free_surface = 1 fuse each step's hh_init with the next step's A;
        // their reuse steps recompute hhq / hhu_p / hhv_p in fused B, which then filters sshp into
        // the second buffer (the ring launch completes it on the halo ring)
        ca = flip_call && c->sw.full_free_surface == 1;
        // one-pass steps 2..K-1 (all SW terms on, no tracers: expl_tracer reads hh_init's hhu / hhv /
        // hhq_p, which a one-pass step keeps in registers; row divisors in udiv's range) -- the first
        // step too when hh_init's stored depths match the state (hh_consistent)
        one_call = ca && c->onepass && (n >= 3 || (n >= 2 && first_one)) && c->sw.trans_terms > 0 &&
                   c->sw.ksw_lat > 0 && tr_ok && udiv_ok;
    };
    decide(N);
    // one-pass steps with one 2-deep exchange each (one_step_x2) where there are exchanges
    const bool x2_call = one_call && x2_ok && c->last_hybrid;   // (its sequences end in the hybrid last step)
    // the last step run is a one-pass step (one launch per block, or an x2 step): the tail may wait
    const bool lazy_end = lazy_cand && one_call && (nsteps >= 2 || first_one) &&
                          (x2_call || (!c->ring_sea && !has_exchange(c)));
    if (!lazy_end && N != nsteps) decide(N = nsteps);
    c->x2_used = x2_call && one_call;
    c->flip_used = flip_call;
    c->tr_call = c->sw.use_tracers > 0 && one_call;
    c->tr_pending = false;
    if (c->tr_call && !c->tr_alt_ok) {   // the second ff1p buffers start as copies
        for (const LBlock &b : c->blocks)
            for (int t = 1; t <= c->sw.tracer_num; ++t)
                HIPCHK(hipMemcpyAsync(b.ffp_alt[(size_t)t - 1], b.ptr[field_slot(OCN_FF1P(t))], field_bytes(b),
                                      hipMemcpyDeviceToDevice, c->stream));
        c->tr_alt_ok = true;
    }
    c->hh_consistent = false;   // until this call's last step has run
    // the last step as one march + hh_init too (single block, no exchange, no ring work)
    // (with exchanges or ring work: the hybrid last step, OCN_OPT_ONEPASS_LAST)
    const bool last_one = one_call && ((c->blocks.size() == 1 && !has_exchange(c) && !has_comm(c) && !c->ring_sea) ||
                                       c->last_hybrid);
    c->one_used = one_call;
    if (x2_call && one_call) {
        if (!c->hrx_ok || has_comm(c)) RC(refresh_hrx(c));   // (with RCCL: every rank, every call)
        RC(prebuild_x2(c));
    }
    if (one_call) {
        RC(prepare_kc(c, x2_call));
        RC(await_kc(c, x2_call, nsteps));
    }
    const bool rc_call = ca && c->recompute && !one_call;
    if (rc_call) c->alt_ok = false;
    if (one_call && !c->alt_ok) {   // the second buffers start as copies (they agree outside a8's write set)
        for (const LBlock &b : c->blocks) {
            HIPCHK(hipMemcpyAsync(b.sshp_alt, b.ptr[field_slot(OCN_SSHP)], field_bytes(b), hipMemcpyDeviceToDevice,
                                  c->stream));
            HIPCHK(hipMemcpyAsync(b.up_alt, b.ptr[field_slot(OCN_UBRTRP)], field_bytes(b), hipMemcpyDeviceToDevice,
                                  c->stream));
            HIPCHK(hipMemcpyAsync(b.vp_alt, b.ptr[field_slot(OCN_VBRTRP)], field_bytes(b), hipMemcpyDeviceToDevice,
                                  c->stream));
        }
        c->alt_ok = true;
    }
    c->rc_used = rc_call && N >= 3;
    if (rc_call)   // the second sshp buffer starts as a copy: the two agree outside a8's write set
        for (const LBlock &b : c->blocks)
            HIPCHK(hipMemcpyAsync(b.sshp_alt, b.ptr[field_slot(OCN_SSHP)], field_bytes(b), hipMemcpyDeviceToDevice,
                                  c->stream));
    RC(join_sync(c));
    // two one-pass steps per launch where both are plain one-pass steps and the second is not the
    // last one run (a lazy tail redoes that one from the state before it, which a pair never writes)
    // (with exchanges: pairs of x2 steps with one 4-deep exchange each, one_step_x4)
    const bool x4_call = one_call && x2_call && x4_now(c);
    c->x4_used = x4_call;
    const bool pairs = one_call && (x2_call ? x4_call : pair_ok(c));
    auto plain_one = [&](int s) {   // step s is a one-pass step that needs nothing around its launch
        const bool one = one_call && (s >= 2 || first_one) && s <= N - 1, next_one = one_call && s + 1 <= N - 1;
        const bool next_a = ca && flip_call && s != N && !next_one && !(last_one && s + 1 == N);
        return one && !next_a && !(last_one && s == N);
    };
    int rc = OCN_OK;
    for (int s = 1; s <= nsteps && rc == OCN_OK; ++s) {
        StepKind k;
        k.check = check_every > 0 && (s % check_every == 0);
        k.first = s == 1;
        k.last = s == N;
        k.flip = flip_call && !k.last;
        k.one = one_call && (s >= 2 || first_one) && s <= N - 1;
        k.next_one = one_call && s + 1 <= N - 1;
        k.one_last = last_one && k.last;
        k.a_done = ca && !k.first;
        k.next_a = ca && k.flip && !k.next_one && !(last_one && s + 1 == N);
        k.next_reuse = k.next_a && s + 1 < N;
        k.rc = rc_call && k.flip && !k.first;
        k.rc_next = rc_call && s + 1 < N;
        k.x2 = x2_call && k.one;
        k.x2_save = k.x2 && !c->ring2_saved;
        k.x2_end = k.one_last && c->ring2_saved;
        if (k.x2_save) c->ring2_saved = true;
        if (k.x2_end) c->ring2_saved = false;
        if (pairs && k.one && s + 1 < nsteps && plain_one(s + 1)) {
            k.pair = true;
            k.check2 = check_every > 0 && ((s + 1) % check_every == 0);
            k.next_one = one_call && s + 2 <= N - 1;
            k.next_a = k.next_reuse = false;
            ++s;
            c->pair_used = true;
        }
        rc = graph_ok ? graph_step(c, tau, k) : run_step(c, tau, k);
    }
    if (lazy_end && rc == OCN_OK) {   // the pending tail: complete_open
        c->open = true;
        c->open_pair = false;   // (the call's last step ran single)
        c->deferred = 0;
        c->open_tau = tau;
        c->open_x2 = x2_call;
        return OCN_OK;
    }
    return finish_call(c, rc);
}

static int step_entry(ocn_ctx *c, double tau, int32_t nsteps, int32_t check_every)
{
    if (!c) return set_error(OCN_ERR_ARG, "null ctx");
    // (a usage error before any collective: no peer waits on this rank yet, the communicator stays)
    if (!c->initialized) return set_error(OCN_ERR_STATE, "ocn_ctx_init_state not called");
    return fail_fatal(c, step_impl(c, tau, nsteps, check_every));
}

int ocn_ctx_step(ocn_ctx *c, double tau, int32_t nsteps, int32_t check_every)
{
    if (!c) return set_error(OCN_ERR_ARG, "null ctx");
    return guarded(c, "ocn_ctx_step", [&] { return step_entry(c, tau, nsteps, check_every); });
}

static int complete_entry(ocn_ctx *c)
{
    if (!c) return set_error(OCN_ERR_ARG, "null ctx");
    return complete_open(c);
}

int ocn_ctx_complete(ocn_ctx *c)
{
    if (!c) return set_error(OCN_ERR_ARG, "null ctx");
    return guarded(c, "ocn_ctx_complete", [&] { return complete_entry(c); });
}

// The steps an open sequence deferred (ocn_ctx_step leaves up to two requested steps not yet
// enqueued while pairs run), run now -- by the calls that look at what the steps did (their
// check_ssh_err counts, their launch times): as a pair or alone, the tail stays pending.
static int run_deferred(ocn_ctx *c)
{
    if (!c->open || !c->deferred) return OCN_OK;
    StepKind k{};
    k.check = c->deferred_check[0];
    k.flip = k.one = k.next_one = k.a_done = true;
    k.pair = c->deferred == 2;   // (a pair only where pairs ran: pair_ok / x4_now held when they were deferred)
    k.check2 = k.pair && c->deferred_check[1];
    k.x2 = c->open_x2;
    c->open_pair = k.pair;
    c->deferred = 0;
    if (const int rc = run_step(c, c->open_tau, k)) { c->open = false; return finish_call(c, rc); }
    return OCN_OK;
}

// check_ssh_err_kernel's verdict (vel_ssh.f90:40-67): abort_model -> mpi_abort on the cart
// communicator (shared/errors.f90:30-37) stops every rank together, so with ranks the counts are
// max-reduced (one int32: ncclAllReduce, or the loopback vote) and every rank returns
// OCN_ERR_BLOWUP from the same synchronize.
static int sync_impl(ocn_ctx *c)
{
    HIPCHK(hipSetDevice(c->dec.device));
    RC(run_deferred(c));
    RC(join_sync(c));
    int32_t *cnt = c->d_nbad;
    if (has_comm(c)) {   // every rank's synchronize takes part (the collective of the check)
        cnt = c->d_nbad + 56;
        HIPCHK(hipMemcpyAsync(cnt, c->d_nbad, sizeof(int32_t), hipMemcpyDeviceToDevice, c->stream));
        RC(allreduce_max(c, cnt, c->stream));
    }
    HIPCHK(hipStreamSynchronize(c->stream));
    learn_fb(c);
    int32_t nbad = 0, berr = 0;
    HIPCHK(hipMemcpy(&nbad, cnt, sizeof(nbad), hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(&berr, c->d_nbad + 61, sizeof(berr), hipMemcpyDeviceToHost));
    if (berr) {   // reported once: the flag is cleared (ocn_ctx_init_state starts the state over)
        HIPCHK(hipMemset(c->d_nbad + 61, 0, sizeof(berr)));
        return set_error(OCN_ERR_HIP, "multi-step launch: a grid barrier timed out (results invalid)");
    }
    if (nbad) return set_error(OCN_ERR_BLOWUP, "SIGFPRE predict error: |ssh| >= 1e4 on " + std::to_string(nbad) +
                                                   (has_comm(c) ? " sea points of a block (the most of any rank;"
                                                                  " check_ssh_err_kernel)"
                                                                : " sea points (check_ssh_err_kernel)"));
    return OCN_OK;
}

static int synchronize_entry(ocn_ctx *c)
{
    if (!c) return set_error(OCN_ERR_ARG, "null ctx");
    return fail_fatal(c, sync_impl(c));
}

int ocn_ctx_synchronize(ocn_ctx *c)
{
    if (!c) return set_error(OCN_ERR_ARG, "null ctx");
    return guarded(c, "ocn_ctx_synchronize", [&] { return synchronize_entry(c); });
}

int ocn_ctx_stage_times(ocn_ctx *c, double *ms, int64_t *counts) { return ocn_ctx_stage_stats(c, ms, counts, nullptr); }

int ocn_ctx_stage_stats(ocn_ctx *c, double *ms, int64_t *counts, double *ms_max)
{
    if (!c || !ms || !counts) return set_error(OCN_ERR_ARG, "null argument");
    HIPCHK(hipSetDevice(c->dec.device));
    RC(run_deferred(c));   // (their launches belong to this report, not the next one)
    RC(join_sync(c));
    HIPCHK(hipStreamSynchronize(c->stream));
    learn_fb(c);
    for (auto &r : c->recs) {
        float t = 0.f;
        if (r.stage == OCN_TIMER_EXPOSED) {   // events on two streams: the comm chain may end first
            if (hipEventElapsedTime(&t, r.a, r.b) != hipSuccess || !(t > 0.f)) t = 0.f;
        } else {
            HIPCHK(hipEventElapsedTime(&t, r.a, r.b));
        }
        c->stage_ms[r.stage] += t;
        c->stage_n[r.stage] += 1;
        c->stage_max[r.stage] = std::max(c->stage_max[r.stage], (double)t);
        c->event_pool.push_back(r.a); c->event_pool.push_back(r.b);
    }
    c->recs.clear();
    for (int i = 0; i < OCN_NUM_TIMERS; ++i) {
        ms[i] = c->stage_ms[i]; counts[i] = c->stage_n[i];
        if (ms_max) ms_max[i] = c->stage_max[i];
    }
    for (int i = 0; i < OCN_NUM_TIMERS; ++i) { c->stage_ms[i] = 0; c->stage_n[i] = 0; c->stage_max[i] = 0; }
    return OCN_OK;
}

static int download_entry(ocn_ctx *c, int k, int id, void *host)
{
    if (!c || !host || k < 0 || k >= (int)c->blocks.size() || !has_field(c, id))
        return set_error(OCN_ERR_ARG, "download: bad argument");
    HIPCHK(hipSetDevice(c->dec.device));
    RC(complete_open(c));
    const LBlock &b = c->blocks[k];
    const size_t es = is_r4(id) ? 4 : 8;
    const size_t w = (size_t)(b.g.bnd_x2 - b.g.bnd_x1 + 1), rows = (size_t)(b.g.bnd_y2 - b.g.bnd_y1 + 1);
    HIPCHK(hipStreamSynchronize(c->stream));
    learn_fb(c);
    HIPCHK(hipMemcpy2D(host, w * es, b.ptr[field_slot(id)], (size_t)b.g.pitch * es, w * es, rows,
                       hipMemcpyDeviceToHost));
    return OCN_OK;
}

int ocn_ctx_download(ocn_ctx *c, int k, int id, void *host)
{
    if (!c) return set_error(OCN_ERR_ARG, "null ctx");
    return guarded(c, "ocn_ctx_download", [&] { return download_entry(c, k, id, host); });
}

static int output_r4_entry(ocn_ctx *c, int k, int id, float undef, float *host)
{
    if (!c || !host || k < 0 || k >= (int)c->blocks.size() || !has_field(c, id))
        return set_error(OCN_ERR_ARG, "output_r4: bad argument");
    HIPCHK(hipSetDevice(c->dec.device));
    RC(complete_open(c));
    const LBlock &b = c->blocks[k];
    const int w = b.g.nx_end - b.g.nx_start + 1, h = b.g.ny_end - b.g.ny_start + 1;
    if (w <= 0 || h <= 0) return OCN_OK;
    const long off = (long)(b.g.ny_start - b.g.bnd_y1) * b.g.pitch + (b.g.nx_start - b.g.bnd_x1);
    float *d = nullptr;
    HIPCHK(hipMallocAsync((void **)&d, (size_t)w * h * sizeof(float), c->stream));
    const float *lu = b.f<float>(OCN_LU) + off;
    const dim3 grid((unsigned)((w + 255) / 256), (unsigned)h);
    if (is_r4(id))
        hipLaunchKernelGGL(k_output_r4<float>, grid, dim3(256), 0, c->stream, b.f<float>(id) + off, lu,
                           (long)b.g.pitch, w, h, undef, d);
    else
        hipLaunchKernelGGL(k_output_r4<double>, grid, dim3(256), 0, c->stream, b.f<double>(id) + off, lu,
                           (long)b.g.pitch, w, h, undef, d);
    int rc = check_launch();
    if (rc == OCN_OK && hipMemcpyAsync(host, d, (size_t)w * h * sizeof(float), hipMemcpyDeviceToHost, c->stream) != hipSuccess)
        rc = set_error(OCN_ERR_HIP, "output_r4: copy");
    (void)hipFreeAsync(d, c->stream);
    HIPCHK(hipStreamSynchronize(c->stream));
    learn_fb(c);
    return rc;
}

int ocn_ctx_output_r4(ocn_ctx *c, int k, int id, float undef, float *host)
{
    if (!c) return set_error(OCN_ERR_ARG, "null ctx");
    return guarded(c, "ocn_ctx_output_r4", [&] { return output_r4_entry(c, k, id, undef, host); });
}

static int upload_entry(ocn_ctx *c, int k, int id, const void *host)
{
    if (!c || !host || k < 0 || k >= (int)c->blocks.size() || !has_field(c, id))
        return set_error(OCN_ERR_ARG, "upload: bad argument");
    HIPCHK(hipSetDevice(c->dec.device));
    RC(complete_open(c));
    HIPCHK(hipStreamSynchronize(c->stream));
    if (is_r4(id)) { c->static_dirty = true; c->ext_ok = false; }
    // (the x2 checks also cover sshp / ubrtrp / vbrtrp and h_r: check_coherence)
    if (is_flip_field(id) || is_alt_field(id) || id == OCN_HHQ_REST || id == OCN_MU) c->coherent_known = false;
    if (is_alt_field(id)) c->alt_ok = false;
    if (is_tracer_field(id)) c->tr_alt_ok = false;
    if (id == OCN_HHQ_REST) c->hrx_ok = false;
    if (id == OCN_HHQ_REST || id == OCN_HHQ_N) c->hqn_stale = true;
    c->hh_consistent = false;
    c->hn_fresh = false;
    c->fb_state = kFbUnchecked;
    return upload_field(c, c->blocks[k], id, host, false);
}

int ocn_ctx_upload(ocn_ctx *c, int k, int id, const void *host)
{
    if (!c) return set_error(OCN_ERR_ARG, "null ctx");
    return guarded(c, "ocn_ctx_upload", [&] { return upload_entry(c, k, id, host); });
}

int ocn_ctx_set_option(ocn_ctx *c, int32_t key, int64_t value)
{
    if (!c) return set_error(OCN_ERR_ARG, "null ctx");
    // an option may change what the next launches are: a pending call tail is formed first
    if (key != OCN_OPT_STAGE_TIMING) {
        HIPCHK(hipSetDevice(c->dec.device));
        RC(complete_open(c));
    }
    switch (key) {
    case OCN_OPT_GRAPH: c->use_graph = value != 0; return OCN_OK;
    case OCN_OPT_STAGE_TIMING:
        c->stage_timing = value != 0;
        if (c->stage_timing) HIPCHK(hipSetDevice(c->dec.device));
        while (c->stage_timing && c->event_pool.size() < 256) {
            hipEvent_t e;
            RC(make_timer_event(e));
            c->event_pool.push_back(e);
        }
        return OCN_OK;
    case OCN_OPT_FUSED:
        if (c->fused != (value != 0)) drop_graphs(c);
        c->fused = value != 0;
        return OCN_OK;
    case OCN_OPT_OVERLAP:
        if (c->overlap != value) drop_graphs(c);
        c->overlap = value < 0 ? -1 : value > 2 ? 2 : (int)value;
        if (c->overlap < 0) c->ov_state = 0;   // (auto again: measured again)
        return OCN_OK;
    case OCN_OPT_XCHG_DELAY: c->xdelay_us = value < 0 ? 0 : value > 1000000 ? 1000000 : (int)value; return OCN_OK;
    case OCN_OPT_MARCH:
        if (c->march != (value != 0)) drop_graphs(c);
        c->march = value != 0;
        return OCN_OK;
    case OCN_OPT_FLIP: c->flip = value != 0; return OCN_OK;
    case OCN_OPT_RECOMPUTE: c->recompute = value != 0; return OCN_OK;
    case OCN_OPT_ONEPASS: c->onepass = value != 0; return OCN_OK;
    case OCN_OPT_ONEPASS_LAST: c->last_hybrid = value != 0; return OCN_OK;
    case OCN_OPT_KNOWN_CONSTANTS:
        c->known_const = value != 0;   // (the check's verdict stays valid: it describes the arrays)
        return OCN_OK;
    case OCN_OPT_LAZY_TAIL: c->lazy = value != 0; return OCN_OK;
    case OCN_OPT_X2: c->x2 = value != 0; c->coherent_known = false; return OCN_OK;
    case OCN_OPT_PAIR: c->pair = value < 0 ? 0 : value > 2 ? 2 : (int)value; return OCN_OK;
    case OCN_OPT_MULTI: c->multi = value != 0; return OCN_OK;
    case OCN_OPT_TRACER_STEP:   // (the x2 vote checks mu's halo only for tracer steps: vote again)
        c->tr_step = value != 0;
        c->coherent_known = false;
        return OCN_OK;
    case OCN_OPT_MULTI_SPIN: c->multi_spin = value < 1 ? 1 : value > kMultiSpin ? kMultiSpin : (int)value; return OCN_OK;
    case OCN_OPT_X4:
        c->x4 = value <= 0 ? 0 : value >= 3 ? 3 : 1;
        c->coherent_known = false;
        c->hrx_ok = false;   // (h_r's copy 2 or 4 rings deep: refresh_hrx)
        return OCN_OK;
    case OCN_OPT_CO_LAUNCH: c->co_launch = value != 0; return OCN_OK;
    case OCN_OPT_BATCH:
        if (c->batch != (value != 0)) drop_graphs(c);
        c->batch = value != 0;
        return OCN_OK;
    case OCN_OPT_COMPACT:   // (re)arms the compact tables: rebuilt from the real(4) fields at the next step
        c->compact_req = value != 0;
        c->r4_escaped = false;
        c->static_dirty = true;
        return OCN_OK;
    default: return set_error(OCN_ERR_ARG, "unknown option");
    }
}

int ocn_ctx_get_option(const ocn_ctx *c, int32_t key, int64_t *value)
{
    if (!c || !value) return set_error(OCN_ERR_ARG, "null argument");
    switch (key) {
    case OCN_OPT_GRAPH: *value = c->use_graph; return OCN_OK;
    case OCN_OPT_STAGE_TIMING: *value = c->stage_timing; return OCN_OK;
    case OCN_OPT_FUSED: *value = c->fused; return OCN_OK;
    case OCN_OPT_OVERLAP: *value = overlap_level(c); return OCN_OK;
    case OCN_OPT_COMPACT: *value = c->compact; return OCN_OK;
    case OCN_OPT_MARCH: *value = c->march; return OCN_OK;
    case OCN_OPT_FLIP: *value = c->flip && c->flip_used; return OCN_OK;
    case OCN_OPT_RECOMPUTE: *value = c->recompute && c->rc_used; return OCN_OK;
    case OCN_OPT_ONEPASS: {
        // 2: the known-constant variant ran, 3: the known-constant variant reading h_r (chosen by the
        // host, or by the device check whose verdict the host has read since)
        const bool z = c->kc_mode == OCN_KC_KNOWN || (c->kc_mode == OCN_KC_DEVICE && c->fb_state == kFbZero);
        const bool h = c->kc_mode == OCN_KC_KNOWN_HR || (c->kc_mode == OCN_KC_DEVICE && c->fb_state == kFbHr);
        *value = c->onepass && c->one_used ? (z ? 2 : h ? 3 : 1) : 0;
        return OCN_OK;
    }
    case OCN_OPT_KNOWN_CONSTANTS: *value = c->known_const; return OCN_OK;
    case OCN_OPT_ONEPASS_LAST: *value = c->last_hybrid; return OCN_OK;
    case OCN_OPT_LAZY_TAIL: *value = c->open ? 2 : c->lazy; return OCN_OK;
    case OCN_OPT_X2: *value = c->x2 && c->x2_used; return OCN_OK;
    case OCN_OPT_BATCH: *value = c->batch; return OCN_OK;
    case OCN_OPT_PAIR: *value = c->pair_used ? 2 : c->pair > 0; return OCN_OK;
    case OCN_OPT_MULTI: *value = c->multi_used ? 2 : c->multi; return OCN_OK;
    case OCN_OPT_TRACER_STEP: *value = c->tr_call ? 2 : c->tr_step; return OCN_OK;
    case OCN_OPT_MULTI_SPIN: *value = c->multi_spin; return OCN_OK;
    case OCN_OPT_X4: *value = c->x4_used ? 2 : c->x4 ? 1 : 0; return OCN_OK;
    case OCN_OPT_CO_LAUNCH: *value = c->co_used ? 2 : c->co_launch; return OCN_OK;
    case OCN_OPT_XCHG_DELAY: *value = c->xdelay_us; return OCN_OK;
    default: return set_error(OCN_ERR_ARG, "unknown option");
    }
}

}  // extern "C"
