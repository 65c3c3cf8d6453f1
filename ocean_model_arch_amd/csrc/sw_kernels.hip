// sw_kernels.hip -- HIP/CDNA4 kernels of the shallow-water barotropic step (gfx950).
//
// One kernel per SW stage of control/shallow_water/shallow_water.f90:36-92, each a
// bitwise-exact restatement of the reference loop nest (kernel/shallow_water/*.f90):
// same write set, same floating-point evaluation order, real(4)*real(4) sub-expressions in
// float (Fortran mixed-kind rules).  Built with -ffp-contract=off (no FMA contraction) and
// IEEE division/sqrt (hipcc defaults), so results equal the reference CPU build bit for bit.
//
// Mapping (HBM-bound fp64 stencils, no MFMA): a workgroup is 64 x 4 threads and owns a
// 64-column x OCN_ROWS-row strip of the block; lane = m (coalesced column-major rows), the
// 4 thread-rows march down the strip in steps of 4 so the n-1 / n+1 rows a thread needs
// were just touched by its own workgroup (L1/L2 hits).  Each array is therefore streamed
// from HBM about once per stage; the +-1 neighbours come from cache.
//
// Code shape for memory-level parallelism: every operand is loaded unconditionally (all
// addresses are inside the block array), values are computed unconditionally, and only the
// stores are predicated by the reference's masks.  Masks therefore never serialise a second
// round of loads behind the mask load, and all loads of a cell can be in flight together.
// Offsets are 32-bit element indices from a wave-uniform base (the kernel-argument pointer),
// so loads use the SGPR-base + 32-bit VGPR-offset form instead of a 64-bit VGPR address
// per array.
#include <hip/hip_runtime.h>

#include <climits>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <type_traits>

#include "ocn_internal.h"
#include "sw_stencils.h"

namespace ocn {

#define RC_KB(x) do { int _rc = (x); if (_rc) return _rc; } while (0)

// ------------------------------------------------------------------ launch scaffolding
// A workgroup owns a tile of OCN_TW columns x OCN_ROWS rows: OCN_TW lanes across (a multiple
// of the 64-lane wave), OCN_WY = 256 / OCN_TW waves stacked vertically that step through the
// tile rows together.  Tile t = (t % ntx, t / ntx).  With OCN_XCD_REMAP the linear workgroup
// id is remapped so that each of the 8 XCDs (workgroups are dealt round-robin, id % 8) works
// on one contiguous band of tiles: horizontally adjacent tiles then run back to back on the
// same XCD and their shared +-1 columns / rows are L2 hits instead of refetches.
// Tiles start at column w0 <= m0 (an aligned column, see launch_range); lanes left of m0 idle.
template <typename Body>
__device__ __forceinline__ void range_tile(int w0, int m0, int m1, int n0, int n1, int ntx, int tile, const Body &body)
{
    const int tx = tile % ntx, ty = tile / ntx;
    const int m = w0 + tx * OCN_TW + (int)threadIdx.x;
    if (m < m0 || m > m1) return;
    const int nb = n0 + ty * OCN_ROWS;
    const int ne = min(n1, nb + OCN_ROWS - 1);
    // every wave is one thread-row: its row index is wave-uniform (scalar registers)
    const int wy = __builtin_amdgcn_readfirstlane((int)threadIdx.y);
    for (int n = nb + wy; n <= ne; n += OCN_WY) body(m, n);
}

template <typename Body>
__global__ __launch_bounds__(256, OCN_LB_WAVES) void k_range(int w0, int m0, int m1, int n0, int n1, int ntx,
                                                             int ntiles, Body body)
{
    int tile = (int)blockIdx.x;
#if OCN_XCD_REMAP
    const int per = (ntiles + 7) / 8;
    tile = (tile % 8) * per + tile / 8;
    if (tile >= ntiles) return;
#endif
    range_tile(w0, m0, m1, n0, n1, ntx, tile, body);
}

// ------------------------------------------------------------------ block batching (ocn_internal.h Batcher)
// The bodies of a batched launch travel by value in its kernel arguments (as a single body does),
// kPack<Body> (up to 8) of them per launch within a 12 KB argument block: no copies to device
// memory, and the launches stay capturable into graphs.  (Plain launches with 16 KB argument blocks
// run correctly on gfx950 under this ROCm: scripts/kernarg_probe.hip; 8 blocks of a device -- the
// 4 x 2 layouts -- then take one launch instead of two.)
constexpr int kBatchMax = 32;   // ranges / rects per batched launch
constexpr int kArgBudget = 12288 - kBatchMax * 48 - 64;
template <class Body> constexpr int kPack = (int)(kArgBudget / sizeof(Body)) < 1 ? 1
                                            : (int)(kArgBudget / sizeof(Body)) > 8 ? 8 : (int)(kArgBudget / sizeof(Body));
template <class Body> struct Pack { Body b[kPack<Body>]; };
// the bodies [b, b + n) as a Pack (bytes: the bodies are trivially copyable launch arguments)
template <class Body> struct PackBuf {
    alignas(Pack<Body>) unsigned char raw[sizeof(Pack<Body>)] = {};
    PackBuf(const Body *b, size_t n) { std::memcpy(raw, (const void *)b, n * sizeof(Body)); }
    const Pack<Body> &get() const { return *reinterpret_cast<const Pack<Body> *>(raw); }
};
struct RangeB { int w0, m0, m1, n0, n1, ntx, tiles, blk; };
struct RangeGridB { int nr, ntiles; RangeB r[kBatchMax]; };
template <typename Body>
__global__ __launch_bounds__(256, OCN_LB_WAVES) void k_range_b(RangeGridB g, Pack<Body> bodies)
{
    int tile = (int)blockIdx.x;
#if OCN_XCD_REMAP
    const int per = (g.ntiles + 7) / 8;
    tile = (tile % 8) * per + tile / 8;
    if (tile >= g.ntiles) return;
#endif
    int k = 0;   // workgroup-uniform
    while (k + 1 < g.nr && tile >= g.r[k].tiles) { tile -= g.r[k].tiles; ++k; }
    const RangeB R = g.r[k];
    range_tile(R.w0, R.m0, R.m1, R.n0, R.n1, R.ntx, tile, bodies.b[__builtin_amdgcn_readfirstlane(R.blk)]);
}

thread_local Batcher *g_batcher = nullptr;
// a launch on stream s joins the active batch
static bool batching(hipStream_t s) { return g_batcher && g_batcher->active && g_batcher->s == s; }
// the entry of kernel `kind` in the active batch for the current block (created on first use; the
// batch is flushed first if this block's launches would lose their order)
template <class E> static E *batch_entry(const void *kind, int &rc)
{
    Batcher &bt = *g_batcher;
    int p = -1;
    for (size_t i = 0; i < bt.entries.size(); ++i)
        if (bt.entries[i]->kind == kind) p = (int)i;
    if (p >= 0 && p <= bt.cur) {
        rc = bt.flush();
        p = -1;
    }
    if (p < 0) {
        E *e = new E();
        e->kind = kind;
        bt.entries.push_back(e);
        p = (int)bt.entries.size() - 1;
    }
    bt.cur = p;
    return static_cast<E *>(bt.entries[(size_t)p]);
}

template <typename Body> struct RangeBatch : BatchEntry {
    std::vector<Body> bodies;
    std::vector<RangeB> ranges;   // one per body (blk = its index)
    int flush(hipStream_t s) override
    {
        for (size_t i = 0; i < bodies.size(); i += kPack<Body>) {
            const size_t n = std::min(bodies.size() - i, (size_t)kPack<Body>);
            if (n == 1) {
                const RangeB &r = ranges[i];
                const int nblocks = OCN_XCD_REMAP ? 8 * ((r.tiles + 7) / 8) : r.tiles;
                hipLaunchKernelGGL(k_range<Body>, dim3((unsigned)nblocks), dim3(OCN_TW, OCN_WY), 0, s, r.w0, r.m0, r.m1,
                                   r.n0, r.n1, r.ntx, r.tiles, bodies[i]);
                RC_KB(check_launch());
                continue;
            }
            RangeGridB g{};
            const PackBuf<Body> pk(&bodies[i], n);
            for (size_t j = 0; j < n; ++j) {
                g.r[g.nr] = ranges[i + j];
                g.r[g.nr].blk = (int)j;
                g.ntiles += ranges[i + j].tiles;
                ++g.nr;
            }
            const int nblocks = OCN_XCD_REMAP ? 8 * ((g.ntiles + 7) / 8) : g.ntiles;
            hipLaunchKernelGGL(k_range_b<Body>, dim3((unsigned)nblocks), dim3(OCN_TW, OCN_WY), 0, s, g, pk.get());
            RC_KB(check_launch());
        }
        return OCN_OK;
    }
};

// wa: a column whose row addresses start a 256-B line (the block's nx_start in the library's
// allocation): the tiles' columns then start on whole lines, so no wave stores a partial line at
// both of its ends (partial-line stores cost HBM bandwidth).  INT_MIN: tiles from m0.
#ifndef OCN_RANGE_ALIGN
#define OCN_RANGE_ALIGN 1
#endif
template <typename Body>
static int launch_range(int m0, int m1, int n0, int n1, const Body &body, hipStream_t s, int wa = INT_MIN)
{
    if (m1 < m0 || n1 < n0) return OCN_OK;
    int w0 = m0;
    if (OCN_RANGE_ALIGN && wa != INT_MIN) {
        const int d = m0 - wa;
        w0 = wa + 64 * (d >= 0 ? d / 64 : -((63 - d) / 64));
    }
    const int ntx = (m1 - w0 + OCN_TW) / OCN_TW, nty = (n1 - n0 + OCN_ROWS) / OCN_ROWS;
    const int ntiles = ntx * nty;
    if (batching(s)) {
        int rc = OCN_OK;
        auto *e = batch_entry<RangeBatch<Body>>((const void *)&k_range<Body>, rc);
        e->ranges.push_back(RangeB{w0, m0, m1, n0, n1, ntx, ntiles, (int)e->bodies.size()});
        e->bodies.push_back(body);
        return rc;
    }
    const int nblocks = OCN_XCD_REMAP ? 8 * ((ntiles + 7) / 8) : ntiles;
    hipLaunchKernelGGL(k_range<Body>, dim3((unsigned)nblocks), dim3(OCN_TW, OCN_WY), 0, s, w0, m0, m1, n0, n1, ntx,
                       ntiles, body);
    return check_launch();
}

// the frame part of a split range (sw_stencils.h frame_rects): one thread per point, one wave
// per workgroup.  The frame's columns touch one cache line per point and array, so the loads a
// CU can have in flight bound these launches: small workgroups spread them over more CUs.
#ifndef OCN_FRAME_WG
#define OCN_FRAME_WG 64
#endif
template <typename Body>
__global__ __launch_bounds__(OCN_FRAME_WG) void k_frame(Rects q, int total, Body body)
{
    const int t = (int)(blockIdx.x * OCN_FRAME_WG + threadIdx.x);
    if (t >= total) return;
    int m, n;
    frame_point(q, t, m, n);
    body(m, n);
}

// batched: entry k's points take workgroups [w0[k], w0[k+1])
struct FrameGridB { int n; int w0[9]; int total[8]; int blk[8]; Rects q[8]; };   // (kPack <= 8)
template <typename Body>
__global__ __launch_bounds__(OCN_FRAME_WG) void k_frame_b(FrameGridB g, Pack<Body> bodies)
{
    const int w = (int)blockIdx.x;
    int k = 0;
    while (k + 1 < g.n && w >= g.w0[k + 1]) ++k;
    const int t = (w - g.w0[k]) * OCN_FRAME_WG + (int)threadIdx.x;
    if (t >= g.total[k]) return;
    int m, n;
    frame_point(g.q[k], t, m, n);
    bodies.b[__builtin_amdgcn_readfirstlane(g.blk[k])](m, n);
}

template <typename Body> struct FrameBatch : BatchEntry {
    std::vector<Body> bodies;
    std::vector<Rects> q;
    std::vector<int> total;
    int flush(hipStream_t s) override
    {
        for (size_t i = 0; i < bodies.size(); i += kPack<Body>) {
            const size_t n = std::min(bodies.size() - i, (size_t)kPack<Body>);
            if (n == 1) {
                hipLaunchKernelGGL(k_frame<Body>, dim3((unsigned)((total[i] + OCN_FRAME_WG - 1) / OCN_FRAME_WG)),
                                   dim3(OCN_FRAME_WG), 0, s, q[i], total[i], bodies[i]);
                RC_KB(check_launch());
                continue;
            }
            FrameGridB g{};
            const PackBuf<Body> pk(&bodies[i], n);
            for (size_t j = 0; j < n; ++j) {
                g.q[g.n] = q[i + j]; g.total[g.n] = total[i + j]; g.blk[g.n] = (int)j;
                g.w0[g.n + 1] = g.w0[g.n] + (total[i + j] + OCN_FRAME_WG - 1) / OCN_FRAME_WG;
                ++g.n;
            }
            hipLaunchKernelGGL(k_frame_b<Body>, dim3((unsigned)g.w0[g.n]), dim3(OCN_FRAME_WG), 0, s, g, pk.get());
            RC_KB(check_launch());
        }
        return OCN_OK;
    }
};

// part: OCN_PART_ALL = R, OCN_PART_FRAME = R minus `inner`, OCN_PART_INNER = R clipped to `inner`
template <typename Body>
static int launch_part(const Range &r, const Range &inner, int part, const Body &body, hipStream_t s)
{
    if (part == OCN_PART_INNER) {
        const Range i = range_clip(r, inner);
        return launch_range(i.m0, i.m1, i.n0, i.n1, body, s);
    }
    if (part == OCN_PART_FRAME) {
        const Rects q = frame_rects(r, inner);
        const int total = q.total();
        if (total == 0) return OCN_OK;
        if (batching(s)) {
            int rc = OCN_OK;
            auto *e = batch_entry<FrameBatch<Body>>((const void *)&k_frame<Body>, rc);
            e->q.push_back(q);
            e->total.push_back(total);
            e->bodies.push_back(body);
            return rc;
        }
        hipLaunchKernelGGL(k_frame<Body>, dim3((unsigned)((total + OCN_FRAME_WG - 1) / OCN_FRAME_WG)), dim3(OCN_FRAME_WG),
                           0, s, q, total, body);
        return check_launch();
    }
    return launch_range(r.m0, r.m1, r.n0, r.n1, body, s);
}

// ------------------------------------------------------------------ register march
// For stencils over many arrays the k_range mapping issues one load instruction per
// (array, neighbour): fused B issues 76 per cell, and the L1/TA path -- not HBM -- limits it
// (SQ_WAIT_INST_ANY ~70 % of wave time; profiles/r01b).  The march mapping loads each array
// once per cell instead:
//   * a wave owns 64 consecutive columns and marches down OCN_MARCH_ROWS rows;
//   * the n-1 / n / n+1 rows of an array stay in registers and rotate as the wave moves down, so
//     each iteration loads only row n+1 (or row n for arrays read at n-1 and n);
//   * m+1 / m-1 neighbours come from the adjacent lane (DPP wave_shl:1 / wave_shr:1);
//   * the per-row metrics of the compact tables are wave-uniform (scalar loads).
// Two lane layouts (Body::kAligned):
//   * aligned: the 64 columns of a wave start on a 512-B boundary (A(nx_start + 64 j, n)) and all
//     64 lanes produce output, so every store writes whole 128-B lines.  Lane 0's m-1 and lane
//     63's m+1 neighbours come from one extra load per (array, row) with only those two lanes
//     active ("edge" values, merged in by the DPP move's bound control).  Partial-line stores
//     cost HBM bandwidth (scripts/mixbench.hip: write-only streams 5.3 TB/s aligned, 3.6 TB/s
//     with 62-column waves offset by one column), so the store-heavy launches use this layout;
//   * offset: lanes 1..62 produce output and lanes 0 / 63 only load the m-1 / m+1 columns (no
//     edge loads, fewer registers; fused B, which stores two arrays).
// Four waves of a workgroup sit side by side; XCD-banded tile order as k_range.  Whole waves
// stay active through the loop (the lane shifts need every lane).
#ifndef OCN_MARCH_ROWS
#define OCN_MARCH_ROWS 8
#endif

// x of lane + dx (dx in {-1, 0, 1}); the lane without a source (0 for -1, 63 for +1) gets e
__device__ __forceinline__ int dpp_shift(int x, int e, int dx)
{
    if (dx > 0) return __builtin_amdgcn_update_dpp(e, x, 0x130, 0xf, 0xf, false);   // wave_shl:1
    return __builtin_amdgcn_update_dpp(e, x, 0x138, 0xf, 0xf, false);               // wave_shr:1
}
__device__ __forceinline__ double lane_shift(double x, double e, int dx)
{
    if (dx == 0) return x;
    const int lo = dpp_shift(__double2loint(x), __double2loint(e), dx);
    const int hi = dpp_shift(__double2hiint(x), __double2hiint(e), dx);
    return __hiloint2double(hi, lo);
}
__device__ __forceinline__ unsigned lane_shift(unsigned x, unsigned e, int dx)
{
    return dx == 0 ? x : (unsigned)dpp_shift((int)x, (int)e, dx);
}
__device__ __forceinline__ float lane_shift(float x, float e, int dx)
{
    return dx == 0 ? x : __int_as_float(dpp_shift(__float_as_int(x), __float_as_int(e), dx));
}

// Never defined: a view access outside the rows a march keeps fails to link.
extern "C" __device__ void ocn_march_bad_access();

// Rows n-1 (s), n (c), n+1 (nn) of one array at this lane's column; S / N: whether s / nn are
// kept; E: the rows' edge values es / ec / enn are kept (aligned layout, arrays read at m+-1).
template <class T, bool S, bool N, bool E = false> struct Rows {
    T s, c, nn, es, ec, enn;
    __device__ __forceinline__ T at(int dx, int dy) const
    {
        if ((dy < 0 && !S) || (dy > 0 && !N) || dy < -1 || dy > 1) ocn_march_bad_access();
        const T v = dy < 0 ? s : dy == 0 ? c : nn;
        const T e = dy < 0 ? es : dy == 0 ? ec : enn;
        return lane_shift(v, E ? e : v, dx);
    }
    __device__ __forceinline__ void rotate() { s = c; c = nn; es = ec; ec = enn; }
};
template <bool S, bool N, bool E = false> using RowsD = Rows<double, S, N, E>;
template <bool S, bool N, bool E = false> using RowsF = Rows<float, S, N, E>;   // a real(4) 2-D array
// mask bytes of the compact tables: bit id of the byte
template <bool S, bool N, bool E = false> struct BitRows : Rows<unsigned, S, N, E> {
    __device__ __forceinline__ float mask(int id, int dx, int dy) const
    {
        return (this->at(dx, dy) >> id) & 1u ? 1.0f : 0.0f;
    }
};

// value of an array read only at (m, n)
template <class T> struct HereT {
    T v;
    __device__ __forceinline__ T at(int dx, int dy) const
    {
        if (dx != 0 || dy != 0) ocn_march_bad_access();
        return v;
    }
};
using Here = HereT<double>;
using HereF = HereT<float>;

// per-row metrics of the compact tables (wave-uniform) for rows n-1, n, n+1
struct MetRows {
    float g[kRowTable][3];
    __device__ __forceinline__ float at(int id, int dy) const
    {
        if (dy < -1 || dy > 1) ocn_march_bad_access();
        return g[id - OCN_DX][dy + 1];
    }
    // rows n-1 <- n <- n+1 = next (one value per metric field)
    __device__ __forceinline__ void shift(const float *next)
    {
        for (int k = 0; k < kRowTable; ++k) { g[k][0] = g[k][1]; g[k][1] = g[k][2]; g[k][2] = next[k]; }
    }
    // rows n-1 and n before the first row of a march (table rows[(id - OCN_DX) * nrows + r])
    __device__ __forceinline__ void preload(const float *rows, unsigned nrows, unsigned r_prev, unsigned r_cur)
    {
        for (int k = 0; k < kRowTable; ++k) {
            g[k][1] = ld(rows, (unsigned)k * nrows + r_prev);
            g[k][2] = ld(rows, (unsigned)k * nrows + r_cur);
        }
    }
    // The row tables are read-only while any step kernel runs: read them through the constant
    // address space, so the wave-uniform loads are scalar (s_load, lgkmcnt) and never wait
    // behind the vector loads of the rows in flight.
    __device__ __forceinline__ static void load(float *q, const float *rows, unsigned nrows, unsigned r)
    {
        typedef const __attribute__((address_space(4))) float cfloat;
        const cfloat *t = (const cfloat *)rows;
        r = __builtin_amdgcn_readfirstlane(r);
        for (int k = 0; k < kRowTable; ++k) q[k] = t[(unsigned)k * nrows + r];
    }
};
#define OCN_MV(name, reg) \
    __device__ __forceinline__ double name(int dx, int dy) const { return reg.at(dx, dy); }
#define OCN_MG(name, id) \
    __device__ __forceinline__ float name(int, int dy) const { return met.at(id, dy); }
#define OCN_MG_ALL                                                                                         \
    OCN_MG(dx, OCN_DX) OCN_MG(dy, OCN_DY) OCN_MG(dxt, OCN_DXT) OCN_MG(dyt, OCN_DYT) OCN_MG(dxh, OCN_DXH)     \
    OCN_MG(dyh, OCN_DYH) OCN_MG(dxb, OCN_DXB) OCN_MG(dyb, OCN_DYB)                                           \
    __device__ __forceinline__ float sratio(int k) const { return met.at(OCN_DX + kNumRowFields + k, 0); }

// One lane of a march: its loaded column m, its edge column me (aligned layout: lane 0 m-1,
// lane 63 m+1, both clamped into the block array), whether it is an edge lane, whether it
// produces output.
// Two-step launches (a body's kPair): pr = 1 for the producer waves, 2 for the consumers, j = the
// lane's column in the workgroup's LDS ring, ccol = the lane's column is the workgroup's (counted).
struct Lane { int m, me; bool edge, out; int pr = 0, j = 0; bool ccol = true; };

// Loaded columns are clamped to [mlo, mhi] (inside the block array); a lane whose column was
// clamped never produces output and its value is read by no output lane.
#ifndef OCN_MARCH_LB
#define OCN_MARCH_LB 1   // minimum waves per SIMD asked of the register allocator
#endif
// A march launch covers up to 4 rectangles (one, or the frame bands of a split range): each
// has its own wave origin w0, tile columns ntx, tile count, column clamps, rows per tile, and
// workgroup shape (vert: the 4 waves take 4 row tiles of one wave column -- narrow bands).
struct MarchRect { int m0, m1, n0, n1, w0, ntx, tiles, mlo, mhi, rows, vert; };
struct MarchGrid { int nr, ntiles; MarchRect r[4]; };

// waves per SIMD a march body asks of the register allocator (Body::kWaves, else OCN_MARCH_LB)
template <class B, class = void> struct WavesOf { static constexpr int v = OCN_MARCH_LB; };
template <class B> struct WavesOf<B, std::void_t<decltype(B::kWaves)>> { static constexpr int v = B::kWaves; };

// a body with a workgroup prologue (Body::prologue(R, ty), called by all 4 waves of a workgroup)
template <class B, class = void> struct HasPrologue { static constexpr bool v = false; };
template <class B> struct HasPrologue<B, std::void_t<decltype(B::kPrologue)>> { static constexpr bool v = B::kPrologue; };
// a two-step body (Body::kPair: MarchStep PAIR; march_tile deals its waves the two roles)
template <class B, class = void> struct HasPair { static constexpr bool v = false; };
template <class B> struct HasPair<B, std::void_t<decltype(B::kPair)>> { static constexpr bool v = B::kPair; };
// a two-step body with halo exchanges (MarchStep PAIR + X2: ocn_ctx.hip one_step_x4): its producers
// also update the halo points neighbour blocks own, 2 deep
template <class B, class = void> struct HasX2 { static constexpr bool v = false; };
template <class B> struct HasX2<B, std::void_t<decltype(B::kX2)>> { static constexpr bool v = B::kX2; };
// a body whose launch may be void at run time (Body::enabled(), a device-side predicate read by
// every workgroup before anything else: the one-pass step's two variants, one of which a device
// check selected -- ocn_ctx.hip launches both and never waits for the verdict)
template <class B, class = void> struct HasGate { static constexpr bool v = false; };
template <class B> struct HasGate<B, std::void_t<decltype(B::kGate)>> { static constexpr bool v = B::kGate; };

template <class Body, bool PRO = true> __device__ __forceinline__ void march_tile(const MarchRect &R, int tile, const Body &body);

// Shader-clock telemetry of the two-step launches (ocn_ctx_clock_info): workgroup 0 of every pair
// launch adds the s_memtime ticks of its tiles, their 100 MHz s_memrealtime ticks and 1, with vector
// atomics -- the clock the dominant kernel ran at, measured while it runs (the device's launches
// since the last reset, every context on it)
__device__ unsigned long long g_clk[3];
struct ClockSample {
    unsigned long long c0 = 0, w0 = 0;
    __device__ __forceinline__ void begin()
    {
        if (blockIdx.x == 0) { c0 = clock64(); w0 = wall_clock64(); }
    }
    __device__ __forceinline__ void end() const
    {
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            const unsigned long long c1 = clock64(), w1 = wall_clock64();
            atomicAdd(&g_clk[0], c1 - c0);
            atomicAdd(&g_clk[1], w1 - w0);
            atomicAdd(&g_clk[2], 1ull);
        }
    }
};

int clock_read(bool reset, unsigned long long out[3])
{
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_clk), sizeof(g_clk)) != hipSuccess)
        return set_error(OCN_ERR_HIP, "clock telemetry read");
    if (reset) {
        const unsigned long long z[3] = {0, 0, 0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_clk), z, sizeof(z)) != hipSuccess)
            return set_error(OCN_ERR_HIP, "clock telemetry reset");
    }
    return OCN_OK;
}

template <class Body>
__global__ __launch_bounds__(256, WavesOf<Body>::v) void k_march(MarchGrid g, Body body)
{
    if constexpr (HasGate<Body>::v)
        if (!body.enabled()) return;   // workgroup-uniform (a value in memory)
    int tile = (int)blockIdx.x;
#if OCN_XCD_REMAP
    const int per = (g.ntiles + 7) / 8;
    tile = (tile % 8) * per + tile / 8;
    if (tile >= g.ntiles) return;
#endif
    int k = 0;   // workgroup-uniform
    while (k + 1 < g.nr && tile >= g.r[k].tiles) { tile -= g.r[k].tiles; ++k; }
#if OCN_CLOCK_PROBE   // diagnostic build only (scripts/gpu_clock_probe.sh): workgroup 0's shader clock
    const unsigned long long c0 = clock64(), w0 = wall_clock64();
#endif
    ClockSample clk;
    if constexpr (HasPair<Body>::v) clk.begin();
    march_tile(g.r[k], tile, body);
    if constexpr (HasPair<Body>::v) clk.end();
#if OCN_CLOCK_PROBE
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        const unsigned long long c1 = clock64(), w1 = wall_clock64();
        printf("clockprobe %d %.4f GHz %.1f us\n", (int)sizeof(Body), (double)(c1 - c0) / ((double)(w1 - w0) * 10.0),
               (double)(w1 - w0) * 0.01);
    }
#endif
}

// batched (ocn_internal.h Batcher): every block's rects in one grid, rect k marched with body blk[k]
struct MarchGridB { int nr, ntiles; MarchRect r[kBatchMax]; int blk[kBatchMax]; };
template <class Body>
__global__ __launch_bounds__(256, WavesOf<Body>::v) void k_march_b(MarchGridB g, Pack<Body> bodies)
{
    int tile = (int)blockIdx.x;
#if OCN_XCD_REMAP
    const int per = (g.ntiles + 7) / 8;
    tile = (tile % 8) * per + tile / 8;
    if (tile >= g.ntiles) return;
#endif
    int k = 0;   // workgroup-uniform
    while (k + 1 < g.nr && tile >= g.r[k].tiles) { tile -= g.r[k].tiles; ++k; }
    const Body &body = bodies.b[__builtin_amdgcn_readfirstlane(g.blk[k])];
    if constexpr (HasGate<Body>::v)
        if (!body.enabled()) return;
    ClockSample clk;
    if constexpr (HasPair<Body>::v) clk.begin();
    march_tile(g.r[k], tile, body);
    if constexpr (HasPair<Body>::v) clk.end();
}

template <class Body> struct MarchBatch;
template <class MB> static bool march_tracer_flush(MarchBatch<MB> &m, BatchEntry *next, hipStream_t s, int &rc);
// a march body whose batch may be co-launched with the tracer step's (k_march_tracer_b)
template <class B, class = void> struct CoTracer { static constexpr bool v = false; };
template <class B> struct CoTracer<B, std::void_t<decltype(B::kCoTracer)>> { static constexpr bool v = B::kCoTracer; };
template <class Body> struct MarchBatch : BatchEntry {
    std::vector<Body> bodies;
    std::vector<MarchRect> rects;
    std::vector<int> blk;
    bool co_flush(BatchEntry *next, hipStream_t s, int &rc) override
    {
        if constexpr (CoTracer<Body>::v) return march_tracer_flush(*this, next, s, rc);
        (void)next; (void)s; (void)rc;
        return false;
    }
    int flush(hipStream_t s) override
    {
        constexpr int P = kPack<Body> < kBatchMax / 4 ? kPack<Body> : kBatchMax / 4;   // (a body has <= 4 rects)
        for (size_t i = 0; i < bodies.size(); i += P) {
            const size_t n = std::min(bodies.size() - i, (size_t)P);
            if (n == 1) {   // one body: its rects (at most 4) in the plain launch
                MarchGrid g{};
                for (size_t j = 0; j < rects.size(); ++j)
                    if (blk[j] == (int)i && g.nr < 4) { g.r[g.nr++] = rects[j]; g.ntiles += rects[j].tiles; }
                if (!g.nr) continue;
                const int nblocks = OCN_XCD_REMAP ? 8 * ((g.ntiles + 7) / 8) : g.ntiles;
                hipLaunchKernelGGL(k_march<Body>, dim3((unsigned)nblocks), dim3(256), 0, s, g, bodies[i]);
                RC_KB(check_launch());
                continue;
            }
            MarchGridB g{};
            const PackBuf<Body> pk(&bodies[i], n);
            for (size_t j = 0; j < rects.size(); ++j)
                if (blk[j] >= (int)i && blk[j] < (int)(i + n)) {
                    g.r[g.nr] = rects[j]; g.blk[g.nr] = blk[j] - (int)i; g.ntiles += rects[j].tiles; ++g.nr;
                }
            if (!g.nr) continue;
            const int nblocks = OCN_XCD_REMAP ? 8 * ((g.ntiles + 7) / 8) : g.ntiles;
            hipLaunchKernelGGL(k_march_b<Body>, dim3((unsigned)nblocks), dim3(256), 0, s, g, pk.get());
            RC_KB(check_launch());
        }
        return OCN_OK;
    }
};

// a march launch of grid g with one body: issued, or added to the active batch
template <class Body> static int issue_march(const MarchGrid &g, const Body &body, hipStream_t s)
{
    if (!g.nr) return OCN_OK;
    if (batching(s)) {
        int rc = OCN_OK;
        auto *e = batch_entry<MarchBatch<Body>>((const void *)&k_march<Body>, rc);
        const int i = (int)e->bodies.size();
        e->bodies.push_back(body);
        for (int k = 0; k < g.nr; ++k) { e->rects.push_back(g.r[k]); e->blk.push_back(i); }
        return rc;
    }
    const int nblocks = OCN_XCD_REMAP ? 8 * ((g.ntiles + 7) / 8) : g.ntiles;
    hipLaunchKernelGGL(k_march<Body>, dim3((unsigned)nblocks), dim3(256), 0, s, g, body);
    return check_launch();
}

// PRO = false: the body's workgroup prologue has run already (k_march_multi: once for all its steps)
template <class Body, bool PRO> __device__ __forceinline__ void march_tile(const MarchRect &R, int tile, const Body &body)
{
    const int tx = tile % R.ntx, ty = tile / R.ntx;
    const int lane = (int)threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
    constexpr int cols = Body::kAligned ? 64 : 64 - 2 * Body::kHalo;
    const int mw = R.w0 + (R.vert ? tx : tx * 4 + wave) * cols;   // first output column of this wave
    const int nb = R.n0 + (R.vert ? ty * 4 + wave : ty) * R.rows, ne = min(R.n1, nb + R.rows - 1);
    if constexpr (PRO && HasPrologue<Body>::v) body.prologue(R, ty);   // all 4 waves (a barrier)
    if constexpr (HasPair<Body>::v) {
        // two steps in one launch (MarchStep PAIR): 4 waves side by side, waves 0 / 1 produce the
        // first step on columns [c0 - 2, c0 + 118) (60 each, into LDS), waves 2 / 3 the second on
        // [c0, c0 + 116) from there -- every wave of the workgroup takes part in its barriers
        if (nb > R.n1) return;   // workgroup-uniform
        const int c0 = R.w0 + tx * Body::kPairCols, p = wave & 1;
        const bool prod = wave < 2;
        const int m = (prod ? c0 - 2 + 60 * p : c0 + 60 * p) - 2 + lane;
        Lane L;
        L.pr = prod ? 1 : 2;
        L.j = min(max(m - (c0 - 2), 0), 2 * 60 - 1);
        // (X2: the producers' columns reach 2 into the halo; iteration keeps the points neighbours own)
        constexpr int xh = HasX2<Body>::v ? 2 : 0;
        L.out = lane >= 2 && lane < 62 &&
                (prod ? m >= R.m0 - xh && m <= R.m1 + xh : m >= R.m0 && m <= min(R.m1, c0 + Body::kPairCols - 1));
        // a producer counts its workgroup's (interior) columns only
        L.ccol = m >= c0 && m < c0 + Body::kPairCols && m >= R.m0 && m <= R.m1;
        L.m = L.me = min(max(m, R.mlo), R.mhi);
        L.edge = false;
        body.march(L, nb, ne);
        return;
    }
    if (mw > R.m1 || nb > R.n1) return;                            // wave-uniform
    Lane L;
    if (Body::kAligned) {
        const int m = mw + lane;
        L.out = m >= R.m0 && m <= R.m1;
        L.m = min(max(m, R.mlo), R.mhi);
        L.me = min(max(lane == 0 ? m - 1 : m + 1, R.mlo), R.mhi);
        L.edge = lane == 0 || lane == 63;
    } else {   // kHalo lanes on each side only load (the m -/+ kHalo neighbour columns)
        const int m = mw - Body::kHalo + lane;
        L.out = lane >= Body::kHalo && lane < 64 - Body::kHalo && m <= R.m1;
        L.m = L.me = min(max(m, R.mlo), R.mhi);
        L.edge = false;
    }
    body.march(L, nb, ne);
}

template <typename Body>
static MarchRect march_rect(const ocn_block *b, const Range &r, int rows = OCN_MARCH_ROWS, bool vert = false)
{
    int w0 = r.m0, cols = 64 - 2 * Body::kHalo, mlo = max(r.m0 - Body::kHalo, b->bnd_x1),
        mhi = min(r.m1 + Body::kHalo, b->bnd_x2);
    if (Body::kAligned) {   // waves start at nx_start + 64 j (256-B aligned rows, ocn_ctx.hip allocate)
        const int d = r.m0 - b->nx_start;
        w0 = b->nx_start + 64 * (d >= 0 ? d / 64 : -((63 - d) / 64));
        cols = 64;
        mlo = b->bnd_x1;
        mhi = b->bnd_x2;
    }
    const int wg_cols = (vert ? 1 : 4) * cols, wg_rows = (vert ? 4 : 1) * rows;
    const int ntx = (r.m1 - w0 + wg_cols) / wg_cols, nty = (r.n1 - r.n0 + wg_rows) / wg_rows;
    return MarchRect{r.m0, r.m1, r.n0, r.n1, w0, ntx, ntx * nty, mlo, mhi, rows, vert ? 1 : 0};
}

// Rows per wave tile for a range: `rows`, halved (not below OCN_MIN_ROWS) while the launch has
// fewer waves than fill the chip (256 CUs x 4 SIMDs x 2 waves).  A march wave's rows are a
// dependent chain of loads, so on small blocks (the Black Sea basin's 285 x 159, a 1024^2 box)
// a launch of few long tiles is latency-bound; shorter tiles trade warm-up rows for waves.
#ifndef OCN_FILL_WAVES
#define OCN_FILL_WAVES 2048
#endif
#ifndef OCN_MIN_ROWS
#define OCN_MIN_ROWS 2
#endif
template <typename Body> static int fit_rows(const Range &r, int rows)
{
    const int cols = Body::kAligned ? 64 : 64 - 2 * Body::kHalo;
    const long wx = (r.m1 - r.m0 + cols) / cols + (Body::kAligned ? 1 : 0);
    while (rows > OCN_MIN_ROWS && wx * ((r.n1 - r.n0 + rows) / rows) < OCN_FILL_WAVES) rows /= 2;
    return rows < OCN_MIN_ROWS ? OCN_MIN_ROWS : rows;
}

// rows = rows per tile (0: OCN_MARCH_ROWS, fitted to the range); vert: see MarchRect
template <typename Body>
static int launch_march_rects(const ocn_block *b, const Range *rs, int nr, const Body &body, hipStream_t s,
                              int rows = 0, bool vert = false)
{
    MarchGrid g{};
    for (int i = 0; i < nr; ++i)
        if (!range_empty(rs[i])) {
            g.r[g.nr] = march_rect<Body>(b, rs[i], rows > 0 ? rows : fit_rows<Body>(rs[i], OCN_MARCH_ROWS),
                                         vert && i >= 2);
            g.ntiles += g.r[g.nr].tiles;
            ++g.nr;
        }
    return issue_march(g, body, s);
}

template <typename Body>
static int launch_march(const ocn_block *b, const Range &r, const Body &body, hipStream_t s)
{
    return launch_march_rects(b, &r, 1, body, s);
}

// Halo-overlap split of a march launch's range: the inner part keeps 64 columns and 8 rows
// (a wave's width, a tile's height) away from the interior's edges, the frame is the rest as up
// to 4 bands, marched in one launch with short tiles (OCN_FRAME_ROWS rows; the left / right
// bands one wave wide with 4 row tiles per workgroup) -- a frame launch has too few waves to
// hide a long march's latency.  Inner points read no halo value and produce nothing a
// neighbour receives (the stencils reach +-1), so the inner part may run while an exchange is
// in flight.
#ifndef OCN_FRAME_ROWS
#define OCN_FRAME_ROWS 2
#endif
static Range march_inner(const ocn_block *b)
{
    return {b->nx_start + 64, b->nx_end - 64, b->ny_start + OCN_MARCH_ROWS, b->ny_end - OCN_MARCH_ROWS};
}
// the points of `all` outside `inner`, as up to 4 bands in one launch
template <typename Body>
static int launch_march_frame(const ocn_block *b, const Range &all, const Range &inner, const Body &body, hipStream_t s)
{
    const Range in = range_clip(all, inner);
    if (range_empty(in)) return launch_march(b, all, body, s);
    const Rects q = frame_rects(all, in);
    Range rs[4];
    for (int i = 0; i < 4; ++i) rs[i] = {q.m0[i], q.m0[i] + q.w[i] - 1, q.n0[i], q.n0[i] + q.h[i] - 1};
    return launch_march_rects(b, rs, 4, body, s, OCN_FRAME_ROWS, true);
}
template <typename Body>
static int launch_march_part(const ocn_block *b, const Range &all, int part, const Body &body, hipStream_t s)
{
    if (part == OCN_PART_INNER) return launch_march(b, range_clip(all, march_inner(b)), body, s);
    if (part == OCN_PART_FRAME) return launch_march_frame(b, all, march_inner(b), body, s);
    return launch_march(b, all, body, s);
}

// The march loop shared by every march body F: F::Batch holds one row's loads, F::load fills it,
// F::row consumes it (rotate the kept rows, compute, store).  Row n+1's loads are issued after row
// n's compute (issuing them before it, one iteration ahead, was measured slower: register pressure).
template <class F, class V>
__device__ __forceinline__ void march_rows(const F &k, V &x, const Lane &L, int nb, int ne)
{
    typename F::Batch cur, nxt;
    k.load(cur, L, nb);
    for (int n = nb; n <= ne; ++n) {
        k.row(x, cur, L, n);
        if (n < ne) {
            k.load(nxt, L, n + 1);
            cur = nxt;
        }
    }
}

// The view of fused B's three stages (sw_stencils.h uv_trans_math / uv_diff2_math /
// sw_update_uv_math) over the march registers.  Accessor names follow the stage functors; an
// array named twice there (u = ubrtr, hu = hhu, hh = hhh) is one register set here.
// RC ("recompute"): hhq = h_r + ssh * ffs is formed from h_r and ssh (hh_init's whole-array
// formula) instead of being read; hhu_p / hhv_p are set by the march from sshp (see MarchFusedB).
template <bool RC> struct MarchViewB {
    RowsD<true, true> rU, rV, rHV, rMU;                // ubrtr, vbrtr, hhv, mu
    RowsD<false, true> rHU, rHQ, rSTT, rSSH, rHR, rSHP; // hhu, hhq (or h_r, sshp when RC), str_t, ssh
    RowsD<true, false> rVORT, rHH, rSTS;               // vort, hhh, str_s
    Here hhun_, hhup_, hhvn_, hhvp_, ubrtrp_, vbrtrp_, rhsx_, rhsy_;
    BitRows<true, true> bits;                          // mask bytes (row n+1 only when RC)
    MetRows met;                                       // metric rows n-1, n, n+1 (compact tables)
    double tau, f;
    __device__ __forceinline__ double quot(double a, double b, int, int) const { return a / b; }
    __device__ __forceinline__ double qtau(double a) const { return a / tau; }
    OCN_MV(u, rU) OCN_MV(ubrtr, rU) OCN_MV(v, rV) OCN_MV(vbrtr, rV) OCN_MV(hu, rHU) OCN_MV(hhu, rHU)
    OCN_MV(hv, rHV) OCN_MV(hhv, rHV) OCN_MV(hh, rHH) OCN_MV(hhh, rHH) OCN_MV(mu, rMU)
    OCN_MV(vort, rVORT) OCN_MV(str_t, rSTT) OCN_MV(str_s, rSTS) OCN_MV(ssh, rSSH)
    OCN_MV(hhun, hhun_) OCN_MV(hhup, hhup_) OCN_MV(hhvn, hhvn_) OCN_MV(hhvp, hhvp_) OCN_MV(ubrtrp, ubrtrp_)
    OCN_MV(vbrtrp, vbrtrp_) OCN_MV(RHSx, rhsx_) OCN_MV(RHSy, rhsy_)
    OCN_MV(h_r, rHR) OCN_MV(shp, rSHP)
    OCN_MG_ALL OCN_MG(rlh_s, OCN_RLH_S) OCN_MG(rdis, OCN_R_DISS)
    __device__ __forceinline__ double hq(int dx, int dy) const
    {
        if constexpr (RC) return rHR.at(dx, dy) + rSSH.at(dx, dy) * f;   // depth.f90:48 hq = h_r + sh*ffs
        else return rHQ.at(dx, dy);
    }
    __device__ __forceinline__ float luu(int dx, int dy) const
    {
        if (dx != 0 || dy < -1 || dy > 0) ocn_march_bad_access();
        return (bits.at(0, dy) & (1u << OCN_LUU)) ? 1.0f : 0.0f;
    }
    __device__ __forceinline__ float lu(int dx, int dy) const { return bits.at(dx, dy) & (1u << OCN_LU) ? 1.0f : 0.0f; }
};

// fused B (sw_stencils.h FusedB) as a register march (offset layout); compact static fields only.
// C1F: the "role-flip" form of the step (ocn_ctx.hip one_step_fused): the launch also runs a8
// sw_next_step's time filters on the interior (sshp, ubrtrp, vbrtrp updated in place -- each is
// read only at its own point) and check_ssh_err on the new ssh (= sshn on sea points); a8's
// copies ssh := sshn, ubrtr := ubrtrn, vbrtr := vbrtrn are not made -- the host swaps the roles
// of the two buffers of each pair instead, so nothing this launch reads at a neighbour is written.
// RC (role-flip reuse steps after a MarchCA<false>, which did not store hhq, hhu_p, hhv_p on
// the interior): hhq is formed from h_r + ssh * ffs, and hhu_p / hhv_p are hh_init's level-1
// interpolations of h_r + sshp * ffs (sw_stencils.h interp_u / interp_v, the same operands and
// arithmetic as the hh_init that would have stored them; sshp has not changed since) where
// llu / llv is set, and the array's never-written value elsewhere.  sshp is read at m+1 / n+1
// here, so a8's new sshp goes to the second sshp buffer (sshp_out), which the host swaps in.
// ALT (one-pass calls with halo exchanges, the frame around the one-pass step's inner part): a8's
// filtered sshp / ubrtrp / vbrtrp all go to the second buffers (sshp_out, up_out, vp_out), as the
// one-pass step writes them, since it reads the current ones at neighbours.
template <bool C1F, bool RC = false, bool ALT = false> struct MarchFusedB {
    static constexpr bool kAligned = false;
    static constexpr int kHalo = 1;
    ocn_block b; Tab<true> t; ocn_sw_params sw; double tau; bool full, reuse; int32_t *nbad; double *sshp_out;
    double *up_out = nullptr, *vp_out = nullptr;
    using View = MarchViewB<RC>;
    struct Fn {
        FusedB<true> k; const Tab<true> &t; SwNextStep<true> a8; HhInit<true> c2; int *nbad; double *sshp_out;
        double *up_out, *vp_out;
        // row n: ubrtr, vbrtr, hhv, mu, hhu, hhq (RC: h_r and sshp), str_t, ssh at n+1; vort, hhh,
        // str_s, mask bytes (RC: at n+1) and the pointwise operands at n; metric row n+1
        struct Batch { double nn[9], c[3], h[8], p[2]; unsigned bits; float g[kRowTable]; };
        __device__ __forceinline__ void load(Batch &q, const Lane &L, int n) const
        {
            const SwUpdateUv<true> &a7 = k.a7;
            const Pt c = a7.I(L.m, n), cn = a7.I(L.m, n + 1);
            q.nn[0] = ld(a7.ubrtr, cn); q.nn[1] = ld(a7.vbrtr, cn); q.nn[2] = ld(a7.hhv, cn);
            q.nn[3] = ld(k.a6.mu, cn); q.nn[4] = ld(a7.hhu, cn);
            if (RC) { q.nn[5] = ld(c2.h_r, cn); q.nn[8] = ld(a8.sshp, cn); }
            else q.nn[5] = ld(k.a6.hq, cn);
            q.nn[6] = ld(k.a6.str_t, cn); q.nn[7] = ld(a7.ssh, cn);
            q.c[0] = ld(k.a4.vort, c); q.c[1] = ld(a7.hhh, c); q.c[2] = ld(k.a6.str_s, c);
            q.bits = ld(t.bits, RC ? cn : c);
            if (!(RC && k.a7.hhun == k.a7.hhu)) { q.h[0] = ld(a7.hhun, c); q.h[2] = ld(a7.hhvn, c); }
            if (!RC) { q.h[1] = ld(a7.hhup, c); q.h[3] = ld(a7.hhvp, c); }
            q.h[4] = ld(a7.ubrtrp, c); q.h[5] = ld(a7.vbrtrp, c); q.h[6] = ld(a7.RHSx, c); q.h[7] = ld(a7.RHSy, c);
            if (C1F) { q.p[0] = ld(a8.sshn, c); if (!RC) q.p[1] = ld(a8.sshp, c); }
            MetRows::load(q.g, t.rows, t.nrows, cn.r);
        }
        __device__ __forceinline__ void row(View &x, const Batch &q, const Lane &L, int n) const
        {
            const SwUpdateUv<true> &a7 = k.a7;
            const Pt c = a7.I(L.m, n);
            x.rVORT.s = x.rVORT.c; x.rHH.s = x.rHH.c; x.rSTS.s = x.rSTS.c;
            x.met.shift(q.g);
            x.rU.nn = q.nn[0]; x.rV.nn = q.nn[1]; x.rHV.nn = q.nn[2]; x.rMU.nn = q.nn[3];
            x.rHU.nn = q.nn[4]; x.rSTT.nn = q.nn[6]; x.rSSH.nn = q.nn[7];
            if (RC) { x.rHR.nn = q.nn[5]; x.rSHP.nn = q.nn[8]; x.bits.nn = q.bits; }
            else { x.rHQ.nn = q.nn[5]; x.bits.s = x.bits.c; x.bits.c = q.bits; }
            x.rVORT.c = q.c[0]; x.rHH.c = q.c[1]; x.rSTS.c = q.c[2];
            if (RC && k.a7.hhun == k.a7.hhu) { x.hhun_.v = x.rHU.c; x.hhvn_.v = x.rHV.c; }   // reuse: the same arrays
            else { x.hhun_.v = q.h[0]; x.hhvn_.v = q.h[2]; }
            x.ubrtrp_.v = q.h[4]; x.vbrtrp_.v = q.h[5]; x.rhsx_.v = q.h[6]; x.rhsy_.v = q.h[7];
            const unsigned bc = x.bits.c;
            if (RC) {   // hh_init's level 1 (depth.f90:76-97 with hqp = h_r + sshp*ffs)
                const double f = x.f;
                const double b00 = x.rHR.c + x.rSHP.c * f;
                const double b10 = x.h_r(1, 0) + x.shp(1, 0) * f, b01 = x.rHR.nn + x.rSHP.nn * f;
                const double up = interp_u(x, b00, b10), vp = interp_v(x, b00, b01);
                x.hhup_.v = (bc & (1u << OCN_LLU)) ? up : ld(c2.hup, c);
                x.hhvp_.v = (bc & (1u << OCN_LLV)) ? vp : ld(c2.hvp, c);
            } else {
                x.hhup_.v = q.h[1]; x.hhvp_.v = q.h[3];
            }

            double rxa, rya, rxd, ryd;
            if (k.do_adv) uv_trans_math(x, rxa, rya);
            else { rxa = ld(a7.RHSx_adv, c); rya = ld(a7.RHSy_adv, c); }
            if (k.do_dif) uv_diff2_math(x, rxd, ryd);
            else { rxd = ld(a7.RHSx_dif, c); ryd = ld(a7.RHSy_dif, c); }
            double un, vn;
            sw_update_uv_math(x, rxa, rxd, rya, ryd, un, vn);
            if (L.out) {
                if (bc & (1u << OCN_LCU)) {
                    if (k.do_adv && k.full) st(k.a4.RHSx, c, rxa);
                    if (k.do_dif && k.full) st(k.a6.RHSx, c, rxd);
                    st(a7.ubrtrn, c, un);
                }
                if (bc & (1u << OCN_LCV)) {
                    if (k.do_adv && k.full) st(k.a4.RHSy, c, rya);
                    if (k.do_dif && k.full) st(k.a6.RHSy, c, ryd);
                    st(a7.vbrtrn, c, vn);
                }
            }
            if (C1F) {   // a8 on this interior point (SwNextStep::step without the copies)
                const double ts = a8.ts, xn = q.p[0];
                const double fx = asselin(x.rSSH.c, xn, RC ? x.rSHP.c : q.p[1], ts);
                const double fa = asselin(x.rU.c, un, x.ubrtrp_.v, ts), fb = asselin(x.rV.c, vn, x.vbrtrp_.v, ts);
                if (L.out) {
                    const bool bl = bc & (1u << OCN_LU);
                    if (bl) st(RC || ALT ? sshp_out : a8.sshp, c, fx);   // RC: sshp is read at neighbours here
                    if (bc & (1u << OCN_LCU)) st(ALT ? up_out : a8.up, c, fa);
                    if (bc & (1u << OCN_LCV)) st(ALT ? vp_out : a8.vp, c, fb);
                    if (nbad && bl && !(xn < 10000.0 && xn > -10000.0)) OCN_ATOMIC_INC(nbad);
                }
            }
            x.rU.rotate(); x.rV.rotate(); x.rHV.rotate(); x.rMU.rotate();
            x.rHU.rotate(); x.rSTT.rotate(); x.rSSH.rotate();
            if (RC) { x.rHR.rotate(); x.rSHP.rotate(); x.bits.rotate(); }
            else x.rHQ.rotate();
        }
    };
    __device__ void march(const Lane &L, int nb, int ne) const
    {
        const Fn f{make_fused_b(&b, t, sw, tau, full, reuse), t, make_sw_next_step(&b, t, sw.time_smooth),
                   make_hh_init(&b, t, (int)sw.full_free_surface, false), (int *)nbad, sshp_out, up_out, vp_out};
        const SwUpdateUv<true> &a7 = f.k.a7;
        View x{};
        x.tau = tau;
        x.f = (double)sw.full_free_surface;
        const Pt s = a7.I(L.m, nb - 1), c = a7.I(L.m, nb);   // rows kept from before the first row
        x.rU.s = ld(a7.ubrtr, s); x.rU.c = ld(a7.ubrtr, c);
        x.rV.s = ld(a7.vbrtr, s); x.rV.c = ld(a7.vbrtr, c);
        x.rHV.s = ld(a7.hhv, s); x.rHV.c = ld(a7.hhv, c);
        x.rMU.s = ld(f.k.a6.mu, s); x.rMU.c = ld(f.k.a6.mu, c);
        x.rHU.c = ld(a7.hhu, c); x.rSTT.c = ld(f.k.a6.str_t, c); x.rSSH.c = ld(a7.ssh, c);
        if (RC) {
            x.rHR.c = ld(f.c2.h_r, c); x.rSHP.c = ld(f.a8.sshp, c);
            x.bits.s = ld(t.bits, s); x.bits.c = ld(t.bits, c);
        } else {
            x.rHQ.c = ld(f.k.a6.hq, c);
            x.bits.c = ld(t.bits, s);
        }
        x.rVORT.c = ld(f.k.a4.vort, s); x.rHH.c = ld(a7.hhh, s); x.rSTS.c = ld(f.k.a6.str_s, s);
        x.met.preload(t.rows, t.nrows, s.r, c.r);
        march_rows(f, x, L, nb, ne);
    }
};

// a4 uv_trans alone (the reference stage over the compact tables, ocn_ctx envoke) as a register
// march (offset layout): its six real(8) operands are read at up to six neighbours each, which
// one thread per point issues as 26 loads per cell; here each is loaded once per cell.
struct MarchViewT {
    RowsD<true, true> rU, rV, rHV;        // ubrtr, vbrtr, hhv: rows n-1 .. n+1
    RowsD<false, true> rHU;               // hhu: rows n, n+1
    RowsD<true, false> rVORT, rHH;        // vort, hhh: rows n-1, n
    BitRows<true, false> bits;            // mask bytes: rows n-1, n
    MetRows met;
    OCN_MV(u, rU) OCN_MV(v, rV) OCN_MV(hu, rHU) OCN_MV(hv, rHV) OCN_MV(vort, rVORT) OCN_MV(hh, rHH)
    OCN_MG_ALL
    __device__ __forceinline__ float luu(int dx, int dy) const
    {
        if (dx != 0) ocn_march_bad_access();
        return (bits.at(0, dy) & (1u << OCN_LUU)) ? 1.0f : 0.0f;
    }
};
struct MarchUvTrans {
    static constexpr bool kAligned = false;
    static constexpr int kHalo = 1;
    ocn_block b; Tab<true> t;
    using View = MarchViewT;
    struct Fn {
        UvTrans<true> k; const Tab<true> &t;
        // row n: ubrtr, vbrtr, hhv, hhu at n+1; vort, hhh, the mask byte at n; metric row n+1
        struct Batch { double nn[4], c[2]; unsigned bits; float g[kRowTable]; };
        __device__ __forceinline__ void load(Batch &q, const Lane &L, int n) const
        {
            const Pt c = k.I(L.m, n), cn = k.I(L.m, n + 1);
            q.nn[0] = ld(k.u, cn); q.nn[1] = ld(k.v, cn); q.nn[2] = ld(k.hv, cn); q.nn[3] = ld(k.hu, cn);
            q.c[0] = ld(k.vort, c); q.c[1] = ld(k.hh, c);
            q.bits = ld(t.bits, c);
            MetRows::load(q.g, t.rows, t.nrows, cn.r);
        }
        __device__ __forceinline__ void row(View &x, const Batch &q, const Lane &L, int n) const
        {
            const Pt c = k.I(L.m, n);
            x.rVORT.s = x.rVORT.c; x.rHH.s = x.rHH.c;
            x.met.shift(q.g);
            x.rU.nn = q.nn[0]; x.rV.nn = q.nn[1]; x.rHV.nn = q.nn[2]; x.rHU.nn = q.nn[3];
            x.rVORT.c = q.c[0]; x.rHH.c = q.c[1];
            x.bits.s = x.bits.c; x.bits.c = q.bits;
            double rx, ry;
            uv_trans_math(x, rx, ry);
            if (L.out) {
                const unsigned bc = x.bits.c;
                if (bc & (1u << OCN_LCU)) st(k.RHSx, c, rx);
                if (bc & (1u << OCN_LCV)) st(k.RHSy, c, ry);
            }
            x.rU.rotate(); x.rV.rotate(); x.rHV.rotate(); x.rHU.rotate();
        }
    };
    __device__ void march(const Lane &L, int nb, int ne) const
    {
        const Fn f{make_uv_trans(&b, t), t};
        View x{};
        const Pt s = f.k.I(L.m, nb - 1), c = f.k.I(L.m, nb);   // rows kept from before the first row
        x.rU.s = ld(f.k.u, s); x.rU.c = ld(f.k.u, c);
        x.rV.s = ld(f.k.v, s); x.rV.c = ld(f.k.v, c);
        x.rHV.s = ld(f.k.hv, s); x.rHV.c = ld(f.k.hv, c);
        x.rHU.c = ld(f.k.hu, c);
        x.rVORT.c = ld(f.k.vort, s); x.rHH.c = ld(f.k.hh, s);
        x.bits.c = ld(t.bits, s);
        x.met.preload(t.rows, t.nrows, s.r, c.r);
        march_rows(f, x, L, nb, ne);
    }
};

// The view of fused A's stages (sw_stencils.h sw_update_ssh_math, hh_update_math,
// uv_trans_vort_math, stress_components_math) over the march registers.  Arrays read at m-1 or
// m+1 keep edge values (aligned layout).
struct MarchViewA {
    RowsD<false, true, true> rU, rUP, rHR, rSH;        // ubrtr, ubrtrp, h_r, ssh
    RowsD<true, false, true> rV, rVP;                  // vbrtr, vbrtrp
    RowsD<true, false> rHV;                            // hhv
    RowsD<false, false, true> rHU;                     // hhu
    Here sshp_;
    BitRows<false, true, true> bits;
    MetRows met;
    double tau;
    __device__ __forceinline__ double tau2() const { return tau; }
    OCN_MV(u, rU) OCN_MV(ubrtr, rU) OCN_MV(v, rV) OCN_MV(vbrtr, rV) OCN_MV(up, rUP) OCN_MV(vp, rVP)
    OCN_MV(hhu, rHU) OCN_MV(hhv, rHV) OCN_MV(sshp, sshp_) OCN_MV(h_r, rHR) OCN_MV(sh, rSH)
    OCN_MG_ALL
    __device__ __forceinline__ float lu(int dx, int dy) const { return bits.mask(OCN_LU, dx, dy); }
};

// fused A (sw_stencils.h FusedA) as a register march (aligned layout); HH = a2 hh_update is part
// of the launch (range [start-1, end]^2, a1/a3/a5 on [start, end]^2) or not (reuse steps,
// [start, end]^2)
template <bool HH> struct MarchFusedA {
    static constexpr bool kAligned = true;
    static constexpr int kHalo = 0;
    ocn_block b; Tab<true> t; ocn_sw_params sw; double tau;
    using View = MarchViewA;
    struct Fn {
        FusedA<true> k; const Tab<true> &t;
        // row n: ubrtr, ubrtrp, mask bytes, h_r, ssh at n+1; vbrtr, hhv, vbrtrp, hhu, sshp at n;
        // edge values of the arrays read at m+-1; metric row n+1
        struct Batch { double nn[4], c[5], enn[4], ec[3]; unsigned bits, ebits; float g[kRowTable]; };
        __device__ __forceinline__ void load(Batch &q, const Lane &L, int n) const
        {
            const SwUpdateSsh<true> &a1 = k.a1;
            for (int i = 0; i < 4; ++i) q.enn[i] = 0.0;
            for (int i = 0; i < 3; ++i) q.ec[i] = 0.0;
            q.ebits = 0;
            const Pt c = a1.I(L.m, n), cn = a1.I(L.m, n + 1);
            q.nn[0] = ld(a1.ubrtr, cn); q.nn[1] = ld(k.a5.u, cn); q.bits = ld(t.bits, cn);
            if (HH) { q.nn[2] = ld(k.a2.h_r, cn); q.nn[3] = ld(k.a2.sh, cn); }
            q.c[0] = ld(a1.vbrtr, c); q.c[1] = ld(a1.hhv, c); q.c[2] = ld(k.a5.v, c);
            q.c[3] = ld(a1.hhu, c); q.c[4] = ld(a1.sshp, c);
            if (L.edge) {
                const Pt e = a1.I(L.me, n), en = a1.I(L.me, n + 1);
                q.enn[0] = ld(a1.ubrtr, en); q.enn[1] = ld(k.a5.u, en); q.ebits = ld(t.bits, en);
                if (HH) { q.enn[2] = ld(k.a2.h_r, en); q.enn[3] = ld(k.a2.sh, en); }
                q.ec[0] = ld(a1.vbrtr, e); q.ec[1] = ld(k.a5.v, e); q.ec[2] = ld(a1.hhu, e);
            }
            MetRows::load(q.g, t.rows, t.nrows, cn.r);
        }
        __device__ __forceinline__ void row(View &x, const Batch &q, const Lane &L, int n) const
        {
            const Pt c = k.a1.I(L.m, n);
            x.rV.s = x.rV.c; x.rV.es = x.rV.ec; x.rHV.s = x.rHV.c; x.rVP.s = x.rVP.c; x.rVP.es = x.rVP.ec;
            x.met.shift(q.g);
            x.rU.nn = q.nn[0]; x.rUP.nn = q.nn[1]; x.bits.nn = q.bits;
            x.rU.enn = q.enn[0]; x.rUP.enn = q.enn[1]; x.bits.enn = q.ebits;
            if (HH) { x.rHR.nn = q.nn[2]; x.rSH.nn = q.nn[3]; x.rHR.enn = q.enn[2]; x.rSH.enn = q.enn[3]; }
            x.rV.c = q.c[0]; x.rHV.c = q.c[1]; x.rVP.c = q.c[2]; x.rHU.c = q.c[3]; x.sshp_.v = q.c[4];
            x.rV.ec = q.ec[0]; x.rVP.ec = q.ec[1]; x.rHU.ec = q.ec[2];
            const unsigned bc = x.bits.c;
            if (n >= k.sy) {   // wave-uniform
                const bool in = L.out && L.m >= k.sx;
                const double r = sw_update_ssh_math(x);
                if (in && (bc & (1u << OCN_LU))) st(k.a1.sshn, c, r);
                if (k.do_vort) {
                    const double v = uv_trans_vort_math(x);
                    if (in && (bc & (1u << OCN_LUU))) st(k.a3.vort, c, v);
                }
                if (k.do_stress) {
                    double vt, vs;
                    stress_components_math(x, vt, vs);
                    if (in && (bc & (1u << OCN_LU))) st(k.a5.str_t, c, vt);
                    if (in && (bc & (1u << OCN_LUU))) st(k.a5.str_s, c, vs);
                }
            }
            if (HH) {
                double xu, xv, xh;
                hh_update_math(x, x.rHR.c + x.rSH.c, xu, xv, xh);
                if (L.out) {
                    if (bc & (1u << OCN_LLU)) st(k.a2.hun, c, xu);
                    if (bc & (1u << OCN_LLV)) st(k.a2.hvn, c, xv);
                    if (bc & (1u << OCN_LUH)) st(k.a2.hhn, c, xh);
                }
            }
            x.rU.rotate(); x.rUP.rotate(); x.bits.rotate();
            if (HH) { x.rHR.rotate(); x.rSH.rotate(); }
        }
    };
    __device__ void march(const Lane &L, int nb, int ne) const
    {
        const Fn f{make_fused_a(&b, t, sw, tau, !HH), t};
        const SwUpdateSsh<true> &a1 = f.k.a1;
        View x{};
        x.tau = tau;
        const Pt s = a1.I(L.m, nb - 1), c = a1.I(L.m, nb);
        x.rU.c = ld(a1.ubrtr, c); x.rUP.c = ld(f.k.a5.u, c); x.bits.c = ld(t.bits, c);
        if (HH) { x.rHR.c = ld(f.k.a2.h_r, c); x.rSH.c = ld(f.k.a2.sh, c); }
        x.rV.c = ld(a1.vbrtr, s); x.rHV.c = ld(a1.hhv, s); x.rVP.c = ld(f.k.a5.v, s);
        if (L.edge) {
            const Pt es = a1.I(L.me, nb - 1), ec = a1.I(L.me, nb);
            x.rU.ec = ld(a1.ubrtr, ec); x.rUP.ec = ld(f.k.a5.u, ec); x.bits.ec = ld(t.bits, ec);
            if (HH) { x.rHR.ec = ld(f.k.a2.h_r, ec); x.rSH.ec = ld(f.k.a2.sh, ec); }
            x.rV.ec = ld(a1.vbrtr, es); x.rVP.ec = ld(f.k.a5.v, es);
        }
        x.met.preload(t.rows, t.nrows, s.r, c.r);
        march_rows(f, x, L, nb, ne);
    }
};

// The view of hh_init (sw_stencils.h hh_init_math) over the march registers.
struct MarchViewH {
    RowsD<false, true, true> rHR, rSH, rSHP;           // h_r, ssh, sshp
    BitRows<false, true, true> bits;
    MetRows met;
    double cu = 0.0, cv = 0.0;                          // (copies) ubrtr, vbrtr at row n
    OCN_MV(h_r, rHR) OCN_MV(sh, rSH) OCN_MV(shp, rSHP)
    OCN_MG_ALL
    __device__ __forceinline__ float lu(int dx, int dy) const { return bits.mask(OCN_LU, dx, dy); }
};

// fused C2 = a10 hh_init (sw_stencils.h HhInit) as a register march (aligned layout) over any
// part of the whole bnd range: row n+1 is clamped to bnd_y2 (its values are used only where
// n <= end, where it is in range)
#ifndef OCN_HH_NT
#define OCN_HH_NT 0   // the call tail's hh_init stores as nontemporal stores (an A/B switch)
#endif
template <class T> __device__ __forceinline__ void st_hh(T *__restrict__ p, Pt q, T v)
{
    if constexpr (OCN_HH_NT) __builtin_nontemporal_store(v, (T *)((char *)p + q.c * (unsigned)sizeof(T)));
    else st(p, q, v);
}
struct MarchHhInit {
    static constexpr bool kAligned = true;
    static constexpr int kHalo = 0;
    // keep_n (with full): the n level (hqn = h_r and its interpolations hun / hvn / hhn) is not
    // stored -- the arrays hold exactly those values already (ocn_ctx.hip last_finish, hn_fresh)
    // copy (the call tail's a8 copies, ocn_ctx.hip last_finish): sshn := ssh, ubrtrn := ubrtr,
    // vbrtrn := vbrtr over the bnd range with the march -- ssh is the value hh_init reads anyway
    ocn_block b; Tab<true> t; int ffs; bool full; bool keep_n = false;
    const double *cu_src = nullptr, *cv_src = nullptr;
    double *csh_dst = nullptr, *cu_dst = nullptr, *cv_dst = nullptr;
    using View = MarchViewH;
    struct Fn {
        HhInit<true> k; const Tab<true> &t; int ylast; bool keep_n;
        const double *cu_src, *cv_src; double *csh_dst, *cu_dst, *cv_dst;
        // row n: h_r, ssh, sshp, mask bytes (+ edge values) and metrics at row n+1 (copies: ubrtr,
        // vbrtr there too)
        struct Batch { double nn[3], enn[3], uv[2]; unsigned bits, ebits; float g[kRowTable]; };
        __device__ __forceinline__ void load(Batch &q, const Lane &L, int n) const
        {
            const int r = min(n + 1, ylast);
            const Pt cn = k.I(L.m, r);
            q.enn[0] = q.enn[1] = q.enn[2] = 0.0;
            q.ebits = 0;
            q.nn[0] = ld(k.h_r, cn); q.nn[1] = ld(k.sh, cn); q.nn[2] = ld(k.shp, cn); q.bits = ld(t.bits, cn);
            q.uv[0] = q.uv[1] = 0.0;
            if (csh_dst) { q.uv[0] = ld(cu_src, cn); q.uv[1] = ld(cv_src, cn); }   // (a kernel argument: uniform)
            if (L.edge) {
                const Pt en = k.I(L.me, r);
                q.enn[0] = ld(k.h_r, en); q.enn[1] = ld(k.sh, en); q.enn[2] = ld(k.shp, en); q.ebits = ld(t.bits, en);
            }
            MetRows::load(q.g, t.rows, t.nrows, cn.r);
        }
        __device__ __forceinline__ void row(View &x, const Batch &q, const Lane &L, int n) const
        {
            const Pt c = k.I(L.m, n);
            const double f = k.f;
            x.met.shift(q.g);
            x.rHR.nn = q.nn[0]; x.rSH.nn = q.nn[1]; x.rSHP.nn = q.nn[2]; x.bits.nn = q.bits;
            x.rHR.enn = q.enn[0]; x.rSH.enn = q.enn[1]; x.rSHP.enn = q.enn[2]; x.bits.enn = q.ebits;
            const double r00 = x.rHR.c;
            if (csh_dst && L.out) { st_hh(csh_dst, c, x.rSH.c); st_hh(cu_dst, c, x.cu); st_hh(cv_dst, c, x.cv); }
            x.cu = q.uv[0]; x.cv = q.uv[1];
            if (L.out) {
                st_hh(k.hq, c, r00 + x.rSH.c * f);
                if (k.full) {
                    st_hh(k.hqp, c, r00 + x.rSHP.c * f);
                    if (!keep_n) st_hh(k.hqn, c, r00);
                }
            }
            if (n >= k.j0 && n <= k.j1) {   // wave-uniform
                HhInitOut o;
                hh_init_math(x, f, k.full && !keep_n, o);
                if (L.out && L.m >= k.i0 && L.m <= k.i1) {
                    const unsigned bc = x.bits.c;
                    const bool bu = bc & (1u << OCN_LLU), bv = bc & (1u << OCN_LLV), bh = bc & (1u << OCN_LUH);
                    if (bu) { st_hh(k.hu, c, o.u[0]); st_hh(k.hup, c, o.u[1]); }
                    if (bv) { st_hh(k.hv, c, o.v[0]); st_hh(k.hvp, c, o.v[1]); }
                    if (bh) { st_hh(k.hh, c, o.h[0]); st_hh(k.hhp, c, o.h[1]); }
                    if (k.full && !keep_n) {
                        if (bu) st_hh(k.hun, c, o.u[2]);
                        if (bv) st_hh(k.hvn, c, o.v[2]);
                        if (bh) st_hh(k.hhn, c, o.h[2]);
                    }
                }
            }
            x.rHR.rotate(); x.rSH.rotate(); x.rSHP.rotate(); x.bits.rotate();
        }
    };
    __device__ void march(const Lane &L, int nb, int ne) const
    {
        const Fn f{make_hh_init(&b, t, ffs, full), t, b.bnd_y2, keep_n, cu_src, cv_src, csh_dst, cu_dst, cv_dst};
        View x{};
        const Pt c = f.k.I(L.m, nb);
        x.rHR.c = ld(f.k.h_r, c); x.rSH.c = ld(f.k.sh, c); x.rSHP.c = ld(f.k.shp, c); x.bits.c = ld(t.bits, c);
        if (csh_dst) { x.cu = ld(cu_src, c); x.cv = ld(cv_src, c); }
        if (L.edge) {
            const Pt e = f.k.I(L.me, nb);
            x.rHR.ec = ld(f.k.h_r, e); x.rSH.ec = ld(f.k.sh, e); x.rSHP.ec = ld(f.k.shp, e); x.bits.ec = ld(t.bits, e);
        }
        x.met.preload(t.rows, t.nrows, c.r, c.r);
        march_rows(f, x, L, nb, ne);
    }
};

// ------------------------------------------------------------------ kernel entries on 2-D arrays
// The ocn_hh_init / ocn_uv_trans kernel entries read the real(4) masks and metrics the caller
// passes (2-D arrays, no compact tables): the same register marches as MarchHhInit / MarchUvTrans
// with those arrays in rings of their own (one load per array and cell; m+-1 by DPP).

// a10 hh_init (sw_stencils.h HhInit<false>, every level) as an aligned register march over any
// part of the bnd range (row n+1 clamped to bnd_y2: its values are used only where n <= end)
struct MarchViewH2 {
    RowsD<false, true, true> rHR, rSH, rSHP;           // h_r, ssh, sshp: rows n, n+1, columns m, m+1
    RowsF<false, true, true> rLU, rDX, rDY;            // lu, dx, dy at the same corners
    HereF dxt_, dyt_, dxh_, dyh_, dxb_, dyb_;
    OCN_MV(h_r, rHR) OCN_MV(sh, rSH) OCN_MV(shp, rSHP)
    __device__ __forceinline__ float lu(int dx, int dy) const { return rLU.at(dx, dy); }
    __device__ __forceinline__ float dx(int i, int j) const { return rDX.at(i, j); }
    __device__ __forceinline__ float dy(int i, int j) const { return rDY.at(i, j); }
    __device__ __forceinline__ float dxt(int i, int j) const { return dxt_.at(i, j); }
    __device__ __forceinline__ float dyt(int i, int j) const { return dyt_.at(i, j); }
    __device__ __forceinline__ float dxh(int i, int j) const { return dxh_.at(i, j); }
    __device__ __forceinline__ float dyh(int i, int j) const { return dyh_.at(i, j); }
    __device__ __forceinline__ float dxb(int i, int j) const { return dxb_.at(i, j); }
    __device__ __forceinline__ float dyb(int i, int j) const { return dyb_.at(i, j); }
};
struct MarchHhInit2D {
    static constexpr bool kAligned = true;
    static constexpr int kHalo = 0;
    HhInit<false> k; int ylast;
    using View = MarchViewH2;
    struct Fn {
        const HhInit<false> &k; int ylast;
        // row n: h_r, ssh, sshp, lu, dx, dy at row n+1 (+ edge values); the centre-only metrics and
        // the level masks at row n
        struct Batch { double nn[3], enn[3]; float fn[3], efn[3], c[9]; };
        __device__ __forceinline__ void load(Batch &q, const Lane &L, int n) const
        {
            const Interp<false> &W = k.W;
            const Pt cn = k.I(L.m, min(n + 1, ylast)), c = k.I(L.m, n);
            q.nn[0] = ld(k.h_r, cn); q.nn[1] = ld(k.sh, cn); q.nn[2] = ld(k.shp, cn);
            q.fn[0] = ld(W.lu, cn); q.fn[1] = ld(W.dx, cn); q.fn[2] = ld(W.dy, cn);
            for (int i = 0; i < 3; ++i) { q.enn[i] = 0.0; q.efn[i] = 0.0f; }
            if (L.edge) {
                const Pt en = k.I(L.me, min(n + 1, ylast));
                q.enn[0] = ld(k.h_r, en); q.enn[1] = ld(k.sh, en); q.enn[2] = ld(k.shp, en);
                q.efn[0] = ld(W.lu, en); q.efn[1] = ld(W.dx, en); q.efn[2] = ld(W.dy, en);
            }
            q.c[0] = ld(W.dxt, c); q.c[1] = ld(W.dyt, c); q.c[2] = ld(W.dxh, c); q.c[3] = ld(W.dyh, c);
            q.c[4] = ld(W.dxb, c); q.c[5] = ld(W.dyb, c);
            q.c[6] = ld(k.llu, c); q.c[7] = ld(k.llv, c); q.c[8] = ld(k.luh, c);
        }
        __device__ __forceinline__ void row(View &x, const Batch &q, const Lane &L, int n) const
        {
            const Pt c = k.I(L.m, n);
            const double f = k.f;
            x.rHR.nn = q.nn[0]; x.rSH.nn = q.nn[1]; x.rSHP.nn = q.nn[2];
            x.rHR.enn = q.enn[0]; x.rSH.enn = q.enn[1]; x.rSHP.enn = q.enn[2];
            x.rLU.nn = q.fn[0]; x.rDX.nn = q.fn[1]; x.rDY.nn = q.fn[2];
            x.rLU.enn = q.efn[0]; x.rDX.enn = q.efn[1]; x.rDY.enn = q.efn[2];
            x.dxt_.v = q.c[0]; x.dyt_.v = q.c[1]; x.dxh_.v = q.c[2]; x.dyh_.v = q.c[3];
            x.dxb_.v = q.c[4]; x.dyb_.v = q.c[5];
            const double r00 = x.rHR.c;
            if (L.out) {
                st(k.hq, c, r00 + x.rSH.c * f);
                if (k.full) { st(k.hqp, c, r00 + x.rSHP.c * f); st(k.hqn, c, r00); }
            }
            if (n >= k.j0 && n <= k.j1) {   // wave-uniform
                HhInitOut o;
                hh_init_math(x, f, k.full, o);
                if (L.out && L.m >= k.i0 && L.m <= k.i1) {
                    const bool bu = q.c[6] > 0.5f, bv = q.c[7] > 0.5f, bh = q.c[8] > 0.5f;
                    if (bu) { st(k.hu, c, o.u[0]); st(k.hup, c, o.u[1]); }
                    if (bv) { st(k.hv, c, o.v[0]); st(k.hvp, c, o.v[1]); }
                    if (bh) { st(k.hh, c, o.h[0]); st(k.hhp, c, o.h[1]); }
                    if (k.full) {
                        if (bu) st(k.hun, c, o.u[2]);
                        if (bv) st(k.hvn, c, o.v[2]);
                        if (bh) st(k.hhn, c, o.h[2]);
                    }
                }
            }
            x.rHR.rotate(); x.rSH.rotate(); x.rSHP.rotate(); x.rLU.rotate(); x.rDX.rotate(); x.rDY.rotate();
        }
    };
    __device__ void march(const Lane &L, int nb, int ne) const
    {
        const Fn f{k, ylast};
        View x{};
        const Interp<false> &W = k.W;
        const Pt c = k.I(L.m, nb);
        x.rHR.c = ld(k.h_r, c); x.rSH.c = ld(k.sh, c); x.rSHP.c = ld(k.shp, c);
        x.rLU.c = ld(W.lu, c); x.rDX.c = ld(W.dx, c); x.rDY.c = ld(W.dy, c);
        if (L.edge) {
            const Pt e = k.I(L.me, nb);
            x.rHR.ec = ld(k.h_r, e); x.rSH.ec = ld(k.sh, e); x.rSHP.ec = ld(k.shp, e);
            x.rLU.ec = ld(W.lu, e); x.rDX.ec = ld(W.dx, e); x.rDY.ec = ld(W.dy, e);
        }
        march_rows(f, x, L, nb, ne);
    }
};

// a4 uv_trans (sw_stencils.h UvTrans<false>) as an offset-layout register march
struct MarchViewT2 {
    RowsD<true, true> rU, rV, rHV;        // ubrtr, vbrtr, hhv: rows n-1 .. n+1
    RowsD<false, true> rHU;               // hhu: rows n, n+1
    RowsD<true, false> rVORT, rHH;        // vort, hhh: rows n-1, n
    RowsF<true, true> rDXH;               // dxh: rows n-1 .. n+1
    RowsF<false, true> rDYH;              // dyh: rows n, n+1
    RowsF<true, false> rLUU;              // luu: rows n-1, n
    OCN_MV(u, rU) OCN_MV(v, rV) OCN_MV(hu, rHU) OCN_MV(hv, rHV) OCN_MV(vort, rVORT) OCN_MV(hh, rHH)
    __device__ __forceinline__ float dxh(int i, int j) const { return rDXH.at(i, j); }
    __device__ __forceinline__ float dyh(int i, int j) const { return rDYH.at(i, j); }
    __device__ __forceinline__ float luu(int i, int j) const { return rLUU.at(i, j); }
};
struct MarchUvTrans2D {
    static constexpr bool kAligned = false;
    static constexpr int kHalo = 1;
    UvTrans<false> k;
    using View = MarchViewT2;
    struct Fn {
        const UvTrans<false> &k;
        // row n: ubrtr, vbrtr, hhv, hhu, dxh, dyh at n+1; vort, hhh, luu, lcu, lcv at n
        struct Batch { double nn[4], c[2]; float fn[2], fc[3]; };
        __device__ __forceinline__ void load(Batch &q, const Lane &L, int n) const
        {
            const Pt c = k.I(L.m, n), cn = k.I(L.m, n + 1);
            q.nn[0] = ld(k.u, cn); q.nn[1] = ld(k.v, cn); q.nn[2] = ld(k.hv, cn); q.nn[3] = ld(k.hu, cn);
            q.fn[0] = ld(k.dxh, cn); q.fn[1] = ld(k.dyh, cn);
            q.c[0] = ld(k.vort, c); q.c[1] = ld(k.hh, c);
            q.fc[0] = ld(k.luu, c); q.fc[1] = ld(k.lcu, c); q.fc[2] = ld(k.lcv, c);
        }
        __device__ __forceinline__ void row(View &x, const Batch &q, const Lane &L, int n) const
        {
            const Pt c = k.I(L.m, n);
            x.rVORT.s = x.rVORT.c; x.rHH.s = x.rHH.c; x.rLUU.s = x.rLUU.c;
            x.rU.nn = q.nn[0]; x.rV.nn = q.nn[1]; x.rHV.nn = q.nn[2]; x.rHU.nn = q.nn[3];
            x.rDXH.nn = q.fn[0]; x.rDYH.nn = q.fn[1];
            x.rVORT.c = q.c[0]; x.rHH.c = q.c[1]; x.rLUU.c = q.fc[0];
            double rx, ry;
            uv_trans_math(x, rx, ry);
            if (L.out) {
                if (q.fc[1] > 0.5f) st(k.RHSx, c, rx);
                if (q.fc[2] > 0.5f) st(k.RHSy, c, ry);
            }
            x.rU.rotate(); x.rV.rotate(); x.rHV.rotate(); x.rHU.rotate(); x.rDXH.rotate(); x.rDYH.rotate();
        }
    };
    __device__ void march(const Lane &L, int nb, int ne) const
    {
        const Fn f{k};
        View x{};
        const Pt s = k.I(L.m, nb - 1), c = k.I(L.m, nb);   // rows kept from before the first row
        x.rU.s = ld(k.u, s); x.rU.c = ld(k.u, c);
        x.rV.s = ld(k.v, s); x.rV.c = ld(k.v, c);
        x.rHV.s = ld(k.hv, s); x.rHV.c = ld(k.hv, c);
        x.rHU.c = ld(k.hu, c);
        x.rDXH.s = ld(k.dxh, s); x.rDXH.c = ld(k.dxh, c);
        x.rDYH.c = ld(k.dyh, c);
        x.rVORT.c = ld(k.vort, s); x.rHH.c = ld(k.hh, s); x.rLUU.c = ld(k.luu, s);
        march_rows(f, x, L, nb, ne);
    }
};

// a6 uv_diff2 (sw_stencils.h UvDiff2<false>) as an offset-layout register march
struct MarchViewD2 {
    RowsD<true, true> rMU;                // mu: rows n-1 .. n+1
    RowsD<false, true> rHQ, rSTT;         // hhq, str_t: rows n, n+1
    RowsD<true, false> rHH, rSTS;         // hhh, str_s: rows n-1, n
    RowsF<false, false> rDY, rDYB;        // dy, dyb: row n (m-1 .. m+1)
    RowsF<false, true> rDX;               // dx: rows n, n+1
    RowsF<true, false> rDXB;              // dxb: rows n-1, n
    HereF dxt_, dyt_, dxh_, dyh_;
    __device__ __forceinline__ double quot(double a, double b, int, int) const { return a / b; }
    OCN_MV(mu, rMU) OCN_MV(hq, rHQ) OCN_MV(str_t, rSTT) OCN_MV(hh, rHH) OCN_MV(str_s, rSTS)
    __device__ __forceinline__ float dx(int i, int j) const { return rDX.at(i, j); }
    __device__ __forceinline__ float dy(int i, int j) const { return rDY.at(i, j); }
    __device__ __forceinline__ float dxb(int i, int j) const { return rDXB.at(i, j); }
    __device__ __forceinline__ float dyb(int i, int j) const { return rDYB.at(i, j); }
    __device__ __forceinline__ float dxt(int i, int j) const { return dxt_.at(i, j); }
    __device__ __forceinline__ float dyt(int i, int j) const { return dyt_.at(i, j); }
    __device__ __forceinline__ float dxh(int i, int j) const { return dxh_.at(i, j); }
    __device__ __forceinline__ float dyh(int i, int j) const { return dyh_.at(i, j); }
};
struct MarchUvDiff2D {
    static constexpr bool kAligned = false;
    static constexpr int kHalo = 1;
    UvDiff2<false> k;
    using View = MarchViewD2;
    struct Fn {
        const UvDiff2<false> &k;
        // row n: mu, hhq, str_t, dx at n+1; hhh, str_s, dy, dyb, dxb, the centre metrics and lcu, lcv at n
        struct Batch { double nn[3], c[2]; float fn, fc[9]; };
        __device__ __forceinline__ void load(Batch &q, const Lane &L, int n) const
        {
            const Pt c = k.I(L.m, n), cn = k.I(L.m, n + 1);
            q.nn[0] = ld(k.mu, cn); q.nn[1] = ld(k.hq, cn); q.nn[2] = ld(k.str_t, cn);
            q.fn = ld(k.dx, cn);
            q.c[0] = ld(k.hh, c); q.c[1] = ld(k.str_s, c);
            q.fc[0] = ld(k.dy, c); q.fc[1] = ld(k.dyb, c); q.fc[2] = ld(k.dxb, c);
            q.fc[3] = ld(k.dxt, c); q.fc[4] = ld(k.dyt, c); q.fc[5] = ld(k.dxh, c); q.fc[6] = ld(k.dyh, c);
            q.fc[7] = ld(k.lcu, c); q.fc[8] = ld(k.lcv, c);
        }
        __device__ __forceinline__ void row(View &x, const Batch &q, const Lane &L, int n) const
        {
            const Pt c = k.I(L.m, n);
            x.rHH.s = x.rHH.c; x.rSTS.s = x.rSTS.c; x.rDXB.s = x.rDXB.c;
            x.rMU.nn = q.nn[0]; x.rHQ.nn = q.nn[1]; x.rSTT.nn = q.nn[2]; x.rDX.nn = q.fn;
            x.rHH.c = q.c[0]; x.rSTS.c = q.c[1];
            x.rDY.c = q.fc[0]; x.rDYB.c = q.fc[1]; x.rDXB.c = q.fc[2];
            x.dxt_.v = q.fc[3]; x.dyt_.v = q.fc[4]; x.dxh_.v = q.fc[5]; x.dyh_.v = q.fc[6];
            double rx, ry;
            uv_diff2_math(x, rx, ry);
            if (L.out) {
                if (q.fc[7] > 0.5f) st(k.RHSx, c, rx);
                if (q.fc[8] > 0.5f) st(k.RHSy, c, ry);
            }
            x.rMU.rotate(); x.rHQ.rotate(); x.rSTT.rotate(); x.rDX.rotate();
        }
    };
    __device__ void march(const Lane &L, int nb, int ne) const
    {
        const Fn f{k};
        View x{};
        const Pt s = k.I(L.m, nb - 1), c = k.I(L.m, nb);   // rows kept from before the first row
        x.rMU.s = ld(k.mu, s); x.rMU.c = ld(k.mu, c);
        x.rHQ.c = ld(k.hq, c); x.rSTT.c = ld(k.str_t, c); x.rDX.c = ld(k.dx, c);
        x.rHH.c = ld(k.hh, s); x.rSTS.c = ld(k.str_s, s); x.rDXB.c = ld(k.dxb, s);
        march_rows(f, x, L, nb, ne);
    }
};

// a5 stress_components (sw_stencils.h StressComponents<false>) as an offset-layout register march
struct MarchViewS2 {
    RowsD<false, true> rUP;               // ubrtrp: rows n, n+1
    RowsD<true, false> rVP;               // vbrtrp: rows n-1, n
    RowsF<false, false> rDYH, rDYT;       // dyh, dyt: row n (m-1 .. m+1)
    RowsF<true, false> rDXH;              // dxh: rows n-1, n
    RowsF<false, true> rDXT;              // dxt: rows n, n+1
    float rat[4];                         // dy/dx, dx/dy, dxb/dyb, dyb/dxb at the point (mixing.f90:33-34, 43-44)
    OCN_MV(up, rUP) OCN_MV(vp, rVP)
    __device__ __forceinline__ float sratio(int k) const { return rat[k]; }
    __device__ __forceinline__ float dyh(int i, int j) const { return rDYH.at(i, j); }
    __device__ __forceinline__ float dyt(int i, int j) const { return rDYT.at(i, j); }
    __device__ __forceinline__ float dxh(int i, int j) const { return rDXH.at(i, j); }
    __device__ __forceinline__ float dxt(int i, int j) const { return rDXT.at(i, j); }
};
struct MarchStress2D {
    static constexpr bool kAligned = false;
    static constexpr int kHalo = 1;
    StressComponents<false> k;
    using View = MarchViewS2;
    struct Fn {
        const StressComponents<false> &k;
        // row n: ubrtrp, dxt at n+1; vbrtrp, dyh, dyt, dxh, dx, dy, dxb, dyb, lu, luu at n
        struct Batch { double nn, c; float fn, fc[10]; };
        __device__ __forceinline__ void load(Batch &q, const Lane &L, int n) const
        {
            const Pt c = k.I(L.m, n), cn = k.I(L.m, n + 1);
            q.nn = ld(k.u, cn); q.fn = ld(k.dxt, cn);
            q.c = ld(k.v, c);
            q.fc[0] = ld(k.dyh, c); q.fc[1] = ld(k.dyt, c); q.fc[2] = ld(k.dxh, c);
            q.fc[3] = ld(k.dx, c); q.fc[4] = ld(k.dy, c); q.fc[5] = ld(k.dxb, c); q.fc[6] = ld(k.dyb, c);
            q.fc[7] = ld(k.lu, c); q.fc[8] = ld(k.luu, c);
        }
        __device__ __forceinline__ void row(View &x, const Batch &q, const Lane &L, int n) const
        {
            const Pt c = k.I(L.m, n);
            x.rVP.s = x.rVP.c; x.rDXH.s = x.rDXH.c;
            x.rUP.nn = q.nn; x.rDXT.nn = q.fn;
            x.rVP.c = q.c; x.rDYH.c = q.fc[0]; x.rDYT.c = q.fc[1]; x.rDXH.c = q.fc[2];
            const float dx = q.fc[3], dy = q.fc[4], dxb = q.fc[5], dyb = q.fc[6];
            x.rat[0] = dy / dx; x.rat[1] = dx / dy; x.rat[2] = dxb / dyb; x.rat[3] = dyb / dxb;
            double vt, vs;
            stress_components_math(x, vt, vs);
            if (L.out) {
                if (q.fc[7] > 0.5f) st(k.str_t, c, vt);
                if (q.fc[8] > 0.5f) st(k.str_s, c, vs);
            }
            x.rUP.rotate(); x.rDXT.rotate();
        }
    };
    __device__ void march(const Lane &L, int nb, int ne) const
    {
        const Fn f{k};
        View x{};
        const Pt s = k.I(L.m, nb - 1), c = k.I(L.m, nb);   // rows kept from before the first row
        x.rUP.c = ld(k.u, c); x.rDXT.c = ld(k.dxt, c);
        x.rVP.c = ld(k.v, s); x.rDXH.c = ld(k.dxh, s);
        march_rows(f, x, L, nb, ne);
    }
};

// ------------------------------------------------------------------ fused CA = hh_init + next A
// Role-flip calls (ocn_ctx.hip one_step_fused): step k's a10 hh_init and step k+1's fused A in
// one aligned march over the bnd range.  A's a1 reads hhu at (m-1, n), (m, n) and hhv at
// (m, n-1), (m, n): exactly the hu / hv that hh_init computes here (level 0), so they come from
// registers: hv of row n-1 is carried from the previous row (a "warm" first row computes it
// for the tile's first row), hu at m-1 is the next lane's value, and the edge lane 0 evaluates
// interp_u one column to the left itself (same operands, same arithmetic as the neighbouring
// wave's lane 63: the same bits).  Where llu / llv is 0 hh_init stores nothing and a1 reads the
// array's (never written) value from memory.  HH: the next step is not a reuse step, so A's a2
// hh_update stores hun / hvn / hhn -- bit for bit hh_init's level-0 values (the reuse identity,
// full_free_surface = 1), under the same masks on the same range.  Nothing this launch writes
// is read at a neighbour, so there are no races.  hh_init's hhh_p is stored only before the last
// step (HH): its only reader is a9 on the outer ring e+1 (the ring launch), outside hh_init's
// range, which gets it from a neighbour's interior through sync B with halo exchanges; what a9
// derives from the older values is hhh_p on that ring alone (read by a9 only, and exchanged over
// before each use), and the last, standard step works from the current ones.  SKIP (the next step is a recompute step):
// hhq on the interior, hhu_p and hhv_p are not stored either -- their only reader, the next
// step's fused B, recomputes them (MarchFusedB RC); hhq stays stored on the halo rows / columns
// (a9 on the ring reads it there).
struct MarchViewCA {
    RowsD<false, true, true> rHR, rSH, rSHP, rU, rUP;  // h_r, ssh, sshp, ubrtr, ubrtrp
    RowsD<true, false, true> rV, rVP;                  // vbrtr, vbrtrp
    RowsD<false, false, true> rHU;                     // hhu: c = this column, ec = column m-1 (lane 0)
    RowsD<true, false> rHV;                            // hhv: rows n-1, n
    BitRows<false, true, true> bits;
    MetRows met;
    double tau;
    __device__ __forceinline__ double tau2() const { return tau; }
    OCN_MV(h_r, rHR) OCN_MV(sh, rSH) OCN_MV(shp, rSHP) OCN_MV(sshp, rSHP) OCN_MV(u, rU) OCN_MV(ubrtr, rU)
    OCN_MV(up, rUP) OCN_MV(v, rV) OCN_MV(vbrtr, rV) OCN_MV(vp, rVP) OCN_MV(hhu, rHU) OCN_MV(hhv, rHV)
    OCN_MG_ALL
    __device__ __forceinline__ float lu(int dx, int dy) const { return bits.mask(OCN_LU, dx, dy); }
};
// the interpolation operands one column to the left (interp_u at m-1)
struct LeftView {
    const MarchViewCA &x;
    __device__ __forceinline__ float lu(int dx, int dy) const { return x.lu(dx - 1, dy); }
    __device__ __forceinline__ float dx(int i, int dy) const { return x.dx(i - 1, dy); }
    __device__ __forceinline__ float dy(int i, int dy) const { return x.dy(i - 1, dy); }
    __device__ __forceinline__ float dxt(int i, int dy) const { return x.dxt(i - 1, dy); }
    __device__ __forceinline__ float dyh(int i, int dy) const { return x.dyh(i - 1, dy); }
};

template <bool HH, bool SKIP> struct MarchCA {
    static constexpr bool kAligned = true;
    static constexpr int kHalo = 0;
    ocn_block b; Tab<true> t; ocn_sw_params sw; double tau;
    struct Fn {
        HhInit<true> c2; FusedA<true> a; const Tab<true> &t; int ylast;
        // row n: h_r, ssh, sshp, mask bytes, ubrtr, ubrtrp at n+1 (clamped to bnd_y2); vbrtr,
        // vbrtrp at n; their edge values; metric row n+1
        struct Batch { double nn[5], c[2], enn[5], ec[2]; unsigned bits, ebits; float g[kRowTable]; };
        __device__ __forceinline__ void load(Batch &q, const Lane &L, int n) const
        {
            const int r = min(n + 1, ylast), r0 = max(n, (int)c2.I.by1);
            const Pt cn = c2.I(L.m, r), c = c2.I(L.m, r0);
            q.nn[0] = ld(c2.h_r, cn); q.nn[1] = ld(c2.sh, cn); q.nn[2] = ld(c2.shp, cn);
            q.nn[3] = ld(a.a1.ubrtr, cn); q.nn[4] = ld(a.a5.u, cn); q.bits = ld(t.bits, cn);
            q.c[0] = ld(a.a1.vbrtr, c); q.c[1] = ld(a.a5.v, c);
            for (int i = 0; i < 5; ++i) q.enn[i] = 0.0;
            q.ec[0] = q.ec[1] = 0.0;
            q.ebits = 0;
            if (L.edge) {
                const Pt en = c2.I(L.me, r), e = c2.I(L.me, r0);
                q.enn[0] = ld(c2.h_r, en); q.enn[1] = ld(c2.sh, en); q.enn[2] = ld(c2.shp, en);
                q.enn[3] = ld(a.a1.ubrtr, en); q.enn[4] = ld(a.a5.u, en); q.ebits = ld(t.bits, en);
                q.ec[0] = ld(a.a1.vbrtr, e); q.ec[1] = ld(a.a5.v, e);
            }
            MetRows::load(q.g, t.rows, t.nrows, cn.r);
        }
        // warm = the row before the tile's first row: only hv (for a1's hhv(m, n-1)) is computed
        __device__ __forceinline__ void row(MarchViewCA &x, const Batch &q, const Lane &L, int n, bool warm) const
        {
            const Pt c = c2.I(L.m, max(n, (int)c2.I.by1));
            const double f = c2.f;
            x.rV.s = x.rV.c; x.rV.es = x.rV.ec; x.rVP.s = x.rVP.c; x.rVP.es = x.rVP.ec; x.rHV.s = x.rHV.c;
            x.met.shift(q.g);
            x.rHR.nn = q.nn[0]; x.rSH.nn = q.nn[1]; x.rSHP.nn = q.nn[2]; x.rU.nn = q.nn[3]; x.rUP.nn = q.nn[4];
            x.rHR.enn = q.enn[0]; x.rSH.enn = q.enn[1]; x.rSHP.enn = q.enn[2]; x.rU.enn = q.enn[3];
            x.rUP.enn = q.enn[4];
            x.bits.nn = q.bits; x.bits.enn = q.ebits;
            x.rV.c = q.c[0]; x.rVP.c = q.c[1]; x.rV.ec = q.ec[0]; x.rVP.ec = q.ec[1];
            const unsigned bc = x.bits.c;
            const bool llu = bc & (1u << OCN_LLU), llv = bc & (1u << OCN_LLV), luh = bc & (1u << OCN_LUH);
            const bool in_rows = n >= c2.j0 && n <= c2.j1;   // wave-uniform
            if (warm) {
                if (in_rows) {
                    const double a00 = x.rHR.c + x.rSH.c * f, a01 = x.rHR.nn + x.rSH.nn * f;
                    const double v0 = interp_v(x, a00, a01);
                    x.rHV.c = llv ? v0 : ld(c2.hv, c);
                }
                goto rotate;
            }
            {
                const double r00 = x.rHR.c;
                // !HH: the next step's fused B forms hhq itself on the interior (MarchFusedB RC)
                const bool interior = L.m >= a.sx && L.m <= b_xe && n >= a.sy && n <= b_ye;
                if (L.out && (!SKIP || !interior)) st(c2.hq, c, r00 + x.rSH.c * f);
                // tracer runs: expl_tracer reads hh_init's whole-array hqp = h_r + shp * ffs after
                // every step (tran_diff_tracer's hhq_p; its hhq_n = h_r is never changed by the
                // fused step: fused A does not store hh_update's hqn)
                if (L.out && tracers) st(c2.hqp, c, r00 + x.rSHP.c * f);
                if (in_rows) {
                    HhInitOut o;
                    hh_init_math(x, f, false, o);
                    const bool inr = L.out && L.m >= c2.i0 && L.m <= c2.i1;
                    if (inr) {
                        if (llu) { st(c2.hu, c, o.u[0]); if (!SKIP) st(c2.hup, c, o.u[1]); }
                        if (llv) { st(c2.hv, c, o.v[0]); if (!SKIP) st(c2.hvp, c, o.v[1]); }
                        if (luh) { st(c2.hh, c, o.h[0]); if (HH) st(c2.hhp, c, o.h[1]); }   // hhh_p: see below
                        if (HH) {
                            if (llu) st(a.a2.hun, c, o.u[0]);
                            if (llv) st(a.a2.hvn, c, o.v[0]);
                            if (luh) st(a.a2.hhn, c, o.h[0]);
                        }
                    }
                    // a1's hhu / hhv: the values memory holds after this launch
                    x.rHU.c = llu ? o.u[0] : ld(c2.hu, c);
                    x.rHV.c = llv ? o.v[0] : ld(c2.hv, c);
                    {   // hu at m-1 (used by lane 0 only)
                        const LeftView lv{x};
                        const double aw = x.h_r(-1, 0) + x.sh(-1, 0) * f, a00 = r00 + x.rSH.c * f;
                        const double uw = interp_u(lv, aw, a00);
                        const bool lluw = x.bits.at(-1, 0) & (1u << OCN_LLU);
                        x.rHU.ec = lluw ? uw : ld(c2.hu, c2.I(L.me, max(n, (int)c2.I.by1)));
                    }
                }
                if (n >= a.sy && n <= b_ye) {   // A's a1 / a3 / a5 on [start, end]^2 (wave-uniform rows)
                    const bool in = L.out && L.m >= a.sx && L.m <= b_xe;
                    const double rs = sw_update_ssh_math(x);
                    if (in && (bc & (1u << OCN_LU))) st(a.a1.sshn, c, rs);
                    if (a.do_vort) {
                        const double v = uv_trans_vort_math(x);
                        if (in && (bc & (1u << OCN_LUU))) st(a.a3.vort, c, v);
                    }
                    if (a.do_stress) {
                        double vt, vs;
                        stress_components_math(x, vt, vs);
                        if (in && (bc & (1u << OCN_LU))) st(a.a5.str_t, c, vt);
                        if (in && (bc & (1u << OCN_LUU))) st(a.a5.str_s, c, vs);
                    }
                }
            }
        rotate:
            x.rHR.rotate(); x.rSH.rotate(); x.rSHP.rotate(); x.rU.rotate(); x.rUP.rotate(); x.bits.rotate();
        }
        int b_xe, b_ye;
        bool tracers;
    };
    __device__ void march(const Lane &L, int nb, int ne) const
    {
        const Fn f{make_hh_init(&b, t, (int)sw.full_free_surface, false), make_fused_a(&b, t, sw, tau, !HH), t,
                   b.bnd_y2, b.nx_end, b.ny_end, sw.use_tracers > 0};
        MarchViewCA x{};
        x.tau = tau;
        // the warm row nb-1 (when it exists) precedes the tile's rows
        const int n0 = max(nb - 1, b.bnd_y1);
        const Pt c = f.c2.I(L.m, n0);
        x.rHR.c = ld(f.c2.h_r, c); x.rSH.c = ld(f.c2.sh, c); x.rSHP.c = ld(f.c2.shp, c);
        x.rU.c = ld(f.a.a1.ubrtr, c); x.rUP.c = ld(f.a.a5.u, c); x.bits.c = ld(t.bits, c);
        if (L.edge) {
            const Pt e = f.c2.I(L.me, n0);
            x.rHR.ec = ld(f.c2.h_r, e); x.rSH.ec = ld(f.c2.sh, e); x.rSHP.ec = ld(f.c2.shp, e);
            x.rU.ec = ld(f.a.a1.ubrtr, e); x.rUP.ec = ld(f.a.a5.u, e); x.bits.ec = ld(t.bits, e);
        }
        x.met.preload(t.rows, t.nrows, c.r, c.r);
        typename Fn::Batch cur, nxt;
        f.load(cur, L, n0);
        for (int n = n0; n <= ne; ++n) {
            f.row(x, cur, L, n, n < nb);
            if (n < ne) {
                f.load(nxt, L, n + 1);
                cur = nxt;
            }
        }
    }
};

// ------------------------------------------------------------------ one-pass step
#ifndef OCN_STEP_ROWS
#define OCN_STEP_ROWS 32   // rows per wave tile of the one-pass step (2 warm rows per tile)
#endif
#ifndef OCN_STEP_WAVES
#define OCN_STEP_WAVES 2   // waves per SIMD asked of the register allocator
#endif
// A whole role-flip step in one register march (ocn_ctx.hip one_step_fused, "one-pass" steps of
// a single-block call): the state (ssh, sshp, ubrtr, ubrtrp, vbrtr, vbrtrp; h_r, mu, RHSx, RHSy)
// is read once and the next state written once -- 10 + 6 arrays, against fused B + CA's 22 + 12.
// Per wave row n (the march goes down the rows), two lagged computations:
//   D(n+1): what the reference's previous hh_init and this step's fused A store and fused B reads
//     back: hh_init's level-0 hu / hv / hh (interp of h_r + ssh * ffs) and level-1 hu / hv (of
//     h_r + sshp * ffs) on [start-1, end]^2 under llu / llv / luh, a3's vort (interior, luu), a5's
//     str_t (interior, lu) and str_s (interior, luu); hq = h_r + ssh * ffs (whole array).  Where
//     the reference stores nothing (mask 0, or outside the stage's range) the array's value in
//     memory is what it reads, so that is loaded there (those points are never written during
//     the call: one block, no a8 / a9 work on the halo ring).
//   S(n): a1 sw_update_ssh (-> sshn), fused B (a4 + a6 + a7 -> ubrtrn, vbrtrn) and a8's time
//     filters (-> the second sshp / ubrtrp / vbrtrp buffers: the current ones are read at
//     neighbours here) + check_ssh_err, reading D at rows n-1, n, n+1.
// The reference's values are reproduced bit for bit: the same operands (hun = hu, hvn = hv: the
// reuse identity, full_free_surface = 1) and the same arithmetic (sw_stencils.h *_math).
// Lane layout: D needs the state at m +- 1 and S needs D at m +- 1, so a wave loads 64 columns
// and produces 60 (kHalo = 2; output runs start on 32-B boundaries).  Rows n-1 .. n+2 of every
// array and of the metric table stay in registers; the loads of the next row are issued before
// the current row is computed.
// x of lane + dx (dx in {-1, 0, 1}); 0 in the lane without a source (bound_ctrl): the one-pass
// march reads such values only in its halo lanes, so no old value needs to be kept
#ifndef OCN_SHIFT_BPERM
#define OCN_SHIFT_BPERM 0
#endif
__device__ __forceinline__ int dpp_shz(int x, int dx)
{
#if OCN_SHIFT_BPERM
    // (the LDS crossbar instead of a VALU move: the lane without a source gets lane (l + dx) mod 64's
    // value, which -- like bound_ctrl's 0 -- only halo lanes read)
    const int lane = (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
    return __builtin_amdgcn_ds_bpermute((lane + dx) << 2, x);
#else
    if (dx > 0) return __builtin_amdgcn_mov_dpp(x, 0x130, 0xf, 0xf, true);   // wave_shl:1
    return __builtin_amdgcn_mov_dpp(x, 0x138, 0xf, 0xf, true);               // wave_shr:1
#endif
}
__device__ __forceinline__ double shz(double x, int dx)
{
    if (dx == 0) return x;
    return __hiloint2double(dpp_shz(__double2hiint(x), dx), dpp_shz(__double2loint(x), dx));
}
__device__ __forceinline__ unsigned shz(unsigned x, int dx) { return dx == 0 ? x : (unsigned)dpp_shz((int)x, dx); }

// A masked store the wave always issues: a lane with !on gets a byte offset past the buffer's
// range (nbytes = the array's size) and the buffer unit drops its write.  With no exec branch
// around the stores every path through an iteration issues the same number of vector memory
// operations, so the wait for the next row's loads (issued before them) is vmcnt(#stores), not
// vmcnt(0) -- which would also wait for the stores' write acknowledgements.
typedef unsigned ocn_u32x2 __attribute__((ext_vector_type(2)));
// AUX = the store's cache policy: 0 = plain (the line kept in the XCD's L2), 16 = sc1 (write-through:
// the bytes reach memory before the wave's vmcnt drops -- k_march_multi's grid barrier then needs no
// L2 write-back)
template <int AUX = 0>
__device__ __forceinline__ void st_on(double *p, unsigned nbytes, unsigned i, double v, bool on)
{
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(p, (short)0, (int)nbytes, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(ocn_u32x2, v), r, on ? i * 8u : 0xfffffff8u, 0, AUX);
}

// x / d, correctly rounded, for a wave-uniform divisor d with rd = RN(1 / d) (the row table's
// reciprocals): q = RN(x rd) is within one ulp of x / d, the residual x - q d is exact in an fma,
// and RN(q + (x - q d) rd) is the correctly rounded quotient (Markstein's theorem) when nothing
// underflows: for d in [2^-60, 2^60] (launch_prepare flags other divisors, and the one-pass step
// is then not used) and x = 0 or 2^-900 <= |x| < 2^900 the quotient and the residual are normal.
// 3 VALU operations instead of the div_scale / rcp / fma / fixup sequence of an IEEE fp64 division
// (11, one of them quarter rate).  The caller checks the dividend's range (exp_check): a row where
// any dividend is outside it is computed again with IEEE divisions.  Checked bit for bit against
// IEEE division on random operands over that domain (tests/test_udiv.py).
// The residual is formed negated, t = RN(q d - x), and added as RN(q - t rd): the same values as
// RN(q + (x - q d) rd) for x != 0, and the sign of a zero quotient kept (x = -0: q = -0, t = +0,
// -0 - 0 = -0), which IEEE division gives and the uv_diff2 terms carry (mu = 0: dividends of +-0).
// d > 0 (the metrics; launch_prepare flags others).
__device__ __forceinline__ double udiv(double x, double d, double rd)
{
    const double q = x * rd;
    const double t = __builtin_fma(q, d, -x);
    return __builtin_fma(-t, rd, q);
}
// the smallest frexp exponent of the dividends of a row (0 for x = 0)
__device__ __forceinline__ void exp_check(int &acc, double x)
{
    acc = min(acc, __builtin_amdgcn_frexp_exp(x));
}
constexpr int kUdivMinExp = -899;   // frexp exponent >= -899  <=>  |x| >= 2^-900

// The row-uniform operands of the one-pass step, per row r, as the doubles the arithmetic uses
// (each formed exactly as the step forms it from the real(4) row table: promoted metrics, the
// real(4) products and sums of metrics, the reciprocals of udiv's divisors).  The known-constant
// variant (MarchStep::kLds): a workgroup forms them once for its rows into LDS (MarchStep::prologue, a thread per row) and
// its waves read them there (broadcast ds_read: no scalar loads, conversions or SGPR spills;
// 0.554 -> 0.480 ms per 4096^2 step); else they are formed from scalar loads of the row table
// where used.  The general variant keeps the scalar loads: with its loaded h_r, mu, forcing and
// fallback values, the LDS operands push it into VGPR spills.
enum RowC { RC_DX, RC_DY, RC_DXT, RC_DYT, RC_DXH, RC_DYH, RC_DXB, RC_DYB, RC_RDXT, RC_RDYH, RC_RDXH, RC_RDYT,
            RC_RDXB, RC_RDYB, RC_RAT0, RC_RAT1, RC_RAT2, RC_RAT3, RC_RLH, RC_DY2, RC_DX2, RC_AREA, RC_RAREA,
            RC_DXB2, RC_DYB2, RC_RDSELF, RC_RDNEXT, kRowC };
#ifndef OCN_PAIR_WAVES
#define OCN_PAIR_WAVES OCN_STEP_WAVES   // waves per SIMD the two-step launch asks of the register allocator
#endif
#ifndef OCN_PAIR_MAX_ROWS
#define OCN_PAIR_MAX_ROWS 150   // the tallest workgroup tile of the two-step launch (its rows +- 5 in LDS)
#endif
// a workgroup's 4 stacked tiles + 2 rows each side; a two-step workgroup's tile + 5 above, 4 below
constexpr int kStepLdsRows = 4 * OCN_STEP_ROWS + 4 > OCN_PAIR_MAX_ROWS + 10 ? 4 * OCN_STEP_ROWS + 4 : OCN_PAIR_MAX_ROWS + 10;

__shared__ double g_step_rc[kStepLdsRows * kRowC];   // the workgroup's rows [nb - 2, ne + 2]
__shared__ unsigned g_step_rlo;                       // table row of its first row
// Two steps per launch (MarchStep PAIR): the producer waves' new state (ssh, sshp, ubrtr, ubrtrp,
// vbrtr, vbrtrp after the first step, by row mod 4) for the consumer waves.
// (Measured and dropped: a wave's 60-column output rows stored as whole 128-B lines through LDS,
// a workgroup barrier per row -- 0.407-0.424 against 0.391 ms per 4096^2 single launch.)
__shared__ double g_pair[4][6][120];

// row constant k of table row r (rows[(id - OCN_DX) * nrows + r], real(4)); r + 1 for RC_RDNEXT
__device__ __forceinline__ double row_const(const float *rows, unsigned nrows, unsigned r, int k)
{
    auto g = [&](int id) { return rows[(unsigned)(id - OCN_DX) * nrows + r]; };
    auto rc = [&](int j) { return ((const double *)(rows + recip_offset(nrows)))[(unsigned)j * nrows + r]; };
    switch (k) {
    case RC_DX: return D(g(OCN_DX));
    case RC_DY: return D(g(OCN_DY));
    case RC_DXT: return D(g(OCN_DXT));
    case RC_DYT: return D(g(OCN_DYT));
    case RC_DXH: return D(g(OCN_DXH));
    case RC_DYH: return D(g(OCN_DYH));
    case RC_DXB: return D(g(OCN_DXB));
    case RC_DYB: return D(g(OCN_DYB));
    case RC_RDXT: return rc(OCN_RC_DXT);
    case RC_RDYH: return rc(OCN_RC_DYH);
    case RC_RDXH: return rc(OCN_RC_DXH);
    case RC_RDYT: return rc(OCN_RC_DYT);
    case RC_RDXB: return rc(OCN_RC_DXB);
    case RC_RDYB: return rc(OCN_RC_DYB);
    case RC_RAT0: case RC_RAT1: case RC_RAT2: case RC_RAT3:
        return D(rows[(unsigned)(kNumRowFields + k - RC_RAT0) * nrows + r]);
    case RC_RLH: return D(g(OCN_RLH_S));
    case RC_DY2: { const float a = g(OCN_DY); return D(a * a); }
    case RC_DX2: { const float a = g(OCN_DX); return D(a * a); }
    case RC_AREA: { const float a = g(OCN_DX) * g(OCN_DY); return D(a); }
    case RC_RAREA: return rc(OCN_RC_AREA);
    case RC_DXB2: { const float a = g(OCN_DXB); return D(a * a); }
    case RC_DYB2: { const float a = g(OCN_DYB); return D(a * a); }
    case RC_RDSELF: { const float a = g(OCN_R_DISS); const float rd = a + a; return D(rd); }
    case RC_RDNEXT: {
        const float a = g(OCN_R_DISS), an = rows[(unsigned)(OCN_R_DISS - OCN_DX) * nrows + min(r + 1, nrows - 1)];
        const float rd = a + an;
        return D(rd);
    }
    default: return 0.0;
    }
}

// 1 / c for a sea count c in {0, 1, 2, 4} (+inf for 0): a * rcp_count(c) is a / (double)c bit for
// bit -- 1, 1/2, 1/4 are exact, so both round the same real value once; for c = 0, a * inf and
// a / 0 are the same infinity or NaN (0 * inf, 0 / 0); c = 3 takes a division (derive).  The
// counts are integers from the mask bits: no float sums, compares or conversions, and u / v
// (c <= 2) need no wave-wide test.
// rcp_count for a count of at least one (c in {1, 2, 4}): no select.  The one-pass step uses it where
// the average is used only under llu / llv / luh, which lu_lv_init (grid_kernels.f90:40-92) sets
// exactly where the sum of lu over the average's corners is at least one -- Prepare checks that the
// mask bytes say so (else OCN_COMPACT_DIVISOR_RANGE: no one-pass steps); a count of 0 gives 1.0 here,
// a value no store uses
__device__ __forceinline__ double rcp_sea(unsigned c)
{
    return __builtin_bit_cast(double, (unsigned long long)(0x3ff00000u - ((c >> 1) << 20)) << 32);
}
__device__ __forceinline__ double rcp_count(unsigned c)
{
    const unsigned hi = c == 0 ? 0x7ff00000u : 0x3ff00000u - ((c >> 1) << 20);
    return __builtin_bit_cast(double, (unsigned long long)hi << 32);
}

// StepRegs::Win: rows n-1 .. n+2 in a ring of kRing slots, written out for kRing phases (MarchStep::march)
constexpr int kRing = 5;

struct StepRegs {
    // rows n-1, n, n+1, n+2 at this lane's column: a ring of kRing slots, row n + k - 1 in slot
    // (PH + k) % kRing for the iteration's phase PH (n - n0 mod kRing, a template parameter: the
    // march is unrolled kRing times), so that no register moves rotate the rows
    template <class T> struct Win {
        T r[kRing];
        template <int PH> __device__ __forceinline__ T &s(int k) { return r[(PH + k) % kRing]; }
        template <int PH> __device__ __forceinline__ T s(int k) const { return r[(PH + k) % kRing]; }
        template <int PH> __device__ __forceinline__ T at(int dx, int dy) const
        {
            if (dy < -1 || dy > 2) ocn_march_bad_access();
            return shz(s<PH>(dy + 1), dx);
        }
        __device__ __forceinline__ void rotate() { r[0] = r[1]; r[1] = r[2]; r[2] = r[3]; }   // (phase 0 only)
    };
    // state
    Win<double> u, v, up, vp, ssh, shp, hr, mu;
    Win<unsigned> bits;
    double rhsx, rhsy;
    // D rows (computed one row ahead)
    Win<double> hu, hv, hh, hu1, hv1, vort, stt, sts;
    // products shared between lanes / rows (each the reference's own sub-expression, see derive)
    Win<double> w0, w1;               // interp weights ((h * dx) * dy) * lu of levels 0 / 1 (rows n+1, n+2)
    Win<double> pu, pv, vh, t3, cx, rr, dt, dxq;
    Win<double> w0r, vr;              // w0 and v shifted one lane left (their m+1 values): shifted once per row
    // metric rows: read where used, as wave-uniform scalar loads from the (read-only) row table
    // through the constant address space -- no table of 4 rows x 14 values held in SGPRs
    const __attribute__((address_space(4))) float *rows;
    const __attribute__((address_space(4))) double *rcp;   // the rows' reciprocals (sw_stencils.h recip_offset)
    unsigned nrows, rn;               // table stride, row index of n (n - bnd_y1)
    double qb, qc;                     // stress quotients of D's previous row (vp/dxh) and next row (up/dxt)
    double tau, inv_tau, f;
    int32_t *nbp;                      // where this wave's check_ssh_err count goes (null: unchecked)
    bool cnt;                          // the point is counted (PAIR producers: their workgroup's points only)
    int pj;                            // PAIR: the lane's column in the workgroup's LDS ring
    double fyx, fyy, vht, a2t;         // row n-1's n faces (MarchStep::face)
    double hr0, mu0;                   // known-constant variant: the uniform h_r and mu (MarchStep::kc)
    const __attribute__((address_space(3))) double *lds;   // (kLds) the workgroup's row constants
    unsigned rlo;                                            // table row of lds row 0
    // row constant k (RowC) of row n + dy, from LDS or from scalar loads
    template <bool LDS> __device__ __forceinline__ double cst(int k, int dy) const
    {
        if (LDS) return lds[(rn + dy - rlo) * kRowC + k];
        switch (k) {   // the same values from scalar loads of the row table
        case RC_RDXT: return rc(OCN_RC_DXT, dy);
        case RC_RDYH: return rc(OCN_RC_DYH, dy);
        case RC_RDXH: return rc(OCN_RC_DXH, dy);
        case RC_RDYT: return rc(OCN_RC_DYT, dy);
        case RC_RDXB: return rc(OCN_RC_DXB, dy);
        case RC_RDYB: return rc(OCN_RC_DYB, dy);
        case RC_RAREA: return rc(OCN_RC_AREA, dy);
        default: break;
        }
        return row_const_s(k, dy);
    }
    // (the general variant) row constant k from scalar loads
    __device__ __forceinline__ double row_const_s(int k, int dy) const
    {
        auto g = [&](int id) { return met(id, dy); };
        switch (k) {
        case RC_DX: return D(g(OCN_DX));
        case RC_DY: return D(g(OCN_DY));
        case RC_DXT: return D(g(OCN_DXT));
        case RC_DYT: return D(g(OCN_DYT));
        case RC_DXH: return D(g(OCN_DXH));
        case RC_DYH: return D(g(OCN_DYH));
        case RC_DXB: return D(g(OCN_DXB));
        case RC_DYB: return D(g(OCN_DYB));
        case RC_RAT0: case RC_RAT1: case RC_RAT2: case RC_RAT3: return D(met(OCN_DX + kNumRowFields + k - RC_RAT0, dy));
        case RC_RLH: return D(g(OCN_RLH_S));
        case RC_DY2: { const float a = g(OCN_DY); return D(a * a); }
        case RC_DX2: { const float a = g(OCN_DX); return D(a * a); }
        case RC_AREA: { const float a = g(OCN_DX) * g(OCN_DY); return D(a); }
        case RC_DXB2: { const float a = g(OCN_DXB); return D(a * a); }
        case RC_DYB2: { const float a = g(OCN_DYB); return D(a * a); }
        case RC_RDSELF: { const float a = g(OCN_R_DISS); const float rd = a + a; return D(rd); }
        case RC_RDNEXT: { const float rd = g(OCN_R_DISS) + met(OCN_R_DISS, dy + 1); return D(rd); }
        default: return 0.0;
        }
    }
    // table row of row n + dy, clamped into the table (PAIR producers: their rows reach 2 past the
    // block's; what they compute there is not used)
    __device__ __forceinline__ unsigned row(int dy) const
    {
        return min((unsigned)__builtin_amdgcn_readfirstlane(rn + dy), (unsigned)nrows - 1u);
    }
    __device__ __forceinline__ float met(int id, int dy) const
    {
        return rows[(unsigned)(id - OCN_DX) * nrows + row(dy)];
    }
    // 1 / (double)g of row n + dy for the divisor OCN_RC_* k (wave-uniform scalar load)
    __device__ __forceinline__ double rc(int k, int dy) const
    {
        return rcp[(unsigned)k * nrows + row(dy)];
    }
    // the rotating form (every iteration in phase 0): rows n-1 .. n+2 move down one slot
    __device__ __forceinline__ void rotate()
    {
        u.rotate(); v.rotate(); up.rotate(); vp.rotate(); ssh.rotate(); shp.rotate(); hr.rotate(); mu.rotate();
        bits.rotate();
        hu.rotate(); hv.rotate(); hh.rotate(); hu1.rotate(); hv1.rotate(); vort.rotate(); stt.rotate(); sts.rotate();
        w0.rotate(); w1.rotate(); pu.rotate(); pv.rotate(); vh.rotate(); t3.rotate(); cx.rotate(); rr.rotate();
        w0r.rotate(); vr.rotate();
        dt.rotate(); dxq.rotate();
    }
    template <int PH> __device__ __forceinline__ unsigned bit(int id, int dx, int dy) const
    {
        return (bits.at<PH>(dx, dy) >> id) & 1u;
    }
    template <int PH> __device__ __forceinline__ float mk(int id, int dx, int dy) const
    {
        return (bits.at<PH>(dx, dy) >> id) & 1u ? 1.0f : 0.0f;
    }
    // the mask value as a double (D(mk)): 1.0 = 0x3ff00000'00000000 formed from the bit, no select or
    // conversion
    template <int PH> __device__ __forceinline__ double mkd(int id, int dx, int dy) const
    {
        const unsigned hi = ((bits.at<PH>(dx, dy) >> id) & 1u) * 0x3ff00000u;
        return __builtin_bit_cast(double, (unsigned long long)hi << 32);
    }
};

// metric id `id` of row n + dy as a double
#define OCN_MD(id, dy) D(x.met((id), (dy)))

// LAST: the last step of a call (ocn_ctx.hip one_step_last): it also stores what the reference's
// last step leaves in the arrays and no later launch rewrites -- a3's vort and a5's stresses (the
// values D formed, where the reference stores them: the interior under luu / lu / luu) and the
// RHS terms a4 / a6 keep on the last step (sw_stencils.h FusedB `full`).  hh_init's and hh_update's
// levels are not stored: the call's final hh_init rewrites them on the same ranges.
// ZF: every point where D takes the array's value (mask 0, outside the stage's range) holds +0.0
// in those arrays, the external forcing RHSx / RHSy is +0.0 on the interior, and the rest depth
// h_r and the viscosity mu hold one value each over the step's reach (checked by
// launch_fallback_check; true from init on -- no stage ever writes the fallback points, and
// init_data.f90 sets h_r = 100 m and mu = 0 everywhere -- until a field is uploaded): those are
// kernel constants -- no loads (32 B per cell fewer), twelve array pointers fewer in the kernel's
// scalar registers, and the same arithmetic on the same values.
// X2: the block's halo points that neighbour blocks own (`own`, sw_stencils.h own_class bits) hold
// the neighbours' state two points deep (ocn_ctx.hip one_step_x2: one 2-deep exchange per step),
// so D there is formed here as the neighbour forms it on its interior -- what the reference's
// exchanges of D deliver -- and the march covers the whole interior.
// WT: write-through stores (sc1), for the multi-step launch (k_march_multi)
// PAIR + X2 (ocn_ctx.hip one_step_x4): two steps per launch on a block with halo exchanges, over the
// block's geometry widened by kXRing rings (ocn_internal.h; the arrays' bases moved to match): the
// exchange before it delivered the state 4 points deep, the producers update the halo points
// neighbours own 2 deep as those neighbours do (their D 3 deep, from the state 4 deep); the known-
// constant variant only (h_r, mu, the forcing and the fallback values are not read).
template <bool P2, bool LAST = false, bool ZF = false, bool X2 = false, bool HR = false, bool PAIR = false,
          bool WT = false>
struct MarchStep {
    static_assert(!PAIR || !X2 || (ZF && !LAST), "two-step launches with exchanges: the known-constant variants");
    static constexpr int kStAux = WT ? 16 : 0;
    static constexpr bool kPair = PAIR;
    static constexpr bool kX2 = X2;
    // the x2 single step and the x4 pair of the known-constant variant: co-launched with a tracer step
    // (k_march_tracer_b)
    static constexpr bool kCoTracer = X2 && ZF && !HR && !LAST && !WT;
    static constexpr int kPairCols = 116;   // PAIR: a workgroup's output columns (2 x 60 produced, less 2 each side)
    static constexpr bool kAligned = false;
    static constexpr int kHalo = 2;
    static constexpr int kWaves = PAIR ? OCN_PAIR_WAVES : OCN_STEP_WAVES;
    ocn_block b; Tab<true> t; ocn_sw_params sw; double tau; int32_t *nbad;
    double *sshp_out, *up_out, *vp_out;   // a8's filtered sshp / ubrtrp / vbrtrp (the second buffers)
    // ZF: kc[0], kc[1] = the values h_r and mu hold at every point the step reads (device memory,
    // written by launch_fallback_check).  gate: 0 = always run; 1 / 2 = run only if the device
    // check's verdict *fbz is 0 / nonzero (both variants launched, the device picks: no host wait)
    const double *kc; const int32_t *fbz; int gate;
    unsigned own;   // X2: own_class bits of the halo points neighbour blocks own
    int32_t *nbad2 = nullptr;   // PAIR: the second step's check_ssh_err count (nbad: the first step's)
    // PAIR + X2 with tracers (ocn_ctx.hip one_step_x4): the first step's new ssh, sshp, ubrtr, vbrtr --
    // what the producers put into the ring -- also to these arrays (the second tracer step reads them)
    double *trs[4] = {nullptr, nullptr, nullptr, nullptr};
    static constexpr bool kGate = true;
    // gate (OCN_KC_DEVICE): which verdict of the check (launch_fallback_check's flag word: bit 0 =
    // h_r not uniform, bit 1 = anything else) this launch is for -- 1: none, 3: h_r only, 2: bit 1
    __device__ __forceinline__ bool enabled() const
    {
        if (gate == 0) return true;
        const int f = *(const volatile int32_t *)fbz;
        return gate == 1 ? f == 0 : gate == 3 ? f == 1 : (f & 2) != 0;
    }

    // a / tau (sw_update_uv_math qtau).  P2: tau is a power of two, so a / tau is a * (1 / tau) bit
    // for bit (both round the same real value once; exact scalings unless subnormal)
    __device__ __forceinline__ double qtau(const StepRegs &x, double a) const { return P2 ? a * x.inv_tau : a / x.tau; }

    // one row's loads for iteration n (rows of the state the march adds)
    struct Batch { double u, v, up, vp, ssh, shp, hr, mu, rhsx, rhsy; unsigned bits; };
    // RO (PAIR): 1 = a producer wave (rows clamped into the block's arrays: its tile reaches 4 rows
    // past the consumers'), 2 = a consumer wave (the state rows from the LDS ring)
    __device__ __forceinline__ int rowc(int r, int RO) const { return RO == 1 ? min(max(r, b.bnd_y1), b.bnd_y2) : r; }
    template <int RO = 0> __device__ __forceinline__ void load(const StepRegs &x, Batch &q, int m, int n) const
    {
        if constexpr (RO == 2) {
            const Geo I = geo(&b);
            const Pt c2 = I(m, n + 2);
            q.ssh = g_pair[(n + 2) & 3][0][x.pj]; q.shp = g_pair[(n + 2) & 3][1][x.pj];
            q.u = g_pair[(n + 2) & 3][2][x.pj]; q.up = g_pair[(n + 2) & 3][3][x.pj];
            q.v = g_pair[(n + 1) & 3][4][x.pj]; q.vp = g_pair[(n + 1) & 3][5][x.pj];
            q.hr = ZF && !HR ? x.hr0 : ld(t.f(OCN_HHQ_REST), c2);
            q.bits = ld(t.bits, c2);
            if (ZF) {
                q.mu = x.mu0;
                q.rhsx = q.rhsy = 0.0;
            } else {   // (the general variant: mu and the forcing read as a single step reads them)
                q.mu = ld(t.f(OCN_MU), I(m, n + 1));
                q.rhsx = ld(t.f(OCN_RHSX), I(m, n));
                q.rhsy = ld(t.f(OCN_RHSY), I(m, n));
            }
            return;
        }
        const Geo I = geo(&b);
        const Pt c = I(m, rowc(n, RO)), c1 = I(m, rowc(n + 1, RO)), c2 = I(m, rowc(n + 2, RO));
        q.u = ld(t.f(OCN_UBRTR), c2); q.up = ld(t.f(OCN_UBRTRP), c2);
        q.ssh = ld(t.f(OCN_SSH), c2); q.shp = ld(t.f(OCN_SSHP), c2);
        q.hr = ZF && !HR ? x.hr0 : ld(t.f(OCN_HHQ_REST), c2);
        q.bits = ld(t.bits, c2);
        q.v = ld(t.f(OCN_VBRTR), c1); q.vp = ld(t.f(OCN_VBRTRP), c1); q.mu = ZF ? x.mu0 : ld(t.f(OCN_MU), c1);
        if (ZF) q.rhsx = q.rhsy = 0.0;
        else { q.rhsx = ld(t.f(OCN_RHSX), c); q.rhsy = ld(t.f(OCN_RHSY), c); }
    }
    template <int PH> __device__ __forceinline__ static void take(StepRegs &x, const Batch &q)
    {
        x.u.s<PH>(3) = q.u; x.up.s<PH>(3) = q.up; x.ssh.s<PH>(3) = q.ssh; x.shp.s<PH>(3) = q.shp; x.hr.s<PH>(3) = q.hr;
        x.bits.s<PH>(3) = q.bits;
        x.v.s<PH>(2) = q.v; x.vp.s<PH>(2) = q.vp; x.mu.s<PH>(2) = q.mu;
        x.rhsx = q.rhsx; x.rhsy = q.rhsy;
    }

    // hh_init's interpolation weights of row n + dy (slot dy + 1): interp_wt(h) = h * dx * dy * lu
    // (sw_stencils.h) with h = h_r + sh * ffs (level 0) or h_r + shp * ffs (level 1).  The weight
    // of corner (m+1, n) / (m, n+1) of a point is its right / upper neighbour's own weight: dx and
    // dy are constant along a row, so the operands are the same.
    template <int PH> __device__ __forceinline__ static void weights(StepRegs &x, int dy)
    {
        const int k = dy + 1;
        const double gx = x.cst<kLds>(RC_DX, dy), gy = x.cst<kLds>(RC_DY, dy);
        const double l = x.mkd<PH>(OCN_LU, 0, dy);
        // ffs = 1 (launch_onepass requires it): sh * ffs is sh bit for bit
        x.w0.s<PH>(k) = (x.hr.s<PH>(k) + x.ssh.s<PH>(k)) * gx * gy * l;
        x.w1.s<PH>(k) = (x.hr.s<PH>(k) + x.shp.s<PH>(k)) * gx * gy * l;
        x.w0r.s<PH>(k) = shz(x.w0.s<PH>(k), 1);   // its right lane's weight: the corner (m+1) weight
    }

    // Where D takes the value in memory (mask 0 or outside the stage's range): those loads, issued
    // (exec-masked) one iteration ahead, for row r = n + 2 (its mask byte arrives with that row),
    // so that nothing in an iteration waits for the loads the iteration itself issues
    struct Fallback {
        bool llu, llv, luh, vt, st, ss;   // the computed value is used
        double hu, hv, hh, hu1, hv1, vort, stt, sts;
    };
    template <int PH, int RO = 0>
    __device__ __forceinline__ void fallback(const StepRegs &x, Fallback &f, int m, int r, int slot) const
    {
        const Pt c = geo(&b)(m, rowc(r, RO));   // (PAIR producers: their rows reach past the arrays)
        const unsigned bc = x.bits.s<PH>(slot);
        bool hh_rng = m >= b.nx_start - 1 && m <= b.nx_end && r >= b.ny_start - 1 && r <= b.ny_end;
        bool in = m >= b.nx_start && m <= b.nx_end && r >= b.ny_start && r <= b.ny_end;
        if (X2) {   // a point a neighbour owns is in its interior: in both stages' ranges there
            const bool owned = (own >> (own_class(m, b.nx_start, b.nx_end) * 3u + own_class(r, b.ny_start, b.ny_end))) & 1u;
            hh_rng = hh_rng || owned;
            in = in || owned;
        }
        f.llu = hh_rng && (bc & (1u << OCN_LLU));
        f.llv = hh_rng && (bc & (1u << OCN_LLV));
        f.luh = hh_rng && (bc & (1u << OCN_LUH));
        f.vt = in && (bc & (1u << OCN_LUU));
        f.st = in && (bc & (1u << OCN_LU));
        f.ss = f.vt;
        f.hu = f.hv = f.hh = f.hu1 = f.hv1 = f.vort = f.stt = f.sts = 0.0;
        if (ZF) return;
        if (!f.llu) { f.hu = ld(t.f(OCN_HHU), c); f.hu1 = ld(t.f(OCN_HHU_P), c); }
        if (!f.llv) { f.hv = ld(t.f(OCN_HHV), c); f.hv1 = ld(t.f(OCN_HHV_P), c); }
        if (!f.luh) f.hh = ld(t.f(OCN_HHH), c);
        if (!f.vt) { f.vort = ld(t.f(OCN_VORT), c); f.sts = ld(t.f(OCN_STR_S), c); }
        if (!f.st) f.stt = ld(t.f(OCN_STR_T), c);
    }

    // D at row r = n + 1 of this lane (column m): the values the reference's arrays hold there,
    // plus the shared products of that row
    // E: IEEE divisions (the exact re-run of a row some dividend of which is out of udiv's range)
    template <bool E> __device__ __forceinline__ static double dv(double a, double d, double rd)
    {
        if constexpr (E) return a / d;
        else return udiv(a, d, rd);
    }
    // N independent quotients x[i] / d[i], each stage of udiv issued for all N before the next
    // (MarchStep::derive, step): the same operations on the same operands as N separate udivs, written so
    // that N dependency chains are in flight at once rather than one after another
    template <bool E, int N>
    __device__ __forceinline__ static void dvn(const double (&a)[N], const double (&d)[N], const double (&rd)[N],
                                               double (&out)[N])
    {
        if constexpr (E) {
#pragma unroll
            for (int i = 0; i < N; ++i) out[i] = a[i] / d[i];
        } else {
            double q[N], t[N];
#pragma unroll
            for (int i = 0; i < N; ++i) q[i] = a[i] * rd[i];
#pragma unroll
            for (int i = 0; i < N; ++i) t[i] = __builtin_fma(q[i], d[i], -a[i]);
#pragma unroll
            for (int i = 0; i < N; ++i) out[i] = __builtin_fma(-t[i], rd[i], q[i]);
        }
    }
    template <bool E, int PH>
    __device__ __forceinline__ void derive(StepRegs &x, const Fallback &fb, int &acc, double &qb_next,
                                           double &qc_next) const
    {
        weights<PH>(x, 2);   // row n+2 (rows n+1's were formed one iteration ago)
        // hh_init levels 0 and 1 (depth.f90:52-97, sw_stencils.h interp_u / interp_v / interp_h)
        // the sea counts of the averages (sw_stencils.h div_mask_sum: a / s, s the sum of lu)
        const unsigned b00 = x.bit<PH>(OCN_LU, 0, 1), b10 = x.bit<PH>(OCN_LU, 1, 1), b01 = x.bit<PH>(OCN_LU, 0, 2),
                       b11 = x.bit<PH>(OCN_LU, 1, 2);
        const unsigned cu = b00 + b10, cv = b00 + b01, ch = cu + b01 + b11;
        const double dxt = x.cst<kLds>(RC_DXT, 1), dyt = x.cst<kLds>(RC_DYT, 1), dxh = x.cst<kLds>(RC_DXH, 1),
                     dyh = x.cst<kLds>(RC_DYH, 1), dxb = x.cst<kLds>(RC_DXB, 1), dyb = x.cst<kLds>(RC_DYB, 1);
        // the right lane's weights, shifted once per row (weights) and kept in the ring
        const double w00 = x.w0.s<PH>(2), w10 = x.w0r.s<PH>(2), w01 = x.w0.s<PH>(3), w11 = x.w0r.s<PH>(3);
        const double p00 = x.w1.s<PH>(2), p10 = shz(p00, 1), p01 = x.w1.s<PH>(3);
        const double s0 = w00 + w10;
        const double rxt = x.cst<kLds>(RC_RDXT, 1), ryh = x.cst<kLds>(RC_RDYH, 1), rxh = x.cst<kLds>(RC_RDXH, 1),
                     ryt = x.cst<kLds>(RC_RDYT, 1);
        const double ru = rcp_sea(cu), rv = rcp_sea(cv);
        const double a_u0 = s0 * ru, a_v0 = (w00 + w01) * rv, a_u1 = (p00 + p10) * ru, a_v1 = (p00 + p01) * rv;
        // a / 3 (three sea corners): udiv by 3 (the same correctly rounded quotient: its dividend's
        // range is checked with the others below), IEEE division in the re-run -- per lane, no branch
        const double sh = s0 + w01 + w11;
        const double a_h0 = ch == 3 ? (E ? sh / 3.0 : udiv(sh, 3.0, 1.0 / 3.0)) : sh * rcp_sea(ch);
        if (!E) exp_check(acc, sh);
        if (!E) {   // (a / g1) / g2: a's range bounds a / g1's (|g1| <= 2^60)
            exp_check(acc, a_u0); exp_check(acc, a_v0); exp_check(acc, a_h0); exp_check(acc, a_u1);
            exp_check(acc, a_v1); exp_check(acc, x.up.s<PH>(2)); exp_check(acc, x.vp.s<PH>(2)); exp_check(acc, x.up.s<PH>(3));
        }
        // the nine first quotients (hh_init's five, a5's four) at once, then the five second ones
        // (each stage of udiv issued for all of them: independent chains in flight together)
        double q1[9], q2[5];
        dvn<E, 9>({a_u0, a_v0, a_h0, a_u1, a_v1, x.up.s<PH>(2), x.vp.s<PH>(2), x.up.s<PH>(3), x.vp.s<PH>(2)},
                  {dxt, dxh, dxb, dxt, dxh, dyh, dxh, x.cst<kLds>(RC_DXT, 2), dyt},
                  {rxt, rxh, x.cst<kLds>(RC_RDXB, 1), rxt, rxh, ryh, rxh, x.cst<kLds>(RC_RDXT, 2), ryt}, q1);
        dvn<E, 5>({q1[0], q1[1], q1[2], q1[3], q1[4]}, {dyh, dyt, dyb, dyh, dyt},
                  {ryh, ryt, x.cst<kLds>(RC_RDYB, 1), ryh, ryt}, q2);
        const double u0 = q2[0], v0 = q2[1], h0 = q2[2], u1 = q2[3], v1 = q2[4];
        // a3 uv_trans_vort (vel_ssh.f90:247-281, sw_stencils.h uv_trans_vort_math)
        const double u_0 = x.u.s<PH>(2), u_1 = x.u.s<PH>(3), v_0 = x.v.s<PH>(2), v_r = shz(v_0, 1);
        x.vr.s<PH>(2) = v_r;   // S reads it at rows n and n-1 (the same shift of the same values)
        const double vort = (v_r * dyt - v_0 * dyt) - (u_1 * x.cst<kLds>(RC_DXT, 2) - u_0 * dxt)
                            - ((v_r - v_0) * dyb - (u_1 - u_0) * dxb);
        // a5 (mixing.f90:33-44, sw_stencils.h stress_components_math) with its quotients shared:
        // up/dyh at m-1 is the left lane's up/dyh (dyh is constant along the row), vp/dxh at n-1
        // is the previous row's, up/dxt at n+1 the next row's (formed here, kept for the next
        // row), vp/dyt at m+1 the right lane's -- the same operands, so the same values
        const double qa = q1[5], qb = q1[6], qc1 = q1[7], qe = q1[8];
        const double st = x.cst<kLds>(RC_RAT0, 1) * (qa - shz(qa, -1)) - x.cst<kLds>(RC_RAT1, 1) * (qb - x.qb);
        const double ss = x.cst<kLds>(RC_RAT2, 1) * (qc1 - x.qc) + x.cst<kLds>(RC_RAT3, 1) * (shz(qe, 1) - qe);
        qb_next = qb;
        qc_next = qc1;
        const double hu = fb.llu ? u0 : fb.hu;
        const double hv = fb.llv ? v0 : fb.hv;
        const double hh = fb.luh ? h0 : fb.hh;
        const double vt = fb.vt ? vort : fb.vort;
        const double stt = fb.st ? st : fb.stt;
        x.hu.s<PH>(2) = hu; x.hv.s<PH>(2) = hv; x.hh.s<PH>(2) = hh; x.vort.s<PH>(2) = vt; x.stt.s<PH>(2) = stt;
        x.hu1.s<PH>(2) = fb.llu ? u1 : fb.hu1;
        x.hv1.s<PH>(2) = fb.llv ? v1 : fb.hv1;
        x.sts.s<PH>(2) = fb.ss ? ss : fb.sts;
        // shared products of row r (S reads them at m +- 1 and at rows n-1 .. n+1); each is the
        // reference's sub-expression with the same operands in the same order
        x.pu.s<PH>(2) = u_0 * dyh * hu;                                  // uv_trans: u * dyh * hu
        x.pv.s<PH>(2) = v_0 * dxh * hv;                                  // uv_trans: v * dxh * hv
        x.vh.s<PH>(2) = vt * hh;                                         // uv_trans: vort * hh
        x.t3.s<PH>(2) = v_0 * hv * dxh;                                  // sw_update_ssh: vbrtr * hhv * dxh
        const double rr = x.cst<kLds>(RC_RLH, 1) * hh * dxb * dyb;   // sw_update_uv: rlh_s * hhh * dxb * dyb
        x.rr.s<PH>(2) = rr;
        x.cx.s<PH>(2) = rr * (v_r + v_0);                                //   ... * (vbrtr(1,0) + vbrtr)
        const double hq = x.hr.s<PH>(2) + x.ssh.s<PH>(2);                    // depth.f90:48 hq = h_r + sh*ffs (ffs = 1)
        if constexpr (kLds) {   // (the LDS rows hold dy**2 * mu, dx**2 * mu: prologue)
            x.dt.s<PH>(2) = x.cst<kLds>(RC_DY2, 1) * hq * stt;
            x.dxq.s<PH>(2) = x.cst<kLds>(RC_DX2, 1) * hq * stt;
        } else {
            x.dt.s<PH>(2) = x.cst<kLds>(RC_DY2, 1) * x.mu.s<PH>(2) * hq * stt;         // uv_diff2: dy**2 * mu * hq * str_t
            x.dxq.s<PH>(2) = x.cst<kLds>(RC_DX2, 1) * x.mu.s<PH>(2) * hq * stt;        // uv_diff2: dx**2 * mu * hq * str_t
        }
    }

    // (the warm-up row n = nb - 1, after D(nb)) the n+1 faces of row n that S(nb) takes from the
    // row before -- the expressions S(n) forms them with (step)
    template <int PH> __device__ __forceinline__ void face(StepRegs &x) const
    {
        const double u = x.u.s<PH>(1), v = x.v.s<PH>(1), u_n = x.u.s<PH>(2), v_n = x.v.s<PH>(2);
        const double v_r = x.vr.s<PH>(1);
        const double pv = x.pv.s<PH>(1), pvn = x.pv.s<PH>(2), luu = x.mkd<PH>(OCN_LUU, 0, 0);
        x.fyx = (pv + shz(pv, 1)) / 2.0 * (u_n + u) / 2.0 * luu;
        x.vht = x.vh.s<PH>(1) * (v_r + v);
        x.fyy = (pv + pvn) / 2.0 * (v + v_n) / 2.0;
        if constexpr (ZF) {   // (uv_diff2_math's muh_p with mu one value: its lane shifts are the value)
            const double mu = x.mu.s<PH>(1), mu_n = x.mu.s<PH>(2), muh_p = (mu + mu + mu_n + mu_n) / 4.0;
            (void)muh_p;   // (kLds = ZF: the LDS row holds dxb**2 * muh)
            x.a2t = x.cst<kLds>(RC_DXB2, 0) * x.hh.s<PH>(1) * x.sts.s<PH>(1);
        }
    }

    // a row's outputs and where they are stored (store_out, after S's branch)
    struct Out {
        bool lu = false, cu = false, cv = false, uu = false;   // uu: luu (LAST's vort / str_s)
        double sshn = 0.0, fx = 0.0, un = 0.0, fa = 0.0, vn = 0.0, fb = 0.0;
        double vort = 0.0, sts = 0.0, stt = 0.0, rxa = 0.0, rxd = 0.0, rya = 0.0, ryd = 0.0;   // LAST
        double fyx = 0.0, fyy = 0.0, vht = 0.0, a2t = 0.0;   // row n's n+1 faces (see face)
    };
    // S at row n: a1, fused B, a8's filters, check_ssh_err (sw_stencils.h sw_update_ssh_math,
    // uv_trans_math, uv_diff2_math, sw_update_uv_math written out over the shared products)
    template <bool E, int PH>
    __device__ __forceinline__ void step(const StepRegs &x, const Lane &L, int n, int &acc, bool &bad, Out &o) const
    {
        (void)n;
        const double u = x.u.s<PH>(1), v = x.v.s<PH>(1), hu = x.hu.s<PH>(1), hv = x.hv.s<PH>(1), hh = x.hh.s<PH>(1);
        const double dxt = x.cst<kLds>(RC_DXT, 0), dyt = x.cst<kLds>(RC_DYT, 0), dxh = x.cst<kLds>(RC_DXH, 0),
                     dyh = x.cst<kLds>(RC_DYH, 0);
        // a1 sw_update_ssh (vel_ssh.f90:69-106)
        const double t1 = u * hu * dyh;
        const double a_ssh = t1 - shz(t1, -1) + x.t3.s<PH>(1) - x.t3.s<PH>(0);
        if (!E) exp_check(acc, a_ssh);
        // a4 uv_trans (vel_ssh.f90:283-373)
        const double u_r = shz(u, 1), u_n = x.u.s<PH>(2);
        const double v_r = x.vr.s<PH>(1), v_n = x.v.s<PH>(2);
        const double pu = x.pu.s<PH>(1), pun = x.pu.s<PH>(2), pv = x.pv.s<PH>(1), pvn = x.pv.s<PH>(2);
        const double luu = x.mkd<PH>(OCN_LUU, 0, 0);
        double rxa, rya;
        // each face's flux once: the m-1 face is the left lane's m+1 face and the n-1 face the row
        // before's n+1 face (carried in x, face<PH>) -- the same operands, the sums' terms swapped
        // (IEEE addition commutes), so the same values bit for bit
        {
            const double fx_p = (pu + shz(pu, 1)) / 2.0 * (u + u_r) / 2.0;
            const double fx_m = shz(fx_p, -1);
            const double fy_p = (pv + shz(pv, 1)) / 2.0 * (u_n + u) / 2.0 * luu;
            const double cor = x.vh.s<PH>(1) * (v_r + v);
            rxa = -(fx_p - fx_m + fy_p - x.fyx) + (cor + x.vht) / 4.0;
            o.fyx = fy_p;
            o.vht = cor;
        }
        {
            const double fy_p = (pv + pvn) / 2.0 * (v + v_n) / 2.0;
            const double sn = pu + pun;
            const double fx_p = sn / 2.0 * (v_r + v) / 2.0;
            const double fx_m = shz(fx_p, -1);
            const double q = x.vh.s<PH>(1) * (u_n + u);
            rya = -(fx_p - fx_m + fy_p - x.fyy) - (q + shz(q, -1)) / 4.0;
            o.fyy = fy_p;
        }
        // a6 uv_diff2 (vel_ssh.f90:375-452)
        double rxd, ryd;
        double q_ssh = 0.0;   // a1's a_ssh / area
        {
            // ZF: mu is one value over the step's reach, so its neighbours are that value (the lane
            // shifts differ only on the edge lanes, which produce no output and whose mu terms no
            // other lane reads) and the three averages are one loop-invariant value
            auto sh = [](double a, int d) { return ZF ? a : shz(a, d); };
            const double mu = x.mu.s<PH>(1), mu_r = sh(mu, 1), mu_l = sh(mu, -1), mu_n = x.mu.s<PH>(2), mu_s = x.mu.s<PH>(0);
            const double muh_p = (mu + mu_r + mu_n + sh(mu_n, 1)) / 4.0;
            const double muh_m = (mu + mu_r + mu_s + sh(mu_s, 1)) / 4.0;
            const double muh_m2 = (mu + mu_l + mu_n + sh(mu_n, -1)) / 4.0;
            const double dxb2 = x.cst<kLds>(RC_DXB2, 0), dxb2m = x.cst<kLds>(RC_DXB2, -1), dyb2 = x.cst<kLds>(RC_DYB2, 0);
            const double sts = x.sts.s<PH>(1);
            const double dtc = x.dt.s<PH>(1);
            // ZF: the three averages are one value, so a2's second term is the row before's first
            // (carried) and a4's the left lane's first -- the same operands, the same values
            double a2, a4;
            if constexpr (ZF) {
                (void)dxb2m; (void)muh_m; (void)muh_m2;
                // (kLds = ZF: dxb2 / dyb2 are the LDS rows' dxb**2 * muh, dyb**2 * muh -- prologue)
                (void)muh_p;
                const double a2p = dxb2 * hh * sts, a4p = dyb2 * hh * sts;
                a2 = a2p - x.a2t;
                a4 = a4p - shz(a4p, -1);
                o.a2t = a2p;
            } else {
                a2 = dxb2 * muh_p * hh * sts - dxb2m * muh_m * x.hh.s<PH>(0) * x.sts.s<PH>(0);
                a4 = dyb2 * muh_p * hh * sts - dyb2 * muh_m2 * shz(hh, -1) * shz(sts, -1);
            }
            const double a1 = shz(dtc, 1) - dtc, a3 = x.dxq.s<PH>(2) - x.dxq.s<PH>(1);
            {
                if (!E) { exp_check(acc, a1); exp_check(acc, a2); exp_check(acc, a3); exp_check(acc, a4); }
                // a1's quotient with uv_diff2's four, stage by stage (dvn)
                double qd[5];
                dvn<E, 5>({a_ssh, a1, a2, a3, a4}, {x.cst<kLds>(RC_AREA, 0), dyh, dxt, dxh, dyt},
                          {x.cst<kLds>(RC_RAREA, 0), x.cst<kLds>(RC_RDYH, 0), x.cst<kLds>(RC_RDXT, 0),
                           x.cst<kLds>(RC_RDXH, 0), x.cst<kLds>(RC_RDYT, 0)}, qd);
                q_ssh = qd[0];
                rxd = qd[1] + qd[2];
                ryd = -qd[3] + qd[4];
            }
        }
        const double sshn = x.shp.s<PH>(1) + 2.0 * x.tau * (-q_ssh);
        // a7 sw_update_uv (vel_ssh.f90:108-195); hun = hu, hvn = hv (the reuse identity)
        double un, vn;
        {
            const double g = D(OCN_FREE_FALL_ACC);
            const double ssh = x.ssh.s<PH>(1);
            {
                const double bp = qtau(x, hu * dxt * dyh / 2.0);
                const double bp0 = qtau(x, x.hu1.s<PH>(1) * dxt * dyh / 2.0);
                const double slx = -(g * (shz(ssh, 1) - ssh) * dyh * hu);
                // (rdis + rdis) / 2 (kLds: the LDS row holds it halved)
                const double fric = (kLds ? x.cst<kLds>(RC_RDSELF, 0) : x.cst<kLds>(RC_RDSELF, 0) / 2.0) * x.up.s<PH>(1) * dxt *
                                    dyh * hu;
                const double grx = x.rhsx + slx + rxd + rxa - fric + (x.cx.s<PH>(1) + x.cx.s<PH>(0)) / 4.0;
                un = (x.up.s<PH>(1) * bp0 + grx) / (bp);
            }
            {
                const double bp = qtau(x, hv * dyt * dxh / 2.0);
                const double bp0 = qtau(x, x.hv1.s<PH>(1) * dyt * dxh / 2.0);
                const double sly = -(g * (x.ssh.s<PH>(2) - ssh) * dxh * hv);
                // (rdis + rdis(n+1)) / 2 (kLds: halved in the LDS row)
                const double fric = (kLds ? x.cst<kLds>(RC_RDNEXT, 0) : x.cst<kLds>(RC_RDNEXT, 0) / 2.0) * x.vp.s<PH>(1) * dxh *
                                    dyt * hv;
                const double c1 = x.rr.s<PH>(1) * (u_n + u);
                const double gry = x.rhsy + sly + ryd + rya - fric - (c1 + shz(c1, -1)) / 4.0;
                vn = (x.vp.s<PH>(1) * bp0 + gry) / (bp);
            }
        }
        // a8 sw_next_step's filters (vel_ssh.f90:197-245) + check_ssh_err (vel_ssh.f90:40-67)
        const double ts = sw.time_smooth;
        const double fx = asselin(x.ssh.s<PH>(1), sshn, x.shp.s<PH>(1), ts);
        const double fa = asselin(u, un, x.up.s<PH>(1), ts), fb = asselin(v, vn, x.vp.s<PH>(1), ts);
        // the row's stores are issued after the branch (iteration, store_out)
        const unsigned bc = x.bits.s<PH>(1);
        o.lu = L.out && (bc & (1u << OCN_LU));
        o.cu = L.out && (bc & (1u << OCN_LCU));
        o.cv = L.out && (bc & (1u << OCN_LCV));
        o.sshn = sshn; o.fx = fx; o.un = un; o.fa = fa; o.vn = vn; o.fb = fb;
        if (LAST) {
            o.uu = L.out && (bc & (1u << OCN_LUU));
            o.vort = x.vort.s<PH>(1); o.sts = x.sts.s<PH>(1); o.stt = x.stt.s<PH>(1);
            o.rxa = rxa; o.rxd = rxd; o.rya = rya; o.ryd = ryd;
        }
        // check_ssh_err counts each point once: the re-run (E) corrects the first pass's count
        const bool bd = o.lu && !(sshn < 10000.0 && sshn > -10000.0);
        if (__builtin_expect(x.nbp && x.cnt && bd != (E && bad), 0)) atomicAdd(x.nbp, bd ? 1 : -1);
        bad = bd;
    }

    // a row's six stores, issued by every iteration (warm-up rows with every lane dropped) and by
    // no branch: every path to the next row's use of its loads has issued the same six after them
    __device__ __forceinline__ void store_out(const Out &o, unsigned c) const
    {
        const unsigned nbytes = (unsigned)b.pitch * (unsigned)(b.bnd_y2 - b.bnd_y1 + 1) * 8u;
        st_on<kStAux>(t.f(OCN_SSHN), nbytes, c, o.sshn, o.lu);
        st_on<kStAux>(sshp_out, nbytes, c, o.fx, o.lu);
        st_on<kStAux>(t.f(OCN_UBRTRN), nbytes, c, o.un, o.cu);
        st_on<kStAux>(up_out, nbytes, c, o.fa, o.cu);
        st_on<kStAux>(t.f(OCN_VBRTRN), nbytes, c, o.vn, o.cv);
        st_on<kStAux>(vp_out, nbytes, c, o.fb, o.cv);
        if (LAST) {   // what the reference's last step leaves (see MarchStep)
            st_on<kStAux>(t.f(OCN_VORT), nbytes, c, o.vort, o.uu);
            st_on<kStAux>(t.f(OCN_STR_S), nbytes, c, o.sts, o.uu);
            st_on<kStAux>(t.f(OCN_STR_T), nbytes, c, o.stt, o.lu);
            st_on<kStAux>(t.f(OCN_RHSX_ADV), nbytes, c, o.rxa, o.cu);
            st_on<kStAux>(t.f(OCN_RHSX_DIF), nbytes, c, o.rxd, o.cu);
            st_on<kStAux>(t.f(OCN_RHSY_ADV), nbytes, c, o.rya, o.cv);
            st_on<kStAux>(t.f(OCN_RHSY_DIF), nbytes, c, o.ryd, o.cv);
        }
    }

    // PAIR: the workgroup's barrier between iterations (LDS only: the row loads stay in flight)
    __device__ __forceinline__ static void pair_barrier()
    {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
    }
    // PAIR producer: row n of the first step's new state into the ring -- the value formed where
    // the step updates the point (the store flags), the state it read elsewhere: what the buffers
    // the second step reads hold there (outside a8's write sets the pairs and the second buffers
    // agree with the ones read: MarchStep, one_step_fused)
    template <int PH> __device__ __forceinline__ void pair_put(const StepRegs &x, const Out &o, int n) const
    {
        const int lane = (int)threadIdx.x & 63;
        if (lane >= kHalo && lane < 64 - kHalo) {
            double(*r)[120] = g_pair[n & 3];
            r[0][x.pj] = o.lu ? o.sshn : x.ssh.s<PH>(1);
            r[1][x.pj] = o.lu ? o.fx : x.shp.s<PH>(1);
            r[2][x.pj] = o.cu ? o.un : x.u.s<PH>(1);
            r[3][x.pj] = o.cu ? o.fa : x.up.s<PH>(1);
            r[4][x.pj] = o.cv ? o.vn : x.v.s<PH>(1);
            r[5][x.pj] = o.cv ? o.fb : x.vp.s<PH>(1);
        }
    }
    // row constants in LDS: the known-constant variant (the general one keeps scalar loads of the row
    // table -- with its loaded h_r, mu, forcing and fallback values the LDS operands spill VGPRs:
    // 0.83 vs 0.64 ms at 4096^2)
    static constexpr bool kLds = ZF;
    // the march unrolled over the register ring (StepRegs::Win) -- the known-constant variant; the
    // general one (loaded h_r, mu, forcing, fallback values) keeps the rotating loop: unrolled,
    // its scalar and vector registers spill
    static constexpr bool kUnroll = ZF;
    static constexpr bool kPrologue = kLds;
    // the row constants of the workgroup's rows into LDS (rows fit: launch_step's tiles have at
    // most OCN_STEP_ROWS rows)
    __device__ void prologue(const MarchRect &R, int ty) const
    {
        const int h = R.vert ? 4 * R.rows : R.rows, nb = R.n0 + ty * h;
        if (nb > R.n1) return;   // workgroup-uniform
        // rows [nb - 2, ne + 2]; PAIR: [nb - 5, ne + 4] (the producers' rows reach 2 past the consumers')
        const int ne = min(R.n1, nb + h - 1), lo = nb - (PAIR ? 5 : 2) - b.bnd_y1, i = (int)threadIdx.x;
        if (i < ne - nb + (PAIR ? 10 : 5)) {   // a thread per row
            const unsigned r = (unsigned)min(max(lo + i, 0), (int)t.nrows - 1);
            // (the known-constant variant: mu is the one value mu0 = kc[1], so the row-uniform leading
            // factors of four products -- dy**2 * mu, dx**2 * mu, dxb**2 * muh, dyb**2 * muh with muh
            // = (mu + mu + mu + mu) / 4 as uv_diff2_math forms it -- and the friction's (rdis + rdis') / 2
            // are formed here once per row: the same operations on the same operands)
            const double mu0 = kc[1], muh = (mu0 + mu0 + mu0 + mu0) / 4.0;
#pragma unroll
            for (int k = 0; k < kRowC; ++k) {
                double v = row_const(t.rows, t.nrows, r, k);
                if (k == RC_DY2 || k == RC_DX2) v = v * mu0;
                else if (k == RC_DXB2 || k == RC_DYB2) v = v * muh;
                else if (k == RC_RDSELF || k == RC_RDNEXT) v = v / 2.0;
                g_step_rc[i * kRowC + k] = v;
            }
        }
        if (threadIdx.x == 0) g_step_rlo = (unsigned)lo;
        // PAIR: the workgroup meets after its producers have issued their first state loads
        // (march_role<1>, the consumers' first barrier) -- the table's and the state's memory
        // latencies overlap instead of following each other
        if constexpr (!PAIR) __syncthreads();
    }

    // PAIR (two steps in one launch, single block, a variant chosen on the host): the producer waves march the
    // first step over the workgroup's rows +- 2 and put its new state into the LDS ring, the
    // consumer waves march the second step over the workgroup's rows from there, 6 iterations
    // behind (an iteration's ring reads are rows the producers finished before the last barrier);
    // every wave passes R + 8 barriers (R = the tile's rows): at barrier interval t the producers
    // write row nb - 4 + t, the consumers read rows nb - 5 + t and nb - 6 + t (their first reads,
    // rows nb - 2 .. nb, in interval 5), so a ring of 4 rows is never read and written at once.  The launch writes
    // the second step's new state where a single step writes (the new-state and second buffers):
    // the pair is one role flip -- the first step's new state never reaches memory
    __device__ void march(const Lane &L, int nb, int ne) const
    {
        if constexpr (PAIR) {
            if (L.pr == 1) {
                march_role<1>(L, nb - 2, ne + 2);
                pair_barrier();
                pair_barrier();
            } else {   // (march_role<2> has one more before its loop: after its first ring reads)
#pragma unroll
                // (+1 with the prologue: its barrier, met by the producers after their first loads)
                for (int k = 0; k < 5 + (kPrologue ? 1 : 0); ++k) pair_barrier();
                march_role<2>(L, nb, ne);
            }
            return;
        }
        march_role<0>(L, nb, ne);
    }
    template <int RO> __device__ void march_role(const Lane &L, int nb, int ne) const
    {
        const Geo I = geo(&b);
        StepRegs x{};
        x.nbp = RO == 2 ? nbad2 : nbad;
        x.cnt = true;
        x.pj = L.j;
        if (kLds) x.lds = (const __attribute__((address_space(3))) double *)g_step_rc;
        x.rows = (const __attribute__((address_space(4))) float *)t.rows;
        x.rcp = (const __attribute__((address_space(4))) double *)(t.rows + recip_offset(t.nrows));
        x.nrows = t.nrows;
        x.rn = (unsigned)(nb - 2 - b.bnd_y1);   // row n0
        x.tau = tau;
        x.inv_tau = 1.0 / tau;
        x.f = (double)sw.full_free_surface;
        if (ZF) { x.hr0 = kc[0]; x.mu0 = kc[1]; }
        // iteration n computes D(n+1) and, from n = nb on, S(n); two warm iterations give D(nb-1)
        // and D(nb).  Before iteration n0 = nb - 2 the rows it does not load itself: up, ssh, sshp,
        // h_r, bits at n0+1; vp at n0; metric rows n0, n0+1; the weights of row n0+1.
        const int n0 = nb - 2;
        {
            const Pt c = I(L.m, rowc(n0, RO)), c1 = I(L.m, rowc(n0 + 1, RO));
            if constexpr (RO == 2) {   // the first step's new state from the ring
                x.ssh.s<0>(2) = g_pair[(n0 + 1) & 3][0][x.pj]; x.shp.s<0>(2) = g_pair[(n0 + 1) & 3][1][x.pj];
                x.u.s<0>(2) = g_pair[(n0 + 1) & 3][2][x.pj]; x.up.s<0>(2) = g_pair[(n0 + 1) & 3][3][x.pj];
                x.vp.s<0>(1) = g_pair[n0 & 3][5][x.pj];
            } else {
                x.up.s<0>(2) = ld(t.f(OCN_UBRTRP), c1); x.ssh.s<0>(2) = ld(t.f(OCN_SSH), c1);
                x.shp.s<0>(2) = ld(t.f(OCN_SSHP), c1); x.u.s<0>(2) = ld(t.f(OCN_UBRTR), c1);
                x.vp.s<0>(1) = ld(t.f(OCN_VBRTRP), c);
            }
            x.hr.s<0>(2) = ZF && !HR ? x.hr0 : ld(t.f(OCN_HHQ_REST), c1);
            x.bits.s<0>(2) = ld(t.bits, c1);
        }
        Fallback fb;
        fallback<0, RO>(x, fb, L.m, n0 + 1, 2);
        Batch q;
        load<RO>(x, q, L.m, n0);
        // PAIR producer: the workgroup's first barrier (the row constants in LDS: prologue), its loads
        // in flight
        if constexpr (PAIR && RO == 1 && kPrologue) pair_barrier();
        if (kLds) x.rlo = g_step_rlo;
        // the shared stress quotients of rows n0 (vp/dxh) and n0+1 (up/dxt)
        x.qb = x.vp.s<0>(1) / x.cst<kLds>(RC_DXH, 0);
        x.qc = x.up.s<0>(2) / x.cst<kLds>(RC_DXT, 1);
        weights<0>(x, 1);
        if (RO != 1) store_out(Out{}, 0u);   // every lane dropped: the loop entry has six stores after its loads too
        // PAIR consumer: its first ring reads (rows nb - 2 .. nb, finished by the producers 2 barriers
        // ago) precede the barrier after which the producers overwrite row nb - 2's slot with nb + 2
        if constexpr (RO == 2) pair_barrier();
        // the two warm-up rows (D only), then rows nb .. ne with D and S in one basic block
        iteration<0, true, RO>(x, fb, q, L, n0, nb, ne);
        if constexpr (kUnroll) {   // unrolled kRing times: iteration n runs in phase (n - n0) % kRing
            iteration<1, true, RO>(x, fb, q, L, n0 + 1, nb, ne);
            for (int n = nb;; n += kRing) {
                if (iteration<2, false, RO>(x, fb, q, L, n, nb, ne)) break;
                if (iteration<3, false, RO>(x, fb, q, L, n + 1, nb, ne)) break;
                if (iteration<4, false, RO>(x, fb, q, L, n + 2, nb, ne)) break;
                if (iteration<0, false, RO>(x, fb, q, L, n + 3, nb, ne)) break;
                if (iteration<1, false, RO>(x, fb, q, L, n + 4, nb, ne)) break;
            }
        } else {
            x.rotate();
            iteration<0, true, RO>(x, fb, q, L, n0 + 1, nb, ne);
            x.rotate();
            for (int n = nb;; ++n) {
                if (iteration<0, false, RO>(x, fb, q, L, n, nb, ne)) break;
                x.rotate();
            }
        }
    }

    // iteration n (phase PH): D(n+1), and S(n) from n = nb on; true after the last (n = ne).
    // WARM = a warm-up row (n < nb: D only); else D(n+1) and S(n) are one basic block (no branch
    // between them: the scheduler interleaves S's work with D's division chains), each followed by
    // a wave-uniform test that re-runs it with IEEE divisions if any of its dividends was out of
    // udiv's range (nothing is stored before: store_out follows)
    template <int PH, bool WARM = false, int RO = 0>
    __device__ __forceinline__ bool iteration(StepRegs &x, Fallback &fb, Batch &q, const Lane &L0, int n, int nb,
                                              int ne) const
    {
        // the lane's column, opaque to the compiler in every iteration: its addresses are formed
        // where used, not held per phase across the unrolled loop
        Lane L = L0;
        asm volatile("" : "+v"(L.m));
        if (RO == 1) {   // PAIR producer: rows outside the interior keep their state; the count is the
            // workgroup's own points' (its columns, rows nb + 2 .. ne - 2).  X2: a halo point a neighbour
            // owns is one of its interior points -- updated as it updates it (the pair's exchange
            // delivered the state 4 deep: one_step_x4)
            const bool iny = n >= b.ny_start && n <= b.ny_end;
            if constexpr (X2) {
                const bool inx = L.m >= b.nx_start && L.m <= b.nx_end;
                const bool owned =
                    (own >> (own_class(L.m, b.nx_start, b.nx_end) * 3u + own_class(n, b.ny_start, b.ny_end))) & 1u;
                L.out = L.out && ((inx && iny) || owned);
            } else {
                L.out = L.out && iny;
            }
            x.cnt = L.ccol && n >= nb + 2 && n <= ne - 2;
        }
        take<PH>(x, q);
        Fallback fbn;
        if (n < ne) fallback<PH, RO>(x, fbn, L.m, n + 2, 3);   // consumed by the next iteration
        if (n < ne) load<RO>(x, q, L.m, n + 1);   // in flight while this row is computed
        Out o;
        {
            int acc = 0;
            double qb, qc;
            derive<false, PH>(x, fb, acc, qb, qc);
            if (__builtin_expect(__builtin_amdgcn_ballot_w64(acc < kUdivMinExp) != 0, 0))
                derive<true, PH>(x, fb, acc, qb, qc);
            acc = 0;
            if (WARM) {
                if (n == nb - 1) face<PH>(x);
            } else {
                bool bad = false;
                step<false, PH>(x, L, n, acc, bad, o);
                if (__builtin_expect(__builtin_amdgcn_ballot_w64(acc < kUdivMinExp) != 0, 0))
                    step<true, PH>(x, L, n, acc, bad, o);
                x.fyx = o.fyx;
                x.fyy = o.fyy;
                x.vht = o.vht;
                if (ZF) x.a2t = o.a2t;
            }
            x.qb = qb;
            x.qc = qc;
        }
        if constexpr (RO == 1) {   // PAIR producer: the row goes into the ring, not to memory
            if (!WARM) pair_put<PH>(x, o, n);
            if constexpr (X2) {   // (and to the tracer step's arrays: the lanes and rows that hold the state)
                if (!WARM && trs[0]) {
                    const unsigned nbytes = (unsigned)b.pitch * (unsigned)(b.bnd_y2 - b.bnd_y1 + 1) * 8u;
                    const unsigned ci = geo(&b)(L.m, min(max(n, b.bnd_y1), b.bnd_y2)).c;
                    const bool on = L0.out && n >= b.ny_start - 2 && n <= b.ny_end + 2;
                    st_on(trs[0], nbytes, ci, o.lu ? o.sshn : x.ssh.s<PH>(1), on);
                    st_on(trs[1], nbytes, ci, o.lu ? o.fx : x.shp.s<PH>(1), on);
                    st_on(trs[2], nbytes, ci, o.cu ? o.un : x.u.s<PH>(1), on);
                    st_on(trs[3], nbytes, ci, o.cv ? o.vn : x.v.s<PH>(1), on);
                }
            }
            pair_barrier();
            ++x.rn;
            fb = fbn;
            return n >= ne;
        }
        store_out(o, geo(&b)(L.m, n).c);   // warm-up rows: every lane dropped
        if constexpr (RO == 2) pair_barrier();
        ++x.rn;
        fb = fbn;
        return n >= ne;
    }
};
#undef OCN_MD

#define CHECK(...)                                                \
    do {                                                          \
        int _rc = check_block(b);                                 \
        if (_rc) return _rc;                                      \
        _rc = nonnull({__VA_ARGS__});                             \
        if (_rc) return _rc;                                      \
    } while (0)

// ================================================================== C ABI (kernel layer)
static int check_block(const ocn_block *b)
{
    if (!b) return set_error(OCN_ERR_ARG, "null ocn_block");
    if (b->nx_start > b->nx_end || b->ny_start > b->ny_end)
        return set_error(OCN_ERR_ARG, "empty interior");
    if (b->bnd_x1 > b->nx_start - 1 || b->bnd_x2 < b->nx_end + 1 || b->bnd_y1 > b->ny_start - 1 ||
        b->bnd_y2 < b->ny_end + 1)
        return set_error(OCN_ERR_ARG, "array bounds must include a 1-wide halo ring");
    if (b->pitch < (int64_t)(b->bnd_x2 - b->bnd_x1 + 1))
        return set_error(OCN_ERR_ARG, "pitch smaller than bnd_x2-bnd_x1+1");
    if (b->pitch * (int64_t)(b->bnd_y2 - b->bnd_y1 + 1) >= (int64_t(1) << 29))
        return set_error(OCN_ERR_ARG, "block array of 2^29 elements or more (32-bit byte offsets of r8 fields)");
    return OCN_OK;
}

static int nonnull(std::initializer_list<const void *> ps)
{
    for (const void *p : ps)
        if (!p) return set_error(OCN_ERR_ARG, "null array pointer");
    return OCN_OK;
}

#define RC_K(x) do { int _rc = (x); if (_rc) return _rc; } while (0)

// ------------------------------------------------------------------ fused launches
// cp == nullptr: the real(4) fields are read from the 2-D arrays; otherwise from the block's
// compact tables (sw_stencils.h "compact static fields", built by launch_prepare).
template <template <bool> class K, typename... A>
static int launch_fused(const Range &r, const Range &inner, int part, const ocn_block *b, void *const *ptr,
                        int nptr, const Compact *cp, int tracer, hipStream_t s, A... a)
{
    RC_K(check_block(b));
    if (cp)
        return launch_part(r, inner, part,
                           K<true>{*b, make_tab<true>(ptr, nptr, cp->bits, cp->rows, block_rows(b), tracer), a...}, s);
    return launch_part(r, inner, part, K<false>{*b, make_tab<false>(ptr, nptr, nullptr, nullptr, 0, tracer), a...},
                       s);
}

// With the compact tables and OCN_OPT_MARCH, fused A, fused B and hh_init run as register
// marches, their halo-overlap parts split as launch_march_part does (bands of a wave's width);
// otherwise one thread per point, split as sw_stencils.h frame_rects does (thin strips).
static bool use_march(const Compact *cp) { return cp && cp->march; }

int launch_fused_a(const ocn_block *b, void *const *ptr, int nptr, const Compact *cp, int part,
                   const ocn_sw_params &sw, double tau, bool reuse, hipStream_t s)
{
    const Range all = range_fused_a(b, sw, reuse);
    if (use_march(cp)) {
        RC_K(check_block(b));
        const Tab<true> t = make_tab<true>(ptr, nptr, cp->bits, cp->rows, block_rows(b), 0);
        if (sw.full_free_surface > 0 && !reuse)
            return launch_march_part(b, all, part, MarchFusedA<true>{*b, t, sw, tau}, s);
        return launch_march_part(b, all, part, MarchFusedA<false>{*b, t, sw, tau}, s);
    }
    return launch_fused<KFusedA>(all, inner_interior_shrunk(b), part, b, ptr, nptr, cp, 0, s, sw, tau, reuse);
}

int launch_fused_b(const ocn_block *b, void *const *ptr, int nptr, const Compact *cp, int part,
                   const ocn_sw_params &sw, double tau, bool full, bool reuse, hipStream_t s, int32_t *flip_nbad,
                   bool flip, bool rc, double *sshp_out, double *up_out, double *vp_out, const Range *inner)
{
    if (rc && (!flip || !reuse || sw.full_free_surface != 1 || !sshp_out))
        return set_error(OCN_ERR_ARG, "recomputed depths only on role-flip reuse steps with full_free_surface = 1");
    if (up_out || vp_out || inner) {   // the frame of a one-pass step with halo exchanges
        if (!flip || rc || !sshp_out || !up_out || !vp_out || !inner || !use_march(cp))
            return set_error(OCN_ERR_ARG, "fused B into the second buffers: role-flip, no recompute, three buffers, "
                                          "a frame, the march");
        RC_K(check_block(b));
        const Tab<true> t = make_tab<true>(ptr, nptr, cp->bits, cp->rows, block_rows(b), 0);
        MarchFusedB<true, false, true> k{*b, t, sw, tau, full, reuse, flip_nbad, sshp_out};
        k.up_out = up_out;
        k.vp_out = vp_out;
        return launch_march_frame(b, range_interior(b), *inner, k, s);
    }
    if (use_march(cp)) {
        RC_K(check_block(b));
        const Tab<true> t = make_tab<true>(ptr, nptr, cp->bits, cp->rows, block_rows(b), 0);
        const Range r = range_interior(b);
        if (flip && rc)
            return launch_march_part(b, r, part, MarchFusedB<true, true>{*b, t, sw, tau, full, reuse, flip_nbad, sshp_out},
                                     s);
        if (flip)
            return launch_march_part(b, r, part, MarchFusedB<true>{*b, t, sw, tau, full, reuse, flip_nbad, nullptr}, s);
        return launch_march_part(b, r, part, MarchFusedB<false>{*b, t, sw, tau, full, reuse, nullptr, nullptr}, s);
    }
    if (flip) return set_error(OCN_ERR_ARG, "the role-flip step needs the compact tables and the march");
    return launch_fused<KFusedB>(range_interior(b), inner_interior_shrunk(b), part, b, ptr, nptr, cp, 0, s, sw, tau,
                                 full, reuse);
}

int launch_fused_c1(const ocn_block *b, void *const *ptr, int nptr, const Compact *cp, int part,
                    const ocn_sw_params &sw, int32_t *nbad, hipStream_t s, const double *sshp_in,
                    const double *up_in, const double *vp_in)
{
    return launch_fused<KFusedC1>(range_ring(b), range_interior(b), part, b, ptr, nptr, cp, 0, s, sw, nbad, sshp_in,
                                  up_in, vp_in);
}

int launch_fused_c2(const ocn_block *b, void *const *ptr, int nptr, const Compact *cp, int part,
                    const ocn_sw_params &sw, bool full, hipStream_t s, bool keep_n, const TailCopy *copy)
{
    if (use_march(cp)) {
        RC_K(check_block(b));
        MarchHhInit k{*b, make_tab<true>(ptr, nptr, cp->bits, cp->rows, block_rows(b), 0),
                      (int)sw.full_free_surface, full, keep_n && full};
        if (copy) {
            if (part != OCN_PART_ALL || copy->src[0] != ptr[ocn_field_slot(OCN_SSH)])
                return set_error(OCN_ERR_ARG, "hh_init with the tail's copies: the whole bnd range, ssh as read");
            k.cu_src = copy->src[1]; k.cv_src = copy->src[2];
            k.csh_dst = copy->dst[0]; k.cu_dst = copy->dst[1]; k.cv_dst = copy->dst[2];
        }
        return launch_march_part(b, range_bnd(b), part, k, s);
    }
    if (copy) return set_error(OCN_ERR_ARG, "hh_init with the tail's copies: the march path only");
    return launch_fused<KHhInit>(range_bnd(b), inner_interior_shrunk(b), part, b, ptr, nptr, cp, 0, s,
                                 (int)sw.full_free_surface, full);
}

int launch_fused_ca(const ocn_block *b, void *const *ptr, int nptr, const Compact *cp, int part,
                    const ocn_sw_params &sw, double tau_next, bool next_reuse, bool skip_rc, hipStream_t s,
                    const Range *inner)
{
    if (!cp || !cp->march || sw.full_free_surface != 1 || (skip_rc && !next_reuse))
        return set_error(OCN_ERR_ARG, "fused hh_init + A needs the compact tables, the march and full_free_surface = 1");
    RC_K(check_block(b));
    const Tab<true> t = make_tab<true>(ptr, nptr, cp->bits, cp->rows, block_rows(b), 0);
    const Range r = range_bnd(b);
    if (inner) {   // the frame of a one-pass step with halo exchanges: the bnd range outside *inner
        if (skip_rc) return set_error(OCN_ERR_ARG, "fused CA frame: no recompute steps");
        if (!next_reuse)   // the call's last step: A stores hh_update's levels (its sync exchanges them)
            return launch_march_frame(b, r, *inner, MarchCA<true, false>{*b, t, sw, tau_next}, s);
        return launch_march_frame(b, r, *inner, MarchCA<false, false>{*b, t, sw, tau_next}, s);
    }
    if (skip_rc) return launch_march_part(b, r, part, MarchCA<false, true>{*b, t, sw, tau_next}, s);
    if (next_reuse) return launch_march_part(b, r, part, MarchCA<false, false>{*b, t, sw, tau_next}, s);
    return launch_march_part(b, r, part, MarchCA<true, false>{*b, t, sw, tau_next}, s);
}

// The one-pass step's grid: OCN_STEP_VERT = the 4 waves of a workgroup take 4 consecutive row
// tiles of one 60-column wave column (the rows a wave warms up with are its upper neighbour's,
// in the same CU's L1); else 4 wave columns side by side.
#ifndef OCN_STEP_VERT
#define OCN_STEP_VERT 1
#endif
// Rows per wave tile of the one-pass step: a wave spends rows + 2 (warm-up) iterations, and the
// launch runs in ceil(waves / slots) rounds of 2 waves per SIMD (256 CUs x 4 SIMDs); the tile
// height in [OCN_STEP_MIN_ROWS, OCN_STEP_ROWS] with the fewest iterations in total.  (A launch of 2.25 rounds
// spends a third of its time in a quarter-full last round.)
#ifndef OCN_STEP_SLOTS
#define OCN_STEP_SLOTS 2048
#endif
#ifndef OCN_STEP_MIN_ROWS
#define OCN_STEP_MIN_ROWS 1   // the shortest tile the cost model may pick (1: Black Sea 0.0159 -> 0.0148 ms per step)
#endif
template <class Body> static int step_rows(const Range &r, bool vert)
{
    const long wx = (r.m1 - r.m0 + 60) / 60, h = r.n1 - r.n0 + 1, wgx = (r.m1 - r.m0 + 240) / 240;
    int best = OCN_STEP_ROWS;
    long cost = -1;
    for (int rows = OCN_STEP_ROWS; rows >= OCN_STEP_MIN_ROWS; --rows) {
        // vert: 4 vertically stacked waves per workgroup; else 4 side by side (240 columns)
        const long tiles = vert ? (h + 4 * rows - 1) / (4 * rows) : (h + rows - 1) / rows;
        const long waves = vert ? 4 * tiles * wx : 4 * tiles * wgx, rounds = (waves + OCN_STEP_SLOTS - 1) / OCN_STEP_SLOTS;
        const long c = rounds * (rows + 2);
        if (cost < 0 || c < cost) { cost = c; best = rows; }
    }
    return best;
}
template <class Body> static int launch_step(const ocn_block *b, const Range &r, const Body &body, hipStream_t s)
{
    MarchGrid g{};
    g.r[0] = march_rect<Body>(b, r, step_rows<Body>(r, OCN_STEP_VERT != 0), OCN_STEP_VERT != 0);
    g.nr = 1;
    g.ntiles = g.r[0].tiles;
    return issue_march(g, body, s);
}

// The one-pass step over the frame of `all` outside `inner` (up to 4 bands in one launch: the
// overlapped x2 step's part that waits for the exchange): short tiles, the side bands with 4
// vertically stacked tiles per workgroup -- a band is a few points wide, so its waves are few
// and their length is the launch's latency
#ifndef OCN_FRAME_STEP_ROWS
#define OCN_FRAME_STEP_ROWS 4
#endif
template <class Body>
static int launch_step_frame(const ocn_block *b, const Range &all, const Range &inner, const Body &body, hipStream_t s)
{
    const Range in = range_clip(all, inner);
    if (range_empty(in)) return launch_step(b, all, body, s);
    const Rects q = frame_rects(all, in);
    MarchGrid g{};
    for (int i = 0; i < 4; ++i) {
        if (q.w[i] <= 0 || q.h[i] <= 0) continue;
        const Range r{q.m0[i], q.m0[i] + q.w[i] - 1, q.n0[i], q.n0[i] + q.h[i] - 1};
        g.r[g.nr] = march_rect<Body>(b, r, OCN_FRAME_STEP_ROWS, i >= 2);
        g.ntiles += g.r[g.nr].tiles;
        ++g.nr;
    }
    return issue_march(g, body, s);
}

// D's fallback points within r +- 1 (the points the one-pass step over r may take D from
// memory at) all hold +0.0 in the arrays it would read there: OR 1 into *flag otherwise
struct FallbackCheck {
    ocn_block b; const uint8_t *bits; const double *hu, *hu1, *hv, *hv1, *hh, *vort, *stt, *sts, *rx, *ry; int *flag;
    Range r;   // the points the step updates: RHSx / RHSy are read there
    const double *hr, *mu;   // uniform over r +- 2 (h_r) / r +- 1 (mu): equal to their values at (r.m0, r.n0)
    double *kc;              // <- h_r, mu at (r.m0, r.n0): the known-constant variant's constants
    unsigned own;            // MarchStep X2: halo points neighbours own are no fallback points
    OCN_HD void operator()(int m, int n) const
    {
        const Pt c = geo(&b)(m, n), c0 = geo(&b)(r.m0, r.n0);
        if (m == r.m0 && n == r.n0) { kc[0] = ld(hr, c0); kc[1] = ld(mu, c0); }
        if (fbits64(ld(hr, c)) != fbits64(ld(hr, c0))) OCN_ATOMIC_OR(flag, 1);   // bit 0: h_r varies
        if (m < r.m0 - 1 || m > r.m1 + 1 || n < r.n0 - 1 || n > r.n1 + 1) return;   // the ring of r +- 2
        if (fbits64(ld(mu, c)) != fbits64(ld(mu, c0))) OCN_ATOMIC_OR(flag, 2);
        const unsigned bc = ld(bits, c);
        const bool owned = (own >> (own_class(m, b.nx_start, b.nx_end) * 3u + own_class(n, b.ny_start, b.ny_end))) & 1u;
        const bool hh_rng = owned || (m >= b.nx_start - 1 && m <= b.nx_end && n >= b.ny_start - 1 && n <= b.ny_end);
        const bool in = owned || (m >= b.nx_start && m <= b.nx_end && n >= b.ny_start && n <= b.ny_end);
        auto nz = [&](const double *p) { return fbits64(ld(p, c)) != 0; };
        bool bad = false;
        if (!(hh_rng && (bc & (1u << OCN_LLU)))) bad |= nz(hu) || nz(hu1);
        if (!(hh_rng && (bc & (1u << OCN_LLV)))) bad |= nz(hv) || nz(hv1);
        if (!(hh_rng && (bc & (1u << OCN_LUH)))) bad |= nz(hh);
        if (!(in && (bc & (1u << OCN_LUU)))) bad |= nz(vort) || nz(sts);
        if (!(in && (bc & (1u << OCN_LU)))) bad |= nz(stt);
        if (m >= r.m0 && m <= r.m1 && n >= r.n0 && n <= r.n1) bad |= nz(rx) || nz(ry);
        if (bad) OCN_ATOMIC_OR(flag, 2);   // bit 1: a fallback value or the forcing is not +0.0, or mu varies
    }
};

int launch_fallback_check(const ocn_block *b, void *const *ptr, const uint8_t *bits, const Range &r, int32_t *flag,
                          double *kc, hipStream_t s, unsigned own)
{
    RC_K(check_block(b));
    auto f = [&](int id) { return (const double *)ptr[ocn_field_slot(id)]; };
    const FallbackCheck k{*b, bits, f(OCN_HHU), f(OCN_HHU_P), f(OCN_HHV), f(OCN_HHV_P), f(OCN_HHH), f(OCN_VORT),
                          f(OCN_STR_T), f(OCN_STR_S), f(OCN_RHSX), f(OCN_RHSY), (int *)flag, r, f(OCN_HHQ_REST),
                          f(OCN_MU), kc, own};
    const int m0 = max(r.m0 - 2, b->bnd_x1), m1 = min(r.m1 + 2, b->bnd_x2);
    const int n0 = max(r.n0 - 2, b->bnd_y1), n1 = min(r.n1 + 2, b->bnd_y2);
    if (m0 > m1 || n0 > n1) return OCN_OK;
    return launch_range(m0, m1, n0, n1, k, s);
}

int launch_onepass(const ocn_block *b, void *const *ptr, int nptr, const Compact *cp, const ocn_sw_params &sw,
                   double tau, int32_t *nbad, double *sshp_out, double *up_out, double *vp_out, hipStream_t s,
                   const Range *range, bool last, const OnepassKC &kc, unsigned own, const Range *frame_of)
{
    if (!cp || !cp->march || sw.full_free_surface != 1 || sw.trans_terms <= 0 || sw.ksw_lat <= 0 || !sshp_out ||
        !up_out || !vp_out)
        return set_error(OCN_ERR_ARG, "one-pass step: compact tables, march, full_free_surface = 1, trans_terms and "
                                      "ksw_lat on, three second buffers");
    if (kc.mode != OCN_KC_GENERAL && (!kc.kc || (kc.mode == OCN_KC_DEVICE && !kc.flag)))
        return set_error(OCN_ERR_ARG, "one-pass step: known constants without their device words");
    if (own && last) return set_error(OCN_ERR_ARG, "one-pass step over neighbour-owned halos: not a last step");
    RC_K(check_block(b));
    const Tab<true> t = make_tab<true>(ptr, nptr, cp->bits, cp->rows, block_rows(b), 0);
    const Range r = range ? range_clip(range_interior(b), *range) : range_interior(b);
    if (range_empty(r)) return OCN_OK;
    int ex;
    const bool p2 = std::frexp(tau, &ex) == 0.5 && ex > -1020 && ex < 1020;   // tau = 2^k
    // OCN_KC_DEVICE: the known-constant variant runs if the device check found its conditions, the
    // general one otherwise (each launch's workgroups read the verdict and return at once if it
    // is not theirs)
    const bool dev = kc.mode == OCN_KC_DEVICE;
    const int gz = dev ? 1 : 0, gh = dev ? 3 : 0, gg = dev ? 2 : 0;
#define OCN_STEP_LAUNCH(P, L, Z, X, H, G)                                                                        \
    do {                                                                                                          \
        const MarchStep<P, L, Z, X, H> k_{*b, t, sw, tau, nbad, sshp_out, up_out, vp_out, kc.kc, kc.flag, G, own}; \
        RC_K(frame_of ? launch_step_frame(b, r, *frame_of, k_, s) : launch_step(b, r, k_, s));                   \
    } while (0)
#define OCN_STEP_VARIANT(Z, H, G)                                                                                \
    do {                                                                                                         \
        if (own) { if (p2) OCN_STEP_LAUNCH(true, false, Z, true, H, G); else OCN_STEP_LAUNCH(false, false, Z, true, H, G); } \
        else if (last) { if (p2) OCN_STEP_LAUNCH(true, true, Z, false, H, G); else OCN_STEP_LAUNCH(false, true, Z, false, H, G); } \
        else if (p2) OCN_STEP_LAUNCH(true, false, Z, false, H, G);                                                 \
        else OCN_STEP_LAUNCH(false, false, Z, false, H, G);                                                        \
    } while (0)
    if (kc.mode == OCN_KC_KNOWN || dev) {
        OCN_STEP_VARIANT(true, false, gz);
        if (!dev) return OCN_OK;
    }
    if (kc.mode == OCN_KC_KNOWN_HR || dev) {
        OCN_STEP_VARIANT(true, true, gh);
        if (!dev) return OCN_OK;
    }
    OCN_STEP_VARIANT(false, false, gg);
#undef OCN_STEP_VARIANT
#undef OCN_STEP_LAUNCH
    return OCN_OK;
}

// ------------------------------------------------------------------ several steps per launch
// Small single blocks (the Black Sea basin's 285 x 159: a one-pass launch of a few microseconds) are
// launch-latency bound: the host's enqueue and the gap between dependent launches cost more than the
// march.  k_march_multi runs nsteps one-pass steps in ONE launch: every workgroup keeps its tile
// through the steps (its row constants formed once), and a grid-wide barrier separates the steps
// (each step reads at +-2 points what the previous one wrote).  Step s runs body b[s & 1]: the two
// bodies differ only in the buffers of the role pairs and the second buffers, swapped, as the host's
// role flips between single launches swap them.  The bodies store write-through (MarchStep WT: sc1
// buffer stores), so the barrier needs no L2 write-back: every wave drains its stores (vmcnt(0)),
// the workgroup meets (__syncthreads), one lane adds to a device-scope counter and awaits the
// step's total with a bounded relaxed spin -- a workgroup that waits ~0.5 s ORs 1 into *err and ends
// (every wave reaches an exit: no hang; the host reports OCN_ERR_HIP) -- and then invalidates its
// caches (agent-scope acquire) before the next step's loads (the fan-in below).  Every workgroup is resident at once:
// the grid is at most kMultiMaxTiles workgroups and is checked against the occupancy.
// Measured on the Black Sea (98 steps in one launch, 195 workgroups of 1-row wave tiles), per step:
// plain stores + a release fence (L2 write-back) per workgroup + one counter 17.2 us; write-through
// stores, no release 10.9; the grouped fan-in below 7.7 (the march alone 4.5, 3.9 with plain
// stores; the acquire 1.1).  Taller tiles (fewer workgroups) lose: 4 / 8 / 16 rows 10.4 / 15.6 /
// 26 us.  The same kernel launched by hipLaunchCooperativeKernel ran 4.5x slower -- a plain launch.
// The barrier's fan-in is split over 8 groups of workgroups (blockIdx % 8: for speed, the workgroups
// of one XCD as the dispatcher deals them; correctness does not depend on it): bar[32 (1 + g)] counts
// group g's arrivals, the group's last arriver adds to bar[0] and, once all groups are in, publishes
// the epoch in bar[32 (9 + g)], which the group's other workgroups await -- 8 words polled instead of
// one, and each atomic queue 1/8 as long.  (Words 128 B apart.)
__device__ __forceinline__ bool grid_barrier(unsigned *bar, unsigned epoch, int32_t *err, int spin)
{
    __shared__ int ok_s;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's write-through stores reached memory
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned n = gridDim.x, g = blockIdx.x & 7u, ng = (n - g + 7u) / 8u, groups = n < 8u ? n : 8u;
        const unsigned t = __hip_atomic_fetch_add(bar + 32 * (1 + g), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        int k = 0;
        if (t + 1 == ng * epoch) {   // the group's last arrival of this epoch
            __hip_atomic_fetch_add(bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            while (__hip_atomic_load(bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < groups * epoch && ++k < spin)
                __builtin_amdgcn_s_sleep(1);
            __hip_atomic_store(bar + 32 * (9 + g), epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            while (__hip_atomic_load(bar + 32 * (9 + g), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < epoch &&
                   ++k < spin)
                __builtin_amdgcn_s_sleep(1);
        }
        const bool ok = k < spin;
        if (!ok) atomicOr(err, 1);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");   // drop stale lines: the next step's loads
        ok_s = ok;
    }
    __syncthreads();
    return ok_s != 0;
}

template <class Body> struct BodyPair { Body b[2]; };
template <class Body>
__global__ __launch_bounds__(256, WavesOf<Body>::v) void k_march_multi(MarchGrid g, BodyPair<Body> bp, int nsteps,
                                                                       unsigned *ctr, int32_t *err, int spin)
{
    const MarchRect &R = g.r[0];
    const int tile = (int)blockIdx.x;   // one tile per workgroup (gridDim.x = R.tiles)
    if constexpr (HasPrologue<Body>::v) bp.b[0].prologue(R, tile / R.ntx);   // the same rows every step
    for (int s = 0; s < nsteps; ++s) {
        // ONE inlined march, the step's body picked at run time (two inlined copies: 93 KB of code)
        march_tile<Body, false>(R, tile, bp.b[__builtin_amdgcn_readfirstlane(s & 1)]);
        if (s + 1 < nsteps && !grid_barrier(ctr, (unsigned)(s + 1), err, spin)) return;
    }
}

// rows per wave tile of a multi-step launch: the shortest tile whose grid (4 vertically stacked
// waves per workgroup) stays within kMultiMaxTiles workgroups, or 0 if none up to 16 rows does
static constexpr int kMultiMaxTiles = 256;   // one workgroup per CU: resident with room to spare
static int multi_rows(const Range &r)
{
    const long wx = (r.m1 - r.m0 + 60) / 60, h = r.n1 - r.n0 + 1;
    for (int rows = 1; rows <= 16; ++rows)
        if (wx * ((h + 4 * rows - 1) / (4 * rows)) <= kMultiMaxTiles) return rows;
    return 0;
}

// The multi-step kernels' resident capacity on the current device, in workgroups: the fewest of any
// variant's occupancy x the device's CUs (a device with fewer CUs, a partition mode, another
// compile of the march), queried once per device; 0 if a query fails (no multi-step launch then)
template <bool P, bool Z, bool H> using MultiBody = MarchStep<P, false, Z, false, H, false, true>;
static long multi_capacity()
{
    static std::mutex mu;
    static std::map<int, long> cap;
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 0;
    std::lock_guard<std::mutex> g(mu);
    const auto it = cap.find(dev);
    if (it != cap.end()) return it->second;
    long c = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess ? LONG_MAX : 0;
    auto occ = [&](auto kern) {
        int per = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kern, 256, 0) != hipSuccess) per = 0;
        c = std::min(c, (long)per * cus);
    };
    occ(k_march_multi<MultiBody<true, false, false>>);
    occ(k_march_multi<MultiBody<false, false, false>>);
    occ(k_march_multi<MultiBody<true, true, true>>);
    occ(k_march_multi<MultiBody<false, true, true>>);
    occ(k_march_multi<MultiBody<true, true, false>>);
    occ(k_march_multi<MultiBody<false, true, false>>);
    return cap[dev] = c;
}

static long multi_tiles(const Range &r, int rows)
{
    return (long)((r.m1 - r.m0 + 60) / 60) * ((r.n1 - r.n0 + 4 * rows) / (4 * rows));
}

int onepass_multi_fits(const ocn_block *b)
{
    const Range r = range_interior(b);
    const int rows = multi_rows(r);
    return rows > 0 && multi_tiles(r, rows) <= multi_capacity();
}

int launch_onepass_multi(const ocn_block *b, void *const *ptr, int nptr, const Compact *cp, const ocn_sw_params &sw,
                         double tau, int nsteps, int32_t *nbad, double *sshp_alt, double *up_alt, double *vp_alt,
                         unsigned *ctr, int32_t *err, hipStream_t s, const OnepassKC &kc, int spin)
{
    if (!cp || !cp->march || sw.full_free_surface != 1 || sw.trans_terms <= 0 || sw.ksw_lat <= 0 || !sshp_alt ||
        !up_alt || !vp_alt || !ctr || !err || nsteps < 1)
        return set_error(OCN_ERR_ARG, "multi-step launch: compact tables, march, full_free_surface = 1, trans_terms "
                                      "and ksw_lat on, three second buffers, barrier words");
    if (kc.mode == OCN_KC_DEVICE || (kc.mode != OCN_KC_GENERAL && !kc.kc))
        return set_error(OCN_ERR_ARG, "multi-step launch: a variant chosen on the host");
    RC_K(check_block(b));
    const Range r = range_interior(b);
    if (range_empty(r)) return OCN_OK;
    const int rows = multi_rows(r);
    if (!rows) return set_error(OCN_ERR_ARG, "multi-step launch: block too large for one resident grid");
    // the odd steps' table: the role pairs and the second buffers swapped (ocn_ctx.hip swap_roles / swap_alt3)
    std::vector<void *> odd(ptr, ptr + nptr);
    for (const auto &pr : {std::make_pair(OCN_SSH, OCN_SSHN), std::make_pair(OCN_UBRTR, OCN_UBRTRN),
                           std::make_pair(OCN_VBRTR, OCN_VBRTRN)})
        std::swap(odd[ocn_field_slot(pr.first)], odd[ocn_field_slot(pr.second)]);
    double *alt[3] = {sshp_alt, up_alt, vp_alt};
    const int ids[3] = {OCN_SSHP, OCN_UBRTRP, OCN_VBRTRP};
    for (int i = 0; i < 3; ++i) std::swap(odd[ocn_field_slot(ids[i])], *(void **)&alt[i]);
    const Tab<true> t0 = make_tab<true>(ptr, nptr, cp->bits, cp->rows, block_rows(b), 0);
    const Tab<true> t1 = make_tab<true>(odd.data(), nptr, cp->bits, cp->rows, block_rows(b), 0);
    MarchGrid g{};
    g.r[0] = MarchRect{};
    int ex;
    const bool p2 = std::frexp(tau, &ex) == 0.5 && ex > -1020 && ex < 1020;   // tau = 2^k
    if (batching(s)) return batch_violation();   // (a multi-step launch is not batched)
    RC_K(check_hip(hipMemsetAsync(ctr, 0, kMultiBarBytes, s), "multi-step launch: barrier words"));
    auto go = [&](auto k0, auto k1) -> int {
        using Body = decltype(k0);
        g.r[0] = march_rect<Body>(b, r, rows, true);
        g.nr = 1;
        g.ntiles = g.r[0].tiles;
        // residency from the grid size alone (a plain launch: hipLaunchCooperativeKernel's check costs
        // 15-20 us per launch): the callers ask onepass_multi_fits first; this is the assert
        if (g.ntiles != multi_tiles(r, rows) || g.ntiles > multi_capacity())
            return set_error(OCN_ERR_ARG, "multi-step launch: grid larger than the resident capacity");
        count_launch();
        k_march_multi<Body><<<dim3((unsigned)g.ntiles), dim3(256), 0, s>>>(g, BodyPair<Body>{{k0, k1}}, nsteps, ctr, err,
                                                                             spin < 1 ? 1 : spin);
        return check_hip(hipGetLastError(), "multi-step launch");
    };
#define OCN_MULTI(P, Z, H)                                                                                       \
    return go(MarchStep<P, false, Z, false, H, false, true>{*b, t0, sw, tau, nbad, sshp_alt, up_alt, vp_alt, kc.kc,  \
                                                           nullptr, 0, 0u},                                       \
              MarchStep<P, false, Z, false, H, false, true>{*b, t1, sw, tau, nbad, alt[0], alt[1], alt[2], kc.kc,    \
                                                           nullptr, 0, 0u})
    if (kc.mode == OCN_KC_GENERAL) { if (p2) OCN_MULTI(true, false, false); OCN_MULTI(false, false, false); }
    if (kc.mode == OCN_KC_KNOWN_HR) { if (p2) OCN_MULTI(true, true, true); OCN_MULTI(false, true, true); }
    if (p2) OCN_MULTI(true, true, false);
    OCN_MULTI(false, true, false);
#undef OCN_MULTI
}

// Rows per workgroup tile of the two-step launch: the fewest iterations in total, counting
// ceil(waves / slots) rounds of rows + 8 iterations each (MarchStep::march); mult = blocks of this
// size in one launch (a batch: one_step_x4 on several blocks of a device)
// wave slots of the chip for the two-step launch: 256 CUs x 4 SIMDs x its waves per SIMD
constexpr long kPairSlots = 256L * 4L * OCN_PAIR_WAVES;
static int pair_rows(const Range &r, int cols, int mult = 1)
{
    const long wx = (r.m1 - r.m0 + cols) / cols, h = r.n1 - r.n0 + 1;
    // a tuning override (a fixed tile height), read once per process -- not a libc call per launch
    static const int fixed = [] {
        const char *e = getenv("OCN_PAIR_ROWS");
        const int v = e ? atoi(e) : 0;
        return v >= 8 && v <= OCN_PAIR_MAX_ROWS ? v : 0;
    }();
    if (fixed) return fixed;
    int best = 8;
    long cost = -1;
    for (int rows = 8; rows <= OCN_PAIR_MAX_ROWS; ++rows) {
        const long tiles = (h + rows - 1) / rows, waves = 4 * tiles * wx * mult,
                   rounds = (waves + kPairSlots - 1) / kPairSlots, c = rounds * (rows + 8);
        if (cost < 0 || c < cost) { cost = c; best = rows; }
    }
    return best;
}

int launch_onepass_pair(const ocn_block *b, void *const *ptr, int nptr, const Compact *cp, const ocn_sw_params &sw,
                        double tau, int32_t *nbad1, int32_t *nbad2, double *sshp_out, double *up_out, double *vp_out,
                        hipStream_t s, const OnepassKC &kc, bool last)
{
    if (!cp || !cp->march || sw.full_free_surface != 1 || sw.trans_terms <= 0 || sw.ksw_lat <= 0 || !sshp_out ||
        !up_out || !vp_out)
        return set_error(OCN_ERR_ARG, "two-step launch: compact tables, march, full_free_surface = 1, trans_terms and "
                                      "ksw_lat on, three second buffers");
    if (kc.mode == OCN_KC_DEVICE || (kc.mode != OCN_KC_GENERAL && !kc.kc))
        return set_error(OCN_ERR_ARG, "two-step launch: a variant chosen on the host");
    RC_K(check_block(b));
    const Tab<true> t = make_tab<true>(ptr, nptr, cp->bits, cp->rows, block_rows(b), 0);
    const Range r = range_interior(b);
    if (range_empty(r)) return OCN_OK;
    using KP = MarchStep<true, false, true, false, false, true>;
    const int cols = KP::kPairCols, rows = pair_rows(r, cols);
    MarchGrid g{};
    const int ntx = (r.m1 - r.m0 + cols) / cols;
    g.r[0] = MarchRect{r.m0, r.m1, r.n0, r.n1, r.m0, ntx, ntx * ((r.n1 - r.n0 + rows) / rows), max(r.m0 - 4, b->bnd_x1),
                       min(r.m1 + 4, b->bnd_x2), rows, 0};
    g.nr = 1;
    g.ntiles = g.r[0].tiles;
    int ex;
    const bool p2 = std::frexp(tau, &ex) == 0.5 && ex > -1020 && ex < 1020;   // tau = 2^k
#define OCN_PAIR_LAUNCH(P, L, Z, H)                                                                              \
    return issue_march(g, MarchStep<P, L, Z, false, H, true>{*b, t, sw, tau, nbad1, sshp_out, up_out, vp_out,        \
                                                             kc.kc, nullptr, 0, 0u, nbad2}, s)
#define OCN_PAIR_VARIANT(L)                                                                                      \
    if (kc.mode == OCN_KC_GENERAL) { if (p2) OCN_PAIR_LAUNCH(true, L, false, false); OCN_PAIR_LAUNCH(false, L, false, false); } \
    if (kc.mode == OCN_KC_KNOWN_HR) { if (p2) OCN_PAIR_LAUNCH(true, L, true, true); OCN_PAIR_LAUNCH(false, L, true, true); }    \
    if (p2) OCN_PAIR_LAUNCH(true, L, true, false);                                                                \
    OCN_PAIR_LAUNCH(false, L, true, false)
    if (last) { OCN_PAIR_VARIANT(true); }
    OCN_PAIR_VARIANT(false);
#undef OCN_PAIR_VARIANT
#undef OCN_PAIR_LAUNCH
}

// Two one-pass steps per launch on a block with halo exchanges (ocn_ctx.hip one_step_x4): bx = the
// block widened by kXRing rings, ptr / cp->bits / cp->rows its tables over that geometry (bases at
// A(bnd_x1 - kXRing, bnd_y1 - kXRing)), the state exchanged 4 points deep; the known-constant variant.
// range (default: the interior): the points the consumers write.
int launch_onepass_pair_x4(const ocn_block *bx, void *const *ptr, int nptr, const Compact *cp, const ocn_sw_params &sw,
                           double tau, int32_t *nbad1, int32_t *nbad2, double *sshp_out, double *up_out, double *vp_out,
                           hipStream_t s, const OnepassKC &kc, unsigned own, const Range *range, int nblk,
                           const Range *frame_of, double *const *trs)
{
    if (!cp || !cp->march || sw.full_free_surface != 1 || sw.trans_terms <= 0 || sw.ksw_lat <= 0 || !sshp_out ||
        !up_out || !vp_out)
        return set_error(OCN_ERR_ARG, "x4 two-step launch: compact tables, march, full_free_surface = 1, trans_terms "
                                      "and ksw_lat on, three second buffers");
    if ((kc.mode != OCN_KC_KNOWN && kc.mode != OCN_KC_KNOWN_HR) || !kc.kc)
        return set_error(OCN_ERR_ARG, "x4 two-step launch: a known-constant variant chosen on the host");
    RC_K(check_block(bx));
    if (bx->bnd_x1 > bx->nx_start - 4 || bx->bnd_x2 < bx->nx_end + 4 || bx->bnd_y1 > bx->ny_start - 4 ||
        bx->bnd_y2 < bx->ny_end + 4)
        return set_error(OCN_ERR_ARG, "x4 two-step launch: the geometry must reach 4 points past the interior");
    const Tab<true> t = make_tab<true>(ptr, nptr, cp->bits, cp->rows, block_rows(bx), 0);
    const Range all = range ? *range : range_interior(bx);
    if (range_empty(all)) return OCN_OK;
    using KP = MarchStep<true, false, true, true, false, true>;
    // a batch puts up to P blocks' tiles in one launch (MarchBatch): their waves share its rounds
    constexpr int P = kPack<KP> < kBatchMax / 4 ? kPack<KP> : kBatchMax / 4;
    const int cols = KP::kPairCols, mult = batching(s) ? std::max(1, std::min(nblk, P)) : 1;
    // the rects: the range, or (frame_of) its bands outside *frame_of -- one launch, up to 4 rects
    Range rs[4];
    int nr = 0;
    if (!frame_of) {
        rs[nr++] = all;
    } else {
        const Range &in = *frame_of;
        const Range cand[4] = {{all.m0, all.m1, all.n0, in.n0 - 1}, {all.m0, all.m1, in.n1 + 1, all.n1},
                               {all.m0, in.m0 - 1, in.n0, in.n1}, {in.m1 + 1, all.m1, in.n0, in.n1}};
        for (const Range &q : cand)
            if (!range_empty(q)) rs[nr++] = q;
    }
    MarchGrid g{};
    for (int i = 0; i < nr; ++i) {
        const Range &r = rs[i];
        const int rows = pair_rows(r, cols, mult), ntx = (r.m1 - r.m0 + cols) / cols;
        g.r[g.nr++] = MarchRect{r.m0, r.m1, r.n0, r.n1, r.m0, ntx, ntx * ((r.n1 - r.n0 + rows) / rows),
                                max(r.m0 - 4, bx->bnd_x1), min(r.m1 + 4, bx->bnd_x2), rows, 0};
        g.ntiles += g.r[g.nr - 1].tiles;
    }
    int ex;
    auto go = [&](auto body) {
        if (trs)
            for (int i = 0; i < 4; ++i) body.trs[i] = trs[i];
        return issue_march(g, body, s);
    };
    const bool p2 = std::frexp(tau, &ex) == 0.5 && ex > -1020 && ex < 1020;   // tau = 2^k
    if (kc.mode == OCN_KC_KNOWN_HR) {   // h_r read (a topography: the rest depth varies), its 4 rings exchanged
        if (p2)
            return go(MarchStep<true, false, true, true, true, true>{*bx, t, sw, tau, nbad1, sshp_out, up_out, vp_out,
                                                                     kc.kc, nullptr, 0, own, nbad2});
        return go(MarchStep<false, false, true, true, true, true>{*bx, t, sw, tau, nbad1, sshp_out, up_out, vp_out, kc.kc,
                                                                  nullptr, 0, own, nbad2});
    }
    if (p2)
        return go(MarchStep<true, false, true, true, false, true>{*bx, t, sw, tau, nbad1, sshp_out, up_out, vp_out, kc.kc,
                                                                  nullptr, 0, own, nbad2});
    return go(MarchStep<false, false, true, true, false, true>{*bx, t, sw, tau, nbad1, sshp_out, up_out, vp_out, kc.kc,
                                                               nullptr, 0, own, nbad2});
}

// mask bytes of one_step_x4 over the widened geometry bx: at the halo points neighbour blocks own
// (own_class bits), up to kXRing rings past the reference's arrays, lu_init + lu_lv_init of the basin
// mask as the neighbour's init forms them on its interior (init_kernels.hip k_init_grid); elsewhere
// inside the arrays the block's own bytes (Prepare); +0 outside.
__global__ void k_bits_x4(ocn_block bx, ocn_block g, const uint8_t *bits, uint8_t *out, const int32_t *mask, int nx, int ny,
                          unsigned own)
{
    const int w = bx.bnd_x2 - bx.bnd_x1 + 1, h = bx.bnd_y2 - bx.bnd_y1 + 1;
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (long)w * h) return;
    const int m = bx.bnd_x1 + (int)(i % w), n = bx.bnd_y1 + (int)(i / w);
    const unsigned cls = own_class(m, g.nx_start, g.nx_end) * 3u + own_class(n, g.ny_start, g.ny_end);
    unsigned v = 0;
    if (cls != 4u && ((own >> cls) & 1u) && m >= 1 && m < nx && n >= 1 && n < ny) {
        auto lu = [&](int mm, int nn) -> unsigned { return mask[(long)(mm - 1) + (long)(nn - 1) * nx] == 0 ? 1u : 0u; };
        const unsigned a = lu(m, n), b = lu(m + 1, n), c = lu(m, n + 1), d = lu(m + 1, n + 1);
        v = (a << OCN_LU) | ((a & b & c & d) << OCN_LUU) | ((a | b | c | d) << OCN_LUH) | ((a & b) << OCN_LCU) |
            ((a & c) << OCN_LCV) | ((a | b) << OCN_LLU) | ((a | c) << OCN_LLV);
    } else if (m >= g.bnd_x1 && m <= g.bnd_x2 && n >= g.bnd_y1 && n <= g.bnd_y2) {
        v = bits[(long)(m - g.bnd_x1) + (long)(n - g.bnd_y1) * g.pitch];
    }
    out[(long)(m - bx.bnd_x1) + (long)(n - bx.bnd_y1) * bx.pitch] = (uint8_t)v;
}

// one_step_x4's row table over the widened rows: the block's rows bnd_y1 + 1 .. bnd_y2 - 1 (the metric
// range) from its compact table, the ext rows (the neighbours' rows bnd_y1 - 2 .. bnd_y1 and bnd_y2 ..
// bnd_y2 + 2, GridInit ext) around them; ORs OCN_COMPACT_DIVISOR_RANGE into *flags if a divisor is out
// of udiv's range
__global__ void k_rows_x4(float *rows4, unsigned nrows4, const float *rows, unsigned nrows, const float *ext, int *flags)
{
    const unsigned r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= nrows4) return;
    float v[kNumRowFields];
    // ext rows: 0 bnd_y1, 1 bnd_y2, 2 bnd_y1 - 1, 3 bnd_y1 - 2, 4 bnd_y2 + 1, 5 bnd_y2 + 2
    const int e = r == 0 ? 3 : r == 1 ? 2 : r == 2 ? 0 : r == nrows4 - 3 ? 1 : r == nrows4 - 2 ? 4 : r == nrows4 - 1 ? 5 : -1;
    for (int k = 0; k < kNumRowFields; ++k)
        v[k] = e >= 0 ? ext[e * kNumRowFields + k] : rows[(unsigned)k * nrows + (r - kXRing)];
    if (!write_table_row(rows4, nrows4, r, v)) atomicOr(flags, (int)OCN_COMPACT_DIVISOR_RANGE);
}

int launch_x4_tables(const ocn_block *g, const uint8_t *bits, const float *rows, const float *ext, uint8_t *bits4,
                     float *rows4, const int32_t *mask, int nx, int ny, unsigned own, int32_t *flags, hipStream_t s)
{
    RC_K(check_block(g));
    ocn_block bx = *g;
    bx.bnd_x1 -= kXRing; bx.bnd_x2 += kXRing; bx.bnd_y1 -= kXRing; bx.bnd_y2 += kXRing;
    const long pts = (long)(bx.bnd_x2 - bx.bnd_x1 + 1) * (bx.bnd_y2 - bx.bnd_y1 + 1);
    hipLaunchKernelGGL(k_bits_x4, dim3((unsigned)((pts + 255) / 256)), dim3(256), 0, s, bx, *g, bits, bits4, mask, nx, ny,
                       own);
    RC_K(check_launch());
    const unsigned nrows = block_rows(g), nrows4 = block_rows(&bx);
    hipLaunchKernelGGL(k_rows_x4, dim3((nrows4 + 63) / 64), dim3(64), 0, s, rows4, nrows4, rows, nrows, ext, (int *)flags);
    return check_launch();
}

// tracer stage `stage` (OCN_TSTAGE_*) of tracer k on one block; factor_mu = 1.0d0 as the PSy
// layer passes it (tracer_interface.f90:47)
int launch_tracer(const ocn_block *b, void *const *ptr, int nptr, const Compact *cp, int stage, int k, double tau,
                  double ts, hipStream_t s)
{
    const Range ri = range_interior(b), rr = range_ring(b);
    switch (stage) {
    case OCN_TSTAGE_TRAN_DIFF_FLUXES:
        return launch_fused<KTranDiffFluxes>(ri, ri, OCN_PART_ALL, b, ptr, nptr, cp, k, s, 1.0);
    case OCN_TSTAGE_TRAN_DIFF_TRACER:
        return launch_fused<KTranDiffTracer>(ri, ri, OCN_PART_ALL, b, ptr, nptr, cp, k, s, tau);
    case OCN_TSTAGE_TRACER_NEXT_STEP:
        return launch_fused<KTracerNextStep>(rr, rr, OCN_PART_ALL, b, ptr, nptr, cp, k, s, ts);
    default: return set_error(OCN_ERR_ARG, "bad tracer stage id");
    }
}

// expl_tracer of tracer k as one launch in a one-pass sequence (sw_stencils.h TracerStep): the full
// free surface factor is 1 (the one-pass steps require it), factor_mu 1.0d0 (tracer_interface.f90:47)
// The tracer step one point per thread in 64 x 4 tiles, each face flux formed once: a thread forms
// the fluxes of its point's east and north faces (TracerStep::fx_at / fy_at at (m, n)) and takes the
// west / south ones from the neighbour threads through LDS (the tile's west column and south row
// form theirs themselves) -- the same expressions on the same operands, so the same values as four
// per point.  The tracer steps of small blocks (the Black Sea as 4 x 2 blocks, 71 x 79 each) are
// latency-bound launches of few waves: a quarter of the serial work per thread, twice the threads.
constexpr int kTrRows = 4;
template <class Body>
__device__ __forceinline__ void tracer_tile(const RangeB &R, int tile, const Body &body, int tx, int ty)
{
    __shared__ double sfx[kTrRows][64], sfy[kTrRows][64];
    const int m = R.w0 + (tile % R.ntx) * 64 + tx, n = R.n0 + (tile / R.ntx) * kTrRows + ty;
    const bool in = m >= R.m0 && m <= R.m1 && n >= R.n0 && n <= R.n1;
    const auto k = body.make();
    double fxe = 0.0, fyn = 0.0;
    if (in) { fxe = k.fx_at(m, n); fyn = k.fy_at(m, n); }
    sfx[ty][tx] = fxe;
    sfy[ty][tx] = fyn;
    __syncthreads();
    // (an extended range: the halo points neighbours own only -- TracerStep::in_fluxes)
    if (!in || !k.in_fluxes(m, n) || !(ld(k.W.lu, k.I(m, n)) > 0.5f)) return;
    const double fxw = tx > 0 ? sfx[ty][tx - 1] : k.fx_at(m - 1, n);
    const double fys = ty > 0 ? sfy[ty - 1][tx] : k.fy_at(m, n - 1);
    k.finish(m, n, fxe, fxw, fyn, fys);
}
template <class Body> __global__ __launch_bounds__(256) void k_tracer_tiles(RangeB R, Body body)
{
    int tile = (int)blockIdx.x;
#if OCN_XCD_REMAP
    const int per = (R.tiles + 7) / 8;
    tile = (tile % 8) * per + tile / 8;
    if (tile >= R.tiles) return;
#endif
    tracer_tile(R, tile, body, (int)threadIdx.x, (int)threadIdx.y);
}
template <class Body> __global__ __launch_bounds__(256) void k_tracer_tiles_b(RangeGridB g, Pack<Body> bodies)
{
    int tile = (int)blockIdx.x;
#if OCN_XCD_REMAP
    const int per = (g.ntiles + 7) / 8;
    tile = (tile % 8) * per + tile / 8;
    if (tile >= g.ntiles) return;
#endif
    int k = 0;   // workgroup-uniform
    while (k + 1 < g.nr && tile >= g.r[k].tiles) { tile -= g.r[k].tiles; ++k; }
    tracer_tile(g.r[k], tile, bodies.b[__builtin_amdgcn_readfirstlane(g.r[k].blk)], (int)threadIdx.x, (int)threadIdx.y);
}
template <typename Body> struct TracerBatch : BatchEntry {
    std::vector<Body> bodies;
    std::vector<RangeB> ranges;
    int flush(hipStream_t s) override
    {
        for (size_t i = 0; i < bodies.size(); i += kPack<Body>) {
            const size_t n = std::min(bodies.size() - i, (size_t)kPack<Body>);
            RangeGridB g{};
            const PackBuf<Body> pk(&bodies[i], n);
            for (size_t j = 0; j < n; ++j) {
                g.r[g.nr] = ranges[i + j];
                g.r[g.nr].blk = (int)j;
                g.ntiles += ranges[i + j].tiles;
                ++g.nr;
            }
            const int nblocks = OCN_XCD_REMAP ? 8 * ((g.ntiles + 7) / 8) : g.ntiles;
            hipLaunchKernelGGL(k_tracer_tiles_b<Body>, dim3((unsigned)nblocks), dim3(64, kTrRows), 0, s, g, pk.get());
            RC_KB(check_launch());
        }
        return OCN_OK;
    }
};
// BatchEntry::co_flush of a one-pass x2 march batch (MarchStep::kCoTracer) followed by the tracer-step
// batch of the previous state (ocn_ctx.hip one_step_x2): ONE launch, workgroups [0, march tiles) march
// the blocks, the rest are tracer tiles (a 256-thread workgroup as the 64 x kTrRows tile) -- in place
// of the march launch and a tracer launch forked beside it on a second stream (two launches, an event
// fork and join per step: the Black Sea + tracer as 4 x 2 blocks is latency-bound).  The two read the
// same exchanged state and write disjoint buffers (Batcher::co_launch).
template <class MB, class TB>
__global__ __launch_bounds__(256, WavesOf<MB>::v) void k_march_tracer_b(MarchGridB gm, Pack<MB> mb, RangeGridB gt,
                                                                         Pack<TB> tb)
{
    int tile = (int)blockIdx.x;
#if OCN_XCD_REMAP
    const int total = gm.ntiles + gt.ntiles;
    const int per = (total + 7) / 8;
    tile = (tile % 8) * per + tile / 8;
    if (tile >= total) return;
#endif
    if (tile < gm.ntiles) {   // (workgroup-uniform)
        int k = 0;
        while (k + 1 < gm.nr && tile >= gm.r[k].tiles) { tile -= gm.r[k].tiles; ++k; }
        const MB &body = mb.b[__builtin_amdgcn_readfirstlane(gm.blk[k])];
        if constexpr (HasGate<MB>::v)
            if (!body.enabled()) return;
        march_tile(gm.r[k], tile, body);
        return;
    }
    tile -= gm.ntiles;
    int k = 0;
    while (k + 1 < gt.nr && tile >= gt.r[k].tiles) { tile -= gt.r[k].tiles; ++k; }
    tracer_tile(gt.r[k], tile, tb.b[__builtin_amdgcn_readfirstlane(gt.r[k].blk)], (int)threadIdx.x & 63,
                (int)threadIdx.x >> 6);
}
// the argument block of a co-launch (two grids, two packs): within the 16 KB plain launches take on
// gfx950 (scripts/kernarg_probe.hip), with a margin
constexpr size_t kCoArgMax = 15360;
template <class MB> static bool march_tracer_flush(MarchBatch<MB> &m, BatchEntry *next, hipStream_t s, int &rc)
{
    using TB = KTracerStep<true>;
    constexpr int P = kPack<MB> < kBatchMax / 4 ? kPack<MB> : kBatchMax / 4;
    constexpr size_t kArgs = sizeof(MarchGridB) + sizeof(Pack<MB>) + sizeof(RangeGridB) + sizeof(Pack<TB>);
    if (kArgs > kCoArgMax || next->kind != (const void *)&k_tracer_tiles<TB>) return false;
    auto *t = static_cast<TracerBatch<TB> *>(next);
    if (m.bodies.empty() || m.bodies.size() > (size_t)P || m.rects.size() > (size_t)kBatchMax ||
        t->bodies.size() > (size_t)kPack<TB> || t->ranges.size() > (size_t)kBatchMax)
        return false;
    MarchGridB gm{};
    const PackBuf<MB> pm(m.bodies.data(), m.bodies.size());
    for (size_t j = 0; j < m.rects.size(); ++j) {
        gm.r[gm.nr] = m.rects[j]; gm.blk[gm.nr] = m.blk[j]; gm.ntiles += m.rects[j].tiles; ++gm.nr;
    }
    RangeGridB gt{};
    const PackBuf<TB> pt(t->bodies.data(), t->bodies.size());
    for (size_t j = 0; j < t->ranges.size(); ++j) {
        gt.r[gt.nr] = t->ranges[j];
        gt.r[gt.nr].blk = (int)j;
        gt.ntiles += t->ranges[j].tiles;
        ++gt.nr;
    }
    const int total = gm.ntiles + gt.ntiles;
    const int nblocks = OCN_XCD_REMAP ? 8 * ((total + 7) / 8) : total;
    hipLaunchKernelGGL((k_march_tracer_b<MB, TB>), dim3((unsigned)nblocks), dim3(256), 0, s, gm, pm.get(), gt, pt.get());
    rc = check_launch();
    return true;
}

template <class Body> static int launch_tracer_tiles(const Range &r, const Body &body, hipStream_t s)
{
    if (range_empty(r)) return OCN_OK;
    const int ntx = (r.m1 - r.m0 + 64) / 64, nty = (r.n1 - r.n0 + kTrRows) / kTrRows;
    const RangeB R{r.m0, r.m0, r.m1, r.n0, r.n1, ntx, ntx * nty, 0};
    if (batching(s)) {
        int rc = OCN_OK;
        auto *e = batch_entry<TracerBatch<Body>>((const void *)&k_tracer_tiles<Body>, rc);
        RangeB q = R;
        q.blk = (int)e->bodies.size();
        e->ranges.push_back(q);
        e->bodies.push_back(body);
        return rc;
    }
    const int nblocks = OCN_XCD_REMAP ? 8 * ((R.tiles + 7) / 8) : R.tiles;
    hipLaunchKernelGGL(k_tracer_tiles<Body>, dim3((unsigned)nblocks), dim3(64, kTrRows), 0, s, R, body);
    return check_launch();
}

int launch_tracer_step(const ocn_block *b, void *const *ptr, int nptr, const Compact *cp, int k, double tau,
                       double ts, double *ffn_out, double *ffp_out, unsigned own, hipStream_t s, bool ext)
{
    if (!ffn_out || !ffp_out) return set_error(OCN_ERR_ARG, "tracer step: output buffers");
    RC_K(check_block(b));
    Range ri = range_interior(b);
    if (ext) {   // + the first halo ring where neighbours own it (the tiles skip the rest)
        if (b->bnd_x1 > b->nx_start - 2 || b->bnd_x2 < b->nx_end + 2 || b->bnd_y1 > b->ny_start - 2 ||
            b->bnd_y2 < b->ny_end + 2)
            return set_error(OCN_ERR_ARG, "tracer step over the first halo ring: a 2-wide halo");
        ri = Range{ri.m0 - 1, ri.m1 + 1, ri.n0 - 1, ri.n1 + 1};
    }
    if (cp)
        return launch_tracer_tiles(ri, KTracerStep<true>{*b, make_tab<true>(ptr, nptr, cp->bits, cp->rows, block_rows(b), k),
                                                         tau, ts, own, ffn_out, ffp_out}, s);
    return launch_tracer_tiles(ri, KTracerStep<false>{*b, make_tab<false>(ptr, nptr, nullptr, nullptr, 0, k), tau, ts,
                                                      own, ffn_out, ffp_out}, s);
}

// One reference stage over the compact tables (ocn_ctx.hip envoke, OCN_OPT_COMPACT): the stage
// functor is built on the device from the block's field table, as the fused launches build theirs,
// and reads the mask byte and the per-row metrics instead of the real(4) arrays -- the same
// operands (launch_prepare checked every point of a row carries the row's metric bits), so the
// same results as the ocn_<stage> entries on the 2-D arrays.
template <int S> struct KStage {
    ocn_block b; Tab<true> t; ocn_sw_params sw; double tau; int32_t *nbad;
    OCN_HD void operator()(int m, int n) const
    {
        if constexpr (S == OCN_STAGE_SW_UPDATE_SSH) make_sw_update_ssh(&b, t, tau)(m, n);
        else if constexpr (S == OCN_STAGE_HH_UPDATE) make_hh_update(&b, t)(m, n);
        else if constexpr (S == OCN_STAGE_UV_TRANS_VORT) make_uv_trans_vort(&b, t)(m, n);
        else if constexpr (S == OCN_STAGE_UV_TRANS) make_uv_trans(&b, t)(m, n);
        else if constexpr (S == OCN_STAGE_STRESS_COMPONENTS) make_stress_components(&b, t)(m, n);
        else if constexpr (S == OCN_STAGE_UV_DIFF2) make_uv_diff2(&b, t)(m, n);
        else if constexpr (S == OCN_STAGE_SW_UPDATE_UV) make_sw_update_uv(&b, t, tau)(m, n);
        else if constexpr (S == OCN_STAGE_SW_NEXT_STEP) make_sw_next_step(&b, t, sw.time_smooth)(m, n);
        else if constexpr (S == OCN_STAGE_HH_SHIFT) make_hh_shift(&b, t, sw.time_smooth)(m, n);
        else if constexpr (S == OCN_STAGE_HH_INIT) make_hh_init(&b, t, (int)sw.full_free_surface, true)(m, n);
        else make_check_ssh_err(&b, t, nbad)(m, n);
    }
};
template <int S>
static int launch_stage_k(const ocn_block *b, const Tab<true> &t, const Range &r, const ocn_sw_params &sw, double tau,
                          int32_t *nbad, hipStream_t s)
{
    return launch_range(r.m0, r.m1, r.n0, r.n1, KStage<S>{*b, t, sw, tau, nbad}, s, b->nx_start);
}

int launch_stage(const ocn_block *b, void *const *ptr, int nptr, const Compact *cp, int stage, const ocn_sw_params &sw,
                 double tau, int32_t *nbad, hipStream_t s)
{
    RC_K(check_block(b));
    if (!cp) return set_error(OCN_ERR_ARG, "launch_stage: the compact tables");
    const Tab<true> t = make_tab<true>(ptr, nptr, cp->bits, cp->rows, block_rows(b), 0);
    const Range ri = range_interior(b), rr = range_ring(b), rb = range_bnd(b);
    switch (stage) {
    case OCN_STAGE_SW_UPDATE_SSH: return launch_stage_k<OCN_STAGE_SW_UPDATE_SSH>(b, t, ri, sw, tau, nbad, s);
    case OCN_STAGE_HH_UPDATE: return launch_stage_k<OCN_STAGE_HH_UPDATE>(b, t, rb, sw, tau, nbad, s);
    case OCN_STAGE_UV_TRANS_VORT: return launch_stage_k<OCN_STAGE_UV_TRANS_VORT>(b, t, ri, sw, tau, nbad, s);
    case OCN_STAGE_UV_TRANS:
        if (use_march(cp)) return launch_march(b, ri, MarchUvTrans{*b, t}, s);
        return launch_stage_k<OCN_STAGE_UV_TRANS>(b, t, ri, sw, tau, nbad, s);
    case OCN_STAGE_STRESS_COMPONENTS: return launch_stage_k<OCN_STAGE_STRESS_COMPONENTS>(b, t, ri, sw, tau, nbad, s);
    case OCN_STAGE_UV_DIFF2: return launch_stage_k<OCN_STAGE_UV_DIFF2>(b, t, ri, sw, tau, nbad, s);
    case OCN_STAGE_SW_UPDATE_UV: return launch_stage_k<OCN_STAGE_SW_UPDATE_UV>(b, t, ri, sw, tau, nbad, s);
    case OCN_STAGE_SW_NEXT_STEP: return launch_stage_k<OCN_STAGE_SW_NEXT_STEP>(b, t, rr, sw, tau, nbad, s);
    case OCN_STAGE_HH_SHIFT: return launch_stage_k<OCN_STAGE_HH_SHIFT>(b, t, rr, sw, tau, nbad, s);
    case OCN_STAGE_HH_INIT:   // every level (full): the register march where the tables allow it
        if (use_march(cp)) return launch_march(b, rb, MarchHhInit{*b, t, (int)sw.full_free_surface, true}, s);
        return launch_stage_k<OCN_STAGE_HH_INIT>(b, t, rb, sw, tau, nbad, s);
    case OCN_STAGE_CHECK_SSH_ERR: return launch_stage_k<OCN_STAGE_CHECK_SSH_ERR>(b, t, ri, sw, tau, nbad, s);
    default: return set_error(OCN_ERR_ARG, "unknown stage id");
    }
}

int launch_coherence(const ocn_block *b, void *const *ptr, const uint8_t *bits, int32_t *flags, hipStream_t s)
{
    RC_K(check_block(b));
    const Range r = range_bnd(b);
    return launch_range(r.m0, r.m1, r.n0, r.n1, make_coherence(b, ptr, bits, (int *)flags), s);
}

// the tracer steps' pairs: ff1 and ff1n of tracer k agree outside the ring range's lu points (what the
// reference's tran_diff_tracer / its exchange and tracer_next_step write: the interior and the halo ring)
int launch_tracer_coherence(const ocn_block *b, void *const *ptr, const uint8_t *bits, int k, int32_t *flags,
                            hipStream_t s)
{
    RC_K(check_block(b));
    const double *ff = (const double *)ptr[ocn_field_slot(OCN_FF1(k))];
    const double *ffn = (const double *)ptr[ocn_field_slot(OCN_FF1N(k))];
    const Coherence q{geo(b), b->nx_start - 1, b->nx_end + 1, b->ny_start - 1, b->ny_end + 1, bits,
                      {ff, ff, ff}, {ffn, ff, ff}, (int *)flags};   // (pairs 2, 3: trivially equal)
    const Range r = range_bnd(b);
    return launch_range(r.m0, r.m1, r.n0, r.n1, q, s);
}

size_t row_table_size(unsigned nrows) { return row_table_floats(nrows); }

Batcher::~Batcher()
{
    for (BatchEntry *e : entries) delete e;
}

int Batcher::flush()
{
    const bool was = active;
    active = false;   // the flush's own launches are issued, not collected
    int rc = OCN_OK;
    co_launched = 0;
    for (size_t i = 0; i < entries.size(); ++i) {
        if (rc == OCN_OK) {
            if (co_launch && i + 1 < entries.size() && entries[i]->co_flush(entries[i + 1], s, rc)) {
                ++co_launched;
                delete entries[i];
                ++i;   // (issued with entry i)
            } else {
                rc = entries[i]->flush(s);
            }
        }
        delete entries[i];
    }
    entries.clear();
    cur = -1;
    active = was;
    return rc;
}

void batch_begin(Batcher *bt, hipStream_t s)
{
    if (!bt) return;
    for (BatchEntry *e : bt->entries) delete e;
    bt->entries.clear();
    bt->s = s;
    bt->cur = -1;
    bt->co_launch = false;
    bt->active = true;
    g_batcher = bt;
}

int batch_end(Batcher *bt)
{
    if (!bt) return OCN_OK;
    const int rc = bt->flush();
    bt->active = false;
    g_batcher = nullptr;
    return rc;
}

int batch_violation()
{
    return set_error(OCN_ERR_STATE, "a kernel launch bypassed the open block batch (sw_kernels.hip Batcher)");
}

int launch_prepare(const ocn_block *b, void *const *ptr, uint8_t *bits, float *rows, int32_t *flags, hipStream_t s,
                   unsigned own)
{
    RC_K(check_block(b));
    const Range r = range_bnd(b);
    return launch_range(r.m0, r.m1, r.n0, r.n1, make_prepare(b, ptr, bits, rows, (int *)flags, own), s);
}

__global__ void k_rows_ext(float *rows_x, unsigned nrows, const float *ext, int *flags)
{
    const int i = (int)threadIdx.x;
    if (i >= 2) return;
    if (!write_table_row(rows_x, nrows, i == 0 ? 0u : nrows - 1u, ext + i * kNumRowFields))
        atomicOr(flags, (int)OCN_COMPACT_DIVISOR_RANGE);
}

int launch_rows_ext(const ocn_block *b, const float *rows, float *rows_x, const float *ext, int32_t *flags,
                    hipStream_t s)
{
    RC_K(check_block(b));
    const unsigned nrows = block_rows(b);
    if (hipMemcpyAsync(rows_x, rows, row_table_floats(nrows) * sizeof(float), hipMemcpyDeviceToDevice, s) != hipSuccess)
        return set_error(OCN_ERR_HIP, "rows_ext: copy");
    hipLaunchKernelGGL(k_rows_ext, dim3(1), dim3(64), 0, s, rows_x, nrows, ext, (int *)flags);
    return check_launch();
}

}  // namespace ocn

using namespace ocn;

// ocn_hh_init, ocn_uv_trans, ocn_uv_diff2, ocn_stress_components run as register marches over the
// arrays they are given (MarchHhInit2D, MarchUvTrans2D, MarchUvDiff2D, MarchStress2D); the other
// entries one thread per point

extern "C" {

int ocn_sw_update_ssh(const ocn_block *b, double tau, const float *lu, const float *dx, const float *dy,
                      const float *dxh, const float *dyh, const double *hhu, const double *hhv, double *sshn,
                      const double *sshp, const double *ubrtr, const double *vbrtr, void *stream)
{
    CHECK(lu, dx, dy, dxh, dyh, hhu, hhv, sshn, sshp, ubrtr, vbrtr);
    SwUpdateSsh<false> k{geo(b), tau, lu, dx, dy, dxh, dyh, hhu, hhv, sshn, sshp, ubrtr, vbrtr};
    return launch_range(b->nx_start, b->nx_end, b->ny_start, b->ny_end, k, (hipStream_t)stream, b->nx_start);
}

int ocn_hh_update(const ocn_block *b, const float *lu, const float *llu, const float *llv, const float *luh,
                  const float *dx, const float *dy, const float *dxt, const float *dyt, const float *dxh,
                  const float *dyh, const float *dxb, const float *dyb, double *hqn, double *hun, double *hvn,
                  double *hhn, const double *sh, const double *h_r, void *stream)
{
    CHECK(lu, llu, llv, luh, dx, dy, dxt, dyt, dxh, dyh, dxb, dyb, hqn, hun, hvn, hhn, sh, h_r);
    HhUpdate<false> k{geo(b), b->nx_start - 1, b->nx_end, b->ny_start - 1, b->ny_end,
               Interp<false>{lu, dx, dy, dxt, dyt, dxh, dyh, dxb, dyb}, llu, llv, luh, hqn, hun, hvn, hhn, sh, h_r};
    return launch_range(b->bnd_x1, b->bnd_x2, b->bnd_y1, b->bnd_y2, k, (hipStream_t)stream, b->nx_start);
}

int ocn_uv_trans_vort(const ocn_block *b, const float *luu, const float *dxt, const float *dyt, const float *dxb,
                      const float *dyb, const double *u, const double *v, double *vort, void *stream)
{
    CHECK(luu, dxt, dyt, dxb, dyb, u, v, vort);
    UvTransVort<false> k{geo(b), luu, dxt, dyt, dxb, dyb, u, v, vort};
    return launch_range(b->nx_start, b->nx_end, b->ny_start, b->ny_end, k, (hipStream_t)stream, b->nx_start);
}

int ocn_uv_trans(const ocn_block *b, const float *lcu, const float *lcv, const float *luu, const float *dxh,
                 const float *dyh, const double *u, const double *v, const double *vort, const double *hq,
                 const double *hu, const double *hv, const double *hh, double *RHSx, double *RHSy, void *stream)
{
    (void)hq;
    CHECK(lcu, lcv, luu, dxh, dyh, u, v, vort, hu, hv, hh, RHSx, RHSy);
    UvTrans<false> k{geo(b), lcu, lcv, luu, dxh, dyh, u, v, vort, hu, hv, hh, RHSx, RHSy};
    return launch_march(b, range_interior(b), MarchUvTrans2D{k}, (hipStream_t)stream);
}

int ocn_stress_components(const ocn_block *b, const float *lu, const float *luu, const float *dx, const float *dy,
                          const float *dxt, const float *dyt, const float *dxh, const float *dyh, const float *dxb,
                          const float *dyb, const double *u, const double *v, double *str_t, double *str_s,
                          void *stream)
{
    CHECK(lu, luu, dx, dy, dxt, dyt, dxh, dyh, dxb, dyb, u, v, str_t, str_s);
    StressComponents<false> k{geo(b), lu, luu, dx, dy, dxt, dyt, dxh, dyh, dxb, dyb, u, v, str_t, str_s};
    return launch_march(b, range_interior(b), MarchStress2D{k}, (hipStream_t)stream);
}

int ocn_uv_diff2(const ocn_block *b, const float *lcu, const float *lcv, const float *dx, const float *dy,
                 const float *dxt, const float *dyt, const float *dxh, const float *dyh, const float *dxb,
                 const float *dyb, const double *mu, const double *str_t, const double *str_s, const double *hq,
                 const double *hu, const double *hv, const double *hh, double *RHSx, double *RHSy, void *stream)
{
    (void)hu; (void)hv;
    CHECK(lcu, lcv, dx, dy, dxt, dyt, dxh, dyh, dxb, dyb, mu, str_t, str_s, hq, hh, RHSx, RHSy);
    UvDiff2<false> k{geo(b), lcu, lcv, dx, dy, dxt, dyt, dxh, dyh, dxb, dyb, mu, str_t, str_s, hq, hh, RHSx, RHSy};
    return launch_march(b, range_interior(b), MarchUvDiff2D{k}, (hipStream_t)stream);
}

int ocn_sw_update_uv(const ocn_block *b, double tau, const float *lcu, const float *lcv, const float *dxt,
                     const float *dyt, const float *dxh, const float *dyh, const float *dxb, const float *dyb,
                     const double *hhu, const double *hhun, const double *hhup, const double *hhv,
                     const double *hhvn, const double *hhvp, const double *hhh, const double *ssh,
                     const double *ubrtr, double *ubrtrn, const double *ubrtrp, const double *vbrtr,
                     double *vbrtrn, const double *vbrtrp, const float *rdis, const float *rlh_s,
                     const double *RHSx, const double *RHSy, const double *RHSx_adv, const double *RHSy_adv,
                     const double *RHSx_dif, const double *RHSy_dif, void *stream)
{
    CHECK(lcu, lcv, dxt, dyt, dxh, dyh, dxb, dyb, hhu, hhun, hhup, hhv, hhvn, hhvp, hhh, ssh, ubrtr, ubrtrn,
          ubrtrp, vbrtr, vbrtrn, vbrtrp, rdis, rlh_s, RHSx, RHSy, RHSx_adv, RHSy_adv, RHSx_dif, RHSy_dif);
    SwUpdateUv<false> k{geo(b), tau, lcu, lcv, dxt, dyt, dxh, dyh, dxb, dyb, hhu, hhun, hhup, hhv, hhvn, hhvp, hhh, ssh,
                 ubrtr, ubrtrn, ubrtrp, vbrtr, vbrtrn, vbrtrp, rdis, rlh_s, RHSx, RHSy, RHSx_adv, RHSy_adv,
                 RHSx_dif, RHSy_dif};
    return launch_range(b->nx_start, b->nx_end, b->ny_start, b->ny_end, k, (hipStream_t)stream, b->nx_start);
}

int ocn_sw_next_step(const ocn_block *b, double time_smooth, const float *lu, const float *lcu, const float *lcv,
                     double *ssh, double *sshn, double *sshp, double *ubrtr, double *ubrtrn, double *ubrtrp,
                     double *vbrtr, double *vbrtrn, double *vbrtrp, void *stream)
{
    CHECK(lu, lcu, lcv, ssh, sshn, sshp, ubrtr, ubrtrn, ubrtrp, vbrtr, vbrtrn, vbrtrp);
    SwNextStep<false> k{geo(b), time_smooth, lu, lcu, lcv, ssh, sshn, sshp, ubrtr, ubrtrn, ubrtrp, vbrtr, vbrtrn, vbrtrp};
    return launch_range(b->nx_start - 1, b->nx_end + 1, b->ny_start - 1, b->ny_end + 1, k, (hipStream_t)stream, b->nx_start);
}

int ocn_hh_shift(const ocn_block *b, double time_smooth, const float *lu, const float *llu, const float *llv,
                 const float *luh, double *hq, double *hqp, double *hqn, double *hu, double *hup, double *hun,
                 double *hv, double *hvp, double *hvn, double *hh, double *hhp, double *hhn, void *stream)
{
    CHECK(lu, llu, llv, luh, hq, hqp, hqn, hu, hup, hun, hv, hvp, hvn, hh, hhp, hhn);
    HhShift<false> k{geo(b), time_smooth, lu, llu, llv, luh, hq, hqp, hqn, hu, hup, hun, hv, hvp, hvn, hh, hhp, hhn};
    return launch_range(b->nx_start - 1, b->nx_end + 1, b->ny_start - 1, b->ny_end + 1, k, (hipStream_t)stream, b->nx_start);
}

int ocn_hh_init(const ocn_block *b, int32_t full_free_surface, const float *lu, const float *llu,
                const float *llv, const float *luh, const float *dx, const float *dy, const float *dxt,
                const float *dyt, const float *dxh, const float *dyh, const float *dxb, const float *dyb,
                double *hq, double *hqp, double *hqn, double *hu, double *hup, double *hun, double *hv,
                double *hvp, double *hvn, double *hh, double *hhp, double *hhn, const double *sh,
                const double *shp, const double *h_r, void *stream)
{
    CHECK(lu, llu, llv, luh, dx, dy, dxt, dyt, dxh, dyh, dxb, dyb, hq, hqp, hqn, hu, hup, hun, hv, hvp, hvn, hh,
          hhp, hhn, sh, shp, h_r);
    HhInit<false> k{geo(b), b->nx_start - 1, b->nx_end, b->ny_start - 1, b->ny_end, (double)full_free_surface, true,
             Interp<false>{lu, dx, dy, dxt, dyt, dxh, dyh, dxb, dyb}, llu, llv, luh,
             hq, hqp, hqn, hu, hup, hun, hv, hvp, hvn, hh, hhp, hhn, sh, shp, h_r};
    return launch_march(b, range_bnd(b), MarchHhInit2D{k, b->bnd_y2}, (hipStream_t)stream);
}

int ocn_tran_diff_fluxes(const ocn_block *b, const float *lcu, const float *lcv, const float *dxt, const float *dyt,
                         const float *dxh, const float *dyh, const double *hhu, const double *hhv, const double *ff,
                         const double *ffp, const double *uu, const double *vv, const double *mu, double factor_mu,
                         double *flux_x, double *flux_y, void *stream)
{
    (void)ffp;   // passed and unused by the reference kernel ("Try ff instead of ffp")
    CHECK(lcu, lcv, dxt, dyt, dxh, dyh, hhu, hhv, ff, uu, vv, mu, flux_x, flux_y);
    TranDiffFluxes<false> k{geo(b), factor_mu, lcu, lcv, dxt, dyt, dxh, dyh, hhu, hhv, ff, uu, vv, mu, flux_x, flux_y};
    return launch_range(b->nx_start, b->nx_end, b->ny_start, b->ny_end, k, (hipStream_t)stream, b->nx_start);
}

int ocn_tran_diff_tracer(const ocn_block *b, const float *lu, const float *dx, const float *dy, double tau,
                         const double *hhqn, const double *hhqp, const double *flux_x, const double *flux_y,
                         const double *ffp, double *ffn, void *stream)
{
    CHECK(lu, dx, dy, hhqn, hhqp, flux_x, flux_y, ffp, ffn);
    TranDiffTracer<false> k{geo(b), tau, lu, dx, dy, hhqn, hhqp, flux_x, flux_y, ffp, ffn};
    return launch_range(b->nx_start, b->nx_end, b->ny_start, b->ny_end, k, (hipStream_t)stream, b->nx_start);
}

int ocn_tracer_next_step(const ocn_block *b, double time_smooth, const float *lu, const double *ffn, double *ffp,
                         double *ff, void *stream)
{
    CHECK(lu, ffn, ffp, ff);
    TracerNextStep<false> k{geo(b), time_smooth, lu, ffn, ffp, ff};
    return launch_range(b->nx_start - 1, b->nx_end + 1, b->ny_start - 1, b->ny_end + 1, k, (hipStream_t)stream, b->nx_start);
}

int ocn_check_ssh_err(const ocn_block *b, const float *lu, const double *ssh, int32_t *nbad_device, void *stream)
{
    CHECK(lu, ssh, nbad_device);
    CheckSshErr<false> k{geo(b), lu, ssh, (int *)nbad_device};
    return launch_range(b->nx_start, b->nx_end, b->ny_start, b->ny_end, k, (hipStream_t)stream, b->nx_start);
}

}  // extern "C"
