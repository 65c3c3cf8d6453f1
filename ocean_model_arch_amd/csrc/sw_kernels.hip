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

#include "ocn_internal.h"
#include "sw_stencils.h"

namespace ocn {

// ------------------------------------------------------------------ launch scaffolding
// A workgroup owns a tile of OCN_TW columns x OCN_ROWS rows: OCN_TW lanes across (a multiple
// of the 64-lane wave), OCN_WY = 256 / OCN_TW waves stacked vertically that step through the
// tile rows together.  Tile t = (t % ntx, t / ntx).  With OCN_XCD_REMAP the linear workgroup
// id is remapped so that each of the 8 XCDs (workgroups are dealt round-robin, id % 8) works
// on one contiguous band of tiles: horizontally adjacent tiles then run back to back on the
// same XCD and their shared +-1 columns / rows are L2 hits instead of refetches.
template <typename Body>
__global__ __launch_bounds__(256, OCN_LB_WAVES) void k_range(int m0, int m1, int n0, int n1, int ntx, int ntiles,
                                                             Body body)
{
    int tile = (int)blockIdx.x;
#if OCN_XCD_REMAP
    const int per = (ntiles + 7) / 8;
    tile = (tile % 8) * per + tile / 8;
    if (tile >= ntiles) return;
#endif
    const int tx = tile % ntx, ty = tile / ntx;
    const int m = m0 + tx * OCN_TW + (int)threadIdx.x;
    if (m > m1) return;
    const int nb = n0 + ty * OCN_ROWS;
    const int ne = min(n1, nb + OCN_ROWS - 1);
    // every wave is one thread-row: its row index is wave-uniform (scalar registers)
    const int wy = __builtin_amdgcn_readfirstlane((int)threadIdx.y);
    for (int n = nb + wy; n <= ne; n += OCN_WY) body(m, n);
}

template <typename Body>
static int launch_range(int m0, int m1, int n0, int n1, const Body &body, hipStream_t s)
{
    if (m1 < m0 || n1 < n0) return OCN_OK;
    const int ntx = (m1 - m0 + OCN_TW) / OCN_TW, nty = (n1 - n0 + OCN_ROWS) / OCN_ROWS;
    const int ntiles = ntx * nty;
    const int nblocks = OCN_XCD_REMAP ? 8 * ((ntiles + 7) / 8) : ntiles;
    hipLaunchKernelGGL(k_range<Body>, dim3((unsigned)nblocks), dim3(OCN_TW, OCN_WY), 0, s, m0, m1, n0, n1, ntx,
                       ntiles, body);
    return check_launch();
}

// the frame part of a split range (sw_stencils.h frame_rects): one thread per point
template <typename Body>
__global__ __launch_bounds__(256) void k_frame(Rects q, int total, Body body)
{
    const int t = (int)(blockIdx.x * 256 + threadIdx.x);
    if (t >= total) return;
    int m, n;
    frame_point(q, t, m, n);
    body(m, n);
}

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
        hipLaunchKernelGGL(k_frame<Body>, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, q, total, body);
        return check_launch();
    }
    return launch_range(r.m0, r.m1, r.n0, r.n1, body, s);
}

// ------------------------------------------------------------------ register march
// For stencils over many arrays the k_range mapping issues one load instruction per
// (array, neighbour): fused B issues 76 per cell, and the L1/TA path -- not HBM -- limits it
// (SQ_WAIT_INST_ANY ~70 % of wave time; profiles/r01b).  The march mapping loads each array
// once per cell instead:
//   * a wave owns 64 consecutive columns and marches down kMarchRows rows; lanes 1..62 produce
//     output, lanes 0 and 63 only load the m-1 / m+1 neighbour columns;
//   * the n-1 / n / n+1 rows of an array stay in registers and rotate as the wave moves down, so
//     each iteration loads only row n+1 (or row n for arrays read at n-1 and n);
//   * m+1 / m-1 neighbours come from the adjacent lane (DPP wave_shl:1 / wave_shr:1);
//   * the per-row metrics of the compact tables are wave-uniform (scalar loads).
// Four waves of a workgroup sit side by side (248 output columns); XCD-banded tile order as
// k_range.  Whole waves stay active through the loop (the lane shifts need every lane).
constexpr int kMarchCols = 62;
#ifndef OCN_MARCH_ROWS
#define OCN_MARCH_ROWS 16
#endif

__device__ __forceinline__ double lane_shift(double x, int dx)   // x of lane + dx, dx in {-1, 0, 1}
{
    if (dx == 0) return x;
    int lo = __double2loint(x), hi = __double2hiint(x);
    if (dx > 0) {   // wave_shl:1: lane i <- lane i+1
        lo = __builtin_amdgcn_mov_dpp(lo, 0x130, 0xf, 0xf, false);
        hi = __builtin_amdgcn_mov_dpp(hi, 0x130, 0xf, 0xf, false);
    } else {        // wave_shr:1: lane i <- lane i-1
        lo = __builtin_amdgcn_mov_dpp(lo, 0x138, 0xf, 0xf, false);
        hi = __builtin_amdgcn_mov_dpp(hi, 0x138, 0xf, 0xf, false);
    }
    return __hiloint2double(hi, lo);
}

// Never defined: a view access outside the rows a march keeps fails to link.
extern "C" __device__ void ocn_march_bad_access();

// rows n-1 (s), n (c), n+1 (nn) of one r8 array at this lane's column; S / N: whether s / nn are kept
template <bool S, bool N> struct Rows {
    double s, c, nn;
    __device__ __forceinline__ double at(int dx, int dy) const
    {
        if ((dy < 0 && !S) || (dy > 0 && !N) || dy < -1 || dy > 1) ocn_march_bad_access();
        return lane_shift(dy < 0 ? s : dy == 0 ? c : nn, dx);
    }
    __device__ __forceinline__ void rotate() { s = c; c = nn; }
};

// value of an array read only at (m, n)
struct Here {
    double v;
    __device__ __forceinline__ double at(int dx, int dy) const
    {
        if (dx != 0 || dy != 0) ocn_march_bad_access();
        return v;
    }
};

template <class Body>
__global__ __launch_bounds__(256) void k_march(int m0, int m1, int n0, int n1, int ntx, int ntiles, Body body)
{
    int tile = (int)blockIdx.x;
#if OCN_XCD_REMAP
    const int per = (ntiles + 7) / 8;
    tile = (tile % 8) * per + tile / 8;
    if (tile >= ntiles) return;
#endif
    const int tx = tile % ntx, ty = tile / ntx;
    const int lane = (int)threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
    const int mw = m0 + (tx * 4 + wave) * kMarchCols;   // first output column of this wave
    if (mw > m1) return;                                 // wave-uniform
    const int m = mw - 1 + lane;                         // loaded column (m1 + 1 at most is read)
    const bool out = lane >= 1 && lane <= kMarchCols && m <= m1;
    const int nb = n0 + ty * OCN_MARCH_ROWS, ne = min(n1, nb + OCN_MARCH_ROWS - 1);
    body.march(min(m, m1 + 1), out, nb, ne);
}

template <typename Body>
static int launch_march(int m0, int m1, int n0, int n1, const Body &body, hipStream_t s)
{
    if (m1 < m0 || n1 < n0) return OCN_OK;
    const int wg_cols = 4 * kMarchCols;
    const int ntx = (m1 - m0 + wg_cols) / wg_cols, nty = (n1 - n0 + OCN_MARCH_ROWS) / OCN_MARCH_ROWS;
    const int ntiles = ntx * nty;
    const int nblocks = OCN_XCD_REMAP ? 8 * ((ntiles + 7) / 8) : ntiles;
    hipLaunchKernelGGL(k_march<Body>, dim3((unsigned)nblocks), dim3(256), 0, s, m0, m1, n0, n1, ntx, ntiles, body);
    return check_launch();
}

// The view of fused B's three stages (sw_stencils.h uv_trans_math / uv_diff2_math /
// sw_update_uv_math) over the march registers.  Accessor names follow the stage functors; an
// array named twice there (u = ubrtr, hu = hhu, hh = hhh) is one register set here.
struct MarchViewB {
    Rows<true, true> rU, rV, rHV, rMU;                 // ubrtr, vbrtr, hhv, mu
    Rows<false, true> rHU, rHQ, rSTT, rSSH;            // hhu, hhq, str_t, ssh
    Rows<true, false> rVORT, rHH, rSTS;                // vort, hhh, str_s
    Here hhun_, hhup_, hhvn_, hhvp_, ubrtrp_, vbrtrp_, rhsx_, rhsy_;
    unsigned bits_s, bits_c;                           // mask bytes at (m, n-1), (m, n)
    float g[kNumRowFields][3];                         // metric rows n-1, n, n+1 (compact tables)
    double tau;
    __device__ __forceinline__ double quot(double a, double b, int, int) const { return a / b; }
    __device__ __forceinline__ double qtau(double a) const { return a / tau; }
#define OCN_MV(name, reg) \
    __device__ __forceinline__ double name(int dx, int dy) const { return reg.at(dx, dy); }
    OCN_MV(u, rU) OCN_MV(ubrtr, rU) OCN_MV(v, rV) OCN_MV(vbrtr, rV) OCN_MV(hu, rHU) OCN_MV(hhu, rHU)
    OCN_MV(hv, rHV) OCN_MV(hhv, rHV) OCN_MV(hh, rHH) OCN_MV(hhh, rHH) OCN_MV(mu, rMU) OCN_MV(hq, rHQ)
    OCN_MV(vort, rVORT) OCN_MV(str_t, rSTT) OCN_MV(str_s, rSTS) OCN_MV(ssh, rSSH)
    OCN_MV(hhun, hhun_) OCN_MV(hhup, hhup_) OCN_MV(hhvn, hhvn_) OCN_MV(hhvp, hhvp_) OCN_MV(ubrtrp, ubrtrp_)
    OCN_MV(vbrtrp, vbrtrp_) OCN_MV(RHSx, rhsx_) OCN_MV(RHSy, rhsy_)
#undef OCN_MV
#define OCN_MG(name, id) \
    __device__ __forceinline__ float name(int, int dy) const { return g[id - OCN_DX][dy + 1]; }
    OCN_MG(dx, OCN_DX) OCN_MG(dy, OCN_DY) OCN_MG(dxt, OCN_DXT) OCN_MG(dyt, OCN_DYT) OCN_MG(dxh, OCN_DXH)
    OCN_MG(dyh, OCN_DYH) OCN_MG(dxb, OCN_DXB) OCN_MG(dyb, OCN_DYB) OCN_MG(rlh_s, OCN_RLH_S) OCN_MG(rdis, OCN_R_DISS)
#undef OCN_MG
    __device__ __forceinline__ float luu(int dx, int dy) const
    {
        if (dx != 0 || dy < -1 || dy > 0) ocn_march_bad_access();
        return ((dy < 0 ? bits_s : bits_c) & (1u << OCN_LUU)) ? 1.0f : 0.0f;
    }
};

// fused B (sw_stencils.h FusedB) as a register march; compact static fields only
struct MarchFusedB {
    ocn_block b; Tab<true> t; ocn_sw_params sw; double tau; bool full, reuse;
    __device__ void march(int m, bool out, int nb, int ne) const
    {
        const FusedB<true> k = make_fused_b(&b, t, sw, tau, full, reuse);
        const UvTrans<true> &a4 = k.a4;
        const UvDiff2<true> &a6 = k.a6;
        const SwUpdateUv<true> &a7 = k.a7;
        const Geo I = a7.I;
        const unsigned nrows = t.nrows;
        auto row_met = [&](int id, int n) { return t.rows[(unsigned)(id - OCN_DX) * nrows + (unsigned)(n - b.bnd_y1)]; };
        MarchViewB x;
        x.tau = tau;
        {
            const Pt s = I(m, nb - 1), c = I(m, nb);
            x.rU.s = ld(a7.ubrtr, s); x.rU.c = ld(a7.ubrtr, c);
            x.rV.s = ld(a7.vbrtr, s); x.rV.c = ld(a7.vbrtr, c);
            x.rHV.s = ld(a7.hhv, s); x.rHV.c = ld(a7.hhv, c);
            x.rMU.s = ld(a6.mu, s); x.rMU.c = ld(a6.mu, c);
            x.rHU.c = ld(a7.hhu, c); x.rHQ.c = ld(a6.hq, c); x.rSTT.c = ld(a6.str_t, c); x.rSSH.c = ld(a7.ssh, c);
            x.rVORT.c = ld(a4.vort, s); x.rHH.c = ld(a7.hhh, s); x.rSTS.c = ld(a6.str_s, s);
            x.bits_c = ld(t.bits, s);
            for (int id = OCN_DX; id < OCN_NUM_R4; ++id) {
                x.g[id - OCN_DX][1] = row_met(id, nb - 1);
                x.g[id - OCN_DX][2] = row_met(id, nb);
            }
        }
        for (int n = nb; n <= ne; ++n) {
            const Pt c = I(m, n), cn = I(m, n + 1);
            // rotate the rows kept at n-1 / n; load row n+1 (or n)
            x.rVORT.s = x.rVORT.c; x.rHH.s = x.rHH.c; x.rSTS.s = x.rSTS.c; x.bits_s = x.bits_c;
            for (int r = 0; r < kNumRowFields; ++r) { x.g[r][0] = x.g[r][1]; x.g[r][1] = x.g[r][2]; }
            x.rU.nn = ld(a7.ubrtr, cn); x.rV.nn = ld(a7.vbrtr, cn); x.rHV.nn = ld(a7.hhv, cn); x.rMU.nn = ld(a6.mu, cn);
            x.rHU.nn = ld(a7.hhu, cn); x.rHQ.nn = ld(a6.hq, cn); x.rSTT.nn = ld(a6.str_t, cn); x.rSSH.nn = ld(a7.ssh, cn);
            x.rVORT.c = ld(a4.vort, c); x.rHH.c = ld(a7.hhh, c); x.rSTS.c = ld(a6.str_s, c);
            x.bits_c = ld(t.bits, c);
            for (int id = OCN_DX; id < OCN_NUM_R4; ++id) x.g[id - OCN_DX][2] = row_met(id, n + 1);
            x.hhun_.v = ld(a7.hhun, c); x.hhup_.v = ld(a7.hhup, c); x.hhvn_.v = ld(a7.hhvn, c);
            x.hhvp_.v = ld(a7.hhvp, c); x.ubrtrp_.v = ld(a7.ubrtrp, c); x.vbrtrp_.v = ld(a7.vbrtrp, c);
            x.rhsx_.v = ld(a7.RHSx, c); x.rhsy_.v = ld(a7.RHSy, c);

            double rxa, rya, rxd, ryd;
            if (k.do_adv) uv_trans_math(x, rxa, rya);
            else { rxa = ld(a7.RHSx_adv, c); rya = ld(a7.RHSy_adv, c); }
            if (k.do_dif) uv_diff2_math(x, rxd, ryd);
            else { rxd = ld(a7.RHSx_dif, c); ryd = ld(a7.RHSy_dif, c); }
            double un, vn;
            sw_update_uv_math(x, rxa, rxd, rya, ryd, un, vn);
            if (out) {
                if (x.bits_c & (1u << OCN_LCU)) {
                    if (k.do_adv && k.full) st(a4.RHSx, c, rxa);
                    if (k.do_dif && k.full) st(a6.RHSx, c, rxd);
                    st(a7.ubrtrn, c, un);
                }
                if (x.bits_c & (1u << OCN_LCV)) {
                    if (k.do_adv && k.full) st(a4.RHSy, c, rya);
                    if (k.do_dif && k.full) st(a6.RHSy, c, ryd);
                    st(a7.vbrtrn, c, vn);
                }
            }
            x.rU.rotate(); x.rV.rotate(); x.rHV.rotate(); x.rMU.rotate();
            x.rHU.rotate(); x.rHQ.rotate(); x.rSTT.rotate(); x.rSSH.rotate();
        }
    }
};

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

int launch_fused_a(const ocn_block *b, void *const *ptr, int nptr, const Compact *cp, int part,
                   const ocn_sw_params &sw, double tau, bool reuse, hipStream_t s)
{
    return launch_fused<KFusedA>(range_fused_a(b, sw, reuse), inner_interior_shrunk(b), part, b, ptr, nptr, cp, 0, s,
                                 sw, tau, reuse);
}

int launch_fused_b(const ocn_block *b, void *const *ptr, int nptr, const Compact *cp, int part,
                   const ocn_sw_params &sw, double tau, bool full, bool reuse, hipStream_t s)
{
    if (cp && cp->march && part != OCN_PART_FRAME) {
        RC_K(check_block(b));
        const Range r = part == OCN_PART_INNER ? range_clip(range_interior(b), inner_interior_shrunk(b))
                                               : range_interior(b);
        const MarchFusedB k{*b, make_tab<true>(ptr, nptr, cp->bits, cp->rows, block_rows(b), 0), sw, tau, full, reuse};
        return launch_march(r.m0, r.m1, r.n0, r.n1, k, s);
    }
    return launch_fused<KFusedB>(range_interior(b), inner_interior_shrunk(b), part, b, ptr, nptr, cp, 0, s, sw, tau,
                                 full, reuse);
}

int launch_fused_c1(const ocn_block *b, void *const *ptr, int nptr, const Compact *cp, int part,
                    const ocn_sw_params &sw, int32_t *nbad, hipStream_t s)
{
    return launch_fused<KFusedC1>(range_ring(b), range_interior(b), part, b, ptr, nptr, cp, 0, s, sw, nbad);
}

int launch_fused_c2(const ocn_block *b, void *const *ptr, int nptr, const Compact *cp, int part,
                    const ocn_sw_params &sw, bool full, hipStream_t s)
{
    return launch_fused<KHhInit>(range_bnd(b), inner_interior_shrunk(b), part, b, ptr, nptr, cp, 0, s,
                                 (int)sw.full_free_surface, full);
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

int launch_prepare(const ocn_block *b, void *const *ptr, uint8_t *bits, float *rows, int32_t *flags, hipStream_t s)
{
    RC_K(check_block(b));
    const Range r = range_bnd(b);
    return launch_range(r.m0, r.m1, r.n0, r.n1, make_prepare(b, ptr, bits, rows, (int *)flags), s);
}

}  // namespace ocn

using namespace ocn;

extern "C" {

int ocn_sw_update_ssh(const ocn_block *b, double tau, const float *lu, const float *dx, const float *dy,
                      const float *dxh, const float *dyh, const double *hhu, const double *hhv, double *sshn,
                      const double *sshp, const double *ubrtr, const double *vbrtr, void *stream)
{
    CHECK(lu, dx, dy, dxh, dyh, hhu, hhv, sshn, sshp, ubrtr, vbrtr);
    SwUpdateSsh<false> k{geo(b), tau, lu, dx, dy, dxh, dyh, hhu, hhv, sshn, sshp, ubrtr, vbrtr};
    return launch_range(b->nx_start, b->nx_end, b->ny_start, b->ny_end, k, (hipStream_t)stream);
}

int ocn_hh_update(const ocn_block *b, const float *lu, const float *llu, const float *llv, const float *luh,
                  const float *dx, const float *dy, const float *dxt, const float *dyt, const float *dxh,
                  const float *dyh, const float *dxb, const float *dyb, double *hqn, double *hun, double *hvn,
                  double *hhn, const double *sh, const double *h_r, void *stream)
{
    CHECK(lu, llu, llv, luh, dx, dy, dxt, dyt, dxh, dyh, dxb, dyb, hqn, hun, hvn, hhn, sh, h_r);
    HhUpdate<false> k{geo(b), b->nx_start - 1, b->nx_end, b->ny_start - 1, b->ny_end,
               Interp<false>{lu, dx, dy, dxt, dyt, dxh, dyh, dxb, dyb}, llu, llv, luh, hqn, hun, hvn, hhn, sh, h_r};
    return launch_range(b->bnd_x1, b->bnd_x2, b->bnd_y1, b->bnd_y2, k, (hipStream_t)stream);
}

int ocn_uv_trans_vort(const ocn_block *b, const float *luu, const float *dxt, const float *dyt, const float *dxb,
                      const float *dyb, const double *u, const double *v, double *vort, void *stream)
{
    CHECK(luu, dxt, dyt, dxb, dyb, u, v, vort);
    UvTransVort<false> k{geo(b), luu, dxt, dyt, dxb, dyb, u, v, vort};
    return launch_range(b->nx_start, b->nx_end, b->ny_start, b->ny_end, k, (hipStream_t)stream);
}

int ocn_uv_trans(const ocn_block *b, const float *lcu, const float *lcv, const float *luu, const float *dxh,
                 const float *dyh, const double *u, const double *v, const double *vort, const double *hq,
                 const double *hu, const double *hv, const double *hh, double *RHSx, double *RHSy, void *stream)
{
    (void)hq;
    CHECK(lcu, lcv, luu, dxh, dyh, u, v, vort, hu, hv, hh, RHSx, RHSy);
    UvTrans<false> k{geo(b), lcu, lcv, luu, dxh, dyh, u, v, vort, hu, hv, hh, RHSx, RHSy};
    return launch_range(b->nx_start, b->nx_end, b->ny_start, b->ny_end, k, (hipStream_t)stream);
}

int ocn_stress_components(const ocn_block *b, const float *lu, const float *luu, const float *dx, const float *dy,
                          const float *dxt, const float *dyt, const float *dxh, const float *dyh, const float *dxb,
                          const float *dyb, const double *u, const double *v, double *str_t, double *str_s,
                          void *stream)
{
    CHECK(lu, luu, dx, dy, dxt, dyt, dxh, dyh, dxb, dyb, u, v, str_t, str_s);
    StressComponents<false> k{geo(b), lu, luu, dx, dy, dxt, dyt, dxh, dyh, dxb, dyb, u, v, str_t, str_s};
    return launch_range(b->nx_start, b->nx_end, b->ny_start, b->ny_end, k, (hipStream_t)stream);
}

int ocn_uv_diff2(const ocn_block *b, const float *lcu, const float *lcv, const float *dx, const float *dy,
                 const float *dxt, const float *dyt, const float *dxh, const float *dyh, const float *dxb,
                 const float *dyb, const double *mu, const double *str_t, const double *str_s, const double *hq,
                 const double *hu, const double *hv, const double *hh, double *RHSx, double *RHSy, void *stream)
{
    (void)hu; (void)hv;
    CHECK(lcu, lcv, dx, dy, dxt, dyt, dxh, dyh, dxb, dyb, mu, str_t, str_s, hq, hh, RHSx, RHSy);
    UvDiff2<false> k{geo(b), lcu, lcv, dx, dy, dxt, dyt, dxh, dyh, dxb, dyb, mu, str_t, str_s, hq, hh, RHSx, RHSy};
    return launch_range(b->nx_start, b->nx_end, b->ny_start, b->ny_end, k, (hipStream_t)stream);
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
    return launch_range(b->nx_start, b->nx_end, b->ny_start, b->ny_end, k, (hipStream_t)stream);
}

int ocn_sw_next_step(const ocn_block *b, double time_smooth, const float *lu, const float *lcu, const float *lcv,
                     double *ssh, double *sshn, double *sshp, double *ubrtr, double *ubrtrn, double *ubrtrp,
                     double *vbrtr, double *vbrtrn, double *vbrtrp, void *stream)
{
    CHECK(lu, lcu, lcv, ssh, sshn, sshp, ubrtr, ubrtrn, ubrtrp, vbrtr, vbrtrn, vbrtrp);
    SwNextStep<false> k{geo(b), time_smooth, lu, lcu, lcv, ssh, sshn, sshp, ubrtr, ubrtrn, ubrtrp, vbrtr, vbrtrn, vbrtrp};
    return launch_range(b->nx_start - 1, b->nx_end + 1, b->ny_start - 1, b->ny_end + 1, k, (hipStream_t)stream);
}

int ocn_hh_shift(const ocn_block *b, double time_smooth, const float *lu, const float *llu, const float *llv,
                 const float *luh, double *hq, double *hqp, double *hqn, double *hu, double *hup, double *hun,
                 double *hv, double *hvp, double *hvn, double *hh, double *hhp, double *hhn, void *stream)
{
    CHECK(lu, llu, llv, luh, hq, hqp, hqn, hu, hup, hun, hv, hvp, hvn, hh, hhp, hhn);
    HhShift<false> k{geo(b), time_smooth, lu, llu, llv, luh, hq, hqp, hqn, hu, hup, hun, hv, hvp, hvn, hh, hhp, hhn};
    return launch_range(b->nx_start - 1, b->nx_end + 1, b->ny_start - 1, b->ny_end + 1, k, (hipStream_t)stream);
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
    return launch_range(b->bnd_x1, b->bnd_x2, b->bnd_y1, b->bnd_y2, k, (hipStream_t)stream);
}

int ocn_tran_diff_fluxes(const ocn_block *b, const float *lcu, const float *lcv, const float *dxt, const float *dyt,
                         const float *dxh, const float *dyh, const double *hhu, const double *hhv, const double *ff,
                         const double *ffp, const double *uu, const double *vv, const double *mu, double factor_mu,
                         double *flux_x, double *flux_y, void *stream)
{
    (void)ffp;   // passed and unused by the reference kernel ("Try ff instead of ffp")
    CHECK(lcu, lcv, dxt, dyt, dxh, dyh, hhu, hhv, ff, uu, vv, mu, flux_x, flux_y);
    TranDiffFluxes<false> k{geo(b), factor_mu, lcu, lcv, dxt, dyt, dxh, dyh, hhu, hhv, ff, uu, vv, mu, flux_x, flux_y};
    return launch_range(b->nx_start, b->nx_end, b->ny_start, b->ny_end, k, (hipStream_t)stream);
}

int ocn_tran_diff_tracer(const ocn_block *b, const float *lu, const float *dx, const float *dy, double tau,
                         const double *hhqn, const double *hhqp, const double *flux_x, const double *flux_y,
                         const double *ffp, double *ffn, void *stream)
{
    CHECK(lu, dx, dy, hhqn, hhqp, flux_x, flux_y, ffp, ffn);
    TranDiffTracer<false> k{geo(b), tau, lu, dx, dy, hhqn, hhqp, flux_x, flux_y, ffp, ffn};
    return launch_range(b->nx_start, b->nx_end, b->ny_start, b->ny_end, k, (hipStream_t)stream);
}

int ocn_tracer_next_step(const ocn_block *b, double time_smooth, const float *lu, const double *ffn, double *ffp,
                         double *ff, void *stream)
{
    CHECK(lu, ffn, ffp, ff);
    TracerNextStep<false> k{geo(b), time_smooth, lu, ffn, ffp, ff};
    return launch_range(b->nx_start - 1, b->nx_end + 1, b->ny_start - 1, b->ny_end + 1, k, (hipStream_t)stream);
}

int ocn_check_ssh_err(const ocn_block *b, const float *lu, const double *ssh, int32_t *nbad_device, void *stream)
{
    CHECK(lu, ssh, nbad_device);
    CheckSshErr<false> k{geo(b), lu, ssh, (int *)nbad_device};
    return launch_range(b->nx_start, b->nx_end, b->ny_start, b->ny_end, k, (hipStream_t)stream);
}

}  // extern "C"
