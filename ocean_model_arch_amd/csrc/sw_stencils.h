// sw_stencils.h -- the per-cell arithmetic of the SW step stages (functors), shared by the
// HIP kernels (sw_kernels.hip, compiled for gfx950) and the host-side memory-safety /
// parity harness (tests/native/stencil_host.cpp).
// Each functor restates one reference loop nest (kernel/shallow_water/*.f90) bit for bit.
//
// Every functor is a template on C ("compact static fields"):
//   C = false  the real(4) masks and grid metrics are the reference's 2-D block arrays;
//   C = true   the 7 masks are bits of one byte per point and the 10 metric fields that are
//              constant along each row over [nx_start-1, nx_end+1] are one value per row
//              (built by Prepare below; exact -- masks hold only 0.0/1.0, row values are
//              the array's own bit patterns -- and used only when that was verified).
// The arithmetic is identical in both; only where a real(4) operand is read from differs.
#pragma once

#include <stdint.h>

#include "../../include/ocn_sw.h"

#ifndef OCN_HD
#define OCN_HD __host__ __device__
#endif
#ifndef OCN_INLINE
#define OCN_INLINE __forceinline__
#endif
#ifndef OCN_ATOMIC_INC
#define OCN_ATOMIC_INC(p) atomicAdd((p), 1)
#endif
#ifndef OCN_ATOMIC_OR
#define OCN_ATOMIC_OR(p, v) atomicOr((p), (v))
#endif
#ifndef OCN_FREE_FALL_ACC
#define OCN_FREE_FALL_ACC 9.8f   // shared/constants.f90:23 FreeFallAcc = 9.8 (real(4))
#endif

namespace ocn {

// A point of a block array: element index of A(m, n) (32-bit; the host checks pitch * rows
// < 2^29) and row index n - bnd_y1.
struct Pt {
    unsigned c, r;
};

struct Geo {
    int bx1, by1;
    unsigned p;
    OCN_HD OCN_INLINE Pt operator()(int m, int n) const
    {
        const unsigned r = (unsigned)(n - by1);
        return Pt{(unsigned)(m - bx1) + r * p, r};
    }
    OCN_HD OCN_INLINE Pt e(Pt q) const { return Pt{q.c + 1, q.r}; }
    OCN_HD OCN_INLINE Pt w(Pt q) const { return Pt{q.c - 1, q.r}; }
    OCN_HD OCN_INLINE Pt n(Pt q) const { return Pt{q.c + p, q.r + 1}; }
    OCN_HD OCN_INLINE Pt s(Pt q) const { return Pt{q.c - p, q.r - 1}; }
    // A(m + dx, n + dy) for constant dx, dy (folded after inlining)
    OCN_HD OCN_INLINE Pt at(Pt q, int dx, int dy) const
    {
        return Pt{q.c + (unsigned)dx + (unsigned)dy * p, q.r + (unsigned)dy};
    }
};

#define D(x) ((double)(x))

// Loads / stores through a 32-bit byte offset from the (wave-uniform) array base: the compiler
// then emits the SGPR-base + 32-bit VGPR-offset global_load/store form (no 64-bit address
// arithmetic per array).  Block arrays hold < 2^29 elements, so every r8 byte offset fits 32 bits (checked on the host).
#ifdef OCN_HOST_BOUNDS_CHECK   // host harness only: every access checked against the block size
extern unsigned ocn_host_limit;
void ocn_host_oob(unsigned i);
#define OCN_CHECK_INDEX(i) do { if ((i) >= ocn_host_limit) ocn_host_oob(i); } while (0)
#else
#define OCN_CHECK_INDEX(i) do { } while (0)
#endif

template <class T> OCN_HD OCN_INLINE T ld(const T *__restrict__ p, unsigned i)
{
    OCN_CHECK_INDEX(i);
    return *(const T *)((const char *)p + i * (unsigned)sizeof(T));
}
template <class T> OCN_HD OCN_INLINE void st(T *__restrict__ p, unsigned i, T v)
{
    OCN_CHECK_INDEX(i);
    *(T *)((char *)p + i * (unsigned)sizeof(T)) = v;
}
template <class T> OCN_HD OCN_INLINE T ld(const T *__restrict__ p, Pt q) { return ld(p, q.c); }
template <class T> OCN_HD OCN_INLINE void st(T *__restrict__ p, Pt q, T v) { st(p, q.c, v); }

// real(4) mask (lu, luu, luh, lcu, lcv, llu, llv) and grid-metric fields
template <bool C> struct Msk;
template <> struct Msk<false> { const float *__restrict__ a; };
template <> struct Msk<true> { const uint8_t *__restrict__ a; unsigned bit; };
template <bool C> struct Met;
template <> struct Met<false> { const float *__restrict__ a; };
template <> struct Met<true> { const float *__restrict__ a; };   // indexed by row

OCN_HD OCN_INLINE float ld(const Msk<false> &f, Pt q) { return ld(f.a, q.c); }
OCN_HD OCN_INLINE float ld(const Msk<true> &f, Pt q) { return (ld(f.a, q.c) & f.bit) ? 1.0f : 0.0f; }
OCN_HD OCN_INLINE float ld(const Met<false> &f, Pt q) { return ld(f.a, q.c); }
OCN_HD OCN_INLINE float ld(const Met<true> &f, Pt q) { return ld(f.a, q.r); }

OCN_HD OCN_INLINE uint32_t fbits(float f)
{
    uint32_t u;
    __builtin_memcpy(&u, &f, sizeof(u));
    return u;
}
OCN_HD OCN_INLINE uint64_t fbits64(double d)
{
    uint64_t u;
    __builtin_memcpy(&u, &d, 8);
    return u;
}

// ------------------------------------------------------------------ views
// The stage arithmetic is written against a "view" x: x.u(dx, dy) is u(m+dx, n+dy) of the
// reference loop, x.dyh(dx, dy) the real(4) metric there, x.lu(dx, dy) the mask value,
// x.quot(a, b, id, dy) = a / b for b = D(metric id at row n+dy), x.qtau(a) = a / tau,
// x.tau2() = tau.  The pointer views below load every operand from its block array (the stage
// kernels, the k_range fused kernels and the host harness); the register marches of
// sw_kernels.hip supply the same values from registers.  Same expressions, same evaluation
// order, same results.
#define OCN_VIEW_LD(name) \
    OCN_HD OCN_INLINE auto name(int dx, int dy) const { return ld(k.name, k.I.at(c, dx, dy)); }
#define OCN_VIEW_LD_AS(name, field) \
    OCN_HD OCN_INLINE auto name(int dx, int dy) const { return ld(k.field, k.I.at(c, dx, dy)); }
#define OCN_VIEW_PTR_COMMON(K)                                                                         \
    const K &k; Pt c;                                                                                  \
    OCN_HD OCN_INLINE double quot(double a, double b, int, int) const { return a / b; }

// ------------------------------------------------------------------ a1 sw_update_ssh
// vel_ssh.f90:69-106; returns sshn at this point
template <class X> OCN_HD OCN_INLINE double sw_update_ssh_math(const X &x)
{
    const double t1 = x.ubrtr(0, 0) * x.hhu(0, 0) * D(x.dyh(0, 0));
    const double t2 = x.ubrtr(-1, 0) * x.hhu(-1, 0) * D(x.dyh(-1, 0));
    const double t3 = x.vbrtr(0, 0) * x.hhv(0, 0) * D(x.dxh(0, 0));
    const double t4 = x.vbrtr(0, -1) * x.hhv(0, -1) * D(x.dxh(0, -1));
    const float area = x.dx(0, 0) * x.dy(0, 0);
    const double div = (t1 - t2 + t3 - t4) / D(area);
    return x.sshp(0, 0) + 2.0 * x.tau2() * (-div);
}

template <bool C> struct SwUpdateSsh {
    Geo I; double tau;
    Msk<C> lu; Met<C> dx, dy, dxh, dyh;
    const double *__restrict__ hhu, *__restrict__ hhv;
    double *__restrict__ sshn;
    const double *__restrict__ sshp, *__restrict__ ubrtr, *__restrict__ vbrtr;
    struct View {
        OCN_VIEW_PTR_COMMON(SwUpdateSsh)
        OCN_HD OCN_INLINE double tau2() const { return k.tau; }
        OCN_VIEW_LD(ubrtr) OCN_VIEW_LD(vbrtr) OCN_VIEW_LD(hhu) OCN_VIEW_LD(hhv) OCN_VIEW_LD(sshp)
        OCN_VIEW_LD(dx) OCN_VIEW_LD(dy) OCN_VIEW_LD(dxh) OCN_VIEW_LD(dyh)
    };
    OCN_HD void operator()(int m, int n) const
    {
        const Pt c = I(m, n);
        const double r = sw_update_ssh_math(View{*this, c});
        if (ld(lu, c) > 0.5f) st(sshn, c, r);
    }
};

// ------------------------------------------------------------------ T->U/V/H interpolation
// kernel/shallow_water/depth.f90:56-97 for one level given its values at the four corners
// (m,n), (m+1,n), (m,n+1), (m+1,n+1); per-corner weights dx*dy*lu (products evaluated per
// use, as the reference does)
// a / s for s a sum of 0/1 masks (0..4): x / 2^k and x * 2^-k are the same correctly rounded
// value, so when every lane of the wave has s = 1, 2 or 4 (the sea interior) the quotient is a
// multiply; otherwise (3, or 0 on land) the IEEE division.  Bitwise the same either way.
#ifndef OCN_WAVE_ALL
#define OCN_WAVE_ALL(p) __all(p)
#endif
OCN_HD OCN_INLINE double div_mask_sum(double a, double s)
{
    const double r = s == 4.0 ? 0.25 : s == 2.0 ? 0.5 : 1.0;
    if (OCN_WAVE_ALL(s == 1.0 || s == 2.0 || s == 4.0)) return a * r;
    return a / s;
}

template <class X> OCN_HD OCN_INLINE double interp_wt(const X &x, double h, int i, int j)
{
    return h * D(x.dx(i, j)) * D(x.dy(i, j)) * D(x.lu(i, j));
}
template <class X> OCN_HD OCN_INLINE double interp_u(const X &x, double h00, double h10)
{
    const double slu = D(x.lu(0, 0) + x.lu(1, 0));
    return div_mask_sum(interp_wt(x, h00, 0, 0) + interp_wt(x, h10, 1, 0), slu) / D(x.dxt(0, 0)) / D(x.dyh(0, 0));
}
template <class X> OCN_HD OCN_INLINE double interp_v(const X &x, double h00, double h01)
{
    const double slu = D(x.lu(0, 0) + x.lu(0, 1));
    return div_mask_sum(interp_wt(x, h00, 0, 0) + interp_wt(x, h01, 0, 1), slu) / D(x.dxh(0, 0)) / D(x.dyt(0, 0));
}
template <class X> OCN_HD OCN_INLINE double interp_h(const X &x, double h00, double h10, double h01, double h11)
{
    const double slu = D(x.lu(0, 0) + x.lu(1, 0) + x.lu(0, 1) + x.lu(1, 1));
    return div_mask_sum(interp_wt(x, h00, 0, 0) + interp_wt(x, h10, 1, 0) + interp_wt(x, h01, 0, 1)
                            + interp_wt(x, h11, 1, 1), slu) / D(x.dxb(0, 0)) / D(x.dyb(0, 0));
}

// a2 hh_update's interpolation (depth.f90:134-160): q = h_r + sh at each corner, q00 given
template <class X> OCN_HD OCN_INLINE void hh_update_math(const X &x, double q00, double &xu, double &xv, double &xh)
{
    const double q10 = x.h_r(1, 0) + x.sh(1, 0), q01 = x.h_r(0, 1) + x.sh(0, 1), q11 = x.h_r(1, 1) + x.sh(1, 1);
    xu = interp_u(x, q00, q10);
    xv = interp_v(x, q00, q01);
    xh = interp_h(x, q00, q10, q01, q11);
}

// a10 hh_init's interpolation (depth.f90:52-97) of the levels hq = h_r + sh*f (index 0),
// hqp = h_r + shp*f (1) and, when `full`, hqn = h_r (2)
struct HhInitOut { double u[3], v[3], h[3]; };
template <class X> OCN_HD OCN_INLINE void hh_init_math(const X &x, double f, bool full, HhInitOut &o)
{
    const double r00 = x.h_r(0, 0), r10 = x.h_r(1, 0), r01 = x.h_r(0, 1), r11 = x.h_r(1, 1);
    const double a00 = r00 + x.sh(0, 0) * f, a10 = r10 + x.sh(1, 0) * f, a01 = r01 + x.sh(0, 1) * f,
                 a11 = r11 + x.sh(1, 1) * f;
    const double b00 = r00 + x.shp(0, 0) * f, b10 = r10 + x.shp(1, 0) * f, b01 = r01 + x.shp(0, 1) * f,
                 b11 = r11 + x.shp(1, 1) * f;
    o.u[0] = interp_u(x, a00, a10); o.u[1] = interp_u(x, b00, b10);
    o.v[0] = interp_v(x, a00, a01); o.v[1] = interp_v(x, b00, b01);
    o.h[0] = interp_h(x, a00, a10, a01, a11); o.h[1] = interp_h(x, b00, b10, b01, b11);
    if (full) {
        o.u[2] = interp_u(x, r00, r10); o.v[2] = interp_v(x, r00, r01); o.h[2] = interp_h(x, r00, r10, r01, r11);
    }
}

template <bool C> struct Interp {
    Msk<C> lu; Met<C> dx, dy, dxt, dyt, dxh, dyh, dxb, dyb;
};
// pointer-view accessors of the Interp operands (member W of the functor)
#define OCN_VIEW_W(name) \
    OCN_HD OCN_INLINE auto name(int dx, int dy) const { return ld(k.W.name, k.I.at(c, dx, dy)); }
#define OCN_VIEW_INTERP                                                                             \
    OCN_VIEW_W(lu) OCN_VIEW_W(dx) OCN_VIEW_W(dy) OCN_VIEW_W(dxt) OCN_VIEW_W(dyt) OCN_VIEW_W(dxh)    \
    OCN_VIEW_W(dyh) OCN_VIEW_W(dxb) OCN_VIEW_W(dyb)

// ------------------------------------------------------------------ a2 hh_update
// depth.f90:101-162.  Thread grid = whole bnd range (hqn = h_r + sh, :129); the
// interpolation part runs on [start-1, end]^2.
template <bool C> struct HhUpdate {
    Geo I; int i0, i1, j0, j1;
    Interp<C> W;
    Msk<C> llu, llv, luh;
    double *__restrict__ hqn, *__restrict__ hun, *__restrict__ hvn, *__restrict__ hhn;
    const double *__restrict__ sh, *__restrict__ h_r;
    struct View {
        const HhUpdate &k; Pt c;
        OCN_VIEW_INTERP OCN_VIEW_LD(sh) OCN_VIEW_LD(h_r)
    };
    // the [start-1, end]^2 interpolation part (depth.f90:134-160); q00 = h_r + sh here
    OCN_HD OCN_INLINE void interp(Pt c, double q00) const
    {
        double xu, xv, xh;
        hh_update_math(View{*this, c}, q00, xu, xv, xh);
        if (ld(llu, c) > 0.5f) st(hun, c, xu);
        if (ld(llv, c) > 0.5f) st(hvn, c, xv);
        if (ld(luh, c) > 0.5f) st(hhn, c, xh);
    }
    OCN_HD void operator()(int m, int n) const
    {
        const Pt c = I(m, n);
        const double q00 = ld(h_r, c) + ld(sh, c);
        st(hqn, c, q00);
        if (m < i0 || m > i1 || n < j0 || n > j1) return;
        interp(c, q00);
    }
};

// ------------------------------------------------------------------ a10 hh_init
// depth.f90:14-99: hq = h_r + sh*ffs, hqp = h_r + shp*ffs, hqn = h_r (whole array), then the
// three levels interpolated on [start-1, end]^2.
// full = false (fused step, every step of an ocn_ctx_step call but the last) skips stores
// whose values no later kernel reads before they are rewritten:
//   hqn = h_r and hun/hvn/hhn = interp(h_r): hqn is never changed by the fused step (fused A
//     does not store hh_update's hqn), and hun/hvn/hhn are rewritten on exactly these points
//     by the next step's hh_update before anything reads them;
//   hqp: read only by hh_shift's hq/hqp update, whose results this kernel overwrites
//     whole-array one launch later.
template <bool C> struct HhInit {
    Geo I; int i0, i1, j0, j1; double f; bool full;
    Interp<C> W;
    Msk<C> llu, llv, luh;
    double *__restrict__ hq, *__restrict__ hqp, *__restrict__ hqn;
    double *__restrict__ hu, *__restrict__ hup, *__restrict__ hun;
    double *__restrict__ hv, *__restrict__ hvp, *__restrict__ hvn;
    double *__restrict__ hh, *__restrict__ hhp, *__restrict__ hhn;
    const double *__restrict__ sh, *__restrict__ shp, *__restrict__ h_r;
    struct View {
        const HhInit &k; Pt c;
        OCN_VIEW_INTERP OCN_VIEW_LD(sh) OCN_VIEW_LD(shp) OCN_VIEW_LD(h_r)
    };
    OCN_HD void operator()(int m, int n) const
    {
        const Pt c = I(m, n);
        const double r00 = ld(h_r, c);
        st(hq, c, r00 + ld(sh, c) * f);
        if (full) { st(hqp, c, r00 + ld(shp, c) * f); st(hqn, c, r00); }
        if (m < i0 || m > i1 || n < j0 || n > j1) return;
        HhInitOut o;
        hh_init_math(View{*this, c}, f, full, o);
        const bool bu = ld(llu, c) > 0.5f, bv = ld(llv, c) > 0.5f, bh = ld(luh, c) > 0.5f;
        if (bu) { st(hu, c, o.u[0]); st(hup, c, o.u[1]); }
        if (bv) { st(hv, c, o.v[0]); st(hvp, c, o.v[1]); }
        if (bh) { st(hh, c, o.h[0]); st(hhp, c, o.h[1]); }
        if (full) {
            if (bu) st(hun, c, o.u[2]);
            if (bv) st(hvn, c, o.v[2]);
            if (bh) st(hhn, c, o.h[2]);
        }
    }
};

// ------------------------------------------------------------------ a3 uv_trans_vort
// vel_ssh.f90:247-281
template <class X> OCN_HD OCN_INLINE double uv_trans_vort_math(const X &x)
{
    const double a = x.v(1, 0) * D(x.dyt(1, 0)) - x.v(0, 0) * D(x.dyt(0, 0));
    const double b = x.u(0, 1) * D(x.dxt(0, 1)) - x.u(0, 0) * D(x.dxt(0, 0));
    const double d = (x.v(1, 0) - x.v(0, 0)) * D(x.dyb(0, 0)) - (x.u(0, 1) - x.u(0, 0)) * D(x.dxb(0, 0));
    return a - b - d;
}

template <bool C> struct UvTransVort {
    Geo I;
    Msk<C> luu; Met<C> dxt, dyt, dxb, dyb;
    const double *__restrict__ u, *__restrict__ v;
    double *__restrict__ vort;
    struct View {
        OCN_VIEW_PTR_COMMON(UvTransVort)
        OCN_VIEW_LD(u) OCN_VIEW_LD(v) OCN_VIEW_LD(dxt) OCN_VIEW_LD(dyt) OCN_VIEW_LD(dxb) OCN_VIEW_LD(dyb)
    };
    OCN_HD void operator()(int m, int n) const
    {
        const Pt c = I(m, n);
        const double r = uv_trans_vort_math(View{*this, c});
        if (ld(luu, c) > 0.5f) st(vort, c, r);
    }
};

// ------------------------------------------------------------------ a4 uv_trans
// vel_ssh.f90:283-373
template <class X> OCN_HD OCN_INLINE void uv_trans_math(const X &x, double &rx, double &ry)
{
    {
        const double fu_c = x.u(0, 0) * D(x.dyh(0, 0)) * x.hu(0, 0);
        const double fx_p = (fu_c + x.u(1, 0) * D(x.dyh(1, 0)) * x.hu(1, 0)) / 2.0 * (x.u(0, 0) + x.u(1, 0)) / 2.0;
        const double fx_m = (fu_c + x.u(-1, 0) * D(x.dyh(-1, 0)) * x.hu(-1, 0)) / 2.0 * (x.u(0, 0) + x.u(-1, 0)) / 2.0;
        const double fy_p = (x.v(0, 0) * D(x.dxh(0, 0)) * x.hv(0, 0) + x.v(1, 0) * D(x.dxh(1, 0)) * x.hv(1, 0)) / 2.0
                            * (x.u(0, 1) + x.u(0, 0)) / 2.0 * D(x.luu(0, 0));
        const double fy_m = (x.v(0, -1) * D(x.dxh(0, -1)) * x.hv(0, -1) + x.v(1, -1) * D(x.dxh(1, -1)) * x.hv(1, -1)) / 2.0
                            * (x.u(0, -1) + x.u(0, 0)) / 2.0 * D(x.luu(0, -1));
        rx = -(fx_p - fx_m + fy_p - fy_m)
             + (x.vort(0, 0) * x.hh(0, 0) * (x.v(1, 0) + x.v(0, 0))
                + x.vort(0, -1) * x.hh(0, -1) * (x.v(1, -1) + x.v(0, -1))) / 4.0;
    }
    {
        const double fv_c = x.v(0, 0) * D(x.dxh(0, 0)) * x.hv(0, 0);
        const double fy_p = (fv_c + x.v(0, 1) * D(x.dxh(0, 1)) * x.hv(0, 1)) / 2.0 * (x.v(0, 0) + x.v(0, 1)) / 2.0;
        const double fy_m = (fv_c + x.v(0, -1) * D(x.dxh(0, -1)) * x.hv(0, -1)) / 2.0 * (x.v(0, 0) + x.v(0, -1)) / 2.0;
        const double fx_p = (x.u(0, 0) * D(x.dyh(0, 0)) * x.hu(0, 0) + x.u(0, 1) * D(x.dyh(0, 1)) * x.hu(0, 1)) / 2.0
                            * (x.v(1, 0) + x.v(0, 0)) / 2.0;
        const double fx_m = (x.u(-1, 0) * D(x.dyh(-1, 0)) * x.hu(-1, 0) + x.u(-1, 1) * D(x.dyh(-1, 1)) * x.hu(-1, 1)) / 2.0
                            * (x.v(-1, 0) + x.v(0, 0)) / 2.0;
        ry = -(fx_p - fx_m + fy_p - fy_m)
             - (x.vort(0, 0) * x.hh(0, 0) * (x.u(0, 1) + x.u(0, 0))
                + x.vort(-1, 0) * x.hh(-1, 0) * (x.u(-1, 1) + x.u(-1, 0))) / 4.0;
    }
}

template <bool C> struct UvTrans {
    Geo I;
    Msk<C> lcu, lcv, luu; Met<C> dxh, dyh;
    const double *__restrict__ u, *__restrict__ v, *__restrict__ vort;
    const double *__restrict__ hu, *__restrict__ hv, *__restrict__ hh;
    double *__restrict__ RHSx, *__restrict__ RHSy;
    struct View {
        OCN_VIEW_PTR_COMMON(UvTrans)
        OCN_VIEW_LD(u) OCN_VIEW_LD(v) OCN_VIEW_LD(vort) OCN_VIEW_LD(hu) OCN_VIEW_LD(hv) OCN_VIEW_LD(hh)
        OCN_VIEW_LD(dxh) OCN_VIEW_LD(dyh) OCN_VIEW_LD(luu)
    };
    OCN_HD OCN_INLINE void eval(Pt c, double &rx, double &ry) const { uv_trans_math(View{*this, c}, rx, ry); }
    OCN_HD void operator()(int m, int n) const
    {
        const Pt c = I(m, n);
        double rx, ry;
        eval(c, rx, ry);
        if (ld(lcu, c) > 0.5f) st(RHSx, c, rx);
        if (ld(lcv, c) > 0.5f) st(RHSy, c, ry);
    }
};

// ------------------------------------------------------------------ a5 stress_components
// mixing.f90:14-58
// The reference kernel's u, v are the previous time level (the PSy layer passes ubrtrp /
// vbrtrp, sw_interface.f90:110-142); the view names them up / vp.
// The four real(4) metric ratios (dy/dx, dx/dy, dxb/dyb, dyb/dxb at the point) come from
// x.sratio(k): divided per point by the pointer views, read from the compact row tables (where
// Prepare divided the same row values) by the march views.
template <class X> OCN_HD OCN_INLINE void stress_components_math(const X &x, double &vt, double &vs)
{
    const float r1 = x.sratio(0);
    const float r2 = x.sratio(1);
    vt = D(r1) * (x.up(0, 0) / D(x.dyh(0, 0)) - x.up(-1, 0) / D(x.dyh(-1, 0)))
         - D(r2) * (x.vp(0, 0) / D(x.dxh(0, 0)) - x.vp(0, -1) / D(x.dxh(0, -1)));
    const float q1 = x.sratio(2);
    const float q2 = x.sratio(3);
    vs = D(q1) * (x.up(0, 1) / D(x.dxt(0, 1)) - x.up(0, 0) / D(x.dxt(0, 0)))
         + D(q2) * (x.vp(1, 0) / D(x.dyt(1, 0)) - x.vp(0, 0) / D(x.dyt(0, 0)));
}

template <bool C> struct StressComponents {
    Geo I;
    Msk<C> lu, luu; Met<C> dx, dy, dxt, dyt, dxh, dyh, dxb, dyb;
    const double *__restrict__ u, *__restrict__ v;
    double *__restrict__ str_t, *__restrict__ str_s;
    struct View {
        OCN_VIEW_PTR_COMMON(StressComponents)
        OCN_HD OCN_INLINE float sratio(int k) const   // mixing.f90:33-34, 43-44
        {
            return k == 0 ? ld(this->k.dy, c) / ld(this->k.dx, c) : k == 1 ? ld(this->k.dx, c) / ld(this->k.dy, c)
                 : k == 2 ? ld(this->k.dxb, c) / ld(this->k.dyb, c) : ld(this->k.dyb, c) / ld(this->k.dxb, c);
        }
        OCN_VIEW_LD_AS(up, u) OCN_VIEW_LD_AS(vp, v)
        OCN_VIEW_LD(dx) OCN_VIEW_LD(dy) OCN_VIEW_LD(dxt) OCN_VIEW_LD(dyt) OCN_VIEW_LD(dxh) OCN_VIEW_LD(dyh)
        OCN_VIEW_LD(dxb) OCN_VIEW_LD(dyb)
    };
    OCN_HD void operator()(int m, int n) const
    {
        const Pt c = I(m, n);
        double vt, vs;
        stress_components_math(View{*this, c}, vt, vs);
        if (ld(lu, c) > 0.5f) st(str_t, c, vt);
        if (ld(luu, c) > 0.5f) st(str_s, c, vs);
    }
};

// ------------------------------------------------------------------ a6 uv_diff2
// vel_ssh.f90:375-452
template <class X> OCN_HD OCN_INLINE void uv_diff2_math(const X &x, double &rx, double &ry)
{
    {
        const double muh_p = (x.mu(0, 0) + x.mu(1, 0) + x.mu(0, 1) + x.mu(1, 1)) / 4.0;
        const double muh_m = (x.mu(0, 0) + x.mu(1, 0) + x.mu(0, -1) + x.mu(1, -1)) / 4.0;
        const float dy2p = x.dy(1, 0) * x.dy(1, 0), dy2 = x.dy(0, 0) * x.dy(0, 0);
        const float dxb2 = x.dxb(0, 0) * x.dxb(0, 0), dxb2m = x.dxb(0, -1) * x.dxb(0, -1);
        rx = x.quot(D(dy2p) * x.mu(1, 0) * x.hq(1, 0) * x.str_t(1, 0) - D(dy2) * x.mu(0, 0) * x.hq(0, 0) * x.str_t(0, 0),
                    D(x.dyh(0, 0)), OCN_DYH, 0)
             + x.quot(D(dxb2) * muh_p * x.hh(0, 0) * x.str_s(0, 0) - D(dxb2m) * muh_m * x.hh(0, -1) * x.str_s(0, -1),
                      D(x.dxt(0, 0)), OCN_DXT, 0);
    }
    {
        const double muh_p = (x.mu(0, 0) + x.mu(1, 0) + x.mu(0, 1) + x.mu(1, 1)) / 4.0;
        const double muh_m = (x.mu(0, 0) + x.mu(-1, 0) + x.mu(0, 1) + x.mu(-1, 1)) / 4.0;
        const float dx2p = x.dx(0, 1) * x.dx(0, 1), dx2 = x.dx(0, 0) * x.dx(0, 0);
        const float dyb2 = x.dyb(0, 0) * x.dyb(0, 0), dyb2m = x.dyb(-1, 0) * x.dyb(-1, 0);
        ry = x.quot(-(D(dx2p) * x.mu(0, 1) * x.hq(0, 1) * x.str_t(0, 1) - D(dx2) * x.mu(0, 0) * x.hq(0, 0) * x.str_t(0, 0)),
                    D(x.dxh(0, 0)), OCN_DXH, 0)
             + x.quot(D(dyb2) * muh_p * x.hh(0, 0) * x.str_s(0, 0) - D(dyb2m) * muh_m * x.hh(-1, 0) * x.str_s(-1, 0),
                      D(x.dyt(0, 0)), OCN_DYT, 0);
    }
}

template <bool C> struct UvDiff2 {
    Geo I;
    Msk<C> lcu, lcv; Met<C> dx, dy, dxt, dyt, dxh, dyh, dxb, dyb;
    const double *__restrict__ mu, *__restrict__ str_t, *__restrict__ str_s, *__restrict__ hq, *__restrict__ hh;
    double *__restrict__ RHSx, *__restrict__ RHSy;
    struct View {
        OCN_VIEW_PTR_COMMON(UvDiff2)
        OCN_VIEW_LD(mu) OCN_VIEW_LD(str_t) OCN_VIEW_LD(str_s) OCN_VIEW_LD(hq) OCN_VIEW_LD(hh)
        OCN_VIEW_LD(dx) OCN_VIEW_LD(dy) OCN_VIEW_LD(dxt) OCN_VIEW_LD(dyt) OCN_VIEW_LD(dxh) OCN_VIEW_LD(dyh)
        OCN_VIEW_LD(dxb) OCN_VIEW_LD(dyb)
    };
    OCN_HD OCN_INLINE void eval(Pt c, double &rx, double &ry) const { uv_diff2_math(View{*this, c}, rx, ry); }
    OCN_HD void operator()(int m, int n) const
    {
        const Pt c = I(m, n);
        double rx, ry;
        eval(c, rx, ry);
        if (ld(lcu, c) > 0.5f) st(RHSx, c, rx);
        if (ld(lcv, c) > 0.5f) st(RHSy, c, ry);
    }
};

// ------------------------------------------------------------------ a7 sw_update_uv
// vel_ssh.f90:108-195.  rxa/rxd/rya/ryd: RHSx_adv, RHSx_dif, RHSy_adv, RHSy_dif at this point.
template <class X>
OCN_HD OCN_INLINE void sw_update_uv_math(const X &x, double rxa, double rxd, double rya, double ryd, double &un,
                                         double &vn)
{
    const double g = D(OCN_FREE_FALL_ACC);
    {
        const double bp = x.qtau(x.hhun(0, 0) * D(x.dxt(0, 0)) * D(x.dyh(0, 0)) / 2.0);
        const double bp0 = x.qtau(x.hhup(0, 0) * D(x.dxt(0, 0)) * D(x.dyh(0, 0)) / 2.0);
        const double slx = -(g * (x.ssh(1, 0) - x.ssh(0, 0)) * D(x.dyh(0, 0)) * x.hhu(0, 0));
        const float rd = x.rdis(0, 0) + x.rdis(1, 0);
        const double fric = D(rd) / 2.0 * x.ubrtrp(0, 0) * D(x.dxt(0, 0)) * D(x.dyh(0, 0)) * x.hhu(0, 0);
        const double c1 = D(x.rlh_s(0, 0)) * x.hhh(0, 0) * D(x.dxb(0, 0)) * D(x.dyb(0, 0)) * (x.vbrtr(1, 0) + x.vbrtr(0, 0));
        const double c2 = D(x.rlh_s(0, -1)) * x.hhh(0, -1) * D(x.dxb(0, -1)) * D(x.dyb(0, -1))
                          * (x.vbrtr(1, -1) + x.vbrtr(0, -1));
        const double grx = x.RHSx(0, 0) + slx + rxd + rxa - fric + (c1 + c2) / 4.0;
        un = (x.ubrtrp(0, 0) * bp0 + grx) / (bp);
    }
    {
        const double bp = x.qtau(x.hhvn(0, 0) * D(x.dyt(0, 0)) * D(x.dxh(0, 0)) / 2.0);
        const double bp0 = x.qtau(x.hhvp(0, 0) * D(x.dyt(0, 0)) * D(x.dxh(0, 0)) / 2.0);
        const double sly = -(g * (x.ssh(0, 1) - x.ssh(0, 0)) * D(x.dxh(0, 0)) * x.hhv(0, 0));
        const float rd = x.rdis(0, 0) + x.rdis(0, 1);
        const double fric = D(rd) / 2.0 * x.vbrtrp(0, 0) * D(x.dxh(0, 0)) * D(x.dyt(0, 0)) * x.hhv(0, 0);
        const double c1 = D(x.rlh_s(0, 0)) * x.hhh(0, 0) * D(x.dxb(0, 0)) * D(x.dyb(0, 0)) * (x.ubrtr(0, 1) + x.ubrtr(0, 0));
        const double c2 = D(x.rlh_s(-1, 0)) * x.hhh(-1, 0) * D(x.dxb(-1, 0)) * D(x.dyb(-1, 0))
                          * (x.ubrtr(-1, 1) + x.ubrtr(-1, 0));
        const double gry = x.RHSy(0, 0) + sly + ryd + rya - fric - (c1 + c2) / 4.0;
        vn = (x.vbrtrp(0, 0) * bp0 + gry) / (bp);
    }
}

template <bool C> struct SwUpdateUv {
    Geo I; double tau;
    Msk<C> lcu, lcv; Met<C> dxt, dyt, dxh, dyh, dxb, dyb;
    const double *__restrict__ hhu, *__restrict__ hhun, *__restrict__ hhup;
    const double *__restrict__ hhv, *__restrict__ hhvn, *__restrict__ hhvp;
    const double *__restrict__ hhh, *__restrict__ ssh;
    const double *__restrict__ ubrtr; double *__restrict__ ubrtrn; const double *__restrict__ ubrtrp;
    const double *__restrict__ vbrtr; double *__restrict__ vbrtrn; const double *__restrict__ vbrtrp;
    Met<C> rdis, rlh_s;
    const double *__restrict__ RHSx, *__restrict__ RHSy, *__restrict__ RHSx_adv, *__restrict__ RHSy_adv;
    const double *__restrict__ RHSx_dif, *__restrict__ RHSy_dif;
    struct View {
        OCN_VIEW_PTR_COMMON(SwUpdateUv)
        OCN_HD OCN_INLINE double qtau(double a) const { return a / k.tau; }
        OCN_VIEW_LD(hhu) OCN_VIEW_LD(hhun) OCN_VIEW_LD(hhup) OCN_VIEW_LD(hhv) OCN_VIEW_LD(hhvn) OCN_VIEW_LD(hhvp)
        OCN_VIEW_LD(hhh) OCN_VIEW_LD(ssh) OCN_VIEW_LD(ubrtr) OCN_VIEW_LD(ubrtrp) OCN_VIEW_LD(vbrtr) OCN_VIEW_LD(vbrtrp)
        OCN_VIEW_LD(RHSx) OCN_VIEW_LD(RHSy)
        OCN_VIEW_LD(dxt) OCN_VIEW_LD(dyt) OCN_VIEW_LD(dxh) OCN_VIEW_LD(dyh) OCN_VIEW_LD(dxb) OCN_VIEW_LD(dyb)
        OCN_VIEW_LD(rdis) OCN_VIEW_LD(rlh_s)
    };
    OCN_HD OCN_INLINE void eval(Pt c, double rxa, double rxd, double rya, double ryd, double &un, double &vn) const
    {
        sw_update_uv_math(View{*this, c}, rxa, rxd, rya, ryd, un, vn);
    }
    OCN_HD void operator()(int m, int n) const
    {
        const Pt c = I(m, n);
        double un, vn;
        eval(c, ld(RHSx_adv, c), ld(RHSx_dif, c), ld(RHSy_adv, c), ld(RHSy_dif, c), un, vn);
        if (ld(lcu, c) > 0.5f) st(ubrtrn, c, un);
        if (ld(lcv, c) > 0.5f) st(vbrtrn, c, vn);
    }
};

// ------------------------------------------------------------------ a8 sw_next_step
// vel_ssh.f90:197-245 (interior + halo ring).  asselin = the time filter of one field
// (vel_ssh.f90:230, 234, 238), in the reference's evaluation order.
OCN_HD OCN_INLINE double asselin(double x, double xn, double xp, double ts) { return x + ts * (xn - 2.0 * x + xp) / 2.0; }

template <bool C> struct SwNextStep {
    Geo I; double ts;
    Msk<C> lu, lcu, lcv;
    double *__restrict__ ssh, *__restrict__ sshn, *sshp;
    double *__restrict__ u, *__restrict__ un, *__restrict__ up;
    double *__restrict__ v, *__restrict__ vn, *__restrict__ vp;
    // where sshp / ubrtrp / vbrtrp are read from when they are filtered into other buffers
    // (ocn_ctx.hip recompute and one-pass steps with a8 work on the halo ring); nullptr = in place
    const double *sshp_in = nullptr, *up_in = nullptr, *vp_in = nullptr;
    // returns the ssh value after the update (for check_ssh_err)
    OCN_HD OCN_INLINE double step(Pt i) const
    {
        const double x = ld(ssh, i), xn = ld(sshn, i), xp = ld(sshp_in ? sshp_in : sshp, i);
        const double a = ld(u, i), an = ld(un, i), ap = ld(up_in ? up_in : up, i);
        const double b = ld(v, i), bn = ld(vn, i), bp = ld(vp_in ? vp_in : vp, i);
        const double fx = asselin(x, xn, xp, ts), fa = asselin(a, an, ap, ts), fb = asselin(b, bn, bp, ts);
        const bool bl = ld(lu, i) > 0.5f;
        if (bl) { st(sshp, i, fx); st(ssh, i, xn); }
        if (ld(lcu, i) > 0.5f) { st(up, i, fa); st(u, i, an); }
        if (ld(lcv, i) > 0.5f) { st(vp, i, fb); st(v, i, bn); }
        return bl ? xn : x;
    }
    OCN_HD void operator()(int m, int n) const { (void)step(I(m, n)); }
};

// ------------------------------------------------------------------ a9 hh_shift
// depth.f90:164-211 (interior + halo ring)
template <bool C> struct HhShift {
    Geo I; double ts;
    Msk<C> lu, llu, llv, luh;
    double *__restrict__ hq, *__restrict__ hqp, *__restrict__ hqn;
    double *__restrict__ hu, *__restrict__ hup, *__restrict__ hun;
    double *__restrict__ hv, *__restrict__ hvp, *__restrict__ hvn;
    double *__restrict__ hh, *__restrict__ hhp, *__restrict__ hhn;
    OCN_HD static OCN_INLINE void shift(bool mask, double *x, double *xp, const double *xn, Pt i, double ts)
    {
        const double a = ld(x, i), an = ld(xn, i), ap = ld(xp, i);
        const double f = a + ts * (an - 2.0 * a + ap) / 2.0;
        if (mask) { st(xp, i, f); st(x, i, an); }
    }
    OCN_HD void operator()(int m, int n) const
    {
        const Pt i = I(m, n);
        shift(ld(llu, i) > 0.5f, hu, hup, hun, i, ts);
        shift(ld(llv, i) > 0.5f, hv, hvp, hvn, i, ts);
        shift(ld(lu, i) > 0.5f, hq, hqp, hqn, i, ts);
        shift(ld(luh, i) > 0.5f, hh, hhp, hhn, i, ts);
    }
};

// ------------------------------------------------------------------ check_ssh_err
// vel_ssh.f90:40-67 as a device reduction (one atomic per thread with a bad point; the
// count only needs to be non-zero).
template <bool C> struct CheckSshErr {
    Geo I;
    Msk<C> lu; const double *__restrict__ ssh; int *nbad;
    OCN_HD void operator()(int m, int n) const
    {
        const Pt c = I(m, n);
        const double s = ld(ssh, c);
        if (ld(lu, c) > 0.5f && !(s < 10000.0 && s > -10000.0)) OCN_ATOMIC_INC(nbad);
    }
};

// ================================================================== tracers
// kernel/tracer/leapfrog_tracer.f90:13-92 tran_diff_fluxes_kernel (interior).  flux_gm = 0.0d0
// is still added (x + 0.0 turns -0.0 into +0.0, as the reference does).
template <bool C> struct TranDiffFluxes {
    Geo I; double factor_mu;
    Msk<C> lcu, lcv; Met<C> dxt, dyt, dxh, dyh;
    const double *__restrict__ hhu, *__restrict__ hhv, *__restrict__ ff;
    const double *__restrict__ uu, *__restrict__ vv, *__restrict__ mu;
    double *__restrict__ flux_x, *__restrict__ flux_y;
    OCN_HD void operator()(int m, int n) const
    {
        const Pt c = I(m, n), e = I.e(c), nn = I.n(c);
        const double fc = ld(ff, c), fe = ld(ff, e), fn = ld(ff, nn);
        const double mc = ld(mu, c);
        const double mux = (mc + ld(mu, e)) / 2.0 * factor_mu * D(ld(dyh, c)) / D(ld(dxt, c));
        const double fx = -ld(uu, c) * ld(hhu, c) * D(ld(dyh, c)) * (fc + fe) / 2.0 + mux * ld(hhu, c) * (fe - fc) + 0.0;
        const double muy = (mc + ld(mu, nn)) / 2.0 * factor_mu * D(ld(dxh, c)) / D(ld(dyt, c));
        const double fy = -ld(vv, c) * ld(hhv, c) * D(ld(dxh, c)) * (fc + fn) / 2.0 + muy * ld(hhv, c) * (fn - fc) + 0.0;
        if (ld(lcu, c) > 0.5f) st(flux_x, c, fx);
        if (ld(lcv, c) > 0.5f) st(flux_y, c, fy);
    }
};

// leapfrog_tracer.f90:94-136 tran_diff_tracer_kernel (interior)
template <bool C> struct TranDiffTracer {
    Geo I; double tau;
    Msk<C> lu; Met<C> dx, dy;
    const double *__restrict__ hhqn, *__restrict__ hhqp, *__restrict__ flux_x, *__restrict__ flux_y;
    const double *__restrict__ ffp; double *__restrict__ ffn;
    OCN_HD void operator()(int m, int n) const
    {
        const Pt c = I(m, n), w = I.w(c), s = I.s(c);
        const double bp = ld(hhqn, c) * D(ld(dx, c)) * D(ld(dy, c)) / tau / 2.0;
        const double bp0 = ld(hhqp, c) * D(ld(dx, c)) * D(ld(dy, c)) / tau / 2.0;
        const double rhs = ld(flux_x, c) - ld(flux_x, w) + ld(flux_y, c) - ld(flux_y, s);
        const double eta = bp0 * ld(ffp, c) + rhs;
        if (ld(lu, c) > 0.5f) st(ffn, c, eta / bp);
    }
};

// leapfrog_tracer.f90:138-168 tracer_next_step_kernel (interior + halo ring)
template <bool C> struct TracerNextStep {
    Geo I; double ts;
    Msk<C> lu;
    const double *__restrict__ ffn; double *__restrict__ ffp, *__restrict__ ff;
    OCN_HD void operator()(int m, int n) const
    {
        const Pt c = I(m, n);
        const double x = ld(ff, c), xn = ld(ffn, c), xp = ld(ffp, c);
        const double f = x + ts * (xn - 2.0 * x + xp) / 2.0;
        if (ld(lu, c) > 0.5f) { st(ffp, c, f); st(ff, c, xn); }
    }
};

// expl_tracer for ONE tracer in one launch over the interior, in one-pass sequences (the one-pass
// steps store no hh_init depths): control/tracer.f90:33-62 runs tran_diff_fluxes, tran_diff_tracer
// and tracer_next_step (leapfrog_tracer.f90:13-170) after each step, reading hh_init's hhu, hhv
// (level 0), hhq_n (= h_r) and hhq_p (= h_r + sshp * ffs, depth.f90:48-50) of the new state.  At an
// interior point under lu: the fluxes at the point and at its west / south neighbours -- formed
// here with tran_diff_fluxes' expressions where that stage stores them (the interior, and the halo
// points neighbour blocks own: what their exchange delivers), from hhu / hhv formed with hh_init's
// own interp_u / interp_v where hh_init stores them ([start-1, end]^2 under llu / llv), else the
// arrays' values (never written there) -- then ffn = (bp0 * ffp + rhs) / bp and the time filter.
// Writes ffn (the ffn buffer: it becomes ff with the role flip ff <-> ffn, ff := ffn of
// tracer_next_step) and the filtered ffp (into a second buffer: ffp is read at this point only,
// but the role pairs of every buffer trade places together).  Each value is the reference's
// expression on the same operands: bitwise the stages' results.
OCN_HD inline unsigned own_class(int v, int lo, int hi);
template <bool C> struct TracerStep {
    Geo I; double tau, ts, f, factor_mu;
    int nxs, nxe, nys, nye; unsigned own;   // interior; halo points neighbour blocks own (own_class bits)
    Interp<C> W;
    Msk<C> llu, llv, lcu, lcv;
    const double *__restrict__ ssh, *__restrict__ sshp, *__restrict__ h_r, *__restrict__ uu, *__restrict__ vv;
    const double *__restrict__ mu, *__restrict__ hhu, *__restrict__ hhv, *__restrict__ flux_x, *__restrict__ flux_y;
    const double *__restrict__ ff, *__restrict__ ffp;
    double *__restrict__ ffn_out, *__restrict__ ffp_out;
    struct View {
        const TracerStep &k; Pt c;
        OCN_VIEW_INTERP
    };
    OCN_HD OCN_INLINE bool owned(int m, int n) const
    {
        return (own >> (own_class(m, nxs, nxe) * 3u + own_class(n, nys, nye))) & 1u;
    }
    OCN_HD OCN_INLINE double a0(Pt c) const { return ld(h_r, c) + ld(ssh, c) * f; }   // hh_init level 0
    // hh_init's hhu / hhv at (m, n) (depth.f90:52-97 on [start-1, end]^2; the array's value elsewhere)
    OCN_HD OCN_INLINE double hu_at(int m, int n) const
    {
        const Pt c = I(m, n);
        const bool rng = owned(m, n) || (m >= nxs - 1 && m <= nxe && n >= nys - 1 && n <= nye);
        if (!(rng && ld(llu, c) > 0.5f)) return ld(hhu, c);
        return interp_u(View{*this, c}, a0(c), a0(I.e(c)));
    }
    OCN_HD OCN_INLINE double hv_at(int m, int n) const
    {
        const Pt c = I(m, n);
        const bool rng = owned(m, n) || (m >= nxs - 1 && m <= nxe && n >= nys - 1 && n <= nye);
        if (!(rng && ld(llv, c) > 0.5f)) return ld(hhv, c);
        return interp_v(View{*this, c}, a0(c), a0(I.n(c)));
    }
    // tran_diff_fluxes' flux_x / flux_y at (m, n): TranDiffFluxes' expressions where it stores them
    OCN_HD OCN_INLINE bool in_fluxes(int m, int n) const
    {
        return owned(m, n) || (m >= nxs && m <= nxe && n >= nys && n <= nye);
    }
    OCN_HD OCN_INLINE double fx_at(int m, int n) const
    {
        const Pt c = I(m, n), e = I.e(c);
        if (!(in_fluxes(m, n) && ld(lcu, c) > 0.5f)) return ld(flux_x, c);
        const double fc = ld(ff, c), fe = ld(ff, e), mc = ld(mu, c), hu = hu_at(m, n);
        const double mux = (mc + ld(mu, e)) / 2.0 * factor_mu * D(ld(W.dyh, c)) / D(ld(W.dxt, c));
        return -ld(uu, c) * hu * D(ld(W.dyh, c)) * (fc + fe) / 2.0 + mux * hu * (fe - fc) + 0.0;
    }
    OCN_HD OCN_INLINE double fy_at(int m, int n) const
    {
        const Pt c = I(m, n), nn = I.n(c);
        if (!(in_fluxes(m, n) && ld(lcv, c) > 0.5f)) return ld(flux_y, c);
        const double fc = ld(ff, c), fn = ld(ff, nn), mc = ld(mu, c), hv = hv_at(m, n);
        const double muy = (mc + ld(mu, nn)) / 2.0 * factor_mu * D(ld(W.dxh, c)) / D(ld(W.dyt, c));
        return -ld(vv, c) * hv * D(ld(W.dxh, c)) * (fc + fn) / 2.0 + muy * hv * (fn - fc) + 0.0;
    }
    OCN_HD void operator()(int m, int n) const
    {
        const Pt c = I(m, n);
        if (!(ld(W.lu, c) > 0.5f)) return;
        finish(m, n, fx_at(m, n), fx_at(m - 1, n), fy_at(m, n), fy_at(m, n - 1));
    }
    // the point's update from the four face fluxes (fx at m and m - 1, fy at n and n - 1), each
    // formed by fx_at / fy_at -- here, or by the thread of the neighbour point (k_tracer_tiles)
    OCN_HD void finish(int m, int n, double fxe, double fxw, double fyn, double fys) const
    {
        const Pt c = I(m, n);
        // tran_diff_tracer (leapfrog_tracer.f90:94-136): hhq_n = h_r, hhq_p = h_r + sshp * ffs
        const double hqn = ld(h_r, c), hqp = ld(h_r, c) + ld(sshp, c) * f;
        const double bp = hqn * D(ld(W.dx, c)) * D(ld(W.dy, c)) / tau / 2.0;
        const double bp0 = hqp * D(ld(W.dx, c)) * D(ld(W.dy, c)) / tau / 2.0;
        const double rhs = fxe - fxw + fyn - fys;
        const double xn = (bp0 * ld(ffp, c) + rhs) / bp;
        // tracer_next_step (leapfrog_tracer.f90:138-168)
        const double x = ld(ff, c), xp = ld(ffp, c);
        st(ffp_out, c, x + ts * (xn - 2.0 * x + xp) / 2.0);
        st(ffn_out, c, xn);
    }
};

// ================================================================== fused step groups
// The step's 10 stages regrouped into 4 launches with the same results, write sets and halo
// state as the stage-by-stage reference order (shallow_water.f90:36-92):
//   A  = a1 sw_update_ssh + a2 hh_update + a3 uv_trans_vort + a5 stress_components
//        (mutually independent: none reads another's output) -> one sync of their 7 fields.
//        hh_update's whole-array hqn = h_r + ssh is not stored: its only readers are hh_shift's
//        hq/hqp updates, which hh_init overwrites whole-array later in the same step.
//   B  = a4 uv_trans + a6 uv_diff2 + a7 sw_update_uv: sw_update_uv reads RHS*_adv / RHS*_dif
//        only at its own point, so they are passed in registers -> sync of u/v (and
//        uv_trans's lazy hh*_p sync, whose halos nothing in B reads).  They have no other
//        reader, so they are stored only when `full` (the last step of a call).
//   C1 = a8 sw_next_step + a9 hh_shift on the outer ring only (on [start-1,end]^2 its
//        outputs are dead: hh_init overwrites them) + check_ssh_err.
//   C2 = a10 hh_init (full = false except on the last step of a call) -> sync hhu/hhv/hhh.
// "reuse" steps (full_free_surface == 1, neither the first nor the last step of a call): a2's
// hun/hvn/hhn = interp(h_r + ssh) are bit for bit hh_init's hu/hv/hh = interp(h_r + ssh*1.0)
// of the previous step (same ssh -- nothing writes it in between -- same masks, same range,
// same arithmetic), so A skips a2 and B reads hhu/hhv where a7 reads hhu_n/hhv_n.  Their other
// readers only see them on the halo ring, whose results are overwritten before use (see
// ocn_ctx.hip one_step_fused); the last step of a call recomputes and stores them.
// "full" launches (the last step of every ocn_ctx_step call) store everything the reference
// stores; the others skip stores nobody reads (FusedB, HhInit), so the state after each call
// is the reference's bit for bit.
template <bool C> struct FusedA {
    int sx, sy;
    bool do_hh, do_vort, do_stress;
    SwUpdateSsh<C> a1; HhUpdate<C> a2; UvTransVort<C> a3; StressComponents<C> a5;
    OCN_HD void operator()(int m, int n) const
    {
        if (m >= sx && n >= sy) {
            a1(m, n);
            if (do_vort) a3(m, n);
            if (do_stress) a5(m, n);
        }
        if (do_hh) {
            const Pt c = a2.I(m, n);
            a2.interp(c, ld(a2.h_r, c) + ld(a2.sh, c));
        }
    }
};

template <bool C> struct FusedB {
    bool do_adv, do_dif, full;
    UvTrans<C> a4; UvDiff2<C> a6; SwUpdateUv<C> a7;
    OCN_HD void operator()(int m, int n) const
    {
        const Pt c = a7.I(m, n);
        double rxa, rya, rxd, ryd;
        if (do_adv) a4.eval(c, rxa, rya);
        else { rxa = ld(a7.RHSx_adv, c); rya = ld(a7.RHSy_adv, c); }
        if (do_dif) a6.eval(c, rxd, ryd);
        else { rxd = ld(a7.RHSx_dif, c); ryd = ld(a7.RHSy_dif, c); }
        double un, vn;
        a7.eval(c, rxa, rxd, rya, ryd, un, vn);
        const bool bu = ld(a7.lcu, c) > 0.5f, bv = ld(a7.lcv, c) > 0.5f;
        if (bu) {
            if (do_adv && full) st(a4.RHSx, c, rxa);
            if (do_dif && full) st(a6.RHSx, c, rxd);
            st(a7.ubrtrn, c, un);
        }
        if (bv) {
            if (do_adv && full) st(a4.RHSy, c, rya);
            if (do_dif && full) st(a6.RHSy, c, ryd);
            st(a7.vbrtrn, c, vn);
        }
    }
};

template <bool C> struct FusedC1 {
    int sx, ex, sy, ey;
    bool do_hh;
    int *nbad;
    SwNextStep<C> a8; HhShift<C> a9;
    OCN_HD void operator()(int m, int n) const
    {
        const Pt c = a8.I(m, n);
        const double x = a8.step(c);
        if (do_hh && (m == ex + 1 || n == ey + 1)) a9(m, n);
        if (nbad && m >= sx && m <= ex && n >= sy && n <= ey && ld(a8.lu, c) > 0.5f && !(x < 10000.0 && x > -10000.0))
            OCN_ATOMIC_INC(nbad);
    }
};

// ================================================================== compact static fields
// Mask bits: bit (1 << id) for the mask ids OCN_LU..OCN_LLV (0..6).  Row tables: for the
// metric ids OCN_DX..OCN_R_DISS, rows[(id - OCN_DX) * nrows + (n - bnd_y1)].
constexpr int kNumMasks = OCN_DX;                         // OCN_LU..OCN_LLV
constexpr int kNumRowFields = OCN_NUM_R4 - OCN_DX;        // OCN_DX..OCN_R_DISS
// then four per-row ratios for stress_components: dy/dx, dx/dy, dxb/dyb, dyb/dxb (real(4))
constexpr int kNumRowRatios = 4;
constexpr int kRowTable = kNumRowFields + kNumRowRatios;
// then, as doubles from float offset recip_offset(nrows) on, per row the correctly rounded
// reciprocals 1 / (double)g of the divisors the one-pass step divides by (its uniform-divisor
// division, sw_kernels.hip udiv): dxt, dyh, dxh, dyt, dxb, dyb, and the cell area dx*dy (real(4)
// product, as sw_update_ssh forms it)
enum { OCN_RC_DXT = 0, OCN_RC_DYH, OCN_RC_DXH, OCN_RC_DYT, OCN_RC_DXB, OCN_RC_DYB, OCN_RC_AREA, kNumRecips };
OCN_HD inline unsigned recip_offset(unsigned nrows) { return ((unsigned)kRowTable * nrows + 1u) & ~1u; }
inline size_t row_table_floats(unsigned nrows) { return recip_offset(nrows) + 2u * (unsigned)kNumRecips * nrows; }
enum { OCN_COMPACT_MASK_NOT_BINARY = 1, OCN_COMPACT_METRIC_NOT_ROW_CONSTANT = 2,
       OCN_COMPACT_RING_SEA = 4,     // not a failure: a8 / a9 write somewhere on the halo ring
       OCN_COMPACT_DIVISOR_RANGE = 8,     // not a failure: a divisor outside [2^-60, 2^60], or llu / llv / luh
                                          // set where lu_lv_init would not (no one-pass step)
       OCN_COMPACT_EDGE_RING_SEA = 16 };  // not a failure: a8 writes on the ring of a side no neighbour fills

// Which halo points of a block a neighbour block owns (they are its interior points, filled by the
// exchanges): bit (cx * 3 + cy) with cx = 0 / 1 / 2 for m < nx_start / inside / m > nx_end and cy
// likewise for n -- the 8 directions' bits set where that neighbour exists (ocn_ctx.hip own_mask).
OCN_HD inline unsigned own_class(int v, int lo, int hi) { return v < lo ? 0u : v > hi ? 2u : 1u; }

// One row of the compact row table (rows, nrows: sw_stencils.h kRowTable, recip_offset) from the
// row's metric values v[OCN_DX .. OCN_R_DISS]: the values, the stress ratios and the reciprocals,
// formed exactly as Prepare forms them; false if a divisor is outside udiv's range.
OCN_HD inline bool write_table_row(float *rows, unsigned nrows, unsigned r, const float *v)
{
    for (int k = 0; k < kNumRowFields; ++k) rows[(unsigned)k * nrows + r] = v[k];
    const float dx = v[0], dy = v[OCN_DY - OCN_DX], dxb = v[OCN_DXB - OCN_DX], dyb = v[OCN_DYB - OCN_DX];
    const float rat[kNumRowRatios] = {dy / dx, dx / dy, dxb / dyb, dyb / dxb};
    for (int k = 0; k < kNumRowRatios; ++k) rows[(unsigned)(kNumRowFields + k) * nrows + r] = rat[k];
    const float area = dx * dy;
    const float g[kNumRecips] = {v[OCN_DXT - OCN_DX], v[OCN_DYH - OCN_DX], v[OCN_DXH - OCN_DX], v[OCN_DYT - OCN_DX],
                                 dxb, dyb, area};
    double *rc = (double *)(rows + recip_offset(nrows));
    bool range = true;
    for (int k = 0; k < kNumRecips; ++k) {
        rc[(unsigned)k * nrows + r] = 1.0 / (double)g[k];
        range &= g[k] >= 0x1p-60f && g[k] <= 0x1p60f;   // positive; false for NaN
    }
    return range;
}

// Thread grid = whole bnd range.  Mask bytes everywhere; row values from column nx_start-1
// for the rows [ny_start-1, ny_end+1] the stencils read; every point of [nx_start-1,
// nx_end+1] on those rows must carry the same bit pattern, and every mask value must be
// exactly 0.0f or 1.0f -- otherwise `flags` records why and the caller keeps the 2-D path.
// OCN_COMPACT_RING_SEA also reports whether a8 (halo ring) or a9 (outer ring e+1, as fused C1
// runs it) has a point to write: if not, the role-flip steps skip their ring launch.
struct Prepare {
    Geo I; int ms, me, ns, ne;
    const float *__restrict__ r4[OCN_NUM_R4];
    uint8_t *__restrict__ bits; float *__restrict__ rows; unsigned nrows; int *flags;
    unsigned own;   // halo points neighbour blocks own (own_class bits): OCN_COMPACT_EDGE_RING_SEA tests the rest
    int bx2, by2;   // the arrays' last column / row
    OCN_HD void operator()(int m, int n) const
    {
        const Pt q = I(m, n);
        unsigned b = 0;
        bool bad = false;
        for (int id = 0; id < kNumMasks; ++id) {
            const uint32_t v = fbits(ld(r4[id], q));
            if (v == 0x3f800000u) b |= 1u << id;
            else if (v != 0u) bad = true;
        }
        st(bits, q, (uint8_t)b);
        if (bad) OCN_ATOMIC_OR(flags, (int)OCN_COMPACT_MASK_NOT_BINARY);
        {   // llu / llv / luh where lu_lv_init sets them (grid_kernels.f90:60-86): the one-pass step's
            // averages divide by the sea count without a zero case (sw_kernels.hip rcp_sea)
            auto sea = [&](int dm, int dn) {
                const int mm = m + dm, nn = n + dn;
                return mm <= bx2 && nn <= by2 && fbits(ld(r4[OCN_LU], I(mm, nn))) == 0x3f800000u;
            };
            const bool s00 = (b >> OCN_LU) & 1u, s10 = sea(1, 0), s01 = sea(0, 1), s11 = sea(1, 1);
            if ((((b >> OCN_LLU) & 1u) && !(s00 || s10)) || (((b >> OCN_LLV) & 1u) && !(s00 || s01)) ||
                (((b >> OCN_LUH) & 1u) && !(s00 || s10 || s01 || s11)))
                OCN_ATOMIC_OR(flags, (int)OCN_COMPACT_DIVISOR_RANGE);
        }
        if (m < ms || m > me || n < ns || n > ne) return;
        // a8 on the ring writes under lu / lcu / lcv; a9 (fused C1) on the outer ring e+1 under
        // lu / llu / llv / luh
        const unsigned a8m = (1u << OCN_LU) | (1u << OCN_LCU) | (1u << OCN_LCV);
        const unsigned a9m = (1u << OCN_LU) | (1u << OCN_LLU) | (1u << OCN_LLV) | (1u << OCN_LUH);
        const bool a8w = (m == ms || m == me || n == ns || n == ne) && (b & a8m);
        if (a8w || ((m == me || n == ne) && (b & a9m))) OCN_ATOMIC_OR(flags, (int)OCN_COMPACT_RING_SEA);
        // a8 on a ring point no neighbour block fills (a9 there: see ocn_ctx.hip k_halo_zero)
        const unsigned cls = own_class(m, ms + 1, me - 1) * 3u + own_class(n, ns + 1, ne - 1);
        if (a8w && !((own >> cls) & 1u)) OCN_ATOMIC_OR(flags, (int)OCN_COMPACT_EDGE_RING_SEA);
        const Pt q0 = I(ms, n);
        bool vary = false;
        float v[kNumRowFields];
        for (int k = 0; k < kNumRowFields; ++k) {
            v[k] = ld(r4[OCN_DX + k], q);
            vary |= fbits(v[k]) != fbits(ld(r4[OCN_DX + k], q0));
        }
        // the row values, and the same real(4) divisions as stress_components_math on them
        if (m == ms && !write_table_row(rows, nrows, q.r, v)) OCN_ATOMIC_OR(flags, (int)OCN_COMPACT_DIVISOR_RANGE);
        if (vary) OCN_ATOMIC_OR(flags, (int)OCN_COMPACT_METRIC_NOT_ROW_CONSTANT);
    }
};

// ------------------------------------------------------------------ role-flip coherence
// The role-flip step (ocn_ctx.hip one_step_fused) replaces a8's copies ssh := sshn,
// ubrtr := ubrtrn, vbrtr := vbrtrn by swapping the two buffers of each pair.  That is exact when
// the two buffers of a pair agree bit for bit at every point outside the pair's write set
// (interior points with lu / lcu / lcv; a1 and a7 write there, and a8 makes the pair equal there
// and on the ring): nothing else ever writes those points, so the agreement then holds for good.
// This functor (thread grid = bnd range, compact mask bytes) ORs 1 into *flags where it fails.
struct Coherence {
    Geo I; int ms, me, ns, ne;
    const uint8_t *__restrict__ bits;
    const double *a[3], *b[3];
    int *flags;
    OCN_HD void operator()(int m, int n) const
    {
        const Pt q = I(m, n);
        const bool inside = m >= ms && m <= me && n >= ns && n <= ne;
        const unsigned mb = ld(bits, q);
        const unsigned mask_bit[3] = {1u << OCN_LU, 1u << OCN_LCU, 1u << OCN_LCV};
        bool bad = false;
        for (int k = 0; k < 3; ++k) {
            if (inside && (mb & mask_bit[k])) continue;
            uint64_t x, y;
            const double va = ld(a[k], q), vb = ld(b[k], q);
            __builtin_memcpy(&x, &va, 8);
            __builtin_memcpy(&y, &vb, 8);
            bad |= x != y;
        }
        if (bad) OCN_ATOMIC_OR(flags, 1);
    }
};

// ------------------------------------------------------------------ functor makers
// Built from a block's field table (`ptr`, indexed by ocn_field_slot) -- used by the fused
// launches and by the host harness, so both run exactly the same functors over the same ranges.
inline int ocn_field_slot(int id) { return id < OCN_NUM_R4 ? id : OCN_NUM_R4 + (id - OCN_SSH); }
OCN_HD inline Geo geo(const ocn_block *b) { return Geo{b->bnd_x1, b->bnd_y1, (unsigned)b->pitch}; }
OCN_HD inline unsigned block_rows(const ocn_block *b) { return (unsigned)(b->bnd_y2 - b->bnd_y1 + 1); }

#ifndef OCN_RANGE_DEFINED   // also in ocn_internal.h
#define OCN_RANGE_DEFINED
struct Range { int m0, m1, n0, n1; };   // [m0, m1] x [n0, n1], 1-based global indices
#endif
inline Range range_interior(const ocn_block *b) { return {b->nx_start, b->nx_end, b->ny_start, b->ny_end}; }
inline Range range_ring(const ocn_block *b)
{
    return {b->nx_start - 1, b->nx_end + 1, b->ny_start - 1, b->ny_end + 1};
}
inline Range range_bnd(const ocn_block *b) { return {b->bnd_x1, b->bnd_x2, b->bnd_y1, b->bnd_y2}; }
inline Range range_fused_a(const ocn_block *b, const ocn_sw_params &sw, bool reuse = false)
{
    const int o = sw.full_free_surface > 0 && !reuse ? 1 : 0;
    return {b->nx_start - o, b->nx_end, b->ny_start - o, b->ny_end};
}

// Halo-overlap split of a launch range R (OCN_OPT_OVERLAP): the "inner" part is R clipped to
// a rectangle whose points neither read halo values nor produce values a neighbour receives;
// the "frame" is the rest of R, as up to four rectangles (bottom, top, left, right).
//   fused A, fused B, hh_init: inner = [start+1, end-1]^2 (stencils reach +-1 only inside the
//     interior; the interior's outer lines are what neighbours receive);
//   fused C1 (pointwise): inner = [start, end]^2 (only the halo ring reads exchanged values).
struct Rects {
    int m0[4], n0[4], w[4], h[4];
    int total() const { return w[0] * h[0] + w[1] * h[1] + w[2] * h[2] + w[3] * h[3]; }
};
inline Range range_clip(const Range &r, const Range &i)
{
    return {i.m0 > r.m0 ? i.m0 : r.m0, i.m1 < r.m1 ? i.m1 : r.m1, i.n0 > r.n0 ? i.n0 : r.n0,
            i.n1 < r.n1 ? i.n1 : r.n1};
}
inline bool range_empty(const Range &r) { return r.m1 < r.m0 || r.n1 < r.n0; }
inline Rects frame_rects(const Range &r, const Range &inner)
{
    Rects q{};
    const Range i = range_clip(r, inner);
    if (range_empty(r)) return q;
    if (range_empty(i)) {
        q.m0[0] = r.m0; q.n0[0] = r.n0; q.w[0] = r.m1 - r.m0 + 1; q.h[0] = r.n1 - r.n0 + 1;
        return q;
    }
    const int w = r.m1 - r.m0 + 1;
    q.m0[0] = r.m0; q.n0[0] = r.n0;     q.w[0] = w;             q.h[0] = i.n0 - r.n0;   // bottom
    q.m0[1] = r.m0; q.n0[1] = i.n1 + 1; q.w[1] = w;             q.h[1] = r.n1 - i.n1;   // top
    q.m0[2] = r.m0; q.n0[2] = i.n0;     q.w[2] = i.m0 - r.m0;   q.h[2] = i.n1 - i.n0 + 1;   // left
    q.m0[3] = i.m1 + 1; q.n0[3] = i.n0; q.w[3] = r.m1 - i.m1;   q.h[3] = i.n1 - i.n0 + 1;   // right
    return q;
}
// point t (0 <= t < total) of the frame
inline OCN_HD void frame_point(const Rects &q, int t, int &m, int &n)
{
    for (int k = 0; k < 4; ++k) {
        const int cnt = q.w[k] * q.h[k];
        if (t < cnt) { m = q.m0[k] + t % q.w[k]; n = q.n0[k] + t / q.w[k]; return; }
        t -= cnt;
    }
    m = n = 0;
}
inline Range inner_interior_shrunk(const ocn_block *b)
{
    return {b->nx_start + 1, b->nx_end - 1, b->ny_start + 1, b->ny_end - 1};
}

inline Coherence make_coherence(const ocn_block *b, void *const *ptr, const uint8_t *bits, int *flags)
{
    Coherence k{geo(b), b->nx_start, b->nx_end, b->ny_start, b->ny_end, bits, {}, {}, flags};
    const int pa[3] = {OCN_SSH, OCN_UBRTR, OCN_VBRTR}, pb[3] = {OCN_SSHN, OCN_UBRTRN, OCN_VBRTRN};
    for (int i = 0; i < 3; ++i) {
        k.a[i] = (const double *)ptr[ocn_field_slot(pa[i])];
        k.b[i] = (const double *)ptr[ocn_field_slot(pb[i])];
    }
    return k;
}

inline Prepare make_prepare(const ocn_block *b, void *const *ptr, uint8_t *bits, float *rows, int *flags,
                            unsigned own = 0)
{
    Prepare k{geo(b), b->nx_start - 1, b->nx_end + 1, b->ny_start - 1, b->ny_end + 1, {}, bits, rows,
              block_rows(b), flags, own, b->bnd_x2, b->bnd_y2};
    for (int id = 0; id < OCN_NUM_R4; ++id) k.r4[id] = (const float *)ptr[ocn_field_slot(id)];
    return k;
}

// Field table of one block, passed BY VALUE to the fused kernels, which build their stage
// functors on the device from it (the K* wrappers below): every distinct array pointer then
// occupies one kernel-argument slot and one SGPR pair, however many stages read it.  Slots:
// the SW fields (ocn_field_slot order), flux_x, flux_y, and ff1/ff1p/ff1n of ONE tracer.
// Masks / metrics come from the 2-D arrays (C = false) or from the compact tables (C = true).
constexpr int kTabSlots = OCN_NUM_R4 + OCN_NUM_R8 + 5;
OCN_HD inline int tab_slot(int id)
{
    return id < OCN_NUM_R4 ? id
           : id < OCN_TRACER_BASE ? OCN_NUM_R4 + (id - OCN_SSH)
                                  : OCN_NUM_R4 + OCN_NUM_R8 + 2 + (id - OCN_TRACER_BASE) % 3;
}
template <bool C> struct Tab {
    const void *p[kTabSlots];
    const uint8_t *bits; const float *rows; unsigned nrows;
    OCN_HD OCN_INLINE Msk<C> m(int id) const
    {
        if constexpr (C) return Msk<C>{bits, 1u << id};
        else return Msk<C>{(const float *)p[id]};
    }
    OCN_HD OCN_INLINE Met<C> g(int id) const
    {
        if constexpr (C) return Met<C>{rows + (unsigned)(id - OCN_DX) * nrows};
        else return Met<C>{(const float *)p[id]};
    }
    OCN_HD OCN_INLINE double *f(int id) const { return (double *)p[tab_slot(id)]; }
};
// host: the table of a block from its storage `ptr` (indexed by ocn_field_slot, `nptr` entries:
// SW fields, then flux_x, flux_y, ff1/ff1p/ff1n per tracer), holding tracer `tracer`'s fields
template <bool C>
inline Tab<C> make_tab(void *const *ptr, int nptr, const uint8_t *bits, const float *rows, unsigned nrows,
                       int tracer = 0)
{
    Tab<C> t{};
    for (int i = 0; i < OCN_NUM_R4 + OCN_NUM_R8 + 2 && i < nptr; ++i) t.p[i] = ptr[i];
    if (tracer > 0)
        for (int w = 0; w < 3; ++w) {
            const int slot = ocn_field_slot(OCN_FF1(tracer) + w);
            t.p[OCN_NUM_R4 + OCN_NUM_R8 + 2 + w] = slot < nptr ? ptr[slot] : nullptr;
        }
    t.bits = bits; t.rows = rows; t.nrows = nrows;
    return t;
}

template <bool C> OCN_HD inline Interp<C> make_interp(const Tab<C> &t)
{
    return Interp<C>{t.m(OCN_LU), t.g(OCN_DX), t.g(OCN_DY), t.g(OCN_DXT), t.g(OCN_DYT), t.g(OCN_DXH),
                     t.g(OCN_DYH), t.g(OCN_DXB), t.g(OCN_DYB)};
}
template <bool C> OCN_HD inline SwUpdateSsh<C> make_sw_update_ssh(const ocn_block *b, const Tab<C> &t, double tau)
{
    return SwUpdateSsh<C>{geo(b), tau, t.m(OCN_LU), t.g(OCN_DX), t.g(OCN_DY), t.g(OCN_DXH), t.g(OCN_DYH),
                          t.f(OCN_HHU), t.f(OCN_HHV), t.f(OCN_SSHN), t.f(OCN_SSHP), t.f(OCN_UBRTR), t.f(OCN_VBRTR)};
}
template <bool C> OCN_HD inline HhUpdate<C> make_hh_update(const ocn_block *b, const Tab<C> &t)
{
    return HhUpdate<C>{geo(b), b->nx_start - 1, b->nx_end, b->ny_start - 1, b->ny_end, make_interp(t),
                       t.m(OCN_LLU), t.m(OCN_LLV), t.m(OCN_LUH), t.f(OCN_HHQ_N), t.f(OCN_HHU_N), t.f(OCN_HHV_N),
                       t.f(OCN_HHH_N), t.f(OCN_SSH), t.f(OCN_HHQ_REST)};
}
template <bool C> OCN_HD inline UvTransVort<C> make_uv_trans_vort(const ocn_block *b, const Tab<C> &t)
{
    return UvTransVort<C>{geo(b), t.m(OCN_LUU), t.g(OCN_DXT), t.g(OCN_DYT), t.g(OCN_DXB), t.g(OCN_DYB),
                          t.f(OCN_UBRTR), t.f(OCN_VBRTR), t.f(OCN_VORT)};
}
template <bool C> OCN_HD inline UvTrans<C> make_uv_trans(const ocn_block *b, const Tab<C> &t)
{
    return UvTrans<C>{geo(b), t.m(OCN_LCU), t.m(OCN_LCV), t.m(OCN_LUU), t.g(OCN_DXH), t.g(OCN_DYH),
                      t.f(OCN_UBRTR), t.f(OCN_VBRTR), t.f(OCN_VORT), t.f(OCN_HHU), t.f(OCN_HHV), t.f(OCN_HHH),
                      t.f(OCN_RHSX_ADV), t.f(OCN_RHSY_ADV)};
}
template <bool C> OCN_HD inline StressComponents<C> make_stress_components(const ocn_block *b, const Tab<C> &t)
{
    return StressComponents<C>{geo(b), t.m(OCN_LU), t.m(OCN_LUU), t.g(OCN_DX), t.g(OCN_DY), t.g(OCN_DXT),
                               t.g(OCN_DYT), t.g(OCN_DXH), t.g(OCN_DYH), t.g(OCN_DXB), t.g(OCN_DYB),
                               t.f(OCN_UBRTRP), t.f(OCN_VBRTRP), t.f(OCN_STR_T), t.f(OCN_STR_S)};
}
template <bool C> OCN_HD inline UvDiff2<C> make_uv_diff2(const ocn_block *b, const Tab<C> &t)
{
    return UvDiff2<C>{geo(b), t.m(OCN_LCU), t.m(OCN_LCV), t.g(OCN_DX), t.g(OCN_DY), t.g(OCN_DXT), t.g(OCN_DYT),
                      t.g(OCN_DXH), t.g(OCN_DYH), t.g(OCN_DXB), t.g(OCN_DYB), t.f(OCN_MU), t.f(OCN_STR_T),
                      t.f(OCN_STR_S), t.f(OCN_HHQ), t.f(OCN_HHH), t.f(OCN_RHSX_DIF), t.f(OCN_RHSY_DIF)};
}
template <bool C> OCN_HD inline SwUpdateUv<C> make_sw_update_uv(const ocn_block *b, const Tab<C> &t, double tau)
{
    return SwUpdateUv<C>{geo(b), tau, t.m(OCN_LCU), t.m(OCN_LCV), t.g(OCN_DXT), t.g(OCN_DYT), t.g(OCN_DXH),
                         t.g(OCN_DYH), t.g(OCN_DXB), t.g(OCN_DYB), t.f(OCN_HHU), t.f(OCN_HHU_N), t.f(OCN_HHU_P),
                         t.f(OCN_HHV), t.f(OCN_HHV_N), t.f(OCN_HHV_P), t.f(OCN_HHH), t.f(OCN_SSH), t.f(OCN_UBRTR),
                         t.f(OCN_UBRTRN), t.f(OCN_UBRTRP), t.f(OCN_VBRTR), t.f(OCN_VBRTRN), t.f(OCN_VBRTRP),
                         t.g(OCN_R_DISS), t.g(OCN_RLH_S), t.f(OCN_RHSX), t.f(OCN_RHSY), t.f(OCN_RHSX_ADV),
                         t.f(OCN_RHSY_ADV), t.f(OCN_RHSX_DIF), t.f(OCN_RHSY_DIF)};
}
template <bool C> OCN_HD inline SwNextStep<C> make_sw_next_step(const ocn_block *b, const Tab<C> &t, double ts)
{
    return SwNextStep<C>{geo(b), ts, t.m(OCN_LU), t.m(OCN_LCU), t.m(OCN_LCV), t.f(OCN_SSH), t.f(OCN_SSHN),
                         t.f(OCN_SSHP), t.f(OCN_UBRTR), t.f(OCN_UBRTRN), t.f(OCN_UBRTRP), t.f(OCN_VBRTR),
                         t.f(OCN_VBRTRN), t.f(OCN_VBRTRP)};
}
template <bool C> OCN_HD inline HhShift<C> make_hh_shift(const ocn_block *b, const Tab<C> &t, double ts)
{
    return HhShift<C>{geo(b), ts, t.m(OCN_LU), t.m(OCN_LLU), t.m(OCN_LLV), t.m(OCN_LUH), t.f(OCN_HHQ),
                      t.f(OCN_HHQ_P), t.f(OCN_HHQ_N), t.f(OCN_HHU), t.f(OCN_HHU_P), t.f(OCN_HHU_N), t.f(OCN_HHV),
                      t.f(OCN_HHV_P), t.f(OCN_HHV_N), t.f(OCN_HHH), t.f(OCN_HHH_P), t.f(OCN_HHH_N)};
}
template <bool C> OCN_HD inline HhInit<C> make_hh_init(const ocn_block *b, const Tab<C> &t, int ffs, bool full)
{
    return HhInit<C>{geo(b), b->nx_start - 1, b->nx_end, b->ny_start - 1, b->ny_end, (double)ffs, full,
                     make_interp(t), t.m(OCN_LLU), t.m(OCN_LLV), t.m(OCN_LUH), t.f(OCN_HHQ), t.f(OCN_HHQ_P),
                     t.f(OCN_HHQ_N), t.f(OCN_HHU), t.f(OCN_HHU_P), t.f(OCN_HHU_N), t.f(OCN_HHV), t.f(OCN_HHV_P),
                     t.f(OCN_HHV_N), t.f(OCN_HHH), t.f(OCN_HHH_P), t.f(OCN_HHH_N), t.f(OCN_SSH), t.f(OCN_SSHP),
                     t.f(OCN_HHQ_REST)};
}
template <bool C> OCN_HD inline CheckSshErr<C> make_check_ssh_err(const ocn_block *b, const Tab<C> &t, int32_t *nbad)
{
    return CheckSshErr<C>{geo(b), t.m(OCN_LU), t.f(OCN_SSH), (int *)nbad};
}
// tracer k (1-based); the PSy layer passes factor_mu = 1.0d0 (tracer_interface.f90:47)
template <bool C>
OCN_HD inline TranDiffFluxes<C> make_tran_diff_fluxes(const ocn_block *b, const Tab<C> &t, int k, double factor_mu = 1.0)
{
    return TranDiffFluxes<C>{geo(b), factor_mu, t.m(OCN_LCU), t.m(OCN_LCV), t.g(OCN_DXT), t.g(OCN_DYT), t.g(OCN_DXH),
                             t.g(OCN_DYH), t.f(OCN_HHU), t.f(OCN_HHV), t.f(OCN_FF1(k)), t.f(OCN_UBRTR),
                             t.f(OCN_VBRTR), t.f(OCN_MU), t.f(OCN_FLUX_X), t.f(OCN_FLUX_Y)};
}
template <bool C> OCN_HD inline TranDiffTracer<C> make_tran_diff_tracer(const ocn_block *b, const Tab<C> &t, int k, double tau)
{
    return TranDiffTracer<C>{geo(b), tau, t.m(OCN_LU), t.g(OCN_DX), t.g(OCN_DY), t.f(OCN_HHQ_N), t.f(OCN_HHQ_P),
                             t.f(OCN_FLUX_X), t.f(OCN_FLUX_Y), t.f(OCN_FF1P(k)), t.f(OCN_FF1N(k))};
}
template <bool C> OCN_HD inline TracerNextStep<C> make_tracer_next_step(const ocn_block *b, const Tab<C> &t, int k, double ts)
{
    return TracerNextStep<C>{geo(b), ts, t.m(OCN_LU), t.f(OCN_FF1N(k)), t.f(OCN_FF1P(k)), t.f(OCN_FF1(k))};
}
template <bool C>
OCN_HD inline FusedA<C> make_fused_a(const ocn_block *b, const Tab<C> &t, const ocn_sw_params &sw, double tau, bool reuse = false)
{
    return FusedA<C>{b->nx_start, b->ny_start, sw.full_free_surface > 0 && !reuse, sw.trans_terms > 0, sw.ksw_lat > 0,
                     make_sw_update_ssh(b, t, tau), make_hh_update(b, t), make_uv_trans_vort(b, t),
                     make_stress_components(b, t)};
}
template <bool C>
OCN_HD inline FusedB<C> make_fused_b(const ocn_block *b, const Tab<C> &t, const ocn_sw_params &sw, double tau, bool full,
                       bool reuse = false)
{
    FusedB<C> k{sw.trans_terms > 0, sw.ksw_lat > 0, full, make_uv_trans(b, t), make_uv_diff2(b, t),
                make_sw_update_uv(b, t, tau)};
    if (reuse) { k.a7.hhun = k.a7.hhu; k.a7.hhvn = k.a7.hhv; }
    return k;
}
template <bool C>
OCN_HD inline FusedC1<C> make_fused_c1(const ocn_block *b, const Tab<C> &t, const ocn_sw_params &sw, int32_t *nbad,
                                       const double *sshp_in = nullptr, const double *up_in = nullptr,
                                       const double *vp_in = nullptr)
{
    FusedC1<C> k{b->nx_start, b->nx_end, b->ny_start, b->ny_end, sw.full_free_surface > 0, (int *)nbad,
                 make_sw_next_step(b, t, sw.time_smooth), make_hh_shift(b, t, sw.time_smooth)};
    k.a8.sshp_in = sshp_in;
    k.a8.up_in = up_in;
    k.a8.vp_in = vp_in;
    return k;
}

// ------------------------------------------------------------------ launch functors
// What the fused / tracer kernels receive: the block, its field table and the scalars.  The
// stage functors are built on the device inside operator(), so each distinct array is one
// kernel-argument pointer however many stages read it (no duplicated pointers, no SGPR spills).
template <bool C> struct KFusedA {
    ocn_block b; Tab<C> t; ocn_sw_params sw; double tau; bool reuse;
    OCN_HD void operator()(int m, int n) const { make_fused_a(&b, t, sw, tau, reuse)(m, n); }
};
template <bool C> struct KFusedB {
    ocn_block b; Tab<C> t; ocn_sw_params sw; double tau; bool full, reuse;
    OCN_HD void operator()(int m, int n) const { make_fused_b(&b, t, sw, tau, full, reuse)(m, n); }
};
template <bool C> struct KFusedC1 {
    ocn_block b; Tab<C> t; ocn_sw_params sw; int32_t *nbad;
    const double *sshp_in = nullptr, *up_in = nullptr, *vp_in = nullptr;   // see SwNextStep
    OCN_HD void operator()(int m, int n) const { make_fused_c1(&b, t, sw, nbad, sshp_in, up_in, vp_in)(m, n); }
};
template <bool C> struct KHhInit {
    ocn_block b; Tab<C> t; int ffs; bool full;
    OCN_HD void operator()(int m, int n) const { make_hh_init(&b, t, ffs, full)(m, n); }
};
template <bool C> struct KTranDiffFluxes {      // t holds the tracer's fields
    ocn_block b; Tab<C> t; double factor_mu;
    OCN_HD void operator()(int m, int n) const { make_tran_diff_fluxes(&b, t, 1, factor_mu)(m, n); }
};
template <bool C> struct KTranDiffTracer {
    ocn_block b; Tab<C> t; double tau;
    OCN_HD void operator()(int m, int n) const { make_tran_diff_tracer(&b, t, 1, tau)(m, n); }
};
template <bool C> struct KTracerNextStep {
    ocn_block b; Tab<C> t; double ts;
    OCN_HD void operator()(int m, int n) const { make_tracer_next_step(&b, t, 1, ts)(m, n); }
};
// TracerStep of the table's tracer (one-pass sequences), its outputs into ffn_out / ffp_out
template <bool C> struct KTracerStep {
    ocn_block b; Tab<C> t; double tau, ts; unsigned own; double *ffn_out, *ffp_out;
    OCN_HD TracerStep<C> make() const
    {
        return TracerStep<C>{geo(&b), tau, ts, 1.0, 1.0, b.nx_start, b.nx_end, b.ny_start, b.ny_end, own,
                             make_interp(t), t.m(OCN_LLU), t.m(OCN_LLV), t.m(OCN_LCU), t.m(OCN_LCV),
                             t.f(OCN_SSH), t.f(OCN_SSHP), t.f(OCN_HHQ_REST), t.f(OCN_UBRTR), t.f(OCN_VBRTR),
                             t.f(OCN_MU), t.f(OCN_HHU), t.f(OCN_HHV), t.f(OCN_FLUX_X), t.f(OCN_FLUX_Y),
                             t.f(OCN_FF1(1)), t.f(OCN_FF1P(1)), ffn_out, ffp_out};
    }
    OCN_HD void operator()(int m, int n) const { make()(m, n); }
};

}  // namespace ocn
