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
#include <hip/hip_runtime.h>

#include "ocn_internal.h"

namespace ocn {

// ------------------------------------------------------------------ launch scaffolding
template <typename Body>
__global__ __launch_bounds__(256) void k_range(int m0, int m1, int n0, int n1, Body body)
{
    const int m = m0 + (int)blockIdx.x * 64 + (int)threadIdx.x;
    if (m > m1) return;
    const int nb = n0 + (int)blockIdx.y * OCN_ROWS;
    const int ne = min(n1, nb + OCN_ROWS - 1);
    for (int n = nb + (int)threadIdx.y; n <= ne; n += 4) body(m, n);
}

template <typename Body>
static int launch_range(int m0, int m1, int n0, int n1, const Body &body, hipStream_t s)
{
    if (m1 < m0 || n1 < n0) return OCN_OK;
    dim3 block(64, 4);
    dim3 grid((unsigned)((m1 - m0 + 64) / 64), (unsigned)((n1 - n0 + OCN_ROWS) / OCN_ROWS));
    hipLaunchKernelGGL(k_range<Body>, grid, block, 0, s, m0, m1, n0, n1, body);
    return check_launch();
}

struct Geo {
    int bx1, by1;
    long p;
    __device__ __forceinline__ long operator()(int m, int n) const
    {
        return (long)(m - bx1) + (long)(n - by1) * p;
    }
};
static inline Geo geo(const ocn_block *b) { return Geo{b->bnd_x1, b->bnd_y1, (long)b->pitch}; }

#define D(x) ((double)(x))

// ------------------------------------------------------------------ a1 sw_update_ssh
// vel_ssh.f90:69-106
struct SwUpdateSsh {
    Geo I; double tau;
    const float *__restrict__ lu, *__restrict__ dx, *__restrict__ dy, *__restrict__ dxh, *__restrict__ dyh;
    const double *__restrict__ hhu, *__restrict__ hhv;
    double *__restrict__ sshn;
    const double *__restrict__ sshp, *__restrict__ ubrtr, *__restrict__ vbrtr;
    __device__ void operator()(int m, int n) const
    {
        const long c = I(m, n);
        if (!(lu[c] > 0.5f)) return;
        const long w = I(m - 1, n), s = I(m, n - 1);
        const double t1 = ubrtr[c] * hhu[c] * D(dyh[c]);
        const double t2 = ubrtr[w] * hhu[w] * D(dyh[w]);
        const double t3 = vbrtr[c] * hhv[c] * D(dxh[c]);
        const double t4 = vbrtr[s] * hhv[s] * D(dxh[s]);
        const float area = dx[c] * dy[c];
        const double div = (t1 - t2 + t3 - t4) / D(area);
        sshn[c] = sshp[c] + 2.0 * tau * (-div);
    }
};

// ------------------------------------------------------------------ T->U/V/H interpolation
// kernel/shallow_water/depth.f90:56-97; hq(m,n) = h_r + sh * f recomputed at each point
// (the whole-array assignment precedes the loop in the reference, so every read sees it).
struct Interp {
    Geo I;
    const float *__restrict__ lu, *__restrict__ dx, *__restrict__ dy;
    __device__ __forceinline__ double wt(double h, long i) const { return h * D(dx[i]) * D(dy[i]) * D(lu[i]); }
};

// ------------------------------------------------------------------ a2 hh_update
// depth.f90:101-162.  Thread grid = whole bnd range (hqn = h_r + sh, :129); the
// interpolation part runs on [start-1, end]^2.
struct HhUpdate {
    Geo I; int i0, i1, j0, j1;
    const float *__restrict__ lu, *__restrict__ llu, *__restrict__ llv, *__restrict__ luh;
    const float *__restrict__ dx, *__restrict__ dy, *__restrict__ dxt, *__restrict__ dyt;
    const float *__restrict__ dxh, *__restrict__ dyh, *__restrict__ dxb, *__restrict__ dyb;
    double *__restrict__ hqn, *__restrict__ hun, *__restrict__ hvn, *__restrict__ hhn;
    const double *__restrict__ sh, *__restrict__ h_r;
    // the [start-1, end]^2 interpolation part (depth.f90:134-160)
    __device__ __forceinline__ void interp(int m, int n, long c, double q00) const
    {
        const long e = I(m + 1, n), nn = I(m, n + 1), ne = I(m + 1, n + 1);
        const Interp W{I, lu, dx, dy};
        if (llu[c] > 0.5f) {
            const double slu = D(lu[c] + lu[e]);
            const double q10 = h_r[e] + sh[e];
            hun[c] = (W.wt(q00, c) + W.wt(q10, e)) / slu / D(dxt[c]) / D(dyh[c]);
        }
        if (llv[c] > 0.5f) {
            const double slu = D(lu[c] + lu[nn]);
            const double q01 = h_r[nn] + sh[nn];
            hvn[c] = (W.wt(q00, c) + W.wt(q01, nn)) / slu / D(dxh[c]) / D(dyt[c]);
        }
        if (luh[c] > 0.5f) {
            const double slu = D(lu[c] + lu[e] + lu[nn] + lu[ne]);
            const double q10 = h_r[e] + sh[e], q01 = h_r[nn] + sh[nn], q11 = h_r[ne] + sh[ne];
            hhn[c] = (W.wt(q00, c) + W.wt(q10, e) + W.wt(q01, nn) + W.wt(q11, ne)) / slu / D(dxb[c]) / D(dyb[c]);
        }
    }
    __device__ void operator()(int m, int n) const
    {
        const long c = I(m, n);
        const double q00 = h_r[c] + sh[c];
        hqn[c] = q00;
        if (m < i0 || m > i1 || n < j0 || n > j1) return;
        interp(m, n, c, q00);
    }
};

// ------------------------------------------------------------------ a10 hh_init
// depth.f90:14-99: hq = h_r + sh*ffs, hqp = h_r + shp*ffs, hqn = h_r (whole array), then the
// three levels interpolated on [start-1, end]^2.
struct HhInit {
    Geo I; int i0, i1, j0, j1; double f;
    const float *__restrict__ lu, *__restrict__ llu, *__restrict__ llv, *__restrict__ luh;
    const float *__restrict__ dx, *__restrict__ dy, *__restrict__ dxt, *__restrict__ dyt;
    const float *__restrict__ dxh, *__restrict__ dyh, *__restrict__ dxb, *__restrict__ dyb;
    double *__restrict__ hq, *__restrict__ hqp, *__restrict__ hqn;
    double *__restrict__ hu, *__restrict__ hup, *__restrict__ hun;
    double *__restrict__ hv, *__restrict__ hvp, *__restrict__ hvn;
    double *__restrict__ hh, *__restrict__ hhp, *__restrict__ hhn;
    const double *__restrict__ sh, *__restrict__ shp, *__restrict__ h_r;
    __device__ void operator()(int m, int n) const
    {
        const long c = I(m, n);
        const double r00 = h_r[c];
        const double a00 = r00 + sh[c] * f, b00 = r00 + shp[c] * f;
        hq[c] = a00; hqp[c] = b00; hqn[c] = r00;
        if (m < i0 || m > i1 || n < j0 || n > j1) return;
        const long e = I(m + 1, n), nn = I(m, n + 1), ne = I(m + 1, n + 1);
        const Interp W{I, lu, dx, dy};
        const bool bu = llu[c] > 0.5f, bv = llv[c] > 0.5f, bh = luh[c] > 0.5f;
        if (bu) {
            const double slu = D(lu[c] + lu[e]);
            const double r10 = h_r[e];
            const double a10 = r10 + sh[e] * f, b10 = r10 + shp[e] * f;
            const double x = D(dxt[c]), y = D(dyh[c]);
            hu[c] = (W.wt(a00, c) + W.wt(a10, e)) / slu / x / y;
            hup[c] = (W.wt(b00, c) + W.wt(b10, e)) / slu / x / y;
            hun[c] = (W.wt(r00, c) + W.wt(r10, e)) / slu / x / y;
        }
        if (bv) {
            const double slu = D(lu[c] + lu[nn]);
            const double r01 = h_r[nn];
            const double a01 = r01 + sh[nn] * f, b01 = r01 + shp[nn] * f;
            const double x = D(dxh[c]), y = D(dyt[c]);
            hv[c] = (W.wt(a00, c) + W.wt(a01, nn)) / slu / x / y;
            hvp[c] = (W.wt(b00, c) + W.wt(b01, nn)) / slu / x / y;
            hvn[c] = (W.wt(r00, c) + W.wt(r01, nn)) / slu / x / y;
        }
        if (bh) {
            const double slu = D(lu[c] + lu[e] + lu[nn] + lu[ne]);
            const double r10 = h_r[e], r01 = h_r[nn], r11 = h_r[ne];
            const double a10 = r10 + sh[e] * f, a01 = r01 + sh[nn] * f, a11 = r11 + sh[ne] * f;
            const double b10 = r10 + shp[e] * f, b01 = r01 + shp[nn] * f, b11 = r11 + shp[ne] * f;
            const double x = D(dxb[c]), y = D(dyb[c]);
            hh[c] = (W.wt(a00, c) + W.wt(a10, e) + W.wt(a01, nn) + W.wt(a11, ne)) / slu / x / y;
            hhp[c] = (W.wt(b00, c) + W.wt(b10, e) + W.wt(b01, nn) + W.wt(b11, ne)) / slu / x / y;
            hhn[c] = (W.wt(r00, c) + W.wt(r10, e) + W.wt(r01, nn) + W.wt(r11, ne)) / slu / x / y;
        }
    }
};

// ------------------------------------------------------------------ a3 uv_trans_vort
// vel_ssh.f90:247-281
struct UvTransVort {
    Geo I;
    const float *__restrict__ luu, *__restrict__ dxt, *__restrict__ dyt, *__restrict__ dxb, *__restrict__ dyb;
    const double *__restrict__ u, *__restrict__ v;
    double *__restrict__ vort;
    __device__ void operator()(int m, int n) const
    {
        const long c = I(m, n);
        if (!(luu[c] > 0.5f)) return;
        const long e = I(m + 1, n), nn = I(m, n + 1);
        const double a = v[e] * D(dyt[e]) - v[c] * D(dyt[c]);
        const double b = u[nn] * D(dxt[nn]) - u[c] * D(dxt[c]);
        const double d = (v[e] - v[c]) * D(dyb[c]) - (u[nn] - u[c]) * D(dxb[c]);
        vort[c] = a - b - d;
    }
};

// ------------------------------------------------------------------ a4 uv_trans
// vel_ssh.f90:283-373
struct UvTrans {
    Geo I;
    const float *__restrict__ lcu, *__restrict__ lcv, *__restrict__ luu, *__restrict__ dxh, *__restrict__ dyh;
    const double *__restrict__ u, *__restrict__ v, *__restrict__ vort;
    const double *__restrict__ hu, *__restrict__ hv, *__restrict__ hh;
    double *__restrict__ RHSx, *__restrict__ RHSy;
    __device__ __forceinline__ void eval(int m, int n, long c, bool bu, bool bv, double &rx, double &ry) const
    {
        const long e = I(m + 1, n), w = I(m - 1, n), nn = I(m, n + 1), s = I(m, n - 1);
        if (bu) {
            const long se = I(m + 1, n - 1);
            const double fu_c = u[c] * D(dyh[c]) * hu[c];
            const double fx_p = (fu_c + u[e] * D(dyh[e]) * hu[e]) / 2.0 * (u[c] + u[e]) / 2.0;
            const double fx_m = (fu_c + u[w] * D(dyh[w]) * hu[w]) / 2.0 * (u[c] + u[w]) / 2.0;
            const double fy_p = (v[c] * D(dxh[c]) * hv[c] + v[e] * D(dxh[e]) * hv[e]) / 2.0
                                * (u[nn] + u[c]) / 2.0 * D(luu[c]);
            const double fy_m = (v[s] * D(dxh[s]) * hv[s] + v[se] * D(dxh[se]) * hv[se]) / 2.0
                                * (u[s] + u[c]) / 2.0 * D(luu[s]);
            rx = -(fx_p - fx_m + fy_p - fy_m)
                 + (vort[c] * hh[c] * (v[e] + v[c]) + vort[s] * hh[s] * (v[se] + v[s])) / 4.0;
        }
        if (bv) {
            const long wn = I(m - 1, n + 1);
            const double fv_c = v[c] * D(dxh[c]) * hv[c];
            const double fy_p = (fv_c + v[nn] * D(dxh[nn]) * hv[nn]) / 2.0 * (v[c] + v[nn]) / 2.0;
            const double fy_m = (fv_c + v[s] * D(dxh[s]) * hv[s]) / 2.0 * (v[c] + v[s]) / 2.0;
            const double fx_p = (u[c] * D(dyh[c]) * hu[c] + u[nn] * D(dyh[nn]) * hu[nn]) / 2.0
                                * (v[e] + v[c]) / 2.0;
            const double fx_m = (u[w] * D(dyh[w]) * hu[w] + u[wn] * D(dyh[wn]) * hu[wn]) / 2.0
                                * (v[w] + v[c]) / 2.0;
            ry = -(fx_p - fx_m + fy_p - fy_m)
                 - (vort[c] * hh[c] * (u[nn] + u[c]) + vort[w] * hh[w] * (u[wn] + u[w])) / 4.0;
        }
    }
    __device__ void operator()(int m, int n) const
    {
        const long c = I(m, n);
        const bool bu = lcu[c] > 0.5f, bv = lcv[c] > 0.5f;
        if (!bu && !bv) return;
        double rx = 0.0, ry = 0.0;
        eval(m, n, c, bu, bv, rx, ry);
        if (bu) RHSx[c] = rx;
        if (bv) RHSy[c] = ry;
    }
};

// ------------------------------------------------------------------ a5 stress_components
// mixing.f90:14-58
struct StressComponents {
    Geo I;
    const float *__restrict__ lu, *__restrict__ luu, *__restrict__ dx, *__restrict__ dy;
    const float *__restrict__ dxt, *__restrict__ dyt, *__restrict__ dxh, *__restrict__ dyh;
    const float *__restrict__ dxb, *__restrict__ dyb;
    const double *__restrict__ u, *__restrict__ v;
    double *__restrict__ str_t, *__restrict__ str_s;
    __device__ void operator()(int m, int n) const
    {
        const long c = I(m, n);
        if (lu[c] > 0.5f) {
            const long w = I(m - 1, n), s = I(m, n - 1);
            const float r1 = dy[c] / dx[c];
            const float r2 = dx[c] / dy[c];
            str_t[c] = D(r1) * (u[c] / D(dyh[c]) - u[w] / D(dyh[w]))
                       - D(r2) * (v[c] / D(dxh[c]) - v[s] / D(dxh[s]));
        }
        if (luu[c] > 0.5f) {
            const long e = I(m + 1, n), nn = I(m, n + 1);
            const float r1 = dxb[c] / dyb[c];
            const float r2 = dyb[c] / dxb[c];
            str_s[c] = D(r1) * (u[nn] / D(dxt[nn]) - u[c] / D(dxt[c]))
                       + D(r2) * (v[e] / D(dyt[e]) - v[c] / D(dyt[c]));
        }
    }
};

// ------------------------------------------------------------------ a6 uv_diff2
// vel_ssh.f90:375-452
struct UvDiff2 {
    Geo I;
    const float *__restrict__ lcu, *__restrict__ lcv, *__restrict__ dx, *__restrict__ dy;
    const float *__restrict__ dxt, *__restrict__ dyt, *__restrict__ dxh, *__restrict__ dyh;
    const float *__restrict__ dxb, *__restrict__ dyb;
    const double *__restrict__ mu, *__restrict__ str_t, *__restrict__ str_s, *__restrict__ hq, *__restrict__ hh;
    double *__restrict__ RHSx, *__restrict__ RHSy;
    __device__ __forceinline__ void eval(int m, int n, long c, bool bu, bool bv, double &rx, double &ry) const
    {
        const long e = I(m + 1, n), nn = I(m, n + 1), ne = I(m + 1, n + 1);
        if (bu) {
            const long s = I(m, n - 1), se = I(m + 1, n - 1);
            const double muh_p = (mu[c] + mu[e] + mu[nn] + mu[ne]) / 4.0;
            const double muh_m = (mu[c] + mu[e] + mu[s] + mu[se]) / 4.0;
            const float dy2p = dy[e] * dy[e], dy2 = dy[c] * dy[c];
            const float dxb2 = dxb[c] * dxb[c], dxb2m = dxb[s] * dxb[s];
            rx = (D(dy2p) * mu[e] * hq[e] * str_t[e] - D(dy2) * mu[c] * hq[c] * str_t[c]) / D(dyh[c])
                 + (D(dxb2) * muh_p * hh[c] * str_s[c] - D(dxb2m) * muh_m * hh[s] * str_s[s]) / D(dxt[c]);
        }
        if (bv) {
            const long w = I(m - 1, n), wn = I(m - 1, n + 1);
            const double muh_p = (mu[c] + mu[e] + mu[nn] + mu[ne]) / 4.0;
            const double muh_m = (mu[c] + mu[w] + mu[nn] + mu[wn]) / 4.0;
            const float dx2p = dx[nn] * dx[nn], dx2 = dx[c] * dx[c];
            const float dyb2 = dyb[c] * dyb[c], dyb2m = dyb[w] * dyb[w];
            ry = -(D(dx2p) * mu[nn] * hq[nn] * str_t[nn] - D(dx2) * mu[c] * hq[c] * str_t[c]) / D(dxh[c])
                 + (D(dyb2) * muh_p * hh[c] * str_s[c] - D(dyb2m) * muh_m * hh[w] * str_s[w]) / D(dyt[c]);
        }
    }
    __device__ void operator()(int m, int n) const
    {
        const long c = I(m, n);
        const bool bu = lcu[c] > 0.5f, bv = lcv[c] > 0.5f;
        if (!bu && !bv) return;
        double rx = 0.0, ry = 0.0;
        eval(m, n, c, bu, bv, rx, ry);
        if (bu) RHSx[c] = rx;
        if (bv) RHSy[c] = ry;
    }
};

// ------------------------------------------------------------------ a7 sw_update_uv
// vel_ssh.f90:108-195
struct SwUpdateUv {
    Geo I; double tau;
    const float *__restrict__ lcu, *__restrict__ lcv, *__restrict__ dxt, *__restrict__ dyt;
    const float *__restrict__ dxh, *__restrict__ dyh, *__restrict__ dxb, *__restrict__ dyb;
    const double *__restrict__ hhu, *__restrict__ hhun, *__restrict__ hhup;
    const double *__restrict__ hhv, *__restrict__ hhvn, *__restrict__ hhvp;
    const double *__restrict__ hhh, *__restrict__ ssh;
    const double *__restrict__ ubrtr; double *__restrict__ ubrtrn; const double *__restrict__ ubrtrp;
    const double *__restrict__ vbrtr; double *__restrict__ vbrtrn; const double *__restrict__ vbrtrp;
    const float *__restrict__ rdis, *__restrict__ rlh_s;
    const double *__restrict__ RHSx, *__restrict__ RHSy, *__restrict__ RHSx_adv, *__restrict__ RHSy_adv;
    const double *__restrict__ RHSx_dif, *__restrict__ RHSy_dif;
    // rxa/rxd/rya/ryd: RHSx_adv, RHSx_dif, RHSy_adv, RHSy_dif at this point (used under lcu / lcv)
    __device__ __forceinline__ void eval(int m, int n, long c, bool bu, bool bv, double rxa, double rxd,
                                         double rya, double ryd) const
    {
        const double g = D(OCN_FREE_FALL_ACC);
        if (bu) {
            const long e = I(m + 1, n), s = I(m, n - 1), se = I(m + 1, n - 1);
            const double bp = hhun[c] * D(dxt[c]) * D(dyh[c]) / 2.0 / tau;
            const double bp0 = hhup[c] * D(dxt[c]) * D(dyh[c]) / 2.0 / tau;
            const double slx = -(g * (ssh[e] - ssh[c]) * D(dyh[c]) * hhu[c]);
            const float rd = rdis[c] + rdis[e];
            const double fric = D(rd) / 2.0 * ubrtrp[c] * D(dxt[c]) * D(dyh[c]) * hhu[c];
            const double c1 = D(rlh_s[c]) * hhh[c] * D(dxb[c]) * D(dyb[c]) * (vbrtr[e] + vbrtr[c]);
            const double c2 = D(rlh_s[s]) * hhh[s] * D(dxb[s]) * D(dyb[s]) * (vbrtr[se] + vbrtr[s]);
            const double grx = RHSx[c] + slx + rxd + rxa - fric + (c1 + c2) / 4.0;
            ubrtrn[c] = (ubrtrp[c] * bp0 + grx) / (bp);
        }
        if (bv) {
            const long nn = I(m, n + 1), w = I(m - 1, n), wn = I(m - 1, n + 1);
            const double bp = hhvn[c] * D(dyt[c]) * D(dxh[c]) / 2.0 / tau;
            const double bp0 = hhvp[c] * D(dyt[c]) * D(dxh[c]) / 2.0 / tau;
            const double sly = -(g * (ssh[nn] - ssh[c]) * D(dxh[c]) * hhv[c]);
            const float rd = rdis[c] + rdis[nn];
            const double fric = D(rd) / 2.0 * vbrtrp[c] * D(dxh[c]) * D(dyt[c]) * hhv[c];
            const double c1 = D(rlh_s[c]) * hhh[c] * D(dxb[c]) * D(dyb[c]) * (ubrtr[nn] + ubrtr[c]);
            const double c2 = D(rlh_s[w]) * hhh[w] * D(dxb[w]) * D(dyb[w]) * (ubrtr[wn] + ubrtr[w]);
            const double gry = RHSy[c] + sly + ryd + rya - fric - (c1 + c2) / 4.0;
            vbrtrn[c] = (vbrtrp[c] * bp0 + gry) / (bp);
        }
    }
    __device__ void operator()(int m, int n) const
    {
        const long c = I(m, n);
        const bool bu = lcu[c] > 0.5f, bv = lcv[c] > 0.5f;
        if (!bu && !bv) return;
        double rxa = 0.0, rxd = 0.0, rya = 0.0, ryd = 0.0;
        if (bu) { rxa = RHSx_adv[c]; rxd = RHSx_dif[c]; }
        if (bv) { rya = RHSy_adv[c]; ryd = RHSy_dif[c]; }
        eval(m, n, c, bu, bv, rxa, rxd, rya, ryd);
    }
};

// ------------------------------------------------------------------ a8 sw_next_step
// vel_ssh.f90:197-245 (interior + halo ring)
struct SwNextStep {
    Geo I; double ts;
    const float *__restrict__ lu, *__restrict__ lcu, *__restrict__ lcv;
    double *__restrict__ ssh, *__restrict__ sshn, *__restrict__ sshp;
    double *__restrict__ u, *__restrict__ un, *__restrict__ up;
    double *__restrict__ v, *__restrict__ vn, *__restrict__ vp;
    __device__ void operator()(int m, int n) const
    {
        const long i = I(m, n);
        if (lu[i] > 0.5f) {
            const double x = ssh[i], xn = sshn[i];
            sshp[i] = x + ts * (xn - 2.0 * x + sshp[i]) / 2.0;
            ssh[i] = xn;
        }
        if (lcu[i] > 0.5f) {
            const double x = u[i], xn = un[i];
            up[i] = x + ts * (xn - 2.0 * x + up[i]) / 2.0;
            u[i] = xn;
        }
        if (lcv[i] > 0.5f) {
            const double x = v[i], xn = vn[i];
            vp[i] = x + ts * (xn - 2.0 * x + vp[i]) / 2.0;
            v[i] = xn;
        }
    }
};

// ------------------------------------------------------------------ a9 hh_shift
// depth.f90:164-211 (interior + halo ring)
struct HhShift {
    Geo I; double ts;
    const float *__restrict__ lu, *__restrict__ llu, *__restrict__ llv, *__restrict__ luh;
    double *__restrict__ hq, *__restrict__ hqp, *__restrict__ hqn;
    double *__restrict__ hu, *__restrict__ hup, *__restrict__ hun;
    double *__restrict__ hv, *__restrict__ hvp, *__restrict__ hvn;
    double *__restrict__ hh, *__restrict__ hhp, *__restrict__ hhn;
    __device__ static __forceinline__ void shift(double *x, double *xp, const double *xn, long i, double ts)
    {
        const double a = x[i], an = xn[i];
        xp[i] = a + ts * (an - 2.0 * a + xp[i]) / 2.0;
        x[i] = an;
    }
    __device__ void operator()(int m, int n) const
    {
        const long i = I(m, n);
        if (llu[i] > 0.5f) shift(hu, hup, hun, i, ts);
        if (llv[i] > 0.5f) shift(hv, hvp, hvn, i, ts);
        if (lu[i] > 0.5f) shift(hq, hqp, hqn, i, ts);
        if (luh[i] > 0.5f) shift(hh, hhp, hhn, i, ts);
    }
};

// ------------------------------------------------------------------ check_ssh_err
// vel_ssh.f90:40-67 as a device reduction (one atomic per wave with bad points).
struct CheckSshErr {
    Geo I;
    const float *__restrict__ lu; const double *__restrict__ ssh; int *nbad;
    __device__ void operator()(int m, int n) const
    {
        const long c = I(m, n);
        bool bad = false;
        if (lu[c] > 0.5f) {
            const double s = ssh[c];
            bad = !(s < 10000.0 && s > -10000.0);
        }
        if (bad) atomicAdd(nbad, 1);
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
//        only at its own point, so they are passed in registers (and still stored) -> sync
//        of u/v (and uv_trans's lazy hh*_p sync, whose halos nothing in B reads).
//   C1 = a8 sw_next_step + a9 hh_shift on the outer ring only (on [start-1,end]^2 its
//        outputs are dead: hh_init overwrites them) + check_ssh_err.
//   C2 = a10 hh_init (unchanged) -> sync hhu/hhv/hhh.
struct FusedA {
    int sx, sy;
    bool do_hh, do_vort, do_stress;
    SwUpdateSsh a1; HhUpdate a2; UvTransVort a3; StressComponents a5;
    __device__ void operator()(int m, int n) const
    {
        if (m >= sx && n >= sy) {
            a1(m, n);
            if (do_vort) a3(m, n);
            if (do_stress) a5(m, n);
        }
        if (do_hh) {
            const long c = a2.I(m, n);
            a2.interp(m, n, c, a2.h_r[c] + a2.sh[c]);
        }
    }
};

struct FusedB {
    bool do_adv, do_dif;
    UvTrans a4; UvDiff2 a6; SwUpdateUv a7;
    __device__ void operator()(int m, int n) const
    {
        const long c = a7.I(m, n);
        const bool bu = a7.lcu[c] > 0.5f, bv = a7.lcv[c] > 0.5f;
        if (!bu && !bv) return;
        double rxa = 0.0, rya = 0.0, rxd = 0.0, ryd = 0.0;
        if (do_adv) {
            a4.eval(m, n, c, bu, bv, rxa, rya);
            if (bu) a4.RHSx[c] = rxa;
            if (bv) a4.RHSy[c] = rya;
        } else {
            if (bu) rxa = a7.RHSx_adv[c];
            if (bv) rya = a7.RHSy_adv[c];
        }
        if (do_dif) {
            a6.eval(m, n, c, bu, bv, rxd, ryd);
            if (bu) a6.RHSx[c] = rxd;
            if (bv) a6.RHSy[c] = ryd;
        } else {
            if (bu) rxd = a7.RHSx_dif[c];
            if (bv) ryd = a7.RHSy_dif[c];
        }
        a7.eval(m, n, c, bu, bv, rxa, rxd, rya, ryd);
    }
};

struct FusedC1 {
    int sx, ex, sy, ey;
    bool do_hh;
    int *nbad;
    SwNextStep a8; HhShift a9;
    __device__ void operator()(int m, int n) const
    {
        a8(m, n);
        if (do_hh && (m == ex + 1 || n == ey + 1)) a9(m, n);
        if (nbad && m >= sx && m <= ex && n >= sy && n <= ey) {
            const long c = a8.I(m, n);
            if (a8.lu[c] > 0.5f) {
                const double x = a8.ssh[c];
                if (!(x < 10000.0 && x > -10000.0)) atomicAdd(nbad, 1);
            }
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
#define F4(id) ((const float *)ptr[field_slot(id)])
#define F8(id) ((double *)ptr[field_slot(id)])

static SwUpdateSsh mk_a1(const ocn_block *b, void *const *ptr, double tau)
{
    return SwUpdateSsh{geo(b), tau, F4(OCN_LU), F4(OCN_DX), F4(OCN_DY), F4(OCN_DXH), F4(OCN_DYH), F8(OCN_HHU),
                       F8(OCN_HHV), F8(OCN_SSHN), F8(OCN_SSHP), F8(OCN_UBRTR), F8(OCN_VBRTR)};
}
static HhUpdate mk_a2(const ocn_block *b, void *const *ptr)
{
    return HhUpdate{geo(b), b->nx_start - 1, b->nx_end, b->ny_start - 1, b->ny_end,
                    F4(OCN_LU), F4(OCN_LLU), F4(OCN_LLV), F4(OCN_LUH), F4(OCN_DX), F4(OCN_DY), F4(OCN_DXT),
                    F4(OCN_DYT), F4(OCN_DXH), F4(OCN_DYH), F4(OCN_DXB), F4(OCN_DYB), F8(OCN_HHQ_N), F8(OCN_HHU_N),
                    F8(OCN_HHV_N), F8(OCN_HHH_N), F8(OCN_SSH), F8(OCN_HHQ_REST)};
}

int launch_fused_a(const ocn_block *b, void *const *ptr, const ocn_sw_params &sw, double tau, hipStream_t s)
{
    RC_K(check_block(b));
    FusedA k{b->nx_start, b->ny_start, sw.full_free_surface > 0, sw.trans_terms > 0, sw.ksw_lat > 0,
             mk_a1(b, ptr, tau), mk_a2(b, ptr),
             UvTransVort{geo(b), F4(OCN_LUU), F4(OCN_DXT), F4(OCN_DYT), F4(OCN_DXB), F4(OCN_DYB), F8(OCN_UBRTR),
                         F8(OCN_VBRTR), F8(OCN_VORT)},
             StressComponents{geo(b), F4(OCN_LU), F4(OCN_LUU), F4(OCN_DX), F4(OCN_DY), F4(OCN_DXT), F4(OCN_DYT),
                              F4(OCN_DXH), F4(OCN_DYH), F4(OCN_DXB), F4(OCN_DYB), F8(OCN_UBRTRP), F8(OCN_VBRTRP),
                              F8(OCN_STR_T), F8(OCN_STR_S)}};
    const int o = k.do_hh ? 1 : 0;
    return launch_range(b->nx_start - o, b->nx_end, b->ny_start - o, b->ny_end, k, s);
}

int launch_fused_b(const ocn_block *b, void *const *ptr, const ocn_sw_params &sw, double tau, hipStream_t s)
{
    RC_K(check_block(b));
    FusedB k{sw.trans_terms > 0, sw.ksw_lat > 0,
             UvTrans{geo(b), F4(OCN_LCU), F4(OCN_LCV), F4(OCN_LUU), F4(OCN_DXH), F4(OCN_DYH), F8(OCN_UBRTR),
                     F8(OCN_VBRTR), F8(OCN_VORT), F8(OCN_HHU), F8(OCN_HHV), F8(OCN_HHH), F8(OCN_RHSX_ADV),
                     F8(OCN_RHSY_ADV)},
             UvDiff2{geo(b), F4(OCN_LCU), F4(OCN_LCV), F4(OCN_DX), F4(OCN_DY), F4(OCN_DXT), F4(OCN_DYT), F4(OCN_DXH),
                     F4(OCN_DYH), F4(OCN_DXB), F4(OCN_DYB), F8(OCN_MU), F8(OCN_STR_T), F8(OCN_STR_S), F8(OCN_HHQ),
                     F8(OCN_HHH), F8(OCN_RHSX_DIF), F8(OCN_RHSY_DIF)},
             SwUpdateUv{geo(b), tau, F4(OCN_LCU), F4(OCN_LCV), F4(OCN_DXT), F4(OCN_DYT), F4(OCN_DXH), F4(OCN_DYH),
                        F4(OCN_DXB), F4(OCN_DYB), F8(OCN_HHU), F8(OCN_HHU_N), F8(OCN_HHU_P), F8(OCN_HHV),
                        F8(OCN_HHV_N), F8(OCN_HHV_P), F8(OCN_HHH), F8(OCN_SSH), F8(OCN_UBRTR), F8(OCN_UBRTRN),
                        F8(OCN_UBRTRP), F8(OCN_VBRTR), F8(OCN_VBRTRN), F8(OCN_VBRTRP), F4(OCN_R_DISS),
                        F4(OCN_RLH_S), F8(OCN_RHSX), F8(OCN_RHSY), F8(OCN_RHSX_ADV), F8(OCN_RHSY_ADV),
                        F8(OCN_RHSX_DIF), F8(OCN_RHSY_DIF)}};
    return launch_range(b->nx_start, b->nx_end, b->ny_start, b->ny_end, k, s);
}

int launch_fused_c1(const ocn_block *b, void *const *ptr, const ocn_sw_params &sw, int32_t *nbad, hipStream_t s)
{
    RC_K(check_block(b));
    FusedC1 k{b->nx_start, b->nx_end, b->ny_start, b->ny_end, sw.full_free_surface > 0, (int *)nbad,
              SwNextStep{geo(b), sw.time_smooth, F4(OCN_LU), F4(OCN_LCU), F4(OCN_LCV), F8(OCN_SSH), F8(OCN_SSHN),
                         F8(OCN_SSHP), F8(OCN_UBRTR), F8(OCN_UBRTRN), F8(OCN_UBRTRP), F8(OCN_VBRTR),
                         F8(OCN_VBRTRN), F8(OCN_VBRTRP)},
              HhShift{geo(b), sw.time_smooth, F4(OCN_LU), F4(OCN_LLU), F4(OCN_LLV), F4(OCN_LUH), F8(OCN_HHQ),
                      F8(OCN_HHQ_P), F8(OCN_HHQ_N), F8(OCN_HHU), F8(OCN_HHU_P), F8(OCN_HHU_N), F8(OCN_HHV),
                      F8(OCN_HHV_P), F8(OCN_HHV_N), F8(OCN_HHH), F8(OCN_HHH_P), F8(OCN_HHH_N)}};
    return launch_range(b->nx_start - 1, b->nx_end + 1, b->ny_start - 1, b->ny_end + 1, k, s);
}
#undef F4
#undef F8

}  // namespace ocn

using namespace ocn;

extern "C" {

int ocn_sw_update_ssh(const ocn_block *b, double tau, const float *lu, const float *dx, const float *dy,
                      const float *dxh, const float *dyh, const double *hhu, const double *hhv, double *sshn,
                      const double *sshp, const double *ubrtr, const double *vbrtr, void *stream)
{
    CHECK(lu, dx, dy, dxh, dyh, hhu, hhv, sshn, sshp, ubrtr, vbrtr);
    SwUpdateSsh k{geo(b), tau, lu, dx, dy, dxh, dyh, hhu, hhv, sshn, sshp, ubrtr, vbrtr};
    return launch_range(b->nx_start, b->nx_end, b->ny_start, b->ny_end, k, (hipStream_t)stream);
}

int ocn_hh_update(const ocn_block *b, const float *lu, const float *llu, const float *llv, const float *luh,
                  const float *dx, const float *dy, const float *dxt, const float *dyt, const float *dxh,
                  const float *dyh, const float *dxb, const float *dyb, double *hqn, double *hun, double *hvn,
                  double *hhn, const double *sh, const double *h_r, void *stream)
{
    CHECK(lu, llu, llv, luh, dx, dy, dxt, dyt, dxh, dyh, dxb, dyb, hqn, hun, hvn, hhn, sh, h_r);
    HhUpdate k{geo(b), b->nx_start - 1, b->nx_end, b->ny_start - 1, b->ny_end,
               lu, llu, llv, luh, dx, dy, dxt, dyt, dxh, dyh, dxb, dyb, hqn, hun, hvn, hhn, sh, h_r};
    return launch_range(b->bnd_x1, b->bnd_x2, b->bnd_y1, b->bnd_y2, k, (hipStream_t)stream);
}

int ocn_uv_trans_vort(const ocn_block *b, const float *luu, const float *dxt, const float *dyt, const float *dxb,
                      const float *dyb, const double *u, const double *v, double *vort, void *stream)
{
    CHECK(luu, dxt, dyt, dxb, dyb, u, v, vort);
    UvTransVort k{geo(b), luu, dxt, dyt, dxb, dyb, u, v, vort};
    return launch_range(b->nx_start, b->nx_end, b->ny_start, b->ny_end, k, (hipStream_t)stream);
}

int ocn_uv_trans(const ocn_block *b, const float *lcu, const float *lcv, const float *luu, const float *dxh,
                 const float *dyh, const double *u, const double *v, const double *vort, const double *hq,
                 const double *hu, const double *hv, const double *hh, double *RHSx, double *RHSy, void *stream)
{
    (void)hq;
    CHECK(lcu, lcv, luu, dxh, dyh, u, v, vort, hu, hv, hh, RHSx, RHSy);
    UvTrans k{geo(b), lcu, lcv, luu, dxh, dyh, u, v, vort, hu, hv, hh, RHSx, RHSy};
    return launch_range(b->nx_start, b->nx_end, b->ny_start, b->ny_end, k, (hipStream_t)stream);
}

int ocn_stress_components(const ocn_block *b, const float *lu, const float *luu, const float *dx, const float *dy,
                          const float *dxt, const float *dyt, const float *dxh, const float *dyh, const float *dxb,
                          const float *dyb, const double *u, const double *v, double *str_t, double *str_s,
                          void *stream)
{
    CHECK(lu, luu, dx, dy, dxt, dyt, dxh, dyh, dxb, dyb, u, v, str_t, str_s);
    StressComponents k{geo(b), lu, luu, dx, dy, dxt, dyt, dxh, dyh, dxb, dyb, u, v, str_t, str_s};
    return launch_range(b->nx_start, b->nx_end, b->ny_start, b->ny_end, k, (hipStream_t)stream);
}

int ocn_uv_diff2(const ocn_block *b, const float *lcu, const float *lcv, const float *dx, const float *dy,
                 const float *dxt, const float *dyt, const float *dxh, const float *dyh, const float *dxb,
                 const float *dyb, const double *mu, const double *str_t, const double *str_s, const double *hq,
                 const double *hu, const double *hv, const double *hh, double *RHSx, double *RHSy, void *stream)
{
    (void)hu; (void)hv;
    CHECK(lcu, lcv, dx, dy, dxt, dyt, dxh, dyh, dxb, dyb, mu, str_t, str_s, hq, hh, RHSx, RHSy);
    UvDiff2 k{geo(b), lcu, lcv, dx, dy, dxt, dyt, dxh, dyh, dxb, dyb, mu, str_t, str_s, hq, hh, RHSx, RHSy};
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
    SwUpdateUv k{geo(b), tau, lcu, lcv, dxt, dyt, dxh, dyh, dxb, dyb, hhu, hhun, hhup, hhv, hhvn, hhvp, hhh, ssh,
                 ubrtr, ubrtrn, ubrtrp, vbrtr, vbrtrn, vbrtrp, rdis, rlh_s, RHSx, RHSy, RHSx_adv, RHSy_adv,
                 RHSx_dif, RHSy_dif};
    return launch_range(b->nx_start, b->nx_end, b->ny_start, b->ny_end, k, (hipStream_t)stream);
}

int ocn_sw_next_step(const ocn_block *b, double time_smooth, const float *lu, const float *lcu, const float *lcv,
                     double *ssh, double *sshn, double *sshp, double *ubrtr, double *ubrtrn, double *ubrtrp,
                     double *vbrtr, double *vbrtrn, double *vbrtrp, void *stream)
{
    CHECK(lu, lcu, lcv, ssh, sshn, sshp, ubrtr, ubrtrn, ubrtrp, vbrtr, vbrtrn, vbrtrp);
    SwNextStep k{geo(b), time_smooth, lu, lcu, lcv, ssh, sshn, sshp, ubrtr, ubrtrn, ubrtrp, vbrtr, vbrtrn, vbrtrp};
    return launch_range(b->nx_start - 1, b->nx_end + 1, b->ny_start - 1, b->ny_end + 1, k, (hipStream_t)stream);
}

int ocn_hh_shift(const ocn_block *b, double time_smooth, const float *lu, const float *llu, const float *llv,
                 const float *luh, double *hq, double *hqp, double *hqn, double *hu, double *hup, double *hun,
                 double *hv, double *hvp, double *hvn, double *hh, double *hhp, double *hhn, void *stream)
{
    CHECK(lu, llu, llv, luh, hq, hqp, hqn, hu, hup, hun, hv, hvp, hvn, hh, hhp, hhn);
    HhShift k{geo(b), time_smooth, lu, llu, llv, luh, hq, hqp, hqn, hu, hup, hun, hv, hvp, hvn, hh, hhp, hhn};
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
    HhInit k{geo(b), b->nx_start - 1, b->nx_end, b->ny_start - 1, b->ny_end, (double)full_free_surface,
             lu, llu, llv, luh, dx, dy, dxt, dyt, dxh, dyh, dxb, dyb,
             hq, hqp, hqn, hu, hup, hun, hv, hvp, hvn, hh, hhp, hhn, sh, shp, h_r};
    return launch_range(b->bnd_x1, b->bnd_x2, b->bnd_y1, b->bnd_y2, k, (hipStream_t)stream);
}

int ocn_check_ssh_err(const ocn_block *b, const float *lu, const double *ssh, int32_t *nbad_device, void *stream)
{
    CHECK(lu, ssh, nbad_device);
    CheckSshErr k{geo(b), lu, ssh, (int *)nbad_device};
    return launch_range(b->nx_start, b->nx_end, b->ny_start, b->ny_end, k, (hipStream_t)stream);
}

}  // extern "C"
