/*
 * sw_oracle.c -- CPU restatement of the reference shallow-water barotropic step.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity checker: only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.  The
 * product (ocean_model_arch_amd/, include/) never links or calls it.
 *
 * Every routine restates one reference routine (paths relative to the
 * Andrcraft9/ocean_model_arch tree) with the same loop ranges, the same write
 * sets and the same floating-point evaluation order, including the Fortran
 * mixed-kind rules (real(4)*real(4) sub-expressions are evaluated in float).
 * Build with -O2 -ffp-contract=off (no FMA contraction, no fast-math).
 *
 * Array convention: Fortran column-major A(bnd_x1:bnd_x2, bnd_y1:bnd_y2),
 * pointer = address of A(bnd_x1,bnd_y1), leading dimension bnd_x2-bnd_x1+1.
 * Indices are the reference's 1-based global indices.
 *
 * Pinned against: the tests/golden npz fixtures produced from the compiled reference
 * (oracle/ref.mk -> oracle/_ref/libref.so, oracle/ref_driver.f90).
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

#define BND_ARGS int nxs, int nxe, int nys, int nye, int bx1, int bx2, int by1, int by2
#define LD (bx2 - bx1 + 1)
#define I(m, n) ((long)((m) - bx1) + (long)((n) - by1) * (long)LD)

/* shared/constants.f90:23 FreeFallAcc = 9.8 is real(4); promoted to real(8) on use. */
static const float kFreeFallAcc = 9.8f;
/* shared/constants.f90:14-16 */
static const float kPi = 3.1415926f;
static const double kDPi = 3.14159265358979;
static const double kLatExtr = 89.99999;
static const float kRadEarth = 6371000.0f;
static const float kEarthAngVel = 7.2921159e-5f;

/* ------------------------------------------------------------------------- */
/* kernel/shallow_water/vel_ssh.f90:15-38  gaussian_elimination_kernel        */
void orc_gaussian_elimination(BND_ARGS, const float *lu, double *ssh, double sigma, int nx0, int ny0)
{
    (void)by2;
    for (int n = nys; n <= nye; ++n)
        for (int m = nxs; m <= nxe; ++m)
            if (lu[I(m, n)] > 0.5f) {
                double dx = (double)(m - nx0) / ((double)nx0 * 0.25);
                double dy = (double)(n - ny0) / ((double)ny0 * 0.25);
                /* (1.0 / (dsqrt(2*dPi) * sigma)) * dexp(-((dx*dx + dy*dy) / (2*sigma*sigma))) */
                double a = 1.0 / (sqrt(2.0 * kDPi) * sigma);
                double e = exp(-((dx * dx + dy * dy) / (2.0 * sigma * sigma)));
                ssh[I(m, n)] = a * e;
            }
}

/* vel_ssh.f90:40-67  check_ssh_err_kernel: returns number of bad sea points */
long orc_check_ssh_err(BND_ARGS, const float *lu, const double *ssh)
{
    (void)by2;
    long bad = 0;
    for (int n = nys; n <= nye; ++n)
        for (int m = nxs; m <= nxe; ++m)
            if (lu[I(m, n)] > 0.5f) {
                double s = ssh[I(m, n)];
                if (!(s < 10000.0 && s > -10000.0)) ++bad;
            }
    return bad;
}

/* vel_ssh.f90:69-106  sw_update_ssh_kernel (a1) */
void orc_sw_update_ssh(BND_ARGS, double tau, const float *lu, const float *dx, const float *dy,
                       const float *dxh, const float *dyh, const double *hhu, const double *hhv,
                       double *sshn, const double *sshp, const double *ubrtr, const double *vbrtr)
{
    (void)by2;
    for (int n = nys; n <= nye; ++n)
        for (int m = nxs; m <= nxe; ++m)
            if (lu[I(m, n)] > 0.5f) {
                double t1 = ubrtr[I(m, n)] * hhu[I(m, n)] * (double)dyh[I(m, n)];
                double t2 = ubrtr[I(m - 1, n)] * hhu[I(m - 1, n)] * (double)dyh[I(m - 1, n)];
                double t3 = vbrtr[I(m, n)] * hhv[I(m, n)] * (double)dxh[I(m, n)];
                double t4 = vbrtr[I(m, n - 1)] * hhv[I(m, n - 1)] * (double)dxh[I(m, n - 1)];
                float area = dx[I(m, n)] * dy[I(m, n)]; /* real(4)*real(4) */
                double div = (t1 - t2 + t3 - t4) / (double)area;
                sshn[I(m, n)] = sshp[I(m, n)] + 2.0 * tau * (-div);
            }
}

/* vel_ssh.f90:108-195  sw_update_uv (a7) */
void orc_sw_update_uv(BND_ARGS, double tau, const float *lcu, const float *lcv,
                      const float *dxt, const float *dyt, const float *dxh, const float *dyh,
                      const float *dxb, const float *dyb,
                      const double *hhu, const double *hhun, const double *hhup,
                      const double *hhv, const double *hhvn, const double *hhvp,
                      const double *hhh, const double *ssh,
                      const double *ubrtr, double *ubrtrn, const double *ubrtrp,
                      const double *vbrtr, double *vbrtrn, const double *vbrtrp,
                      const float *rdis, const float *rlh_s,
                      const double *RHSx, const double *RHSy, const double *RHSx_adv,
                      const double *RHSy_adv, const double *RHSx_dif, const double *RHSy_dif)
{
    (void)by2;
    const double g = (double)kFreeFallAcc;
    for (int n = nys; n <= nye; ++n)
        for (int m = nxs; m <= nxe; ++m) {
            if (lcu[I(m, n)] > 0.5f) {
                double bp = hhun[I(m, n)] * (double)dxt[I(m, n)] * (double)dyh[I(m, n)] / 2.0 / tau;
                double bp0 = hhup[I(m, n)] * (double)dxt[I(m, n)] * (double)dyh[I(m, n)] / 2.0 / tau;
                double slx = -(g * (ssh[I(m + 1, n)] - ssh[I(m, n)]) * (double)dyh[I(m, n)] * hhu[I(m, n)]);
                float rd = rdis[I(m, n)] + rdis[I(m + 1, n)];
                double fric = (double)rd / 2.0 * ubrtrp[I(m, n)] * (double)dxt[I(m, n)] * (double)dyh[I(m, n)] * hhu[I(m, n)];
                double c1 = (double)rlh_s[I(m, n)] * hhh[I(m, n)] * (double)dxb[I(m, n)] * (double)dyb[I(m, n)]
                            * (vbrtr[I(m + 1, n)] + vbrtr[I(m, n)]);
                double c2 = (double)rlh_s[I(m, n - 1)] * hhh[I(m, n - 1)] * (double)dxb[I(m, n - 1)] * (double)dyb[I(m, n - 1)]
                            * (vbrtr[I(m + 1, n - 1)] + vbrtr[I(m, n - 1)]);
                double grx = RHSx[I(m, n)] + slx + RHSx_dif[I(m, n)] + RHSx_adv[I(m, n)] - fric + (c1 + c2) / 4.0;
                ubrtrn[I(m, n)] = (ubrtrp[I(m, n)] * bp0 + grx) / (bp);
            }
            if (lcv[I(m, n)] > 0.5f) {
                double bp = hhvn[I(m, n)] * (double)dyt[I(m, n)] * (double)dxh[I(m, n)] / 2.0 / tau;
                double bp0 = hhvp[I(m, n)] * (double)dyt[I(m, n)] * (double)dxh[I(m, n)] / 2.0 / tau;
                double sly = -(g * (ssh[I(m, n + 1)] - ssh[I(m, n)]) * (double)dxh[I(m, n)] * hhv[I(m, n)]);
                float rd = rdis[I(m, n)] + rdis[I(m, n + 1)];
                double fric = (double)rd / 2.0 * vbrtrp[I(m, n)] * (double)dxh[I(m, n)] * (double)dyt[I(m, n)] * hhv[I(m, n)];
                double c1 = (double)rlh_s[I(m, n)] * hhh[I(m, n)] * (double)dxb[I(m, n)] * (double)dyb[I(m, n)]
                            * (ubrtr[I(m, n + 1)] + ubrtr[I(m, n)]);
                double c2 = (double)rlh_s[I(m - 1, n)] * hhh[I(m - 1, n)] * (double)dxb[I(m - 1, n)] * (double)dyb[I(m - 1, n)]
                            * (ubrtr[I(m - 1, n + 1)] + ubrtr[I(m - 1, n)]);
                double gry = RHSy[I(m, n)] + sly + RHSy_dif[I(m, n)] + RHSy_adv[I(m, n)] - fric - (c1 + c2) / 4.0;
                vbrtrn[I(m, n)] = (vbrtrp[I(m, n)] * bp0 + gry) / (bp);
            }
        }
}

/* vel_ssh.f90:197-245  sw_next_step (a8): interior + halo ring */
void orc_sw_next_step(BND_ARGS, double ts, const float *lu, const float *lcu, const float *lcv,
                      double *ssh, double *sshn, double *sshp,
                      double *ubrtr, double *ubrtrn, double *ubrtrp,
                      double *vbrtr, double *vbrtrn, double *vbrtrp)
{
    (void)by2;
    for (int n = nys - 1; n <= nye + 1; ++n)
        for (int m = nxs - 1; m <= nxe + 1; ++m) {
            long i = I(m, n);
            if (lu[i] > 0.5f) {
                sshp[i] = ssh[i] + ts * (sshn[i] - 2.0 * ssh[i] + sshp[i]) / 2.0;
                ssh[i] = sshn[i];
            }
            if (lcu[i] > 0.5f) {
                ubrtrp[i] = ubrtr[i] + ts * (ubrtrn[i] - 2.0 * ubrtr[i] + ubrtrp[i]) / 2.0;
                ubrtr[i] = ubrtrn[i];
            }
            if (lcv[i] > 0.5f) {
                vbrtrp[i] = vbrtr[i] + ts * (vbrtrn[i] - 2.0 * vbrtr[i] + vbrtrp[i]) / 2.0;
                vbrtr[i] = vbrtrn[i];
            }
        }
}

/* vel_ssh.f90:247-281  uv_trans_vort_kernel (a3), nlev = 1 */
void orc_uv_trans_vort(BND_ARGS, const float *luu, const float *dxt, const float *dyt,
                       const float *dxb, const float *dyb, const double *u, const double *v, double *vort)
{
    (void)by2;
    for (int n = nys; n <= nye; ++n)
        for (int m = nxs; m <= nxe; ++m)
            if (luu[I(m, n)] > 0.5f) {
                double a = v[I(m + 1, n)] * (double)dyt[I(m + 1, n)] - v[I(m, n)] * (double)dyt[I(m, n)];
                double b = u[I(m, n + 1)] * (double)dxt[I(m, n + 1)] - u[I(m, n)] * (double)dxt[I(m, n)];
                double c = (v[I(m + 1, n)] - v[I(m, n)]) * (double)dyb[I(m, n)]
                           - (u[I(m, n + 1)] - u[I(m, n)]) * (double)dxb[I(m, n)];
                vort[I(m, n)] = a - b - c;
            }
}

/* vel_ssh.f90:283-373  uv_trans_kernel (a4), nlev = 1; hq is passed but unused */
void orc_uv_trans(BND_ARGS, const float *lcu, const float *lcv, const float *luu,
                  const float *dxh, const float *dyh, const double *u, const double *v,
                  const double *vort, const double *hq, const double *hu, const double *hv,
                  const double *hh, double *RHSx, double *RHSy)
{
    (void)by2; (void)hq;
    for (int n = nys; n <= nye; ++n)
        for (int m = nxs; m <= nxe; ++m) {
            if (lcu[I(m, n)] > 0.5f) {
                double fx_p = (u[I(m, n)] * (double)dyh[I(m, n)] * hu[I(m, n)]
                               + u[I(m + 1, n)] * (double)dyh[I(m + 1, n)] * hu[I(m + 1, n)]) / 2.0
                              * (u[I(m, n)] + u[I(m + 1, n)]) / 2.0;
                double fx_m = (u[I(m, n)] * (double)dyh[I(m, n)] * hu[I(m, n)]
                               + u[I(m - 1, n)] * (double)dyh[I(m - 1, n)] * hu[I(m - 1, n)]) / 2.0
                              * (u[I(m, n)] + u[I(m - 1, n)]) / 2.0;
                double fy_p = (v[I(m, n)] * (double)dxh[I(m, n)] * hv[I(m, n)]
                               + v[I(m + 1, n)] * (double)dxh[I(m + 1, n)] * hv[I(m + 1, n)]) / 2.0
                              * (u[I(m, n + 1)] + u[I(m, n)]) / 2.0 * (double)luu[I(m, n)];
                double fy_m = (v[I(m, n - 1)] * (double)dxh[I(m, n - 1)] * hv[I(m, n - 1)]
                               + v[I(m + 1, n - 1)] * (double)dxh[I(m + 1, n - 1)] * hv[I(m + 1, n - 1)]) / 2.0
                              * (u[I(m, n - 1)] + u[I(m, n)]) / 2.0 * (double)luu[I(m, n - 1)];
                RHSx[I(m, n)] = -(fx_p - fx_m + fy_p - fy_m)
                                + (vort[I(m, n)] * hh[I(m, n)] * (v[I(m + 1, n)] + v[I(m, n)])
                                   + vort[I(m, n - 1)] * hh[I(m, n - 1)] * (v[I(m + 1, n - 1)] + v[I(m, n - 1)])) / 4.0;
            }
            if (lcv[I(m, n)] > 0.5f) {
                double fy_p = (v[I(m, n)] * (double)dxh[I(m, n)] * hv[I(m, n)]
                               + v[I(m, n + 1)] * (double)dxh[I(m, n + 1)] * hv[I(m, n + 1)]) / 2.0
                              * (v[I(m, n)] + v[I(m, n + 1)]) / 2.0;
                double fy_m = (v[I(m, n)] * (double)dxh[I(m, n)] * hv[I(m, n)]
                               + v[I(m, n - 1)] * (double)dxh[I(m, n - 1)] * hv[I(m, n - 1)]) / 2.0
                              * (v[I(m, n)] + v[I(m, n - 1)]) / 2.0;
                double fx_p = (u[I(m, n)] * (double)dyh[I(m, n)] * hu[I(m, n)]
                               + u[I(m, n + 1)] * (double)dyh[I(m, n + 1)] * hu[I(m, n + 1)]) / 2.0
                              * (v[I(m + 1, n)] + v[I(m, n)]) / 2.0;
                double fx_m = (u[I(m - 1, n)] * (double)dyh[I(m - 1, n)] * hu[I(m - 1, n)]
                               + u[I(m - 1, n + 1)] * (double)dyh[I(m - 1, n + 1)] * hu[I(m - 1, n + 1)]) / 2.0
                              * (v[I(m - 1, n)] + v[I(m, n)]) / 2.0;
                RHSy[I(m, n)] = -(fx_p - fx_m + fy_p - fy_m)
                                - (vort[I(m, n)] * hh[I(m, n)] * (u[I(m, n + 1)] + u[I(m, n)])
                                   + vort[I(m - 1, n)] * hh[I(m - 1, n)] * (u[I(m - 1, n + 1)] + u[I(m - 1, n)])) / 4.0;
            }
        }
}

/* vel_ssh.f90:375-452  uv_diff2_kernel (a6), nlev = 1 */
void orc_uv_diff2(BND_ARGS, const float *lcu, const float *lcv,
                  const float *dx, const float *dy, const float *dxt, const float *dyt,
                  const float *dxh, const float *dyh, const float *dxb, const float *dyb,
                  const double *mu, const double *str_t, const double *str_s,
                  const double *hq, const double *hu, const double *hv, const double *hh,
                  double *RHSx, double *RHSy)
{
    (void)by2; (void)hu; (void)hv;
    for (int n = nys; n <= nye; ++n)
        for (int m = nxs; m <= nxe; ++m) {
            if (lcu[I(m, n)] > 0.5f) {
                double muh_p = (mu[I(m, n)] + mu[I(m + 1, n)] + mu[I(m, n + 1)] + mu[I(m + 1, n + 1)]) / 4.0;
                double muh_m = (mu[I(m, n)] + mu[I(m + 1, n)] + mu[I(m, n - 1)] + mu[I(m + 1, n - 1)]) / 4.0;
                float dy2p = dy[I(m + 1, n)] * dy[I(m + 1, n)];
                float dy2 = dy[I(m, n)] * dy[I(m, n)];
                float dxb2 = dxb[I(m, n)] * dxb[I(m, n)];
                float dxb2m = dxb[I(m, n - 1)] * dxb[I(m, n - 1)];
                RHSx[I(m, n)] = ((double)dy2p * mu[I(m + 1, n)] * hq[I(m + 1, n)] * str_t[I(m + 1, n)]
                                 - (double)dy2 * mu[I(m, n)] * hq[I(m, n)] * str_t[I(m, n)]) / (double)dyh[I(m, n)]
                                + ((double)dxb2 * muh_p * hh[I(m, n)] * str_s[I(m, n)]
                                   - (double)dxb2m * muh_m * hh[I(m, n - 1)] * str_s[I(m, n - 1)]) / (double)dxt[I(m, n)];
            }
            if (lcv[I(m, n)] > 0.5f) {
                double muh_p = (mu[I(m, n)] + mu[I(m + 1, n)] + mu[I(m, n + 1)] + mu[I(m + 1, n + 1)]) / 4.0;
                double muh_m = (mu[I(m, n)] + mu[I(m - 1, n)] + mu[I(m, n + 1)] + mu[I(m - 1, n + 1)]) / 4.0;
                float dx2p = dx[I(m, n + 1)] * dx[I(m, n + 1)];
                float dx2 = dx[I(m, n)] * dx[I(m, n)];
                float dyb2 = dyb[I(m, n)] * dyb[I(m, n)];
                float dyb2m = dyb[I(m - 1, n)] * dyb[I(m - 1, n)];
                RHSy[I(m, n)] = -((double)dx2p * mu[I(m, n + 1)] * hq[I(m, n + 1)] * str_t[I(m, n + 1)]
                                  - (double)dx2 * mu[I(m, n)] * hq[I(m, n)] * str_t[I(m, n)]) / (double)dxh[I(m, n)]
                                + ((double)dyb2 * muh_p * hh[I(m, n)] * str_s[I(m, n)]
                                   - (double)dyb2m * muh_m * hh[I(m - 1, n)] * str_s[I(m - 1, n)]) / (double)dyt[I(m, n)];
            }
        }
}

/* kernel/shallow_water/mixing.f90:14-58  stress_components_kernel (a5), nlev = 1 */
void orc_stress_components(BND_ARGS, const float *lu, const float *luu,
                           const float *dx, const float *dy, const float *dxt, const float *dyt,
                           const float *dxh, const float *dyh, const float *dxb, const float *dyb,
                           const double *u, const double *v, double *str_t, double *str_s)
{
    (void)by2;
    for (int n = nys; n <= nye; ++n)
        for (int m = nxs; m <= nxe; ++m) {
            if (lu[I(m, n)] > 0.5f) {
                float r1 = dy[I(m, n)] / dx[I(m, n)];
                float r2 = dx[I(m, n)] / dy[I(m, n)];
                str_t[I(m, n)] = (double)r1 * (u[I(m, n)] / (double)dyh[I(m, n)] - u[I(m - 1, n)] / (double)dyh[I(m - 1, n)])
                                 - (double)r2 * (v[I(m, n)] / (double)dxh[I(m, n)] - v[I(m, n - 1)] / (double)dxh[I(m, n - 1)]);
            }
            if (luu[I(m, n)] > 0.5f) {
                float r1 = dxb[I(m, n)] / dyb[I(m, n)];
                float r2 = dyb[I(m, n)] / dxb[I(m, n)];
                str_s[I(m, n)] = (double)r1 * (u[I(m, n + 1)] / (double)dxt[I(m, n + 1)] - u[I(m, n)] / (double)dxt[I(m, n)])
                                 + (double)r2 * (v[I(m + 1, n)] / (double)dyt[I(m + 1, n)] - v[I(m, n)] / (double)dyt[I(m, n)]);
            }
        }
}

/* Shared interpolation T -> U/V/H points, kernel/shallow_water/depth.f90:56-97 */
static inline double interp_u(BND_ARGS, const double *h, const float *lu, const float *dx, const float *dy,
                              const float *dxt, const float *dyh, int m, int n, double slu)
{
    (void)nxs; (void)nxe; (void)nys; (void)nye; (void)by2;
    return (h[I(m, n)] * (double)dx[I(m, n)] * (double)dy[I(m, n)] * (double)lu[I(m, n)]
            + h[I(m + 1, n)] * (double)dx[I(m + 1, n)] * (double)dy[I(m + 1, n)] * (double)lu[I(m + 1, n)])
           / slu / (double)dxt[I(m, n)] / (double)dyh[I(m, n)];
}
static inline double interp_v(BND_ARGS, const double *h, const float *lu, const float *dx, const float *dy,
                              const float *dxh, const float *dyt, int m, int n, double slu)
{
    (void)nxs; (void)nxe; (void)nys; (void)nye; (void)by2;
    return (h[I(m, n)] * (double)dx[I(m, n)] * (double)dy[I(m, n)] * (double)lu[I(m, n)]
            + h[I(m, n + 1)] * (double)dx[I(m, n + 1)] * (double)dy[I(m, n + 1)] * (double)lu[I(m, n + 1)])
           / slu / (double)dxh[I(m, n)] / (double)dyt[I(m, n)];
}
static inline double interp_h(BND_ARGS, const double *h, const float *lu, const float *dx, const float *dy,
                              const float *dxb, const float *dyb, int m, int n, double slu)
{
    (void)nxs; (void)nxe; (void)nys; (void)nye; (void)by2;
    return (h[I(m, n)] * (double)dx[I(m, n)] * (double)dy[I(m, n)] * (double)lu[I(m, n)]
            + h[I(m + 1, n)] * (double)dx[I(m + 1, n)] * (double)dy[I(m + 1, n)] * (double)lu[I(m + 1, n)]
            + h[I(m, n + 1)] * (double)dx[I(m, n + 1)] * (double)dy[I(m, n + 1)] * (double)lu[I(m, n + 1)]
            + h[I(m + 1, n + 1)] * (double)dx[I(m + 1, n + 1)] * (double)dy[I(m + 1, n + 1)] * (double)lu[I(m + 1, n + 1)])
           / slu / (double)dxb[I(m, n)] / (double)dyb[I(m, n)];
}
#define BARGS nxs, nxe, nys, nye, bx1, bx2, by1, by2

/* depth.f90:14-99  hh_init_kernel (a10); ffs = config_sw_module::full_free_surface */
void orc_hh_init(BND_ARGS, int ffs, const float *lu, const float *llu, const float *llv, const float *luh,
                 const float *dx, const float *dy, const float *dxt, const float *dyt,
                 const float *dxh, const float *dyh, const float *dxb, const float *dyb,
                 double *hq, double *hqp, double *hqn, double *hu, double *hup, double *hun,
                 double *hv, double *hvp, double *hvn, double *hh, double *hhp, double *hhn,
                 const double *sh, const double *shp, const double *h_r)
{
    const long tot = (long)LD * (long)(by2 - by1 + 1);
    const double f = (double)ffs;
    for (long i = 0; i < tot; ++i) {           /* whole-array assignments :48-50 */
        hq[i] = h_r[i] + sh[i] * f;
        hqp[i] = h_r[i] + shp[i] * f;
        hqn[i] = h_r[i];
    }
    for (int n = nys - 1; n <= nye; ++n)
        for (int m = nxs - 1; m <= nxe; ++m) {
            if (llu[I(m, n)] > 0.5f) {
                double slu = (double)(lu[I(m, n)] + lu[I(m + 1, n)]);
                hu[I(m, n)] = interp_u(BARGS, hq, lu, dx, dy, dxt, dyh, m, n, slu);
                hup[I(m, n)] = interp_u(BARGS, hqp, lu, dx, dy, dxt, dyh, m, n, slu);
                hun[I(m, n)] = interp_u(BARGS, hqn, lu, dx, dy, dxt, dyh, m, n, slu);
            }
            if (llv[I(m, n)] > 0.5f) {
                double slu = (double)(lu[I(m, n)] + lu[I(m, n + 1)]);
                hv[I(m, n)] = interp_v(BARGS, hq, lu, dx, dy, dxh, dyt, m, n, slu);
                hvp[I(m, n)] = interp_v(BARGS, hqp, lu, dx, dy, dxh, dyt, m, n, slu);
                hvn[I(m, n)] = interp_v(BARGS, hqn, lu, dx, dy, dxh, dyt, m, n, slu);
            }
            if (luh[I(m, n)] > 0.5f) {
                double slu = (double)(lu[I(m, n)] + lu[I(m + 1, n)] + lu[I(m, n + 1)] + lu[I(m + 1, n + 1)]);
                hh[I(m, n)] = interp_h(BARGS, hq, lu, dx, dy, dxb, dyb, m, n, slu);
                hhp[I(m, n)] = interp_h(BARGS, hqp, lu, dx, dy, dxb, dyb, m, n, slu);
                hhn[I(m, n)] = interp_h(BARGS, hqn, lu, dx, dy, dxb, dyb, m, n, slu);
            }
        }
}

/* depth.f90:101-162  hh_update_kernel (a2) */
void orc_hh_update(BND_ARGS, const float *lu, const float *llu, const float *llv, const float *luh,
                   const float *dx, const float *dy, const float *dxt, const float *dyt,
                   const float *dxh, const float *dyh, const float *dxb, const float *dyb,
                   double *hqn, double *hun, double *hvn, double *hhn, const double *sh, const double *h_r)
{
    const long tot = (long)LD * (long)(by2 - by1 + 1);
    for (long i = 0; i < tot; ++i) hqn[i] = h_r[i] + sh[i];   /* :129 */
    for (int n = nys - 1; n <= nye; ++n)
        for (int m = nxs - 1; m <= nxe; ++m) {
            if (llu[I(m, n)] > 0.5f) {
                double slu = (double)(lu[I(m, n)] + lu[I(m + 1, n)]);
                hun[I(m, n)] = interp_u(BARGS, hqn, lu, dx, dy, dxt, dyh, m, n, slu);
            }
            if (llv[I(m, n)] > 0.5f) {
                double slu = (double)(lu[I(m, n)] + lu[I(m, n + 1)]);
                hvn[I(m, n)] = interp_v(BARGS, hqn, lu, dx, dy, dxh, dyt, m, n, slu);
            }
            if (luh[I(m, n)] > 0.5f) {
                double slu = (double)(lu[I(m, n)] + lu[I(m + 1, n)] + lu[I(m, n + 1)] + lu[I(m + 1, n + 1)]);
                hhn[I(m, n)] = interp_h(BARGS, hqn, lu, dx, dy, dxb, dyb, m, n, slu);
            }
        }
}

/* depth.f90:164-211  hh_shift_kernel (a9): interior + halo ring; ts = config_sw_module::time_smooth */
void orc_hh_shift(BND_ARGS, double ts, const float *lu, const float *llu, const float *llv, const float *luh,
                  double *hq, double *hqp, double *hqn, double *hu, double *hup, double *hun,
                  double *hv, double *hvp, double *hvn, double *hh, double *hhp, double *hhn)
{
    (void)by2;
    for (int n = nys - 1; n <= nye + 1; ++n)
        for (int m = nxs - 1; m <= nxe + 1; ++m) {
            long i = I(m, n);
            if (llu[i] > 0.5f) {
                hup[i] = hu[i] + ts * (hun[i] - 2.0 * hu[i] + hup[i]) / 2.0;
                hu[i] = hun[i];
            }
            if (llv[i] > 0.5f) {
                hvp[i] = hv[i] + ts * (hvn[i] - 2.0 * hv[i] + hvp[i]) / 2.0;
                hv[i] = hvn[i];
            }
            if (lu[i] > 0.5f) {
                hqp[i] = hq[i] + ts * (hqn[i] - 2.0 * hq[i] + hqp[i]) / 2.0;
                hq[i] = hqn[i];
            }
            if (luh[i] > 0.5f) {
                hhp[i] = hh[i] + ts * (hhn[i] - 2.0 * hh[i] + hhp[i]) / 2.0;
                hh[i] = hhn[i];
            }
        }
}

/* ------------------------------------------------------------------------- */
/* Grid setup (runs once).                                                   */

/* ---------------------------------------------------------------- tracers
 * kernel/tracer/leapfrog_tracer.f90:13-92 tran_diff_fluxes_kernel (interior; flux_x on lcu,
 * flux_y on lcv; flux_gm = 0.0d0 is still added, so -0.0 sums become +0.0). */
void orc_tran_diff_fluxes(BND_ARGS, const float *lcu, const float *lcv, const float *dxt, const float *dyt,
                          const float *dxh, const float *dyh, const double *hhu, const double *hhv,
                          const double *ff, const double *ffp, const double *uu, const double *vv,
                          const double *mu, double factor_mu, double *flux_x, double *flux_y)
{
    (void)ffp; (void)by2;
    for (int n = nys; n <= nye; ++n)
        for (int m = nxs; m <= nxe; ++m) {
            const long c = I(m, n), e = I(m + 1, n), nn = I(m, n + 1);
            if (lcu[c] > 0.5f) {
                const double dfdx = ff[e] - ff[c];
                const double mu_1d = (mu[c] + mu[e]) / 2.0 * factor_mu * (double)dyh[c] / (double)dxt[c];
                const double flux_diff = mu_1d * hhu[c] * dfdx;
                const double flux_adv = -uu[c] * hhu[c] * (double)dyh[c] * (ff[c] + ff[e]) / 2.0;
                flux_x[c] = flux_adv + flux_diff + 0.0;
            }
            if (lcv[c] > 0.5f) {
                const double dfdy = ff[nn] - ff[c];
                const double mu_1d = (mu[c] + mu[nn]) / 2.0 * factor_mu * (double)dxh[c] / (double)dyt[c];
                const double flux_diff = mu_1d * hhv[c] * dfdy;
                const double flux_adv = -vv[c] * hhv[c] * (double)dxh[c] * (ff[c] + ff[nn]) / 2.0;
                flux_y[c] = flux_adv + flux_diff + 0.0;
            }
        }
}

/* leapfrog_tracer.f90:94-136 tran_diff_tracer_kernel (interior, lu). */
void orc_tran_diff_tracer(BND_ARGS, const float *lu, const float *dx, const float *dy, double tau,
                          const double *hhqn, const double *hhqp, const double *flux_x, const double *flux_y,
                          const double *ffp, double *ffn)
{
    (void)by2;
    for (int n = nys; n <= nye; ++n)
        for (int m = nxs; m <= nxe; ++m) {
            const long c = I(m, n);
            if (lu[c] > 0.5f) {
                const double bp = hhqn[c] * (double)dx[c] * (double)dy[c] / tau / 2.0;
                const double bp0 = hhqp[c] * (double)dx[c] * (double)dy[c] / tau / 2.0;
                const double rhs = flux_x[c] - flux_x[I(m - 1, n)] + flux_y[c] - flux_y[I(m, n - 1)];
                const double eta = bp0 * ffp[c] + rhs;
                ffn[c] = eta / bp;
            }
        }
}

/* leapfrog_tracer.f90:138-168 tracer_next_step_kernel (interior + halo ring, lu). */
void orc_tracer_next_step(BND_ARGS, double ts, const float *lu, const double *ffn, double *ffp, double *ff)
{
    (void)by2;
    for (int n = nys - 1; n <= nye + 1; ++n)
        for (int m = nxs - 1; m <= nxe + 1; ++m) {
            const long c = I(m, n);
            if (lu[c] > 0.5f) {
                ffp[c] = ff[c] + ts * (ffn[c] - 2.0 * ff[c] + ffp[c]) / 2.0;
                ff[c] = ffn[c];
            }
        }
}

/* kernel/service/grid_kernels.f90:18-38  lu_init_kernel: mask is global (nx, ny) column-major */
void orc_lu_init(int bx1, int bx2, int by1, int by2, int nx, const int32_t *mask, float *lu, float *lu1)
{
    for (int n = by1; n <= by2; ++n)
        for (int m = bx1; m <= bx2; ++m) {
            if (mask[(long)(m - 1) + (long)(n - 1) * nx] == 0) lu[I(m, n)] = 1.0f;
            lu1[I(m, n)] = 1.0f;
        }
}

/* grid_kernels.f90:40-92  lu_lv_init_kernel */
void orc_lu_lv_init(int bx1, int bx2, int by1, int by2, const float *lu, float *luh, float *luu,
                    float *llu, float *llv, float *lcu, float *lcv)
{
    for (int n = by1; n <= by2 - 1; ++n)
        for (int m = bx1; m <= bx2 - 1; ++m) {
            if (lu[I(m, n)] + lu[I(m + 1, n)] + lu[I(m, n + 1)] + lu[I(m + 1, n + 1)] > 0.5f) luh[I(m, n)] = 1.0f;
            if (lu[I(m, n)] * lu[I(m + 1, n)] * lu[I(m, n + 1)] * lu[I(m + 1, n + 1)] > 0.5f) luu[I(m, n)] = 1.0f;
        }
    for (int n = by1; n <= by2 - 1; ++n)
        for (int m = bx1; m <= bx2 - 1; ++m) {
            if (lu[I(m, n)] + lu[I(m + 1, n)] > 0.5f) llu[I(m, n)] = 1.0f;
            if (lu[I(m, n)] + lu[I(m, n + 1)] > 0.5f) llv[I(m, n)] = 1.0f;
            if (lu[I(m, n)] * lu[I(m + 1, n)] > 0.5f) lcu[I(m, n)] = 1.0f;
            if (lu[I(m, n)] * lu[I(m, n + 1)] > 0.5f) lcv[I(m, n)] = 1.0f;
        }
}

static double dsind(double x) { return sin((x / 180.0) * kDPi); }   /* core/math_tools.f90:38-50 */
static double dcosd(double x) { return cos((x / 180.0) * kDPi); }

/* grid_kernels.f90:94-202 (uniform x/y grid) + grid_geo_init_kernel :206-421 for curve_grid 0/1.
 * xt,yt,xu,yv: 1-D coordinate work arrays on bnd ranges (owned by the caller).
 * rot_lon/rot_lat: rotation_on_lon / rotation_on_lat (basin.par lines 13-14). */
void orc_grid_init(BND_ARGS, int mmm, int nnn, double rlon, double rlat, double dxst, double dyst,
                   int curve_grid, double rot_lon, double rot_lat,
                   double *xt, double *yt, double *xu, double *yv,
                   float *dx, float *dy, float *dxt, float *dyt, float *dxh, float *dyh,
                   float *dxb, float *dyb, float *rlh_s, float *rlh_c)
{
    (void)rot_lon;
    const float pip180 = kPi / 180.0f;
    for (int m = bx1; m <= bx2; ++m) xt[m - bx1] = rlon + (double)(m - mmm) * dxst;
    for (int n = by1; n <= by2; ++n) yt[n - by1] = rlat + (double)(n - nnn) * dyst;
    for (int m = bx1; m <= bx2 - 1; ++m) xu[m - bx1] = (xt[m - bx1] + xt[m + 1 - bx1]) / 2.0;
    for (int n = by1; n <= by2 - 1; ++n) yv[n - by1] = (yt[n - by1] + yt[n + 1 - by1]) / 2.0;
    const float sx = (float)dxst * pip180 * kRadEarth;
    const float sy = (float)dyst * pip180 * kRadEarth;
    for (int n = nys - 1; n <= nye + 1; ++n)
        for (int m = nxs - 1; m <= nxe + 1; ++m) {
            dxt[I(m, n)] = sx; dxb[I(m, n)] = sx; dx[I(m, n)] = sx; dxh[I(m, n)] = sx;
        }
    for (int n = nys - 1; n <= nye + 1; ++n)
        for (int m = nxs - 1; m <= nxe + 1; ++m) {
            dyt[I(m, n)] = sy; dyb[I(m, n)] = sy; dy[I(m, n)] = sy; dyh[I(m, n)] = sy;
        }
    const long tot = (long)LD * (long)(by2 - by1 + 1);
    for (long i = 0; i < tot; ++i) { rlh_s[i] = 2.0f * kEarthAngVel; rlh_c[i] = -2.0f * kEarthAngVel; }

    /* grid_geo_init_kernel: four passes (T: xt,yt -> dx,dy; U: xu,yt -> dxt,dyh;
     * V: xt,yv -> dxh,dyt; H: xu,yv -> dxb,dyb + Coriolis) over [start-1, end+1]. */
    for (int pass = 0; pass < 4; ++pass) {
        const double *xm = (pass == 1 || pass == 3) ? xu : xt;
        const double *ym = (pass >= 2) ? yv : yt;
        float *mx = pass == 0 ? dx : pass == 1 ? dxt : pass == 2 ? dxh : dxb;
        float *my = pass == 0 ? dy : pass == 1 ? dyh : pass == 2 ? dyt : dyb;
        const int key_cor = (pass == 3);
        for (int n = nys - 1; n <= nye + 1; ++n) {
            double y = ym[n - by1];
            if (curve_grid == 0) {
                /* grid_parameters.f90:16-78 carthesian */
                for (int m = nxs - 1; m <= nxe + 1; ++m) {
                    mx[I(m, n)] = mx[I(m, n)] * 1.0f;
                    my[I(m, n)] = my[I(m, n)] * 1.0f;
                    if (key_cor) {
                        rlh_s[I(m, n)] = rlh_s[I(m, n)] / sqrtf(2.0f);
                        rlh_c[I(m, n)] = rlh_c[I(m, n)] / sqrtf(2.0f);
                    }
                }
            } else {
                /* grid_parameters.f90:80-181 spherical */
                double lat_mod = fmax(fmin(y, kLatExtr), -kLatExtr);
                double sinlat_extr = dsind(kLatExtr);
                for (int m = nxs - 1; m <= nxe + 1; ++m) {
                    double x = xm[m - bx1];
                    double sin_lat = dsind(y) * dcosd(rot_lat) + dcosd(x) * dcosd(y) * dsind(rot_lat);
                    sin_lat = fmin(fmax(sin_lat, -sinlat_extr), sinlat_extr);
                    double cos_lat = sqrt(1.0 - sin_lat * sin_lat);
                    mx[I(m, n)] = mx[I(m, n)] * (float)dcosd(lat_mod);
                    my[I(m, n)] = my[I(m, n)] * 1.0f;
                    if (key_cor) {
                        rlh_s[I(m, n)] = rlh_s[I(m, n)] * (float)sin_lat;
                        rlh_c[I(m, n)] = rlh_c[I(m, n)] * (float)cos_lat;
                    }
                }
            }
        }
    }
}

/* ------------------------------------------------------------------------- */
/* Halo exchange between blocks of one process: shared/mpp/syncborder_block2D_gen_all.fi
 * :139-251 (block-to-block copies).  Directions follow macros/kernel_macros.fi:4-12:
 * 1 nx+, 2 nx-, 3 ny+, 4 ny-, 5 nx+ny+, 6 nx+ny-, 7 nx-ny+, 8 nx-ny-.
 * The unit is one 1-wide halo region of block k filled from the matching boundary
 * region of neighbour block kn (decomposition.f90:94-290). */
void orc_halo_copy(int dir,
                   int nxs, int nxe, int nys, int nye, int bx1, int bx2, int by1, int by2, double *dst,
                   int snxs, int snxe, int snys, int snye, int sbx1, int sbx2, int sby1, int sby2,
                   const double *src)
{
    (void)by2; (void)sby2;
    int hx0, hx1, hy0, hy1;   /* halo points of the receiving block */
    int sx0, sy0;             /* boundary points of the sending block (inverse dir) */
    switch (dir) {
    case 1: hx0 = nxe + 1; hx1 = nxe + 1; hy0 = nys; hy1 = nye; sx0 = snxs; sy0 = snys; break;
    case 2: hx0 = nxs - 1; hx1 = nxs - 1; hy0 = nys; hy1 = nye; sx0 = snxe; sy0 = snys; break;
    case 3: hx0 = nxs; hx1 = nxe; hy0 = nye + 1; hy1 = nye + 1; sx0 = snxs; sy0 = snys; break;
    case 4: hx0 = nxs; hx1 = nxe; hy0 = nys - 1; hy1 = nys - 1; sx0 = snxs; sy0 = snye; break;
    case 5: hx0 = hx1 = nxe + 1; hy0 = hy1 = nye + 1; sx0 = snxs; sy0 = snys; break;
    case 6: hx0 = hx1 = nxe + 1; hy0 = hy1 = nys - 1; sx0 = snxs; sy0 = snye; break;
    case 7: hx0 = hx1 = nxs - 1; hy0 = hy1 = nye + 1; sx0 = snxe; sy0 = snys; break;
    default: hx0 = hx1 = nxs - 1; hy0 = hy1 = nys - 1; sx0 = snxe; sy0 = snye; break;
    }
    (void)snxe; (void)snye;
    const long sld = (long)(sbx2 - sbx1 + 1);
    for (int n = hy0; n <= hy1; ++n)
        for (int m = hx0; m <= hx1; ++m) {
            int sm = sx0 + (m - hx0), sn = sy0 + (n - hy0);
            dst[I(m, n)] = src[(long)(sm - sbx1) + (long)(sn - sby1) * sld];
        }
}
