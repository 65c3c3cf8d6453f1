// init_kernels.hip -- the initial state on the device (ocn_ctx.hip init_state).
//
// Reference: control/init_data.f90:29-125 (init_grid_data, init_ocean_data) over
//   kernel/service/grid_kernels.f90:18-92   lu_init, lu_lv_init (masks from the basin mask)
//   kernel/service/grid_kernels.f90:94-202  grid_base_init (uniform steps on the metric range)
//   kernel/service/grid_kernels.f90 grid_geo_init + grid_parameters.f90:80-181 (cartesian /
//                                            spherical metric scaling, Coriolis)
//   kernel/shallow_water/vel_ssh.f90:15-38  gaussian_elimination_kernel (ssh, tracers)
// Every 2-D field is formed here, one thread per point of the block array.  What stays on the host
// is O(nx + ny): the separable trigonometric factors of the grid -- cos(lat) per row, sin / cos
// of the rotated latitude's row and column terms -- taken from the host's libm exactly as the
// reference takes them, so the device's products are the reference's bit for bit.  The Gaussian's
// exp is ocn_exp.h (the same libm's algorithm restated).
#include <cmath>

#include "ocn_exp.h"
#include "ocn_internal.h"

namespace ocn {

__global__ __launch_bounds__(256) void k_init_grid(GridInit q)
{
    const ocn_block &g = q.g;
    const int w = g.bnd_x2 - g.bnd_x1 + 1, h = g.bnd_y2 - g.bnd_y1 + 1;
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (long)w * h) return;
    const int m = g.bnd_x1 + (int)(i % w), n = g.bnd_y1 + (int)(i / w);
    const long at = (long)(m - g.bnd_x1) + (long)(n - g.bnd_y1) * g.pitch;
    // lu_init: sea where the basin mask is 0 (mask(m, n), 1-based global indices)
    auto lu = [&](int mm, int nn) -> float { return q.mask[(long)(mm - 1) + (long)(nn - 1) * q.nx] == 0 ? 1.0f : 0.0f; };
    const float a = lu(m, n);
    float luh = 0.0f, luu = 0.0f, llu = 0.0f, llv = 0.0f, lcu = 0.0f, lcv = 0.0f;
    if (m <= g.bnd_x2 - 1 && n <= g.bnd_y2 - 1) {   // lu_lv_init
        const float b = lu(m + 1, n), c = lu(m, n + 1), d = lu(m + 1, n + 1);
        if (a + b + c + d > 0.5f) luh = 1.0f;
        if (a * b * c * d > 0.5f) luu = 1.0f;
        if (a + b > 0.5f) llu = 1.0f;
        if (a + c > 0.5f) llv = 1.0f;
        if (a * b > 0.5f) lcu = 1.0f;
        if (a * c > 0.5f) lcv = 1.0f;
    }
    q.r4[OCN_LU][at] = a;
    q.r4[OCN_LUH][at] = luh; q.r4[OCN_LUU][at] = luu; q.r4[OCN_LLU][at] = llu;
    q.r4[OCN_LLV][at] = llv; q.r4[OCN_LCU][at] = lcu; q.r4[OCN_LCV][at] = lcv;
    // grid_base_init + grid_geo_init on [nx_start-1, nx_end+1] x [ny_start-1, ny_end+1]; the four
    // passes (t, u, v, b points) each scale their own pair of metrics, the b pass the Coriolis term
    float dx = 0.0f, dy = 0.0f, dxt = 0.0f, dyt = 0.0f, dxh = 0.0f, dyh = 0.0f, dxb = 0.0f, dyb = 0.0f;
    float rlh = q.cor;
    if (m >= g.nx_start - 1 && m <= g.nx_end + 1 && n >= g.ny_start - 1 && n <= g.ny_end + 1) {
        const int r = n - g.bnd_y1;
        const float ct = q.curve ? q.cos_t[r] : 1.0f, cv = q.curve ? q.cos_v[r] : 1.0f;   // (float) dcosd(lat_mod)
        dx = q.sx * ct; dy = q.sy * 1.0f;      // t points (xt, yt)
        dxt = q.sx * ct; dyh = q.sy * 1.0f;    // u points (xu, yt)
        dxh = q.sx * cv; dyt = q.sy * 1.0f;    // v points (xt, yv)
        dxb = q.sx * cv; dyb = q.sy * 1.0f;    // b points (xu, yv)
        if (q.curve) {
            double s = q.sin_v[r] * q.cos_rot + q.cos_xu[m - g.bnd_x1] * q.cosy_v[r] * q.sin_rot;
            s = fmin(fmax(s, -q.sin_extr), q.sin_extr);
            rlh = rlh * (float)s;
        } else {
            rlh = rlh / q.sqrt2;
        }
    }
    q.r4[OCN_DX][at] = dx; q.r4[OCN_DY][at] = dy; q.r4[OCN_DXT][at] = dxt; q.r4[OCN_DYT][at] = dyt;
    q.r4[OCN_DXH][at] = dxh; q.r4[OCN_DYH][at] = dyh; q.r4[OCN_DXB][at] = dxb; q.r4[OCN_DYB][at] = dyb;
    q.r4[OCN_RLH_S][at] = rlh;
    q.r4[OCN_R_DISS][at] = 0.0f;
}

// gaussian_elimination_kernel (vel_ssh.f90:15-38): on the interior where lu > 0.5, centre
// (nx/2, ny/2); zero elsewhere in the array
__global__ __launch_bounds__(256) void k_gaussian(ocn_block g, double *p, const float *lu, int nx0, int ny0,
                                                  double coef, double two_s2)
{
    const int w = g.bnd_x2 - g.bnd_x1 + 1, h = g.bnd_y2 - g.bnd_y1 + 1;
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (long)w * h) return;
    const int m = g.bnd_x1 + (int)(i % w), n = g.bnd_y1 + (int)(i / w);
    const long at = (long)(m - g.bnd_x1) + (long)(n - g.bnd_y1) * g.pitch;
    double v = 0.0;
    if (m >= g.nx_start && m <= g.nx_end && n >= g.ny_start && n <= g.ny_end && lu[at] > 0.5f) {
        const double dx = (double)(m - nx0) / ((double)nx0 * 0.25);
        const double dy = (double)(n - ny0) / ((double)ny0 * 0.25);
        v = coef * exp_libm(-((dx * dx + dy * dy) / two_s2));
    }
    p[at] = v;
}

__global__ __launch_bounds__(256) void k_fill_field(ocn_block g, double *p, double v)
{
    const int w = g.bnd_x2 - g.bnd_x1 + 1, h = g.bnd_y2 - g.bnd_y1 + 1;
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (long)w * h) return;
    p[(i % w) + (i / w) * g.pitch] = v;
}

static unsigned grid_of(const ocn_block &g)
{
    const long pts = (long)(g.bnd_x2 - g.bnd_x1 + 1) * (g.bnd_y2 - g.bnd_y1 + 1);
    return (unsigned)((pts + 255) / 256);
}

int launch_init_grid(const GridInit &q, hipStream_t s)
{
    hipLaunchKernelGGL(k_init_grid, dim3(grid_of(q.g)), dim3(256), 0, s, q);
    return check_launch();
}

int launch_fill_field(const ocn_block &g, double *p, double v, hipStream_t s)
{
    hipLaunchKernelGGL(k_fill_field, dim3(grid_of(g)), dim3(256), 0, s, g, p, v);
    return check_launch();
}

int launch_gaussian(const ocn_block &g, double *p, const float *lu, int nx0, int ny0, double sigma, hipStream_t s)
{
    const double kDPi = 3.14159265358979;   // constants.f90:17
    const double coef = 1.0 / (std::sqrt(2.0 * kDPi) * sigma), two_s2 = 2.0 * sigma * sigma;
    hipLaunchKernelGGL(k_gaussian, dim3(grid_of(g)), dim3(256), 0, s, g, p, lu, nx0, ny0, coef, two_s2);
    return check_launch();
}

}  // namespace ocn
