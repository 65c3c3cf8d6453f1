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

// grid_base_init + grid_geo_init at one point of the metric range (grid_kernels.f90:94-202,
// grid_parameters.f90:80-181): the four passes (t, u, v, b points) each scale their own pair of
// metrics, the b pass the Coriolis term.  ct / cv: (float) dcosd(lat_mod) of the row's yt / yv;
// sin_v, cosy_v: dsind / dcosd of its yv; cos_xu: dcosd of the column's xu.  out: OCN_DX .. OCN_R_DISS.
__device__ __forceinline__ void grid_metrics(const GridInit &q, float ct, float cv, double sin_v, double cosy_v,
                                             double cos_xu, float *out)
{
    if (!q.curve) ct = cv = 1.0f;
    out[OCN_DX - OCN_DX] = q.sx * ct; out[OCN_DY - OCN_DX] = q.sy * 1.0f;    // t points (xt, yt)
    out[OCN_DXT - OCN_DX] = q.sx * ct; out[OCN_DYH - OCN_DX] = q.sy * 1.0f;  // u points (xu, yt)
    out[OCN_DXH - OCN_DX] = q.sx * cv; out[OCN_DYT - OCN_DX] = q.sy * 1.0f;  // v points (xt, yv)
    out[OCN_DXB - OCN_DX] = q.sx * cv; out[OCN_DYB - OCN_DX] = q.sy * 1.0f;  // b points (xu, yv)
    float rlh = q.cor;
    if (q.curve) {
        double s = sin_v * q.cos_rot + cos_xu * cosy_v * q.sin_rot;
        s = fmin(fmax(s, -q.sin_extr), q.sin_extr);
        rlh = rlh * (float)s;
    } else {
        rlh = rlh / q.sqrt2;
    }
    out[OCN_RLH_S - OCN_DX] = rlh;
    out[OCN_R_DISS - OCN_DX] = 0.0f;
}

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
    // grid_base_init + grid_geo_init on [nx_start-1, nx_end+1] x [ny_start-1, ny_end+1] (zero
    // elsewhere, the Coriolis term 2 * EarthAngVel)
    float v[OCN_NUM_R4 - OCN_DX] = {0.0f};
    v[OCN_RLH_S - OCN_DX] = q.cor;
    if (m >= g.nx_start - 1 && m <= g.nx_end + 1 && n >= g.ny_start - 1 && n <= g.ny_end + 1) {
        const int r = n - g.bnd_y1;
        grid_metrics(q, q.cos_t[r], q.cos_v[r], q.sin_v[r], q.cosy_v[r], q.cos_xu[m - g.bnd_x1], v);
    }
    for (int id = OCN_DX; id < OCN_NUM_R4; ++id) q.r4[id][at] = v[id - OCN_DX];
}

// The metric values of the rows just outside the block's metric range (bnd_y1 and bnd_y2, where
// the reference leaves 0, and the two rows beyond each, outside its arrays) as the neighbour block
// above / below forms them on its interior -- the same global row, the same arithmetic: the
// one-pass steps form their halo points' depths and stresses there (ocn_ctx.hip one_step_x2,
// one_step_x4).  Column nx_start - 1 (the compact row tables' column).
__global__ void k_ext_rows(GridInit q)
{
    const int i = (int)threadIdx.x;
    if (i >= kExtRows) return;
    grid_metrics(q, q.ext_ct[i], q.ext_cv[i], q.ext_sin_v[i], q.ext_cosy_v[i], q.cos_xu[q.g.nx_start - 1 - q.g.bnd_x1],
                 q.ext + i * (OCN_NUM_R4 - OCN_DX));
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
    int rc = check_launch();
    if (rc || !q.ext) return rc;
    hipLaunchKernelGGL(k_ext_rows, dim3(1), dim3(64), 0, s, q);
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
