// membench.hip -- HBM streaming microbenchmark for the SW stencil kernels' access pattern.
// Sums NI input r8 arrays (+ optional r4 arrays) into NO output r8 arrays over a 2-D
// (pitch x rows) field, using the same 64x4-thread strip walk as sw_kernels.hip, with
// 8-byte (1 cell/lane) or 16-byte (2 cells/lane) accesses.  Prints achieved GB/s.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

struct Args { const double *in[16]; const float *in4[16]; double *out[16]; int ni, ni4, no; long pitch; int w, h; };

template <int ROWS, int VEC>
__global__ __launch_bounds__(256) void k_strip(Args a)
{
    const int m = ((int)blockIdx.x * 64 + (int)threadIdx.x) * VEC;
    if (m >= a.w) return;
    const int nb = (int)blockIdx.y * ROWS;
    const int ne = min(a.h, nb + ROWS);
    for (int n = nb + (int)threadIdx.y; n < ne; n += 4) {
        const long i = (long)m + (long)n * a.pitch;
        if (VEC == 1) {
            double s = 0.0;
            for (int k = 0; k < a.ni; ++k) s += a.in[k][i];
            for (int k = 0; k < a.ni4; ++k) s += (double)a.in4[k][i];
            for (int k = 0; k < a.no; ++k) a.out[k][i] = s + k;
        } else {
            double2 s = make_double2(0.0, 0.0);
            for (int k = 0; k < a.ni; ++k) { double2 v = *(const double2 *)(a.in[k] + i); s.x += v.x; s.y += v.y; }
            for (int k = 0; k < a.ni4; ++k) { float2 v = *(const float2 *)(a.in4[k] + i); s.x += v.x; s.y += v.y; }
            for (int k = 0; k < a.no; ++k) { double2 r = make_double2(s.x + k, s.y + k); *(double2 *)(a.out[k] + i) = r; }
        }
    }
}

template <int ROWS, int VEC>
static float run(Args a, int iters)
{
    dim3 b(64, 4), g((a.w / VEC + 63) / 64, (a.h + ROWS - 1) / ROWS);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    hipLaunchKernelGGL((k_strip<ROWS, VEC>), g, b, 0, 0, a);
    (void)hipEventRecord(e0, 0);
    for (int it = 0; it < iters; ++it) hipLaunchKernelGGL((k_strip<ROWS, VEC>), g, b, 0, 0, a);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms; (void)hipEventElapsedTime(&ms, e0, e1);
    return ms / iters;
}

int main()
{
    const int w = 4096, h = 4100;
    const long pitch = 4160;
    const size_t n = (size_t)pitch * h;
    std::vector<double *> bufs;
    for (int k = 0; k < 32; ++k) { double *p; CHK(hipMalloc(&p, n * 8)); CHK(hipMemset(p, 0, n * 8)); bufs.push_back(p); }
    std::vector<float *> b4;
    for (int k = 0; k < 16; ++k) { float *p; CHK(hipMalloc(&p, n * 4)); CHK(hipMemset(p, 0, n * 4)); b4.push_back(p); }
    struct Cfg { int ni, ni4, no; } cfgs[] = {{1, 0, 1}, {4, 0, 2}, {9, 3, 6}, {10, 14, 12}, {16, 13, 6}, {6, 12, 2}};
    for (auto c : cfgs) {
        if (c.ni > 16 || c.ni4 > 16 || c.no > 16) { printf("bad cfg\n"); return 1; }
        Args a{};
        for (int k = 0; k < c.ni; ++k) a.in[k] = bufs[k];
        for (int k = 0; k < c.ni4; ++k) a.in4[k] = b4[k];
        for (int k = 0; k < c.no; ++k) a.out[k] = bufs[16 + k];
        a.ni = c.ni; a.ni4 = c.ni4; a.no = c.no; a.pitch = pitch; a.w = w; a.h = h;
        const double bytes = (double)w * h * (8.0 * (c.ni + c.no) + 4.0 * c.ni4);
        float t1 = run<32, 1>(a, 10), t2 = run<32, 2>(a, 10), t3 = run<8, 2>(a, 10), t4 = run<128, 2>(a, 10),
              t5 = run<128, 1>(a, 10);
        printf("in8=%2d in4=%2d out8=%2d  B/cell=%3.0f  vec1/r32 %6.0f  vec2/r32 %6.0f  vec2/r8 %6.0f  vec2/r128 %6.0f  vec1/r128 %6.0f GB/s\n",
               c.ni, c.ni4, c.no, bytes / ((double)w * h), bytes / t1 / 1e6, bytes / t2 / 1e6, bytes / t3 / 1e6,
               bytes / t4 / 1e6, bytes / t5 / 1e6);
    }
    return 0;
}
