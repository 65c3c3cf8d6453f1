// stenbench.hip -- microbenchmark: what does a 5-point fp64 stencil over many arrays cost on
// MI355X compared with pure streaming of the same arrays?  Also the calibration kernel for
// rocprofv3 FETCH_SIZE with 8-byte-per-lane loads (pointwise kernel: exactly NI*8 B/cell read).
//   point : out[j][c] = sum_k in[k][c]                              (NI*8 + NO*8 B/cell)
//   sten5 : out[j][c] = sum_k in[k][c] + in[k][c+-1] + in[k][c+-p]  (same algorithmic bytes)
// Same workgroup shape as sw_kernels.hip (64 x 4 threads, ROWS-row strips); optional XCD
// banding of the tile order.  Interior m in [1, W-2], n in [1, H-2]: every access in bounds.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

constexpr int NI = 20, NO = 2, W = 4096, H = 4096, PITCH = 4160, ROWS = 8;

struct Args { const double *in[NI]; double *out[NO]; };

template <int MODE, int REMAP>
__global__ __launch_bounds__(256) void k_bench(Args a, int ntx, int ntiles)
{
    int tile = (int)blockIdx.x;
    if (REMAP) {
        const int per = (ntiles + 7) / 8;
        tile = (tile % 8) * per + tile / 8;
        if (tile >= ntiles) return;
    }
    const int tx = tile % ntx, ty = tile / ntx;
    const int m = 1 + tx * 64 + (int)threadIdx.x;
    if (m > W - 2) return;
    const int nb = 1 + ty * ROWS, ne = min(H - 2, nb + ROWS - 1);
    const unsigned p = PITCH;
    for (int n = nb + __builtin_amdgcn_readfirstlane((int)threadIdx.y); n <= ne; n += 4) {
        const unsigned c = (unsigned)m + (unsigned)n * p;
        double s = 0.0;
#pragma unroll
        for (int k = 0; k < NI; ++k) {
            const double *q = a.in[k];
            if (MODE == 0) s += q[c];
            else s += q[c] + q[c + 1] + q[c - 1] + q[c + p] + q[c - p];
        }
#pragma unroll
        for (int j = 0; j < NO; ++j) a.out[j][c] = s + j;
    }
}

template <int MODE, int REMAP>
static float run(const Args &a, int iters)
{
    const int ntx = (W - 2 + 63) / 64, nty = (H - 2 + ROWS - 1) / ROWS, ntiles = ntx * nty;
    const int nb = REMAP ? 8 * ((ntiles + 7) / 8) : ntiles;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    hipLaunchKernelGGL((k_bench<MODE, REMAP>), dim3(nb), dim3(64, 4), 0, 0, a, ntx, ntiles);
    (void)hipEventRecord(e0, 0);
    for (int it = 0; it < iters; ++it) hipLaunchKernelGGL((k_bench<MODE, REMAP>), dim3(nb), dim3(64, 4), 0, 0, a, ntx, ntiles);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    (void)hipEventDestroy(e0); (void)hipEventDestroy(e1);
    return ms / iters;
}

int main()
{
    const size_t n = (size_t)PITCH * H;
    Args a{};
    std::vector<double *> bufs;
    for (int k = 0; k < NI + NO; ++k) {
        double *q;
        CHK(hipMalloc(&q, n * 8));
        CHK(hipMemset(q, 0, n * 8));
        bufs.push_back(q);
    }
    for (int k = 0; k < NI; ++k) a.in[k] = bufs[k];
    for (int j = 0; j < NO; ++j) a.out[j] = bufs[NI + j];
    const double cells = (double)(W - 2) * (H - 2), bytes = cells * 8.0 * (NI + NO);
    const float t0 = run<0, 0>(a, 10), t1 = run<0, 1>(a, 10), t2 = run<1, 0>(a, 10), t3 = run<1, 1>(a, 10);
    printf("stenbench %dx%d, %d r8 in + %d r8 out (%.0f B/cell algorithmic)\n", W, H, NI, NO, bytes / cells);
    printf("point        %.4f ms  %6.0f GB/s\n", t0, bytes / t0 / 1e6);
    printf("point+xcd    %.4f ms  %6.0f GB/s\n", t1, bytes / t1 / 1e6);
    printf("sten5        %.4f ms  %6.0f GB/s\n", t2, bytes / t2 / 1e6);
    printf("sten5+xcd    %.4f ms  %6.0f GB/s\n", t3, bytes / t3 / 1e6);
    CHK(hipDeviceSynchronize());
    for (double *q : bufs) CHK(hipFree(q));
    return 0;
}
