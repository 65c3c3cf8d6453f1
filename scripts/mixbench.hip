// mixbench.hip -- HBM ceiling for the read/write mixes of the fused SW launches (MI355X).
// Pure streaming (no stencil, no arithmetic beyond a sum) over NI r8 input arrays + one u8
// array into NO r8 output arrays on a 4096^2 interior with the ocean context's layout (pitch
// 4160, rows 4100, fields back to back in one slab, rows 256-B aligned), one cell per lane,
// fully unrolled so every load of a cell is in flight together.  The mixes:
//   fused A (reuse step)  7 in + 4 out     hh_init (mid step)  3 in + 7 out
//   fused B (reuse step) 17 in + 2 out     fused C1            9 in + 6 out
// Prints the achieved GB/s of each mix = the practical ceiling of that launch's byte stream.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

constexpr int W = 4096, H = 4096, PITCH = 4160, ROWS = 4100, MAXA = 24;
struct Args { const double *in[MAXA]; double *out[MAXA]; const unsigned char *bits; };

// 64 x 4 threads, 8-row strips (the k_range mapping), XCD-banded tile order
template <int NI, int NO>
__global__ __launch_bounds__(256) void k_mix(Args a, int ntx, int ntiles)
{
    int tile = (int)blockIdx.x;
    const int per = (ntiles + 7) / 8;
    tile = (tile % 8) * per + tile / 8;
    if (tile >= ntiles) return;
    const int tx = tile % ntx, ty = tile / ntx;
    const int m = 2 + tx * 64 + (int)threadIdx.x;
    if (m > W + 1) return;
    const int nb = 2 + ty * 8, ne = min(H + 1, nb + 7);
    for (int n = nb + (int)threadIdx.y; n <= ne; n += 4) {
        const unsigned c = (unsigned)m + (unsigned)n * PITCH;
        double s = (double)a.bits[c];
#pragma unroll
        for (int k = 0; k < NI; ++k) s += a.in[k][c];
#pragma unroll
        for (int j = 0; j < NO; ++j) a.out[j][c] = s + j;
    }
}

// the register-march shape (sw_kernels.hip k_march): 4 waves side by side, each marching
// 16 rows; ALIGNED = 64 output columns per wave starting on a 512-B boundary, else 62 output
// columns per wave whose loads start one column to the left (the m-1 neighbour lane)
template <int NI, int NO, bool ALIGNED>
__global__ __launch_bounds__(256) void k_mix_march(Args a, int ntx, int ntiles)
{
    int tile = (int)blockIdx.x;
    const int per = (ntiles + 7) / 8;
    tile = (tile % 8) * per + tile / 8;
    if (tile >= ntiles) return;
    const int tx = tile % ntx, ty = tile / ntx;
    const int lane = (int)threadIdx.x & 63, wave = (int)threadIdx.x >> 6;
    const int cols = ALIGNED ? 64 : 62;
    const int mw = 2 + (tx * 4 + wave) * cols;
    if (mw > W + 1) return;
    const int m = ALIGNED ? mw + lane : mw - 1 + lane;
    const bool out = (ALIGNED || (lane >= 1 && lane <= 62)) && m <= W + 1;
    const int nb = 2 + ty * 16, ne = min(H + 1, nb + 15);
    for (int n = nb; n <= ne; ++n) {
        const unsigned c = (unsigned)min(m, W + 2) + (unsigned)n * PITCH;
        double s = (double)a.bits[c];
#pragma unroll
        for (int k = 0; k < NI; ++k) s += a.in[k][c];
        if (out) {
#pragma unroll
            for (int j = 0; j < NO; ++j) a.out[j][c] = s + j;
        }
    }
}

template <int NI, int NO, bool ALIGNED>
static float run_march(const Args &a)
{
    const int cols = 4 * (ALIGNED ? 64 : 62);
    const int ntx = (W + cols - 1) / cols, nty = H / 16, ntiles = ntx * nty;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    hipLaunchKernelGGL((k_mix_march<NI, NO, ALIGNED>), dim3(8 * ((ntiles + 7) / 8)), dim3(256), 0, 0, a, ntx, ntiles);
    (void)hipEventRecord(e0, 0);
    for (int it = 0; it < 10; ++it)
        hipLaunchKernelGGL((k_mix_march<NI, NO, ALIGNED>), dim3(8 * ((ntiles + 7) / 8)), dim3(256), 0, 0, a, ntx, ntiles);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    return ms / 10;
}

template <int NI, int NO>
static float run(const Args &a)
{
    const int ntx = W / 64, nty = H / 8, ntiles = ntx * nty;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    hipLaunchKernelGGL((k_mix<NI, NO>), dim3(8 * ((ntiles + 7) / 8)), dim3(64, 4), 0, 0, a, ntx, ntiles);
    (void)hipEventRecord(e0, 0);
    for (int it = 0; it < 10; ++it)
        hipLaunchKernelGGL((k_mix<NI, NO>), dim3(8 * ((ntiles + 7) / 8)), dim3(64, 4), 0, 0, a, ntx, ntiles);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    return ms / 10;
}

template <int NI, int NO>
static void report(const char *name, const Args &a)
{
    const float ms = run<NI, NO>(a), ma = run_march<NI, NO, true>(a), mm = run_march<NI, NO, false>(a);
    const double cells = (double)W * H, bytes = cells * (8.0 * (NI + NO) + 1.0);
    printf("%-22s %2d in + %2d out  %5.0f B/cell  strip %.4f ms %6.0f GB/s | march64 aligned %.4f ms %6.0f GB/s | "
           "march62 offset %.4f ms %6.0f GB/s\n", name, NI, NO, bytes / cells, ms, bytes / ms / 1e6, ma, bytes / ma / 1e6,
           mm, bytes / mm / 1e6);
}

int main()
{
    const size_t n = (size_t)PITCH * ROWS;
    const size_t fb = ((n * 8 + 16 + 255) / 256) * 256 + 256;   // ocn_ctx.hip allocate()
    char *slab;
    CHK(hipMalloc(&slab, fb * 2 * MAXA + 4096));
    CHK(hipMemset(slab, 0, fb * 2 * MAXA + 4096));
    unsigned char *bits;
    CHK(hipMalloc(&bits, n));
    CHK(hipMemset(bits, 1, n));
    Args a{};
    for (int k = 0; k < MAXA; ++k) a.in[k] = (const double *)(slab + k * fb + 256 - 16);
    for (int k = 0; k < MAXA; ++k) a.out[k] = (double *)(slab + (MAXA + k) * fb + 256 - 16);
    a.bits = bits;
    report<7, 4>("fused A (reuse)", a);
    report<3, 7>("hh_init (mid)", a);
    report<17, 2>("fused B (reuse)", a);
    report<9, 6>("fused C1", a);
    report<1, 1>("copy", a);
    report<0, 8>("write only", a);
    CHK(hipDeviceSynchronize());
    return 0;
}
