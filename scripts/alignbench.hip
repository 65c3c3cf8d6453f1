// alignbench.hip -- HBM rate of a register-march launch shape by the width and alignment of a
// wave's output columns (MI355X).  Same layout as the ocean context (pitch 4160, rows 4100,
// fields back to back, A(nx_start, n) on 256-B boundaries), one cell per lane, 4 waves side by
// side, 16 rows per wave.  A wave loads 64 consecutive columns starting LEFT columns before its
// first output column and stores COLS columns:
//   COLS 64 / LEFT 0: every store covers whole 128-B lines;
//   COLS 62 / LEFT 1: output runs start on any 8-B boundary (the fused B layout);
//   COLS 60 / LEFT 2: output runs start on 32-B boundaries;
//   COLS 56 / LEFT 4: output runs start on 64-B boundaries.
// Question answered: which of these a march that needs +-2 columns of halo lanes should use.
#include <hip/hip_runtime.h>

#include <cstdio>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

constexpr int W = 4096, H = 4096, PITCH = 4160, ROWS = 4100, MAXA = 24;
struct Args { const double *in[MAXA]; double *out[MAXA]; const unsigned char *bits; };

template <int NI, int NO, int COLS, int LEFT>
__global__ __launch_bounds__(256) void k_mix(Args a, int ntx, int ntiles)
{
    int tile = (int)blockIdx.x;
    const int per = (ntiles + 7) / 8;
    tile = (tile % 8) * per + tile / 8;
    if (tile >= ntiles) return;
    const int tx = tile % ntx, ty = tile / ntx;
    const int lane = (int)threadIdx.x & 63, wave = (int)threadIdx.x >> 6;
    const int mw = 2 + (tx * 4 + wave) * COLS;
    if (mw > W + 1) return;
    const int m = mw - LEFT + lane;
    const bool out = lane >= LEFT && lane < LEFT + COLS && m <= W + 1;
    const int nb = 2 + ty * 16, ne = min(H + 1, nb + 15);
    for (int n = nb; n <= ne; ++n) {
        const unsigned c = (unsigned)min(max(m, 0), W + 3) + (unsigned)n * PITCH;
        double s = (double)a.bits[c];
#pragma unroll
        for (int k = 0; k < NI; ++k) s += a.in[k][c];
        if (out) {
#pragma unroll
            for (int j = 0; j < NO; ++j) a.out[j][c] = s + j;
        }
    }
}

template <int NI, int NO, int COLS, int LEFT>
static float run(const Args &a)
{
    const int cols = 4 * COLS;
    const int ntx = (W + cols - 1) / cols, nty = H / 16, ntiles = ntx * nty;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    hipLaunchKernelGGL((k_mix<NI, NO, COLS, LEFT>), dim3(8 * ((ntiles + 7) / 8)), dim3(256), 0, 0, a, ntx, ntiles);
    (void)hipEventRecord(e0, 0);
    for (int it = 0; it < 10; ++it)
        hipLaunchKernelGGL((k_mix<NI, NO, COLS, LEFT>), dim3(8 * ((ntiles + 7) / 8)), dim3(256), 0, 0, a, ntx, ntiles);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    return ms / 10;
}

template <int NI, int NO>
static void report(const char *name, const Args &a)
{
    const double cells = (double)W * H, bytes = cells * (8.0 * (NI + NO) + 1.0);
    const float t64 = run<NI, NO, 64, 0>(a), t62 = run<NI, NO, 62, 1>(a), t60 = run<NI, NO, 60, 2>(a),
                t56 = run<NI, NO, 56, 4>(a);
    printf("%-16s %2d in + %2d out %4.0f B/cell | 64/line %6.0f GB/s | 62/8B %6.0f GB/s | 60/32B %6.0f GB/s | "
           "56/64B %6.0f GB/s\n", name, NI, NO, bytes / cells, bytes / t64 / 1e6, bytes / t62 / 1e6, bytes / t60 / 1e6,
           bytes / t56 / 1e6);
}

int main()
{
    const size_t n = (size_t)PITCH * ROWS;
    const size_t fb = ((n * 8 + 16 + 255) / 256) * 256 + 256;
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
    for (int rep = 0; rep < 2; ++rep) {
        report<0, 8>("write only", a);
        report<1, 1>("copy", a);
        report<17, 5>("B role-flip", a);
        report<17, 12>("B + CA fused", a);
        report<10, 6>("one-pass step", a);
        report<7, 7>("CA", a);
    }
    CHK(hipDeviceSynchronize());
    return 0;
}
