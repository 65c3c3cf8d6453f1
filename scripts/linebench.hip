// linebench.hip -- does the one-pass step's store layout cost HBM bandwidth? (MI355X)
// Pure streaming in the register-march shape (4 waves per workgroup, rows marched, the next
// row's loads issued before the current row's stores, XCD-banded tile order) over the one-pass
// step's mix: 6 r8 arrays + the u8 mask byte in, 6 r8 arrays out (97 B per cell), on a 4096^2
// interior laid out as ocn_ctx.hip allocates (pitch 4160, rows 256-B aligned at nx_start).
// Lane layouts (COLS output columns per wave, HALO load-only lanes each side):
//   64 / 0: outputs start on 512-B boundaries (whole 128-B lines per store)
//   60 / 2: the one-pass step's layout -- runs of 480 B starting on 32-B boundaries, so every
//           wave boundary splits a 128-B line between two waves
//   62 / 1: 8-B offset runs (partial 32-B sectors)
//   48 / 8: 384-B runs on 128-B lines (whole lines, a quarter of the lanes idle)
// Every form runs at 2 workgroups per CU (dynamic LDS padding), the one-pass step's occupancy.
// Prints ms and GB/s of each; 10 timed launches after one warm-up launch.
#include <hip/hip_runtime.h>

#include <cstdio>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

constexpr int W = 4096, H = 4096, PITCH = 4160, ROWS = 4100, MAXA = 12, TR = 28;
struct Args { const double *in[MAXA]; double *out[MAXA]; const unsigned char *bits; };

template <int NI, int NO, int COLS, int HALO>
__global__ __launch_bounds__(256) void k_line(Args a, int ntx, int ntiles)
{
    int tile = (int)blockIdx.x;
    const int per = (ntiles + 7) / 8;
    tile = (tile % 8) * per + tile / 8;
    if (tile >= ntiles) return;
    const int tx = tile % ntx, ty = tile / ntx;
    const int lane = (int)threadIdx.x & 63, wave = (int)threadIdx.x >> 6;
    const int mw = 2 + tx * COLS;                       // waves stacked vertically (OCN_STEP_VERT)
    const int m = mw - HALO + lane;
    const bool out = lane >= HALO && lane < 64 - HALO && m <= W + 1;
    const int nb = 2 + (ty * 4 + wave) * TR, ne = min(H + 1, nb + TR - 1);
    if (nb > H + 1) return;
    const unsigned mc = (unsigned)min(m, W + 3);
    double q[NI + 1];
    {
        const unsigned c = mc + (unsigned)nb * PITCH;
        q[NI] = (double)a.bits[c];
#pragma unroll
        for (int k = 0; k < NI; ++k) q[k] = a.in[k][c];
    }
    for (int n = nb; n <= ne; ++n) {
        double s = q[NI];
#pragma unroll
        for (int k = 0; k < NI; ++k) s += q[k];
        if (n < ne) {
            const unsigned c = mc + (unsigned)(n + 1) * PITCH;
            q[NI] = (double)a.bits[c];
#pragma unroll
            for (int k = 0; k < NI; ++k) q[k] = a.in[k][c];
        }
        const unsigned c = mc + (unsigned)n * PITCH;
        if (NO == 0 && s == -12345.0) a.out[0][c] = s;   // (never: keeps the loads)
        if (out) {
#pragma unroll
            for (int j = 0; j < NO; ++j) a.out[j][c] = s + j;
        }
    }
}

// 60 / 2 lanes, 4 waves side by side (HORIZ), optionally staged through LDS every STAGE rows
// (STAGE > 0: after a workgroup barrier wave w stores columns [64 w, 64 w + 64) of the 240)
template <int NI, int NO, int STAGE>
__global__ __launch_bounds__(256) void k_line_h(Args a, int ntx, int ntiles)
{
    __shared__ double sb[2][STAGE > 0 ? STAGE : 1][NO > 0 ? NO : 1][240];
    int tile = (int)blockIdx.x;
    const int per = (ntiles + 7) / 8;
    tile = (tile % 8) * per + tile / 8;
    if (tile >= ntiles) return;
    const int tx = tile % ntx, ty = tile / ntx;
    const int lane = (int)threadIdx.x & 63, wave = (int)threadIdx.x >> 6;
    const int wg0 = 2 + tx * 240, mw = wg0 + wave * 60;
    const bool full = wg0 + 239 <= W + 1;
    if (!full && STAGE > 0) return;   // (the edge workgroup: not measured in the staged form)
    const int m = mw - 2 + lane;
    const bool out = lane >= 2 && lane < 62 && m <= W + 1;
    const int nb = 2 + ty * TR, ne = min(H + 1, nb + TR - 1);
    const unsigned mc = (unsigned)min(m, W + 3);
    double q[NI + 1];
    {
        const unsigned c = mc + (unsigned)nb * PITCH;
        q[NI] = (double)a.bits[c];
#pragma unroll
        for (int k = 0; k < NI; ++k) q[k] = a.in[k][c];
    }
    for (int n = nb; n <= ne; ++n) {
        double s = q[NI];
#pragma unroll
        for (int k = 0; k < NI; ++k) s += q[k];
        if (n < ne) {
            const unsigned c = mc + (unsigned)(n + 1) * PITCH;
            q[NI] = (double)a.bits[c];
#pragma unroll
            for (int k = 0; k < NI; ++k) q[k] = a.in[k][c];
        }
        if constexpr (STAGE == 0) {
            const unsigned c = mc + (unsigned)n * PITCH;
            if (out) {
#pragma unroll
                for (int j = 0; j < NO; ++j) a.out[j][c] = s + j;
            }
        } else {
            const int k = (n - nb) % STAGE, buf = ((n - nb) / STAGE) & 1;
            if (out) {
#pragma unroll
                for (int j = 0; j < NO; ++j) sb[buf][k][j][wave * 60 + lane - 2] = s + j;
            }
            if (k == STAGE - 1 || n == ne) {
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
                __builtin_amdgcn_s_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
                const int col = wave * 64 + lane, cc = min(col, 239);
                for (int kk = 0; kk <= k; ++kk) {
                    const unsigned c = (unsigned)(wg0 + cc) + (unsigned)(n - k + kk) * PITCH;
                    if (col < 240) {
#pragma unroll
                        for (int j = 0; j < NO; ++j) a.out[j][c] = sb[buf][kk][j][cc];
                    }
                }
            }
        }
    }
}

template <int NI, int NO, int STAGE>
static float run_h(const Args &a)
{
    const int ntx = STAGE > 0 ? W / 240 : (W + 239) / 240, nty = (H + TR - 1) / TR, ntiles = ntx * nty;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    // dynamic LDS pads every form to 2 workgroups per CU (the one-pass step's occupancy)
    const size_t dyn = STAGE == 4 ? 0 : 70 * 1024 - (size_t)2 * (STAGE > 0 ? STAGE : 1) * NO * 240 * 8;
    hipLaunchKernelGGL((k_line_h<NI, NO, STAGE>), dim3(8 * ((ntiles + 7) / 8)), dim3(256), dyn, 0, a, ntx, ntiles);
    (void)hipEventRecord(e0, 0);
    for (int it = 0; it < 10; ++it)
        hipLaunchKernelGGL((k_line_h<NI, NO, STAGE>), dim3(8 * ((ntiles + 7) / 8)), dim3(256), dyn, 0, a, ntx, ntiles);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    return ms / 10;
}

template <int NI, int NO, int COLS, int HALO>
static float run(const Args &a)
{
    const int ntx = (W + COLS - 1) / COLS, nty = (H + 4 * TR - 1) / (4 * TR), ntiles = ntx * nty;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    hipLaunchKernelGGL((k_line<NI, NO, COLS, HALO>), dim3(8 * ((ntiles + 7) / 8)), dim3(256), 70 * 1024, 0, a, ntx, ntiles);
    (void)hipEventRecord(e0, 0);
    for (int it = 0; it < 10; ++it)
        hipLaunchKernelGGL((k_line<NI, NO, COLS, HALO>), dim3(8 * ((ntiles + 7) / 8)), dim3(256), 70 * 1024, 0, a, ntx, ntiles);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    return ms / 10;
}

template <int NI, int NO>
static void report(const char *name, const Args &a)
{
    const double bytes = (double)W * H * (8.0 * (NI + NO) + (NI ? 1.0 : 0.0));
    const float t64 = run<NI, NO, 64, 0>(a), t60 = run<NI, NO, 60, 2>(a), t62 = run<NI, NO, 62, 1>(a),
                t48 = run<NI, NO, 48, 8>(a);
    printf("%-16s %2d in + %2d out | 64/0 %.4f ms %5.0f GB/s | 60/2 %.4f ms %5.0f GB/s | 62/1 %.4f ms %5.0f GB/s | "
           "48/8 %.4f ms %5.0f GB/s\n", name, NI, NO, t64, bytes / t64 / 1e6, t60, bytes / t60 / 1e6, t62,
           bytes / t62 / 1e6, t48, bytes / t48 / 1e6);
    // staged forms cover 4080 of the 4096 columns (full workgroups only): GB/s on the bytes moved
    const double bs = bytes * 4080.0 / 4096.0;
    const float h0 = run_h<NI, NO, 0>(a), h1 = run_h<NI, NO, 1>(a), h2 = run_h<NI, NO, 2>(a), h4 = run_h<NI, NO, 4>(a);
    printf("%-16s   horizontal 60/2 %.4f ms %5.0f GB/s | staged/1 %.4f ms %5.0f GB/s | staged/2 %.4f ms %5.0f GB/s | "
           "staged/4 %.4f ms %5.0f GB/s\n", name, h0, bytes / h0 / 1e6, h1, bs / h1 / 1e6, h2, bs / h2 / 1e6, h4,
           bs / h4 / 1e6);
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
    for (int r = 0; r < 2; ++r) {
        report<6, 6>("one-pass mix", a);
        report<0, 6>("write only", a);
    }
    CHK(hipDeviceSynchronize());
    return 0;
}
