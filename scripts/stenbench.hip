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


// ---- mixed pattern: arrays 0..NS-1 read 5-point, NS..NI-1 pointwise ----
constexpr int NS = 10;
__device__ __forceinline__ double lane_next(double x)   // value of lane + 1 (wave_shl:1)
{
    const int lo = __builtin_amdgcn_mov_dpp(__double2loint(x), 0x130, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(x), 0x130, 0xf, 0xf, false);
    return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double lane_prev(double x)   // value of lane - 1 (wave_shr:1)
{
    const int lo = __builtin_amdgcn_mov_dpp(__double2loint(x), 0x138, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(x), 0x138, 0xf, 0xf, false);
    return __hiloint2double(hi, lo);
}

// plain loads, the sw_kernels.hip mapping (64 x 4 threads, ROWS-row strips)
__global__ __launch_bounds__(256) void k_mix_plain(Args a, int ntx)
{
    const int tile = (int)blockIdx.x, tx = tile % ntx, ty = tile / ntx;
    const int m = 1 + tx * 64 + (int)threadIdx.x;
    if (m > W - 2) return;
    const int nb = 1 + ty * ROWS, ne = min(H - 2, nb + ROWS - 1);
    const unsigned p = PITCH;
    for (int n = nb + __builtin_amdgcn_readfirstlane((int)threadIdx.y); n <= ne; n += 4) {
        const unsigned c = (unsigned)m + (unsigned)n * p;
        double s = 0.0;
#pragma unroll
        for (int k = 0; k < NS; ++k) {
            const double *q = a.in[k];
            s += q[c] + q[c + 1] + q[c - 1] + q[c + p] + q[c - p];
        }
#pragma unroll
        for (int k = NS; k < NI; ++k) s += a.in[k][c];
#pragma unroll
        for (int j = 0; j < NO; ++j) a.out[j][c] = s + j;
    }
}

// register march: a wave owns 62 output columns (64 loaded, neighbours by DPP); 4 waves side
// by side; every thread walks MR rows keeping rows n-1, n, n+1 of the 5-point arrays in registers
template <int MR>
__global__ __launch_bounds__(256) void k_mix_march(Args a, int ntx)
{
    const int tile = (int)blockIdx.x, tx = tile % ntx, ty = tile / ntx;
    const int lane = (int)threadIdx.x & 63, wave = (int)threadIdx.x >> 6;
    const int m = tx * 248 + wave * 62 + lane;                 // loaded column; outputs for lanes 1..62
    const int ml = min(m, W - 1);
    const bool out = lane >= 1 && lane <= 62 && m >= 1 && m <= W - 2;
    const int nb = 1 + ty * MR, ne = min(H - 2, nb + MR - 1);
    const unsigned p = PITCH;
    double r0[NS], r1[NS], r2[NS];
#pragma unroll
    for (int k = 0; k < NS; ++k) {
        r0[k] = a.in[k][(unsigned)ml + (unsigned)(nb - 1) * p];
        r1[k] = a.in[k][(unsigned)ml + (unsigned)nb * p];
    }
    for (int n = nb; n <= ne; ++n) {
        const unsigned c = (unsigned)ml + (unsigned)n * p;
#pragma unroll
        for (int k = 0; k < NS; ++k) r2[k] = a.in[k][c + p];
        double s = 0.0;
#pragma unroll
        for (int k = 0; k < NS; ++k) s += r1[k] + lane_next(r1[k]) + lane_prev(r1[k]) + r2[k] + r0[k];
#pragma unroll
        for (int k = NS; k < NI; ++k) s += a.in[k][c];
        if (out) {
#pragma unroll
            for (int j = 0; j < NO; ++j) a.out[j][c] = s + j;
        }
#pragma unroll
        for (int k = 0; k < NS; ++k) { r0[k] = r1[k]; r1[k] = r2[k]; }
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
    // mixed pattern: plain loads vs register march (+ bitwise agreement of the two)
    const size_t nout = n;
    std::vector<double> o1(nout), o2(nout);
    auto timeit = [&](auto launch) {
        hipEvent_t e0, e1;
        (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
        launch();
        (void)hipEventRecord(e0, 0);
        for (int it = 0; it < 10; ++it) launch();
        (void)hipEventRecord(e1, 0);
        (void)hipEventSynchronize(e1);
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, e0, e1);
        return ms / 10;
    };
    // distinct inputs so that a wrong neighbour would show
    std::vector<double> h(n);
    for (int k = 0; k < NI; ++k) {
        for (size_t i = 0; i < n; ++i) h[i] = (double)((i * 2654435761u + k * 97u) % 1000003u) * 1e-3;
        CHK(hipMemcpy(bufs[k], h.data(), n * 8, hipMemcpyHostToDevice));
    }
    const int ntx_p = (W - 2 + 63) / 64, nty_p = (H - 2 + ROWS - 1) / ROWS;
    const float tp = timeit([&] { hipLaunchKernelGGL(k_mix_plain, dim3(ntx_p * nty_p), dim3(256), 0, 0, a, ntx_p); });
    CHK(hipMemcpy(o1.data(), a.out[0], n * 8, hipMemcpyDeviceToHost));
    CHK(hipMemset(a.out[0], 0, n * 8));
    const int ntx_m = (W + 247) / 248;
    const float t16 = timeit([&] { hipLaunchKernelGGL(k_mix_march<16>, dim3(ntx_m * ((H - 2 + 15) / 16)), dim3(256), 0, 0, a, ntx_m); });
    CHK(hipMemcpy(o2.data(), a.out[0], n * 8, hipMemcpyDeviceToHost));
    long bad = 0;
    for (int nn = 1; nn <= H - 2; ++nn)
        for (int mm = 1; mm <= W - 2; ++mm) {
            const size_t i = (size_t)mm + (size_t)nn * PITCH;
            if (o1[i] != o2[i]) ++bad;
        }
    const float t32 = timeit([&] { hipLaunchKernelGGL(k_mix_march<32>, dim3(ntx_m * ((H - 2 + 31) / 32)), dim3(256), 0, 0, a, ntx_m); });
    const float t64 = timeit([&] { hipLaunchKernelGGL(k_mix_march<64>, dim3(ntx_m * ((H - 2 + 63) / 64)), dim3(256), 0, 0, a, ntx_m); });
    printf("mixed (%d arrays 5-point, %d pointwise): plain %.4f ms %6.0f GB/s | march16 %.4f ms %6.0f GB/s | "
           "march32 %.4f ms %6.0f GB/s | march64 %.4f ms %6.0f GB/s | march vs plain mismatches: %ld\n",
           NS, NI - NS, tp, bytes / tp / 1e6, t16, bytes / t16 / 1e6, t32, bytes / t32 / 1e6, t64, bytes / t64 / 1e6, bad);
    CHK(hipDeviceSynchronize());
    for (double *q : bufs) CHK(hipFree(q));
    return 0;
}
