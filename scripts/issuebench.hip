// issuebench.hip -- VALU issue cost per instruction class on MI355X (gfx950), at 1, 2 and 4 waves
// per SIMD: the classes the one-pass pair launch issues (profiles/sq_valu.json): f64 mul / add / fma,
// DPP lane moves (two v_mov_b32 per f64 lane shift), v_cndmask_b32 (selects), v_cmp (compares),
// int32 ops, v_frexp_exp_i32_f64 (udiv's range checks), and mixes of f64 with 32-bit work.
//
// Each workgroup is 4 waves (one per SIMD of a CU); the grid is 256 CUs x W workgroups, so every SIMD
// holds W waves.  Every wave runs ITER iterations of a block of 16 independent instructions of the
// class (8 register chains, no dependency stall at 1 wave beyond the class's own latency).  Reported:
// SIMD cycles per wave64 instruction = (per-wave shader-clock cycles of the loop, s_memtime) / (W x
// instructions per wave) -- the SIMD's issue throughput for the class -- and the effective clock
// (s_memtime ticks over the 100 MHz s_memrealtime ticks of the same loop).
//
// Build: hipcc --offload-arch=gfx950 -O3 scripts/issuebench.hip -o scripts/issuebench
#include <hip/hip_runtime.h>

#include <cstdio>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

constexpr int ITER = 4096;

enum Op { MUL64, ADD64, FMA64, DPP, CND, CMP64, ADDU32, FREXP, MIX_5F_3D, MIX_5F_3I, MIX_2F_2D, MIX_PAIR, CND_S,
          CMP_CND, ADD64_S, BFE, kOps };
static const char *kName[kOps] = {"v_mul_f64", "v_add_f64", "v_fma_f64", "v_mov_b32 dpp wave_shl:1", "v_cndmask_b32",
                                  "v_cmp_lt_f64", "v_add_u32", "v_frexp_exp_i32_f64",
                                  "mix 10 f64 mul + 6 dpp", "mix 10 f64 mul + 6 add_u32", "mix 8 f64 mul + 8 dpp",
                                  "mix 10 f64 (mul/add/fma) + 2 dpp + 2 cnd + 2 u32",
                                  "v_cndmask_b32_e64 (SGPR-pair condition)",
                                  "v_cmp_lt_f64 s[] + 2 v_cndmask_b32_e64 (f64 select)", "v_add_f64 (SGPR operand)",
                                  "v_bfe_u32"};
// instructions per block of each op (16 everywhere)
constexpr int kPerBlock = 16;

template <int OP>
__global__ __launch_bounds__(256) void k_issue(double seed, unsigned long long *cyc, unsigned long long *rt, double *sink)
{
    double d0 = seed + threadIdx.x, d1 = d0 * 1.5, d2 = d0 + 0.25, d3 = d0 * 0.75, d4 = d0 - 1.0, d5 = d0 * 1.25,
           d6 = d0 + 2.0, d7 = d0 * 0.5;
    const double k = 1.0000001, c = 0.999999;
    unsigned u0 = threadIdx.x, u1 = u0 * 3, u2 = u0 + 7, u3 = u0 ^ 5, u4 = u0 + 1, u5 = u0 * 5, u6 = u0 + 9, u7 = u0 ^ 3;
    unsigned s0 = u0 + 11, s1 = u0 + 13;   // DPP sources: not written inside the loop (no DPP read hazard)
    const unsigned long long smask = __builtin_amdgcn_ballot_w64((threadIdx.x & 1) != 0);
    unsigned long long sc0 = 0, sc1 = 0;
    const double ks = seed;
    __syncthreads();
    const unsigned long long t0 = clock64(), w0 = wall_clock64();
    for (int it = 0; it < ITER; ++it) {
        if constexpr (OP == MUL64) {
#pragma unroll
            for (int r = 0; r < 2; ++r)
                asm volatile("v_mul_f64 %0, %0, %8\n v_mul_f64 %1, %1, %8\n v_mul_f64 %2, %2, %8\n v_mul_f64 %3, %3, %8\n"
                             " v_mul_f64 %4, %4, %8\n v_mul_f64 %5, %5, %8\n v_mul_f64 %6, %6, %8\n v_mul_f64 %7, %7, %8"
                             : "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3), "+v"(d4), "+v"(d5), "+v"(d6), "+v"(d7) : "v"(k));
        } else if constexpr (OP == ADD64) {
#pragma unroll
            for (int r = 0; r < 2; ++r)
                asm volatile("v_add_f64 %0, %0, %8\n v_add_f64 %1, %1, %8\n v_add_f64 %2, %2, %8\n v_add_f64 %3, %3, %8\n"
                             " v_add_f64 %4, %4, %8\n v_add_f64 %5, %5, %8\n v_add_f64 %6, %6, %8\n v_add_f64 %7, %7, %8"
                             : "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3), "+v"(d4), "+v"(d5), "+v"(d6), "+v"(d7) : "v"(k));
        } else if constexpr (OP == FMA64) {
#pragma unroll
            for (int r = 0; r < 2; ++r)
                asm volatile("v_fma_f64 %0, %0, %8, %9\n v_fma_f64 %1, %1, %8, %9\n v_fma_f64 %2, %2, %8, %9\n"
                             " v_fma_f64 %3, %3, %8, %9\n v_fma_f64 %4, %4, %8, %9\n v_fma_f64 %5, %5, %8, %9\n"
                             " v_fma_f64 %6, %6, %8, %9\n v_fma_f64 %7, %7, %8, %9"
                             : "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3), "+v"(d4), "+v"(d5), "+v"(d6), "+v"(d7)
                             : "v"(k), "v"(c));
        } else if constexpr (OP == DPP) {
#pragma unroll
            for (int r = 0; r < 2; ++r)
                asm volatile("v_mov_b32_dpp %0, %8 wave_shl:1 row_mask:0xf bank_mask:0xf\n"
                             " v_mov_b32_dpp %1, %9 wave_shl:1 row_mask:0xf bank_mask:0xf\n"
                             " v_mov_b32_dpp %2, %8 wave_shr:1 row_mask:0xf bank_mask:0xf\n"
                             " v_mov_b32_dpp %3, %9 wave_shr:1 row_mask:0xf bank_mask:0xf\n"
                             " v_mov_b32_dpp %4, %8 wave_shl:1 row_mask:0xf bank_mask:0xf\n"
                             " v_mov_b32_dpp %5, %9 wave_shl:1 row_mask:0xf bank_mask:0xf\n"
                             " v_mov_b32_dpp %6, %8 wave_shr:1 row_mask:0xf bank_mask:0xf\n"
                             " v_mov_b32_dpp %7, %9 wave_shr:1 row_mask:0xf bank_mask:0xf"
                             : "=&v"(u0), "=&v"(u1), "=&v"(u2), "=&v"(u3), "=&v"(u4), "=&v"(u5), "=&v"(u6), "=&v"(u7)
                             : "v"(s0), "v"(s1));
        } else if constexpr (OP == CND) {
#pragma unroll
            for (int r = 0; r < 2; ++r)
                asm volatile("v_cndmask_b32 %0, %0, %8, vcc\n v_cndmask_b32 %1, %1, %8, vcc\n"
                             " v_cndmask_b32 %2, %2, %8, vcc\n v_cndmask_b32 %3, %3, %8, vcc\n"
                             " v_cndmask_b32 %4, %4, %8, vcc\n v_cndmask_b32 %5, %5, %8, vcc\n"
                             " v_cndmask_b32 %6, %6, %8, vcc\n v_cndmask_b32 %7, %7, %8, vcc"
                             : "+v"(u0), "+v"(u1), "+v"(u2), "+v"(u3), "+v"(u4), "+v"(u5), "+v"(u6), "+v"(u7)
                             : "v"(s0) : "vcc");
        } else if constexpr (OP == CMP64) {
#pragma unroll
            for (int r = 0; r < 2; ++r)
                asm volatile("v_cmp_lt_f64 vcc, %0, %8\n v_cmp_lt_f64 vcc, %1, %8\n v_cmp_lt_f64 vcc, %2, %8\n"
                             " v_cmp_lt_f64 vcc, %3, %8\n v_cmp_lt_f64 vcc, %4, %8\n v_cmp_lt_f64 vcc, %5, %8\n"
                             " v_cmp_lt_f64 vcc, %6, %8\n v_cmp_lt_f64 vcc, %7, %8"
                             : "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3), "+v"(d4), "+v"(d5), "+v"(d6), "+v"(d7)
                             : "v"(k) : "vcc");
        } else if constexpr (OP == ADDU32) {
#pragma unroll
            for (int r = 0; r < 2; ++r)
                asm volatile("v_add_u32 %0, %0, %8\n v_add_u32 %1, %1, %8\n v_add_u32 %2, %2, %8\n v_add_u32 %3, %3, %8\n"
                             " v_add_u32 %4, %4, %8\n v_add_u32 %5, %5, %8\n v_add_u32 %6, %6, %8\n v_add_u32 %7, %7, %8"
                             : "+v"(u0), "+v"(u1), "+v"(u2), "+v"(u3), "+v"(u4), "+v"(u5), "+v"(u6), "+v"(u7) : "v"(s0));
        } else if constexpr (OP == FREXP) {
#pragma unroll
            for (int r = 0; r < 2; ++r)
                asm volatile("v_frexp_exp_i32_f64 %0, %8\n v_frexp_exp_i32_f64 %1, %9\n v_frexp_exp_i32_f64 %2, %10\n"
                             " v_frexp_exp_i32_f64 %3, %11\n v_frexp_exp_i32_f64 %4, %8\n v_frexp_exp_i32_f64 %5, %9\n"
                             " v_frexp_exp_i32_f64 %6, %10\n v_frexp_exp_i32_f64 %7, %11"
                             : "=&v"(u0), "=&v"(u1), "=&v"(u2), "=&v"(u3), "=&v"(u4), "=&v"(u5), "=&v"(u6), "=&v"(u7)
                             : "v"(d0), "v"(d1), "v"(d2), "v"(d3));
        } else if constexpr (OP == MIX_5F_3D) {   // 10 f64 + 6 dpp
            asm volatile("v_mul_f64 %0, %0, %8\n v_mov_b32_dpp %9, %12 wave_shl:1 row_mask:0xf bank_mask:0xf\n"
                         " v_mul_f64 %1, %1, %8\n v_mul_f64 %2, %2, %8\n v_mov_b32_dpp %10, %13 wave_shl:1 row_mask:0xf bank_mask:0xf\n"
                         " v_mul_f64 %3, %3, %8\n v_mul_f64 %4, %4, %8\n v_mov_b32_dpp %11, %12 wave_shr:1 row_mask:0xf bank_mask:0xf\n"
                         " v_mul_f64 %5, %5, %8\n v_mov_b32_dpp %9, %13 wave_shr:1 row_mask:0xf bank_mask:0xf\n"
                         " v_mul_f64 %6, %6, %8\n v_mul_f64 %7, %7, %8\n v_mov_b32_dpp %10, %12 wave_shl:1 row_mask:0xf bank_mask:0xf\n"
                         " v_mul_f64 %0, %0, %8\n v_mul_f64 %1, %1, %8\n v_mov_b32_dpp %11, %13 wave_shl:1 row_mask:0xf bank_mask:0xf"
                         : "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3), "+v"(d4), "+v"(d5), "+v"(d6), "+v"(d7)
                         : "v"(k), "v"(u0), "v"(u1), "v"(u2), "v"(s0), "v"(s1));
        } else if constexpr (OP == MIX_5F_3I) {   // 10 f64 + 6 int32 (k = %11, u0..u2 = %8..%10)
            asm volatile("v_mul_f64 %0, %0, %11\n v_add_u32 %8, %8, %12\n"
                         " v_mul_f64 %1, %1, %11\n v_mul_f64 %2, %2, %11\n v_add_u32 %9, %9, %12\n"
                         " v_mul_f64 %3, %3, %11\n v_mul_f64 %4, %4, %11\n v_add_u32 %10, %10, %12\n"
                         " v_mul_f64 %5, %5, %11\n v_add_u32 %8, %8, %13\n"
                         " v_mul_f64 %6, %6, %11\n v_mul_f64 %7, %7, %11\n v_add_u32 %9, %9, %13\n"
                         " v_mul_f64 %0, %0, %11\n v_mul_f64 %1, %1, %11\n v_add_u32 %10, %10, %13"
                         : "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3), "+v"(d4), "+v"(d5), "+v"(d6), "+v"(d7), "+v"(u0),
                           "+v"(u1), "+v"(u2)
                         : "v"(k), "v"(s0), "v"(s1));
        } else if constexpr (OP == MIX_2F_2D) {   // 8 f64 + 8 dpp
#pragma unroll
            for (int r = 0; r < 2; ++r)
                asm volatile("v_mul_f64 %0, %0, %8\n v_mov_b32_dpp %4, %9 wave_shl:1 row_mask:0xf bank_mask:0xf\n"
                             " v_mul_f64 %1, %1, %8\n v_mov_b32_dpp %5, %10 wave_shl:1 row_mask:0xf bank_mask:0xf\n"
                             " v_mul_f64 %2, %2, %8\n v_mov_b32_dpp %6, %9 wave_shr:1 row_mask:0xf bank_mask:0xf\n"
                             " v_mul_f64 %3, %3, %8\n v_mov_b32_dpp %7, %10 wave_shr:1 row_mask:0xf bank_mask:0xf"
                             : "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3), "=&v"(u0), "=&v"(u1), "=&v"(u2), "=&v"(u3)
                             : "v"(k), "v"(s0), "v"(s1));
        } else if constexpr (OP == MIX_PAIR) {   // the pair launch's measured mix, roughly: 10 f64 + 6 other
            asm volatile("v_mul_f64 %0, %0, %8\n v_mov_b32_dpp %12, %15 wave_shl:1 row_mask:0xf bank_mask:0xf\n"
                         " v_add_f64 %1, %1, %8\n v_fma_f64 %2, %2, %8, %9\n v_mov_b32_dpp %13, %16 wave_shl:1 row_mask:0xf bank_mask:0xf\n"
                         " v_mul_f64 %3, %3, %8\n v_cndmask_b32 %10, %10, %15, vcc\n"
                         " v_add_f64 %4, %4, %8\n v_mul_f64 %5, %5, %8\n v_add_u32 %11, %11, %15\n"
                         " v_fma_f64 %6, %6, %8, %9\n v_cndmask_b32 %14, %14, %16, vcc\n"
                         " v_mul_f64 %7, %7, %8\n v_add_f64 %0, %0, %8\n v_add_u32 %10, %10, %16\n"
                         " v_mul_f64 %1, %1, %8"
                         : "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3), "+v"(d4), "+v"(d5), "+v"(d6), "+v"(d7)
                         : "v"(k), "v"(c), "v"(u0), "v"(u1), "v"(u2), "v"(u3), "v"(u4), "v"(s0), "v"(s1) : "vcc");
        }
        if constexpr (OP == CND_S) {
#pragma unroll
            for (int r = 0; r < 2; ++r)
                asm volatile("v_cndmask_b32_e64 %0, %0, %8, %9\n v_cndmask_b32_e64 %1, %1, %8, %9\n"
                             " v_cndmask_b32_e64 %2, %2, %8, %9\n v_cndmask_b32_e64 %3, %3, %8, %9\n"
                             " v_cndmask_b32_e64 %4, %4, %8, %9\n v_cndmask_b32_e64 %5, %5, %8, %9\n"
                             " v_cndmask_b32_e64 %6, %6, %8, %9\n v_cndmask_b32_e64 %7, %7, %8, %9"
                             : "+v"(u0), "+v"(u1), "+v"(u2), "+v"(u3), "+v"(u4), "+v"(u5), "+v"(u6), "+v"(u7)
                             : "v"(s0), "s"(smask));
        } else if constexpr (OP == CMP_CND) {   // 4 x (compare into an SGPR pair, select both halves of an f64)
#pragma unroll
            for (int r = 0; r < 4; ++r)
                asm volatile("v_cmp_lt_f64_e64 %8, %0, %10\n v_cndmask_b32_e64 %4, %4, %11, %8\n v_cndmask_b32_e64 %5, %5, %11, %8\n"
                             " v_cmp_lt_f64_e64 %9, %1, %10\n v_cndmask_b32_e64 %6, %6, %11, %9\n v_cndmask_b32_e64 %7, %7, %11, %9\n"
                             " v_mul_f64 %2, %2, %10\n v_mul_f64 %3, %3, %10"
                             : "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3), "+v"(u0), "+v"(u1), "+v"(u2), "+v"(u3),
                               "=&s"(sc0), "=&s"(sc1)
                             : "v"(k), "v"(s0));
        } else if constexpr (OP == ADD64_S) {
#pragma unroll
            for (int r = 0; r < 2; ++r)
                asm volatile("v_add_f64 %0, %0, %8\n v_add_f64 %1, %1, %8\n v_add_f64 %2, %2, %8\n v_add_f64 %3, %3, %8\n"
                             " v_add_f64 %4, %4, %8\n v_add_f64 %5, %5, %8\n v_add_f64 %6, %6, %8\n v_add_f64 %7, %7, %8"
                             : "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3), "+v"(d4), "+v"(d5), "+v"(d6), "+v"(d7) : "s"(ks));
        } else if constexpr (OP == BFE) {
#pragma unroll
            for (int r = 0; r < 2; ++r)
                asm volatile("v_bfe_u32 %0, %8, 3, 1\n v_bfe_u32 %1, %8, 4, 1\n v_bfe_u32 %2, %8, 5, 1\n v_bfe_u32 %3, %8, 6, 1\n"
                             " v_bfe_u32 %4, %9, 3, 1\n v_bfe_u32 %5, %9, 4, 1\n v_bfe_u32 %6, %9, 5, 1\n v_bfe_u32 %7, %9, 6, 1"
                             : "=&v"(u0), "=&v"(u1), "=&v"(u2), "=&v"(u3), "=&v"(u4), "=&v"(u5), "=&v"(u6), "=&v"(u7)
                             : "v"(s0), "v"(s1));
        }
    }
    const unsigned long long t1 = clock64(), w1 = wall_clock64();
    if ((threadIdx.x & 63) == 0) {
        const unsigned wv = blockIdx.x * 4 + (threadIdx.x >> 6);
        cyc[wv] = t1 - t0;
        rt[wv] = w1 - w0;
    }
    const double s = d0 + d1 + d2 + d3 + d4 + d5 + d6 + d7 + (double)(u0 + u1 + u2 + u3 + u4 + u5 + u6 + u7) +
                     (double)(sc0 ^ sc1);
    if (s == 12345.678) sink[threadIdx.x] = s;   // (never true: keeps the chains live)
}

template <int OP>
static int run(int wps, unsigned long long *cyc, unsigned long long *rt, double *sink, unsigned long long *hc,
               unsigned long long *hr, int ncu)
{
    const int blocks = ncu * wps, waves = blocks * 4;
    hipLaunchKernelGGL(k_issue<OP>, dim3(blocks), dim3(256), 0, 0, 1.0, cyc, rt, sink);   // warm
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    CHK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(k_issue<OP>, dim3(blocks), dim3(256), 0, 0, 1.0, cyc, rt, sink);
    CHK(hipEventRecord(e1, 0));
    CHK(hipEventSynchronize(e1));
    float ms = 0.f;
    CHK(hipEventElapsedTime(&ms, e0, e1));
    CHK(hipMemcpy(hc, cyc, sizeof(unsigned long long) * waves, hipMemcpyDeviceToHost));
    CHK(hipMemcpy(hr, rt, sizeof(unsigned long long) * waves, hipMemcpyDeviceToHost));
    double c = 0.0, r = 0.0;
    for (int i = 0; i < waves; ++i) { c += (double)hc[i]; r += (double)hr[i]; }
    c /= waves;
    r /= waves;
    const double insts = (double)ITER * kPerBlock;         // per wave
    const double cpi_simd = c / (insts * wps);              // SIMD cycles per wave64 instruction
    const double ghz = c / (r * 10.0);                      // s_memtime ticks per ns (s_memrealtime: 100 MHz)
    // whole-chip view from the event time: instructions per SIMD per ns at the measured clock
    const double cpi_ev = (double)ms * 1e6 * ghz / (insts * wps);
    printf("%-48s waves/SIMD %d  cycles/inst/SIMD %.3f (loop clock64)  %.3f (event time x %.2f GHz)\n", kName[OP], wps,
           cpi_simd, cpi_ev, ghz);
    return 0;
}

template <int OP> static int run_all(unsigned long long *cyc, unsigned long long *rt, double *sink,
                                     unsigned long long *hc, unsigned long long *hr, int ncu)
{
    for (int w : {1, 2, 4})
        if (run<OP>(w, cyc, rt, sink, hc, hr, ncu)) return 1;
    return 0;
}

int main()
{
    hipDeviceProp_t p;
    CHK(hipGetDeviceProperties(&p, 0));
    const int ncu = p.multiProcessorCount;
    printf("%s, %d CUs, %s\n", p.name, ncu, p.gcnArchName);
    const int maxw = ncu * 4 * 4;
    unsigned long long *cyc, *rt;
    double *sink;
    CHK(hipMalloc(&cyc, sizeof(unsigned long long) * maxw));
    CHK(hipMalloc(&rt, sizeof(unsigned long long) * maxw));
    CHK(hipMalloc(&sink, sizeof(double) * 256));
    static unsigned long long hc[1 << 14], hr[1 << 14];
    int rc = 0;
    rc |= run_all<MUL64>(cyc, rt, sink, hc, hr, ncu);
    rc |= run_all<ADD64>(cyc, rt, sink, hc, hr, ncu);
    rc |= run_all<FMA64>(cyc, rt, sink, hc, hr, ncu);
    rc |= run_all<DPP>(cyc, rt, sink, hc, hr, ncu);
    rc |= run_all<CND>(cyc, rt, sink, hc, hr, ncu);
    rc |= run_all<CMP64>(cyc, rt, sink, hc, hr, ncu);
    rc |= run_all<ADDU32>(cyc, rt, sink, hc, hr, ncu);
    rc |= run_all<FREXP>(cyc, rt, sink, hc, hr, ncu);
    rc |= run_all<MIX_5F_3D>(cyc, rt, sink, hc, hr, ncu);
    rc |= run_all<MIX_5F_3I>(cyc, rt, sink, hc, hr, ncu);
    rc |= run_all<MIX_2F_2D>(cyc, rt, sink, hc, hr, ncu);
    rc |= run_all<MIX_PAIR>(cyc, rt, sink, hc, hr, ncu);
    rc |= run_all<CND_S>(cyc, rt, sink, hc, hr, ncu);
    rc |= run_all<CMP_CND>(cyc, rt, sink, hc, hr, ncu);
    rc |= run_all<ADD64_S>(cyc, rt, sink, hc, hr, ncu);
    rc |= run_all<BFE>(cyc, rt, sink, hc, hr, ncu);
    CHK(hipDeviceSynchronize());
    return rc;
}
