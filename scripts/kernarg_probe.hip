// Probe: the largest kernel-argument struct a plain launch accepts on this device (the batched
// launches of sw_kernels.hip pass their bodies by value: more bodies per launch if larger argument
// blocks work).  Each kernel sums its argument's words and writes the sum; the host checks it.
#include <hip/hip_runtime.h>

#include <cstdio>

template <int N> struct Arg { unsigned w[N / 4]; };

template <int N> __global__ void k_sum(Arg<N> a, unsigned *out)
{
    unsigned s = 0;
    for (int i = 0; i < N / 4; ++i) s += a.w[i] * (unsigned)(i + 1);
    if (threadIdx.x == 0 && blockIdx.x == 0) out[0] = s;
}

template <int N> static void probe(unsigned *d)
{
    Arg<N> a;
    unsigned want = 0;
    for (int i = 0; i < N / 4; ++i) { a.w[i] = 3u * i + 7u; want += a.w[i] * (unsigned)(i + 1); }
    (void)hipMemset(d, 0, 4);
    hipLaunchKernelGGL(k_sum<N>, dim3(1), dim3(64), 0, 0, a, d);
    hipError_t e = hipGetLastError();
    hipError_t e2 = hipDeviceSynchronize();
    unsigned got = 0;
    (void)hipMemcpy(&got, d, 4, hipMemcpyDeviceToHost);
    std::printf("kernarg %6d B: launch %s, sync %s, %s\n", N, hipGetErrorString(e), hipGetErrorString(e2),
                got == want ? "correct" : "WRONG");
}

int main()
{
    unsigned *d = nullptr;
    if (hipMalloc(&d, 4) != hipSuccess) return 1;
    probe<3584>(d);
    probe<4096>(d);
    probe<6144>(d);
    probe<8192>(d);
    probe<12288>(d);
    probe<16384>(d);
    (void)hipFree(d);
    return 0;
}
