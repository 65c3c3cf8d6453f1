// lanetest.hip -- which source lane does each cross-lane primitive read on gfx950?
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ void k(int *o)
{
    const int l = (int)threadIdx.x;
    o[0 * 64 + l] = __builtin_amdgcn_mov_dpp(l, 0x130, 0xf, 0xf, false);   // wave_shl:1
    o[1 * 64 + l] = __builtin_amdgcn_mov_dpp(l, 0x138, 0xf, 0xf, false);   // wave_shr:1
    o[2 * 64 + l] = __builtin_amdgcn_update_dpp(-1, l, 0x130, 0xf, 0xf, false);
    o[3 * 64 + l] = __builtin_amdgcn_update_dpp(-1, l, 0x138, 0xf, 0xf, false);
    o[4 * 64 + l] = __shfl_down(l, 1);
    o[5 * 64 + l] = __shfl_up(l, 1);
    o[6 * 64 + l] = __builtin_amdgcn_mov_dpp(l, 0x101, 0xf, 0xf, false);   // row_shl:1
}

int main()
{
    int *d, h[7 * 64];
    if (hipMalloc(&d, sizeof(h)) != hipSuccess) return 1;
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
    if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 1;
    const char *nm[] = {"mov_dpp wave_shl:1", "mov_dpp wave_shr:1", "update_dpp(-1) wave_shl:1",
                        "update_dpp(-1) wave_shr:1", "__shfl_down(1)", "__shfl_up(1)", "mov_dpp row_shl:1"};
    for (int r = 0; r < 7; ++r) {
        printf("%-28s", nm[r]);
        for (int l = 0; l < 64; ++l) printf(" %d", h[r * 64 + l]);
        printf("\n");
    }
    return 0;
}
