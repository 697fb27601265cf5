// Checks the lane-exchange paths of the wave sort (binning.hip xor_lane_u32)
// against __shfl_xor on the GPU: every lane's partner value for M = 1..32.
// Build: hipcc --offload-arch=gfx950 -O3 dpp_xor.hip -o dpp_xor ; run: ./dpp_xor
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <int M>
__device__ uint32_t xor_lane(uint32_t x)
{
    const int lane = threadIdx.x & 63;
    if constexpr (M == 32) {
        auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
        return (lane & 32) ? r[0] : r[1];
    } else if constexpr (M == 16) {
        auto r = __builtin_amdgcn_permlane16_swap(x, x, false, false);
        return (lane & 16) ? r[0] : r[1];
    } else if constexpr (M == 8) {
        return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x128, 0xF, 0xF, false);
    } else if constexpr (M == 4) {
        const uint32_t from_below = (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x124, 0xF, 0xF, false);
        const uint32_t from_above = (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x12C, 0xF, 0xF, false);
        return (lane & 4) ? from_below : from_above;
    } else if constexpr (M == 2) {
        return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x4E, 0xF, 0xF, false);
    } else {
        return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xF, 0xF, false);
    }
}

__global__ void k(uint32_t* out)
{
    const uint32_t x = 1000u + threadIdx.x;
    const int l = threadIdx.x;
    out[0 * 64 + l] = xor_lane<1>(x) ^ (uint32_t)__shfl_xor((int)x, 1, 64);
    out[1 * 64 + l] = xor_lane<2>(x) ^ (uint32_t)__shfl_xor((int)x, 2, 64);
    out[2 * 64 + l] = xor_lane<4>(x) ^ (uint32_t)__shfl_xor((int)x, 4, 64);
    out[3 * 64 + l] = xor_lane<8>(x) ^ (uint32_t)__shfl_xor((int)x, 8, 64);
    out[4 * 64 + l] = xor_lane<16>(x) ^ (uint32_t)__shfl_xor((int)x, 16, 64);
    out[5 * 64 + l] = xor_lane<32>(x) ^ (uint32_t)__shfl_xor((int)x, 32, 64);
}

int main()
{
    uint32_t* d = nullptr;
    if (hipMalloc(&d, 6 * 64 * 4) != hipSuccess) return 2;
    k<<<1, 64>>>(d);
    uint32_t h[6 * 64];
    if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 2;
    int bad = 0;
    for (int m = 0; m < 6; m++) {
        int nb = 0;
        for (int l = 0; l < 64; l++) nb += h[m * 64 + l] != 0;
        printf("M=%d mismatching lanes %d\n", 1 << m, nb);
        bad += nb;
    }
    (void)hipFree(d);
    printf(bad ? "FAIL\n" : "OK\n");
    return bad ? 1 : 0;
}
