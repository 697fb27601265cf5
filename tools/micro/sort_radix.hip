// Tile-sort probe at cfg5's bucket sizes: the shipped class kernels
// (lsr::launch_tile_sort: register bitonic + merge path) against an LDS radix
// sort (rocprim::block_radix_sort, 256 threads x 8 keys) of the same
// (depth bits, id) keys, either the full 64-bit key or a compacted one:
// (depth bits - tile minimum) << ID_BITS | id over only the bits the tile's
// keys span.  Every tile is checked against std::sort.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../../langsplatv2_amd/csrc sort_radix.hip -o sort_radix
// Usage: ./sort_radix T lo hi [iters]
#include "../../langsplatv2_amd/csrc/binning.hip"
#include <rocprim/block/block_radix_sort.hpp>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

constexpr int ID_BITS = 23;   // ids < 2^23 (cfg5: 5M Gaussians)

template <int RB, bool COMPACT>
__global__ void __launch_bounds__(256) k_radix(int T, const uint32_t* __restrict__ start, const uint64_t* __restrict__ keys,
                                               uint32_t* __restrict__ out, const uint32_t* __restrict__ list, int ntile)
{
    using sorter = rocprim::block_radix_sort<uint64_t, 256, 8, rocprim::empty_type, 1, 1, RB>;
    __shared__ typename sorter::storage_type st;
    __shared__ uint32_t smin[4], smax[4];
    const int tid = threadIdx.x;
    for (int i = blockIdx.x; i < ntile; i += gridDim.x) {
        const int t = (int)list[i];
        const uint32_t s0 = start[t];
        const int n = (int)(start[t + 1] - s0);
        uint64_t k[8];
        uint32_t lo = 0xffffffffu, hi = 0u;
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const int e = tid * 8 + j;   // blocked arrangement
            k[j] = e < n ? keys[s0 + e] : ~0ull;
            if (e < n) {
                lo = min(lo, (uint32_t)(k[j] >> 32));
                hi = max(hi, (uint32_t)(k[j] >> 32));
            }
        }
        unsigned end_bit = 64;
        if (COMPACT) {
            for (int d = 32; d >= 1; d >>= 1) {
                lo = min(lo, (uint32_t)__shfl_xor((int)lo, d, 64));
                hi = max(hi, (uint32_t)__shfl_xor((int)hi, d, 64));
            }
            if ((tid & 63) == 0) { smin[tid >> 6] = lo; smax[tid >> 6] = hi; }
            __syncthreads();
            lo = min(min(smin[0], smin[1]), min(smin[2], smin[3]));
            hi = max(max(smax[0], smax[1]), max(smax[2], smax[3]));
            __syncthreads();
            const uint32_t span = hi - lo;
            const int sb = span ? 32 - __clz(span) : 0;
            // padding sorts last: all ones over the compacted width
            const uint64_t pad = (sb + ID_BITS >= 64) ? ~0ull : ((1ull << (sb + ID_BITS)) - 1);
#pragma unroll
            for (int j = 0; j < 8; j++)
                k[j] = (tid * 8 + j < n) ? (((uint64_t)((uint32_t)(k[j] >> 32) - lo) << ID_BITS) | (k[j] & ((1u << ID_BITS) - 1)))
                                         : pad;
            end_bit = sb + ID_BITS;
        }
        sorter().sort(k, st, 0, end_bit);
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const int e = tid * 8 + j;
            if (e < n) out[s0 + e] = (uint32_t)(k[j] & (COMPACT ? ((1u << ID_BITS) - 1) : 0xffffffffu));
        }
        __syncthreads();
    }
}

int main(int argc, char** argv)
{
    const int T = argc > 1 ? atoi(argv[1]) : 32400;
    const int lo = argc > 2 ? atoi(argv[2]) : 1600, hi = argc > 3 ? atoi(argv[3]) : 2048;
    const int iters = argc > 4 ? atoi(argv[4]) : 10;
    std::mt19937_64 rng(7);
    std::vector<uint32_t> start(T + 1, 0);
    for (int t = 0; t < T; t++) start[t + 1] = start[t] + lo + (uint32_t)(rng() % (uint64_t)(hi - lo + 1));
    const size_t M = start[T];
    std::vector<uint64_t> keys(M);
    for (size_t i = 0; i < M; i++) {
        const float depth = 2.0f + 10.0f * (float)((rng() >> 11) * (1.0 / 9007199254740992.0));
        uint32_t b;
        std::memcpy(&b, &depth, 4);
        if (rng() % 16 == 0 && i) b = (uint32_t)(keys[i - 1] >> 32);   // some equal depths: ties by id
        keys[i] = ((uint64_t)b << 32) | (uint32_t)((i * 2654435761ull) % 5000000ull);
    }
    uint32_t *d_start, *d_out;
    uint64_t *d_keys, *d_keys0;
    CK(hipMalloc(&d_start, (T + 1) * 4));
    CK(hipMalloc(&d_keys, M * 8));
    CK(hipMalloc(&d_keys0, M * 8));
    CK(hipMalloc(&d_out, M * 4));
    CK(hipMemcpy(d_start, start.data(), (T + 1) * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_keys0, keys.data(), M * 8, hipMemcpyHostToDevice));
    std::vector<uint32_t> cnt(SORT_NCLS, 0), list((size_t)SORT_NCLS * T, 0);
    for (int t = 0; t < T; t++) {
        const int n = (int)(start[t + 1] - start[t]);
        const int c = n <= 0 ? -1 : n <= 512 ? 0 : n <= 1024 ? 1 : n <= 2048 ? 2 : n <= 4096 ? 3 : n <= 8192 ? 4 : 5;
        if (c >= 0) list[(size_t)c * T + cnt[c]++] = t;
    }
    if (cnt[2] != (uint32_t)T) { printf("sizes must all be in (1024, 2048]\n"); return 1; }
    uint32_t *d_cnt, *d_list;
    CK(hipMalloc(&d_cnt, SORT_NCLS * 4));
    CK(hipMalloc(&d_list, list.size() * 4));
    CK(hipMemcpy(d_cnt, cnt.data(), SORT_NCLS * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_list, list.data(), list.size() * 4, hipMemcpyHostToDevice));
    std::vector<std::vector<uint32_t>> ref(T);
    for (int t = 0; t < T; t++) {
        std::vector<uint64_t> s(keys.begin() + start[t], keys.begin() + start[t + 1]);
        std::sort(s.begin(), s.end());
        for (auto v : s) ref[t].push_back((uint32_t)v);
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto run = [&](const char* name, auto launch) {
        float best = 1e30f;
        for (int it = 0; it < iters + 2; it++) {
            CK(hipMemcpy(d_keys, d_keys0, M * 8, hipMemcpyDeviceToDevice));
            CK(hipMemset(d_out, 0xff, M * 4));
            CK(hipEventRecord(e0, 0));
            launch();
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (it >= 2) best = std::min(best, ms);
        }
        std::vector<uint32_t> out(M);
        CK(hipMemcpy(out.data(), d_out, M * 4, hipMemcpyDeviceToHost));
        size_t bad = 0;
        for (int t = 0; t < T; t++)
            for (size_t k = 0; k < ref[t].size(); k++) bad += out[start[t] + k] != ref[t][k];
        printf("%-34s best %.4f ms  %.1f GB/s(12B/key)  mismatches=%zu\n", name, best, M * 12.0 / best / 1e6, bad);
    };
    printf("T=%d sizes=[%d,%d] M=%zu\n", T, lo, hi, M);
    run("shipped (bitonic + merge path)", [&] { CK(lsr::launch_tile_sort(T, d_start, d_keys, d_out, d_cnt, d_list, cnt.data(), 0)); });
    const uint32_t* l2 = d_list + 2 * (size_t)T;
    const int g = std::min(T, 256 * 6);
    run("radix 64-bit, 8 bits/pass", [&] { k_radix<8, false><<<g, 256>>>(T, d_start, d_keys, d_out, l2, T); });
    run("radix 64-bit, 4 bits/pass", [&] { k_radix<4, false><<<g, 256>>>(T, d_start, d_keys, d_out, l2, T); });
    run("radix compacted, 8 bits/pass", [&] { k_radix<8, true><<<g, 256>>>(T, d_start, d_keys, d_out, l2, T); });
    run("radix compacted, 4 bits/pass", [&] { k_radix<4, true><<<g, 256>>>(T, d_start, d_keys, d_out, l2, T); });
    run("radix compacted, 6 bits/pass", [&] { k_radix<6, true><<<g, 256>>>(T, d_start, d_keys, d_out, l2, T); });
    return 0;
}
