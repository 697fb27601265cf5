// Tile-sort microbenchmark: synthetic per-tile buckets of unique
// (depth bits << 32 | id) keys, sorted by lsr::launch_tile_sort; checks every
// tile against std::sort and times the sort with HIP events.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../../langsplatv2_amd/csrc
//        sort_bench.hip -o sort_bench   (SORT_PERSISTENT=1: classify on the GPU, persistent grids)
// Usage: ./sort_bench T lo hi [iters]   (tile sizes uniform in [lo, hi])
#include "../../langsplatv2_amd/csrc/binning.hip"
#include <algorithm>
#include <cstring>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

int main(int argc, char** argv)
{
    const int T = argc > 1 ? atoi(argv[1]) : 8160;
    const int lo = argc > 2 ? atoi(argv[2]) : 900, hi = argc > 3 ? atoi(argv[3]) : 1174;
    const int iters = argc > 4 ? atoi(argv[4]) : 20;
    std::mt19937_64 rng(7);
    std::vector<uint32_t> start(T + 1, 0);
    for (int t = 0; t < T; t++) start[t + 1] = start[t] + lo + (uint32_t)(rng() % (uint64_t)(hi - lo + 1));
    const size_t M = start[T];
    std::vector<uint64_t> keys(M);
    uint32_t id = 0;
    for (size_t i = 0; i < M; i++) {
        const float depth = 2.0f + 10.0f * (float)((rng() >> 11) * (1.0 / 9007199254740992.0));
        uint32_t b;
        std::memcpy(&b, &depth, 4);
        if (rng() % 16 == 0 && i) b = (uint32_t)(keys[i - 1] >> 32);   // some equal depths: ties by id
        keys[i] = ((uint64_t)b << 32) | (id++ * 2654435761u % 0x7fffffffu);
    }
    uint32_t *d_start, *d_out;
    uint64_t *d_keys, *d_keys0;
    CK(hipMalloc(&d_start, (T + 1) * 4));
    CK(hipMalloc(&d_keys, M * 8));
    CK(hipMalloc(&d_keys0, M * 8));
    CK(hipMalloc(&d_out, M * 4));
    CK(hipMemcpy(d_start, start.data(), (T + 1) * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_keys0, keys.data(), M * 8, hipMemcpyHostToDevice));
    // class lists as k_bin_table builds them (host copy of tile_class)
    std::vector<uint32_t> cnt(SORT_NCLS, 0), list((size_t)SORT_NCLS * T, 0);
    for (int t = 0; t < T; t++) {
        const int n = (int)(start[t + 1] - start[t]);
        const int c = n <= 0 ? -1 : n <= 512 ? 0 : n <= 1024 ? 1 : n <= 2048 ? 2 : n <= 4096 ? 3 : n <= 8192 ? 4 : 5;
        if (c >= 0) list[(size_t)c * T + cnt[c]++] = t;
    }
    uint32_t *d_cnt, *d_list;
    CK(hipMalloc(&d_cnt, SORT_NCLS * 4));
    CK(hipMalloc(&d_list, list.size() * 4));
    CK(hipMemcpy(d_cnt, cnt.data(), SORT_NCLS * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_list, list.data(), list.size() * 4, hipMemcpyHostToDevice));
    const bool persistent = getenv("SORT_PERSISTENT") != nullptr;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    float best = 1e30f, tot = 0.f;
    for (int it = 0; it < iters + 2; it++) {
        CK(hipMemcpy(d_keys, d_keys0, M * 8, hipMemcpyDeviceToDevice));
        CK(hipEventRecord(e0, 0));
        CK(lsr::launch_tile_sort(T, d_start, d_keys, d_out, d_cnt, d_list, persistent ? nullptr : cnt.data(), 0));
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (it >= 2) { best = std::min(best, ms); tot += ms; }
    }
    std::vector<uint32_t> out(M);
    CK(hipMemcpy(out.data(), d_out, M * 4, hipMemcpyDeviceToHost));
    size_t bad = 0;
    for (int t = 0; t < T; t++) {
        std::vector<uint64_t> s(keys.begin() + start[t], keys.begin() + start[t + 1]);
        std::sort(s.begin(), s.end());
        for (size_t k = 0; k < s.size(); k++) bad += out[start[t] + k] != (uint32_t)s[k];
    }
    printf("T=%d sizes=[%d,%d] M=%zu persistent=%d  best %.4f ms  mean %.4f ms  %.1f GB/s(12B/key)  mismatches=%zu\n", T, lo,
           hi, M, (int)persistent, best, tot / iters, M * 12.0 / best / 1e6, bad);
    return bad ? 2 : 0;
}
