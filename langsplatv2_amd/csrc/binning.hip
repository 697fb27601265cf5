// binning.hip — tile binning (A.2): scan of tiles_touched, duplicate with
// per-tile counting ranks, scatter into tile buckets, per-tile depth sort.
//
// MI355X design (vs the reference's global 64-bit radix sort over
// 32 + log2(T) bits of M keys): the tile is the bucket.  duplicate takes a
// per-tile rank with one L2 atomic per instance, scatter places each
// instance's key (depth bits << 32 | gaussian id) in its tile bucket, and one
// 256-thread workgroup per tile sorts its bucket in LDS (flip-bitonic on
// unique u64 keys).  The result equals a stable sort by
// (tile, depth bits) with ties broken by Gaussian id — the order of the
// reference's stable radix sort over duplicates emitted in Gaussian order.
#include "lsr_internal.h"

namespace lsr {

// ---------------------------------------------------------------- scan ----
#define SCAN_ITEMS 16
#define SCAN_BLOCK 256
#define SCAN_TILE (SCAN_ITEMS * SCAN_BLOCK)

size_t scan_partials(size_t n) { return (n + SCAN_TILE - 1) / SCAN_TILE + 1; }

__device__ __forceinline__ uint64_t block_excl_scan_u64(uint64_t v, uint64_t* sh, uint64_t& total)
{
    // wave inclusive scan via shuffles, then across the 4 waves through LDS
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint64_t x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        uint64_t y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
    }
    if (lane == 63) sh[w] = x;
    __syncthreads();
    uint64_t wofs = 0, tot = 0;
    for (int k = 0; k < SCAN_BLOCK / 64; k++) {
        if (k < w) wofs += sh[k];
        tot += sh[k];
    }
    __syncthreads();
    total = tot;
    return wofs + x - v;
}

__global__ void __launch_bounds__(SCAN_BLOCK) k_scan_reduce(const uint32_t* __restrict__ in, size_t n,
                                                            uint64_t* __restrict__ part)
{
    __shared__ uint64_t sh[SCAN_BLOCK / 64];
    const size_t base = (size_t)blockIdx.x * SCAN_TILE + (size_t)threadIdx.x * SCAN_ITEMS;
    uint64_t s = 0;
#pragma unroll
    for (int k = 0; k < SCAN_ITEMS; k++)
        if (base + k < n) s += in[base + k];
    uint64_t tot;
    block_excl_scan_u64(s, sh, tot);
    if (threadIdx.x == 0) part[blockIdx.x] = tot;
}

__global__ void __launch_bounds__(SCAN_BLOCK) k_scan_part(uint64_t* __restrict__ part, int nb)
{
    __shared__ uint64_t sh[SCAN_BLOCK / 64];
    uint64_t carry = 0;
    for (int base = 0; base < nb; base += SCAN_BLOCK) {
        const int i = base + threadIdx.x;
        uint64_t v = i < nb ? part[i] : 0;
        uint64_t tot;
        uint64_t ex = block_excl_scan_u64(v, sh, tot);
        __syncthreads();
        if (i < nb) part[i] = carry + ex;
        carry += tot;
        __syncthreads();
    }
    if (threadIdx.x == 0) part[nb] = carry;
}

__global__ void __launch_bounds__(SCAN_BLOCK) k_scan_apply(const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                                           size_t n, const uint64_t* __restrict__ part, int exclusive)
{
    __shared__ uint64_t sh[SCAN_BLOCK / 64];
    const size_t base = (size_t)blockIdx.x * SCAN_TILE + (size_t)threadIdx.x * SCAN_ITEMS;
    uint32_t v[SCAN_ITEMS];
    uint64_t s = 0;
#pragma unroll
    for (int k = 0; k < SCAN_ITEMS; k++) {
        v[k] = (base + k < n) ? in[base + k] : 0u;
        s += v[k];
    }
    uint64_t tot;
    uint64_t run = block_excl_scan_u64(s, sh, tot) + part[blockIdx.x];
#pragma unroll
    for (int k = 0; k < SCAN_ITEMS; k++) {
        const uint64_t incl = run + v[k];
        if (base + k < n) out[base + k] = (uint32_t)(exclusive ? run : incl);
        run = incl;
    }
}

hipError_t launch_scan_u32(const uint32_t* in, uint32_t* out, uint64_t* part, size_t n, bool exclusive, hipStream_t st)
{
    const int nb = (int)((n + SCAN_TILE - 1) / SCAN_TILE);
    if (nb > 0) k_scan_reduce<<<nb, SCAN_BLOCK, 0, st>>>(in, n, part);
    k_scan_part<<<1, SCAN_BLOCK, 0, st>>>(part, nb);
    if (nb > 0) k_scan_apply<<<nb, SCAN_BLOCK, 0, st>>>(in, out, n, part, exclusive ? 1 : 0);
    return hipGetLastError();
}

// ----------------------------------------------------- duplicate / scatter --
__global__ void __launch_bounds__(256) k_duplicate(Cam c, int P, const uint8_t* __restrict__ geom,
                                                   const int32_t* __restrict__ radii, uint32_t* __restrict__ tile_cnt,
                                                   uint32_t* __restrict__ rank)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P) return;
    const int r = radii[i];
    if (r <= 0) return;
    const GeomLayout L = geom_layout(P);
    const float4 A = ((const float4*)(geom + L.splatA))[i];
    const uint32_t* tiles = (const uint32_t*)(geom + L.tiles);
    const uint32_t* offs = (const uint32_t*)(geom + L.offsets);
    uint32_t o = offs[i] - tiles[i];
    int x0, y0, x1, y1;
    get_rect(A.x, A.y, r, c.gx, c.gy, x0, y0, x1, y1);
    for (int y = y0; y < y1; y++)
        for (int x = x0; x < x1; x++) rank[o++] = atomicAdd(&tile_cnt[y * c.gx + x], 1u);
}

hipError_t launch_duplicate(const Cam& c, int P, const uint8_t* geom, const int32_t* radii, uint32_t* tile_cnt,
                            uint32_t* rank, hipStream_t st)
{
    if (P == 0) return hipSuccess;
    k_duplicate<<<(P + 255) / 256, 256, 0, st>>>(c, P, geom, radii, tile_cnt, rank);
    return hipGetLastError();
}

__global__ void __launch_bounds__(256) k_scatter(Cam c, int P, const uint8_t* __restrict__ geom,
                                                 const int32_t* __restrict__ radii,
                                                 const uint32_t* __restrict__ tile_start,
                                                 const uint32_t* __restrict__ rank, uint64_t* __restrict__ keys)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P) return;
    const int r = radii[i];
    if (r <= 0) return;
    const GeomLayout L = geom_layout(P);
    const float4 A = ((const float4*)(geom + L.splatA))[i];
    const float depth = ((const float*)(geom + L.depth))[i];
    const uint32_t* tiles = (const uint32_t*)(geom + L.tiles);
    const uint32_t* offs = (const uint32_t*)(geom + L.offsets);
    uint32_t o = offs[i] - tiles[i];
    const uint64_t key = ((uint64_t)__float_as_uint(depth) << 32) | (uint32_t)i;
    int x0, y0, x1, y1;
    get_rect(A.x, A.y, r, c.gx, c.gy, x0, y0, x1, y1);
    for (int y = y0; y < y1; y++)
        for (int x = x0; x < x1; x++) keys[tile_start[y * c.gx + x] + rank[o++]] = key;
}

hipError_t launch_scatter(const Cam& c, int P, const uint8_t* geom, const int32_t* radii, const uint32_t* tile_start,
                          const uint32_t* rank, uint64_t* keys, hipStream_t st)
{
    if (P == 0) return hipSuccess;
    k_scatter<<<(P + 255) / 256, 256, 0, st>>>(c, P, geom, radii, tile_start, rank, keys);
    return hipGetLastError();
}

// ------------------------------------------------------------ tile sort ---
// Ascending flip-bitonic network over n keys with virtual +inf padding to the
// next power of two: every compare-exchange puts the minimum at the lower
// index, so pairs whose upper index is >= n are no-ops and are skipped.
#define SORT_BLOCK 256
#define SORT_CHUNK 4096

__device__ __forceinline__ void ce(uint64_t* a, int i, int l)
{
    uint64_t x = a[i], y = a[l];
    if (x > y) { a[i] = y; a[l] = x; }
}

// Full network for k = 2..kmax over a[0, n) (n <= kmax), in LDS.
__device__ void bitonic_lds(uint64_t* a, int n, int kmax)
{
    for (int k = 2; k <= kmax; k <<= 1) {
        const int hk = k >> 1;
        for (int p = threadIdx.x; p < kmax / 2; p += SORT_BLOCK) {
            const int blk = p / hk, off = p % hk;
            const int i = blk * k + off, l = blk * k + k - 1 - off;
            if (l < n) ce(a, i, l);
        }
        __syncthreads();
        for (int j = k >> 2; j >= 1; j >>= 1) {
            for (int p = threadIdx.x; p < kmax / 2; p += SORT_BLOCK) {
                const int i = (p / j) * 2 * j + (p % j), l = i + j;
                if (l < n) ce(a, i, l);
            }
            __syncthreads();
        }
    }
}

// Half-cleaner steps j = jmax..1 over a[0, n) in LDS (n <= chunk).
__device__ void halfclean_lds(uint64_t* a, int n, int chunk, int jmax)
{
    for (int j = jmax; j >= 1; j >>= 1) {
        for (int p = threadIdx.x; p < chunk / 2; p += SORT_BLOCK) {
            const int i = (p / j) * 2 * j + (p % j), l = i + j;
            if (l < n) ce(a, i, l);
        }
        __syncthreads();
    }
}

__device__ __forceinline__ int next_pow2(int n)
{
    int p = 1;
    while (p < n) p <<= 1;
    return p;
}

__global__ void __launch_bounds__(SORT_BLOCK) k_tile_sort(int T, const uint32_t* __restrict__ tile_start,
                                                          uint64_t* __restrict__ keys, uint32_t* __restrict__ point_list)
{
    __shared__ uint64_t buf[SORT_CHUNK];
    const int t = xcd_remap(blockIdx.x, gridDim.x);
    if (t >= T) return;
    const uint32_t s0 = tile_start[t], s1 = tile_start[t + 1];
    const int n = (int)(s1 - s0);
    if (n == 0) return;
    uint64_t* g = keys + s0;
    if (n <= SORT_CHUNK) {
        for (int k = threadIdx.x; k < n; k += SORT_BLOCK) buf[k] = g[k];
        __syncthreads();
        bitonic_lds(buf, n, next_pow2(n));
        for (int k = threadIdx.x; k < n; k += SORT_BLOCK) point_list[s0 + k] = (uint32_t)buf[k];
        return;
    }
    // Large tile: chunk-local stages in LDS, cross-chunk stages in global
    // memory (one workgroup owns the tile; __syncthreads orders its passes).
    const int n2 = next_pow2(n);
    const int nch = (n + SORT_CHUNK - 1) / SORT_CHUNK;
    for (int ch = 0; ch < nch; ch++) {
        const int cb = ch * SORT_CHUNK, cn = min(SORT_CHUNK, n - cb);
        for (int k = threadIdx.x; k < cn; k += SORT_BLOCK) buf[k] = g[cb + k];
        __syncthreads();
        bitonic_lds(buf, cn, SORT_CHUNK);
        for (int k = threadIdx.x; k < cn; k += SORT_BLOCK) g[cb + k] = buf[k];
        __syncthreads();
    }
    for (int k = 2 * SORT_CHUNK; k <= n2; k <<= 1) {
        const int hk = k >> 1;
        for (int p = threadIdx.x; p < n2 / 2; p += SORT_BLOCK) {
            const int blk = p / hk, off = p % hk;
            const int i = blk * k + off, l = blk * k + k - 1 - off;
            if (l < n) ce(g, i, l);
        }
        __syncthreads();
        for (int j = k >> 2; j >= SORT_CHUNK; j >>= 1) {
            for (int p = threadIdx.x; p < n2 / 2; p += SORT_BLOCK) {
                const int i = (p / j) * 2 * j + (p % j), l = i + j;
                if (l < n) ce(g, i, l);
            }
            __syncthreads();
        }
        for (int ch = 0; ch < nch; ch++) {
            const int cb = ch * SORT_CHUNK, cn = min(SORT_CHUNK, n - cb);
            for (int q = threadIdx.x; q < cn; q += SORT_BLOCK) buf[q] = g[cb + q];
            __syncthreads();
            halfclean_lds(buf, cn, SORT_CHUNK, SORT_CHUNK / 2);
            for (int q = threadIdx.x; q < cn; q += SORT_BLOCK) g[cb + q] = buf[q];
            __syncthreads();
        }
    }
    for (int k = threadIdx.x; k < n; k += SORT_BLOCK) point_list[s0 + k] = (uint32_t)g[k];
}

hipError_t launch_tile_sort(int T, const uint32_t* tile_start, uint64_t* keys, uint32_t* point_list, hipStream_t st)
{
    if (T == 0) return hipSuccess;
    k_tile_sort<<<T, SORT_BLOCK, 0, st>>>(T, tile_start, keys, point_list);
    return hipGetLastError();
}

}  // namespace lsr
