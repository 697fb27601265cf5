// binning.hip — tile binning (A.2): per-tile instance counts, scatter into
// tile buckets, per-tile depth sort.
//
// MI355X design (vs the reference's global 64-bit radix sort over
// 32 + log2(T) bits of M keys): the tile is the bucket.
//  - count/scatter (k_bin_count / k_bin_table / k_bin_scatter): per-block
//    tile histograms in LDS, a B x T column scan for block bases, LDS-atomic
//    ranks inside the block: no global atomics at all.  (The older
//    k_duplicate / k_scatter pair with one global atomic per instance remains
//    as the fallback when T does not fit LDS.)
//  - per-tile sort of the bucket's unique u64 keys (depth bits << 32 | id):
//    one wave per tile with the keys in registers (k_tile_sort_wave, n <= 1024);
//    a workgroup in LDS for n <= 4096, chunked LDS + global merge above.
// The result equals a stable sort by (tile, depth bits) with ties broken by
// Gaussian id — the order of the reference's stable radix sort over
// duplicates emitted in Gaussian order — of the reference's instances minus
// the ones the tile cull drops: an instance (Gaussian, tile) of the 3-sigma
// rect is emitted only if the Gaussian's cut ellipse meets the tile
// (tile_keep, lsr_device.h); a dropped instance has alpha < 1/255 at every
// pixel of its tile, so no output changes (the oracle checks both lists
// render identically: tests/test_oracle.py).  cfg3: 8.25 M -> 4.73 M.
#include "bin_common.h"

#include <algorithm>

#ifndef LSR_BIN_TARGET
#define LSR_BIN_TARGET 512   // (chunk x band) blocks of the privatised count / scatter
#endif
#ifndef LSR_SORT_WAVE_MAX
#define LSR_SORT_WAVE_MAX 1024  // largest tile sorted by one wave in registers (512, 1024 or 2048): cfg3 tile_sort 0.079 -> 0.073 ms at 1024
#endif
#ifndef LSR_SORT_DPP
#define LSR_SORT_DPP 1
#endif

namespace lsr {

// ---------------------------------------------------------------- scan ----
#define SCAN_ITEMS 16
#define SCAN_BLOCK 256
#define SCAN_TILE (SCAN_ITEMS * SCAN_BLOCK)

size_t scan_partials(size_t n) { return (n + SCAN_TILE - 1) / SCAN_TILE + 1; }

// Block-wide exclusive scan over NB threads (sh: NB / 64 entries).
template <int NB>
__device__ __forceinline__ uint64_t block_excl_scan_u64_n(uint64_t v, uint64_t* sh, uint64_t& total)
{
    // wave inclusive scan via shuffles, then across the waves through LDS
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
    for (int k = 0; k < NB / 64; k++) {
        if (k < w) wofs += sh[k];
        tot += sh[k];
    }
    __syncthreads();
    total = tot;
    return wofs + x - v;
}
__device__ __forceinline__ uint64_t block_excl_scan_u64(uint64_t v, uint64_t* sh, uint64_t& total)
{
    return block_excl_scan_u64_n<SCAN_BLOCK>(v, sh, total);
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

// Publish the scan total: writes it as the closing entry of the tile-start
// array (tile_end, may be null) and, packed with a sequence number, into a
// coherent pinned host word the host spins on (lsr_api.hip wait_published):
// the host needs M to size the binning workspace, and polling one
// PCIe-visible word avoids the staged D2H copy + stream-synchronise wake-up
// latency in the middle of every forward.  Totals >= 2^32 - 1 saturate (the
// host reports LSR_EOVERFLOW).
__global__ void k_publish_total(const uint64_t* __restrict__ total, uint32_t* __restrict__ tile_end,
                                uint64_t* host_slot, uint32_t seq, const uint32_t* __restrict__ cls_cnt)
{
    const uint64_t m = *total;
    const uint32_t m32 = m >= 0xffffffffull ? 0xffffffffu : (uint32_t)m;
    if (tile_end) *tile_end = m32;
    if (cls_cnt) {
        // per-class tile counts ride along in the same pinned line: the host
        // launches exactly the sort classes that have work
        uint32_t* h = (uint32_t*)(host_slot + 1);
#pragma unroll
        for (int k = 0; k < SORT_NCLS; k++) h[k] = cls_cnt[k];
        __atomic_store_n(host_slot + LSR_CLS_SLOT, ((uint64_t)seq << 32) | m32, __ATOMIC_RELEASE);
    }
    __atomic_store_n(host_slot, ((uint64_t)seq << 32) | m32, __ATOMIC_RELEASE);
}

hipError_t launch_publish_total(const uint64_t* total, uint32_t* tile_end, uint64_t* host_slot, uint32_t seq,
                                const uint32_t* cls_cnt, hipStream_t st)
{
    k_publish_total<<<1, 1, 0, st>>>(total, tile_end, host_slot, seq, cls_cnt);
    return hipGetLastError();
}

// Sort size classes: 0 wave sort (n <= 512), 1..4 block merge sorts with
// KPL = 4, 8, 16, 32 (n <= 256*KPL), 5 chunked LDS/global (n > 8192).  Empty
// tiles are in no class.
__device__ __forceinline__ int tile_class(int n)
{
    if (n <= 0) return -1;
    if (n <= LSR_SORT_WAVE_MAX) return 0;
    if (n <= 1024) return 1;
    if (n <= 2048) return 2;
    if (n <= 4096) return 3;
    if (n <= 8192) return 4;
    return 5;
}

// Wave-aggregated append of tile t (lanes with active) to its class list.
// Every lane of the wave must call it.  One atomic instruction for the whole
// wave: lane k adds the wave's class-k count to cls_cnt[k] (the classes'
// adds are independent, so they share one round trip instead of one each).
__device__ __forceinline__ void tile_class_append(bool active, int t, int n, int T, uint32_t* __restrict__ cls_cnt,
                                                  uint32_t* __restrict__ cls_list)
{
    const int c = active ? tile_class(n) : -1;
    const int lane = threadIdx.x & 63;
    const uint64_t below = lane ? (~0ull >> (64 - lane)) : 0ull;
    uint64_t m[SORT_NCLS];
    uint32_t cnt = 0;
#pragma unroll
    for (int k = 0; k < SORT_NCLS; k++) {
        m[k] = __ballot(c == k);
        cnt = lane == k ? (uint32_t)__popcll(m[k]) : cnt;
    }
    uint32_t base = 0;
    if (cnt) base = atomicAdd(&cls_cnt[lane], cnt);
    uint64_t mine = 0;
#pragma unroll
    for (int k = 0; k < SORT_NCLS; k++) mine = c == k ? m[k] : mine;
    const uint32_t b = __shfl(base, c < 0 ? 0 : c, 64);
    if (c >= 0) cls_list[(size_t)c * T + b + __popcll(mine & below)] = (uint32_t)t;
}

// Classification pass for the global-atomic binning path (the privatised path
// classifies inside k_bin_table).  cls_cnt must be zero.
__global__ void __launch_bounds__(256) k_tile_classify(int T, const uint32_t* __restrict__ tile_start,
                                                       uint32_t* __restrict__ cls_cnt, uint32_t* __restrict__ cls_list)
{
    const int t = blockIdx.x * 256 + threadIdx.x;
    const int n = t < T ? (int)(tile_start[t + 1] - tile_start[t]) : 0;
    tile_class_append(t < T, t, n, T, cls_cnt, cls_list);
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
    const float4 B = ((const float4*)(geom + L.splatB))[i];
    const uint32_t* tiles = (const uint32_t*)(geom + L.tiles);
    const uint32_t* offs = (const uint32_t*)(geom + L.offsets);
    uint32_t o = offs[i] - tiles[i];
    int x0, y0, x1, y1;
    get_rect(A.x, A.y, r, c.gx, c.gy, x0, y0, x1, y1);
    const SpanPrep sp = span_prep(A, B);
    int bx0 = x0, by0 = y0, bx1 = x1, by1 = y1;
    cull_box(A.x, A.y, A.z, A.w, B.x, B.z, bx0, by0, bx1, by1);
    for (int y = y0; y < y1; y++) {
        int sx0 = 0, sx1 = 0;
        if (y >= by0 && y < by1) row_span(sp, y, bx0, bx1, sx0, sx1);
        for (int x = x0; x < x1; x++, o++)
            rank[o] = (x >= sx0 && x < sx1) ? atomicAdd(&tile_cnt[y * c.gx + x], 1u) : 0xffffffffu;
    }
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
        for (int x = x0; x < x1; x++, o++)
            if (rank[o] != 0xffffffffu) keys[tile_start[y * c.gx + x] + rank[o]] = key;
}

hipError_t launch_scatter(const Cam& c, int P, const uint8_t* geom, const int32_t* radii, const uint32_t* tile_start,
                          const uint32_t* rank, uint64_t* keys, hipStream_t st)
{
    if (P == 0) return hipSuccess;
    k_scatter<<<(P + 255) / 256, 256, 0, st>>>(c, P, geom, radii, tile_start, rank, keys);
    return hipGetLastError();
}

// --------------------------------------------- privatised count / scatter --
// Block b owns Gaussians [b*chunk, (b+1)*chunk).  k_bin_count builds the
// block's tile histogram with LDS atomics and writes it as row b of the
// B x T table; k_bin_table scans each column (tile) over blocks; k_bin_scatter
// re-walks the chunk and places every instance at tile_start + block base +
// LDS-atomic rank.  No global atomics; the in-bucket order is arbitrary and
// fixed by the per-tile sort.


// Load-balanced expansion of the kept instances.  Lane l of a wave owns
// Gaussian i0 + l: its cull box clipped to the band, h_l rows.  The wave's
// rows are numbered by an exclusive scan of h_l and taken 64 at a time
// (a round): lane j computes row entry r0 + j's kept tile range (row_span,
// owner found by binary search over the row scan), the round's entries are
// scanned by width, and each lane walks a contiguous slice of the round's
// kept instances (one entry search, then along the entries).  Every lane
// does one kept instance per step however unequal the Gaussians are, and no
// instance outside the cull is visited or tested.
struct WaveSpans {
    int rpre[65];      // exclusive scan of the owners' band rows; [64] = total
    int epre[65];      // the round's entries: exclusive scan of kept widths; [64] = total
    float4 P0[64];     // owner's SpanPrep: x, y, vm, vr
    float4 P1[64];     //                   cb, det, tca, ica
    float me[64];      //                   me
    int box[64];       // owner's box columns: bx0 | bx1 << 16
    int y0[64];        // owner's first band row (band-relative)
    int ent[64];       // entry: first kept column | band row << 16 | owner << 24
};

// Wave-uniform: stage the lanes' Gaussians, return the wave's row total.
__device__ __forceinline__ int wave_spans_stage(WaveSpans& ws, int h, int bx0, int bx1, int y0, const SpanPrep& sp)
{
    const int lane = threadIdx.x & 63;
    ws.P0[lane] = make_float4(sp.x, sp.y, sp.vm, sp.vr);
    ws.P1[lane] = make_float4(sp.cb, sp.det, sp.tca, sp.ica);
    ws.me[lane] = sp.me;
    ws.box[lane] = bx0 | (bx1 << 16);
    ws.y0[lane] = y0;
    int s = h;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int t = __shfl_up(s, d, 64);
        if (lane >= d) s += t;
    }
    ws.rpre[lane] = s - h;
    if (lane == 63) ws.rpre[64] = s;
    wave_lds_fence();
    return __shfl(s, 63, 64);
}

// Row entry e of the staged wave: its owner (returned), band row yr and kept
// columns [sx0, sx1).
__device__ __forceinline__ int row_entry(const WaveSpans& ws, int e, int ty0, int& sx0, int& sx1, int& yr)
{
    const int o = wave_search(ws.rpre, e);
    yr = ws.y0[o] + (e - ws.rpre[o]);
    const float4 p0 = ws.P0[o], p1 = ws.P1[o];
    const SpanPrep sp{p0.x, p0.y, p0.z, p0.w, p1.x, p1.y, p1.z, p1.w, ws.me[o]};
    const int bx = ws.box[o];
    row_span(sp, yr + ty0, bx & 0xffff, bx >> 16, sx0, sx1);
    return o;
}

// Wave-uniform: one round's entries (rows r0 .. r0 + 63 of the wave), return
// the round's kept-instance total.
__device__ __forceinline__ int wave_spans_round(WaveSpans& ws, int r0, int R, int ty0)
{
    const int lane = threadIdx.x & 63;
    const int e = r0 + lane;
    int wd = 0, packed = 0;
    if (e < R) {
        int sx0, sx1, yr;
        const int o = row_entry(ws, e, ty0, sx0, sx1, yr);
        wd = sx1 - sx0;
        packed = sx0 | (yr << 16) | (o << 24);
    }
    int s = wd;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int t = __shfl_up(s, d, 64);
        if (lane >= d) s += t;
    }
    ws.epre[lane] = s - wd;
    if (lane == 63) ws.epre[64] = s;
    ws.ent[lane] = packed;
    wave_lds_fence();
    return __shfl(s, 63, 64);
}

// A lane's contiguous slice of a round's kept instances: one entry search,
// then along the entries (LDS reads only when the walk enters the next one).
struct SpanWalk {
    int j, x, xe, y, o;
    __device__ __forceinline__ void enter(const WaveSpans& ws, int k0)
    {
        const int p = ws.ent[j];
        x = (p & 0xffff) + k0;
        xe = (p & 0xffff) + (ws.epre[j + 1] - ws.epre[j]);
        y = (p >> 16) & 0xff;
        o = p >> 24;
    }
    __device__ __forceinline__ SpanWalk(const WaveSpans& ws, int k)
    {
        j = wave_search(ws.epre, k);
        enter(ws, k - ws.epre[j]);
    }
    // advance to the next instance (the caller guarantees there is one)
    __device__ __forceinline__ void next(const WaveSpans& ws)
    {
        if (++x < xe) return;
        do { ++j; } while (ws.epre[j + 1] == ws.epre[j]);
        enter(ws, 0);
    }
};

// Stage the lane's Gaussian for the span walk; returns the wave's row total.
__device__ __forceinline__ int stage_gaussian(WaveSpans& ws, const Cam& c, const Band& bd, const BinRec& g)
{
    int x0, x1, y0;
    const int h = band_box(c, bd, g, x0, x1, y0);
    return wave_spans_stage(ws, h, x0, x1, y0, span_prep(g.A, g.B));
}

template <int BB>
__global__ void __launch_bounds__(BB) k_bin_count(Cam c, int P, int chunk, int rows, int S,
                                                         const uint8_t* __restrict__ geom,
                                                         const int32_t* __restrict__ radii, uint32_t* __restrict__ table,
                                                         uint32_t* __restrict__ cls_cnt, uint64_t* host_slot, uint32_t seq)
{
    extern __shared__ uint32_t hist[];
    __shared__ WaveSpans wss[BB / 64];
    __shared__ uint64_t s_tot;
    const int T = c.gx * c.gy;
#if LSR_COUNT_XCD
    // chunk-major, XCD-aware (as k_bin_scatter): a chunk's bands share an L2
    const int o = xcd_remap(blockIdx.x, gridDim.x);
    const int blk = o / S;
    const Band bd(c, rows, o - blk * S);
#else
    const int blk = blockIdx.x;
    const Band bd(c, rows, blockIdx.y);
#endif
    // k_bin_table appends to the class counts and takes tickets after us
    if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x < SORT_NCLS) cls_cnt[threadIdx.x] = 0;
    if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) cls_cnt[LSR_TICKET_WORD] = 0;
    for (int k = threadIdx.x; k < bd.nt; k += BB) hist[k] = 0;
    if (threadIdx.x == 0) s_tot = 0;
    __syncthreads();
    WaveSpans& ws = wss[threadIdx.x >> 6];
    const int lane = threadIdx.x & 63;
    const int g0 = blk * chunk, g1 = min(P, g0 + chunk);
    BinRec nx;
    if (g0 < g1) nx.load(geom, P, g1, radii, g0 + (threadIdx.x & ~63) + lane, false);
    for (int i0 = g0 + (threadIdx.x & ~63); i0 < g1; i0 += BB) {
        const BinRec cur = nx;
        nx.load(geom, P, g1, radii, i0 + BB + lane, false);
        const int R = stage_gaussian(ws, c, bd, cur);
        // every row entry adds its kept range [sx0, sx1) to the histogram as
        // a difference (+1 at sx0, -1 at sx1 inside the row): two LDS atomics
        // per (Gaussian, row) instead of one per instance
        for (int e = lane; e < R; e += 64) {
            int sx0, sx1, yr;
            row_entry(ws, e, bd.ty0, sx0, sx1, yr);
            if (sx1 > sx0) {
                atomicAdd(&hist[yr * c.gx + sx0], 1u);
                if (sx1 < c.gx) atomicAdd(&hist[yr * c.gx + sx1], 0xffffffffu);
            }
        }
        wave_lds_fence();
    }
    __syncthreads();
    // per band row: counts = running sum of the differences (mod 2^32), written
    // straight into the block's table row; one wave per row, 64 columns a step
    uint32_t* row = table + (size_t)blk * table_stride(T) + bd.t0;
    const int nrows = bd.ty1 - bd.ty0;
    uint64_t mine = 0;   // the lane's share of the block's instances
    for (int r = threadIdx.x >> 6; r < nrows; r += BB / 64) {
        uint32_t carry = 0;
        for (int x0 = 0; x0 < c.gx; x0 += 64) {
            const int x = x0 + lane;
            uint32_t v = x < c.gx ? hist[r * c.gx + x] : 0u;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const uint32_t t = __shfl_up(v, d, 64);
                if (lane >= d) v += t;
            }
            if (x < c.gx) {
                row[r * c.gx + x] = carry + v;
                mine += carry + v;
            }
            carry += __shfl(v, 63, 64);
        }
    }
    // M = the sum of every block's counts, published here rather than by
    // k_bin_table: the host sizes and launches the scatter while the column
    // scan runs (the sort classes follow from k_bin_table).  One agent-scope
    // add per block carries the block total and, in bits 44+, its arrival; the
    // block whose add completes the grid holds M.  The sum word is zeroed by
    // the preprocess (the launch before us).
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) mine += __shfl_xor(mine, d, 64);
    if (lane == 0 && mine) atomicAdd((unsigned long long*)&s_tot, (unsigned long long)mine);
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint64_t add = s_tot + (1ull << 44);
        const uint64_t prev = __hip_atomic_fetch_add((uint64_t*)(cls_cnt + LSR_COUNT_WORD), add, __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_AGENT);
        if ((prev >> 44) == (uint64_t)gridDim.x * gridDim.y - 1) {
            const uint64_t m = (prev + add) & ((1ull << 44) - 1);
            const uint32_t m32 = m >= 0xffffffffull ? 0xffffffffu : (uint32_t)m;
            __hip_atomic_store(host_slot, ((uint64_t)seq << 32) | m32, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

// Column scan: table[b][t] <- sum_{b' < b} table[b'][t]; tile_cnt[t] <- total.
// The table's rows have stride Tp = T rounded up to 4 (columns past T are
// never written by the count and are masked here).  A block owns 64 tiles
// (one tile group): 16 column groups of 4 tiles (one 16-B load per row) x
// SEGS row segments of 16 rows, every row held in registers between the sum
// and the rewrite (the table is read once and written once).
//
// The same launch also finishes the tile scan's top level and publishes M:
// every block stores its group total write-through (sc1) and takes a ticket
// (agent-scope add after every wave drained its stores, behind a workgroup
// barrier); the block holding the last ticket scans the group totals (sc1
// loads, in place), writes tile_start[T] = M and publishes the sort class
// counts with M to the pinned host line (word LSR_CLS_SLOT; k_bin_count
// published M alone in word 0 one launch earlier).  k_tile_start_apply then adds each group's base to the
// in-group scan.  This replaces three scan launches and the publish launch.
// The ticket is zeroed by k_bin_count (the preceding launch).
#define TBL_TILES 64   // tiles per k_bin_table block (and per tile group)
#define TBL_RPT 16     // table rows per thread
struct BinPublish {
    uint64_t* gpart;      // per tile group: total, then (last block) exclusive base; [G] = M
    uint32_t* ticket;     // arrival counter, zero on entry
    uint32_t* tile_end;   // tile_start + T
    uint64_t* host_slot;  // pinned host word LSR_CLS_SLOT (the class counts are words 1..3)
    uint32_t seq;
};
__device__ __forceinline__ uint32_t u4_get(const uint4& v, int j) { return j == 0 ? v.x : j == 1 ? v.y : j == 2 ? v.z : v.w; }
__device__ __forceinline__ uint4 u4_add(const uint4& a, const uint4& b)
{
    return make_uint4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
}

template <int SEGS>
__global__ void __launch_bounds__(16 * SEGS) k_bin_table(int T, int Tp, int B, uint32_t* __restrict__ table,
                                                         uint32_t* __restrict__ tile_cnt,
                                                         uint32_t* __restrict__ cls_cnt,
                                                         uint32_t* __restrict__ cls_list, BinPublish pb)
{
    constexpr int NT = 16 * SEGS;
    __shared__ uint4 seg_sum[SEGS][16];
    __shared__ uint64_t sh[NT / 64];
    __shared__ int s_last;
    const int cg = threadIdx.x & 15, seg = threadIdx.x >> 4;
    const int t4 = blockIdx.x * TBL_TILES + cg * 4;   // this thread's 4 tiles
    const int b0 = seg * TBL_RPT;
    // columns past T (the row padding, or past the last tile) count 0
    const uint4 cmask = make_uint4(t4 < T ? ~0u : 0u, t4 + 1 < T ? ~0u : 0u, t4 + 2 < T ? ~0u : 0u,
                                   t4 + 3 < T ? ~0u : 0u);
    const bool colok = t4 < Tp;
    uint4 v[TBL_RPT];
    uint4 sum = make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
    for (int k = 0; k < TBL_RPT; k++) {
        const int b = b0 + k;
        uint4 x = make_uint4(0u, 0u, 0u, 0u);
        if (colok && b < B) x = *reinterpret_cast<const uint4*>(table + (size_t)b * Tp + t4);
        v[k] = make_uint4(x.x & cmask.x, x.y & cmask.y, x.z & cmask.z, x.w & cmask.w);
        sum = u4_add(sum, v[k]);
    }
    seg_sum[seg][cg] = sum;
    __syncthreads();
    uint4 run = make_uint4(0u, 0u, 0u, 0u), tot = run;
    for (int k = 0; k < SEGS; k++) {
        const uint4 x = seg_sum[k][cg];
        if (k < seg) run = u4_add(run, x);
        tot = u4_add(tot, x);
    }
    if (threadIdx.x < 64) {
        // segment 0 = lanes 0..15 of wave 0 hold the 64 totals, 4 each: lane
        // l takes tile l for the class append (one call for the group)
        const int l = threadIdx.x, src = l >> 2, j = l & 3;
        const uint32_t n0 = __shfl(tot.x, src, 64), n1 = __shfl(tot.y, src, 64);
        const uint32_t n2 = __shfl(tot.z, src, 64), n3 = __shfl(tot.w, src, 64);
        const uint32_t nl = j == 0 ? n0 : j == 1 ? n1 : j == 2 ? n2 : n3;
        const int tl = blockIdx.x * TBL_TILES + l;
        tile_class_append(tl < T, tl, (int)nl, T, cls_cnt, cls_list);
        uint64_t g = seg == 0 ? (uint64_t)tot.x + tot.y + tot.z + tot.w : 0ull;
#pragma unroll
        for (int d = 8; d >= 1; d >>= 1) g += __shfl_xor(g, d, 64);
        if (threadIdx.x == 0) __hip_atomic_store(&pb.gpart[blockIdx.x], g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (seg == 0) {
#pragma unroll
            for (int j = 0; j < 4; j++)
                if (t4 + j < T) tile_cnt[t4 + j] = u4_get(tot, j);
        }
    }
    if (colok) {
#pragma unroll
        for (int k = 0; k < TBL_RPT; k++) {
            const int b = b0 + k;
            if (b < B) *reinterpret_cast<uint4*>(table + (size_t)b * Tp + t4) = run;
            run = u4_add(run, v[k]);
        }
    }
    // ticket: every wave drains its stores (the group total's sc1 store, the
    // class atomics), then one lane arrives for the workgroup
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t prev = __hip_atomic_fetch_add(pb.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_last = prev == gridDim.x - 1;
    }
    __syncthreads();
    if (!s_last) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // keeps the sc1 loads below the ticket
    // the group totals, 8 consecutive ones per thread, all loads in flight at
    // once (one round trip per 8 NT groups)
    const int G = (int)gridDim.x;
    uint64_t carry = 0;
    for (int base = 0; base < G; base += NT * 8) {
        const int i0 = base + threadIdx.x * 8;
        uint64_t gv[8], s = 0;
#pragma unroll
        for (int k = 0; k < 8; k++)
            gv[k] = i0 + k < G ? __hip_atomic_load(&pb.gpart[i0 + k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0ull;
#pragma unroll
        for (int k = 0; k < 8; k++) s += gv[k];
        uint64_t gt;
        uint64_t r = carry + block_excl_scan_u64_n<NT>(s, sh, gt);
#pragma unroll
        for (int k = 0; k < 8; k++) {
            if (i0 + k < G) pb.gpart[i0 + k] = r;
            r += gv[k];
        }
        carry += gt;
    }
    if (threadIdx.x < 64) {
        // the class counts: one load per lane, all in flight; lane 0 stores
        // them and then the releasing sequence word
        const int l = threadIdx.x;
        const uint32_t cnt = l < SORT_NCLS ? __hip_atomic_load(&cls_cnt[l], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
        uint32_t cv[SORT_NCLS];
#pragma unroll
        for (int k = 0; k < SORT_NCLS; k++) cv[k] = __shfl(cnt, k, 64);
        if (l == 0) {
            const uint32_t m32 = carry >= 0xffffffffull ? 0xffffffffu : (uint32_t)carry;
            pb.gpart[G] = carry;
            *pb.tile_end = m32;
            uint32_t* h = (uint32_t*)(pb.host_slot - LSR_CLS_SLOT + 1);
#pragma unroll
            for (int k = 0; k < SORT_NCLS; k++) __hip_atomic_store(&h[k], cv[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            // the counts are written through (system scope) and acknowledged
            // before the sequence word goes out.  No release fence: the host
            // reads nothing else this kernel wrote, and a system-scope release
            // writes back this XCD's whole L2 first (the freshly rewritten
            // table) -- measured ~20 us at cfg5.
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __hip_atomic_store(pb.host_slot, ((uint64_t)pb.seq << 32) | m32, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

// tile_start[t] = group base + exclusive scan of tile_cnt inside the 64-tile
// group (one wave).
__global__ void __launch_bounds__(256) k_tile_start_apply(int T, const uint32_t* __restrict__ tile_cnt,
                                                          const uint64_t* __restrict__ gpart,
                                                          uint32_t* __restrict__ tile_start)
{
    const int t = blockIdx.x * 256 + threadIdx.x;
    const uint32_t v = t < T ? tile_cnt[t] : 0u;
    uint32_t x = v;
    const int l = threadIdx.x & 63;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d, 64);
        if (l >= d) x += y;
    }
    if (t < T) tile_start[t] = (uint32_t)gpart[t / TBL_TILES] + x - v;
}

// The scatter's bands are its own (rows of its own, not the count's): the
// table row of (chunk, tile) does not depend on how tiles are grouped.  The
// 1-D grid is chunk-major and XCD-aware (xcd_remap): the S bands of one chunk
// run back to back on one XCD, so a chunk's geometry is read from that XCD's
// L2 and the partial key lines the XCD has open at once span ~one chunk's
// tiles instead of one per resident block.
template <int BB>
__global__ void __launch_bounds__(BB) k_bin_scatter(Cam c, int P, int chunk, int km, int rows, int S,
                                                           const uint8_t* __restrict__ geom,
                                                           const int32_t* __restrict__ radii,
                                                           const uint32_t* __restrict__ table,
                                                           const uint32_t* __restrict__ tile_start,
                                                           uint64_t* __restrict__ keys)
{
    extern __shared__ uint32_t base[];
    __shared__ WaveSpans wss[BB / 64];
    __shared__ uint64_t wkey[BB];   // the lanes' (depth, id) keys
    const int T = c.gx * c.gy;
    const int o = xcd_remap(blockIdx.x, gridDim.x);
    const int blk = (o / S) * km;   // first of the km count chunks this block places
    const Band bd(c, rows, o - (o / S) * S);
    const uint32_t* row = table + (size_t)blk * table_stride(T) + bd.t0;
    for (int k = threadIdx.x; k < bd.nt; k += BB) base[k] = tile_start[bd.t0 + k] + row[k];
    __syncthreads();
    WaveSpans& ws = wss[threadIdx.x >> 6];
    uint64_t* const key = wkey + (threadIdx.x & ~63);
    const int lane = threadIdx.x & 63;
    const int g0 = blk * chunk, g1 = min(P, g0 + km * chunk);
    BinRec nx;
    if (g0 < g1) nx.load(geom, P, g1, radii, g0 + (threadIdx.x & ~63) + lane, true);
    for (int i0 = g0 + (threadIdx.x & ~63); i0 < g1; i0 += BB) {
        const int i = i0 + lane;
        const BinRec cur = nx;
        nx.load(geom, P, g1, radii, i0 + BB + lane, true);
        key[lane] = ((uint64_t)__float_as_uint(cur.depth) << 32) | (uint32_t)i;
        const int R = stage_gaussian(ws, c, bd, cur);
        for (int r0 = 0; r0 < R; r0 += 64) {
            const int K = wave_spans_round(ws, r0, R, bd.ty0);
            const int q = (K + 63) >> 6;
            int k = lane * q;
            const int kend = min(K, k + q);
            if (k < kend) {
                SpanWalk sw(ws, k);
                // two instances per step: both LDS-atomic returns in flight
                for (;;) {
                    const uint32_t sa = atomicAdd(&base[sw.y * c.gx + sw.x], 1u);
                    const uint64_t ka = key[sw.o];
                    const bool two = k + 1 < kend;
                    uint32_t sb = 0;
                    uint64_t kb = 0;
                    if (two) {
                        sw.next(ws);
                        sb = atomicAdd(&base[sw.y * c.gx + sw.x], 1u);
                        kb = key[sw.o];
                    }
                    keys[sa] = ka;
                    if (two) keys[sb] = kb;
                    k += 2;
                    if (k >= kend) break;
                    sw.next(ws);
                }
            }
            wave_lds_fence();
        }
    }
}

// Tile rows per band: the largest band whose histogram fits LSR_BAND_LDS.
// At most LSR_BAND_ROWS rows: at cfg3 (68 tile rows) two bands of 34 halve
// the chunk count for the same ~512 blocks — a smaller B x T table and longer
// per-(chunk, tile) key runs: bin_count 0.0756 -> 0.0691 ms, scatter +0.002 (r02
// A/B; cfg2 count -10 %; cfg5 already has 34-row bands, 24 / 17 were slower).
// Below 4M Gaussians up to 68 rows in up to 2 x LSR_BAND_LDS (r05: cfg3 is then
// one band, its ~512 blocks 512 chunks, and the scatter's blocks twice as many:
// bin_scatter 0.0806 -> 0.0586 ms, whole step 1.1085 -> 1.0984 ms; at cfg5 68-row
// bands were slower, count 0.313 -> 0.363 ms; profiles/r05s3_ab_bands_cfg*.txt).
#ifndef LSR_BAND_ROWS
#define LSR_BAND_ROWS 34
#endif
#ifndef LSR_BAND_ROWS_SMALL
#define LSR_BAND_ROWS_SMALL 68
#endif
static int bin_band_rows(const Cam& c, int P)
{
    const bool big = P >= (4 << 20);
    const int cap = big ? LSR_BAND_ROWS : LSR_BAND_ROWS_SMALL;
    const int lds = big ? LSR_BAND_LDS : 2 * LSR_BAND_LDS;
    return std::max(1, std::min(std::min(c.gy, cap), lds / (4 * c.gx)));
}

// Tile rows per scatter band: the largest band whose LDS bases fit
// LSR_SCATTER_LDS bytes (narrower bands than the count's measured slower:
// every band re-walks its chunk).
#ifndef LSR_SCATTER_LDS
#define LSR_SCATTER_LDS LSR_BAND_LDS
#endif
#ifndef LSR_SCATTER_ROWS
#define LSR_SCATTER_ROWS 0   // > 0: tile rows per scatter band (A/B)
#endif
// Count chunks per scatter block: their table rows are consecutive, so the
// block's run per tile is the concatenation of theirs (longer runs, fewer
// partially written lines).  From 4M Gaussians up 4 (cfg5 bin_scatter 0.900 ->
// 0.839 ms; 2 measured 1.08), below 1 (cfg3: 2 / 4 slower, 4 with 17-row
// bands equal; r03q A/B).  LSR_SCATTER_MERGE > 0 forces a factor (A/B).
#ifndef LSR_SCATTER_MERGE
#define LSR_SCATTER_MERGE 0
#endif
int scatter_merge(int P) { return LSR_SCATTER_MERGE > 0 ? LSR_SCATTER_MERGE : (P >= (4 << 20) ? 4 : 1); }
int bin_scatter_rows(const Cam& c)
{
    if (LSR_SCATTER_ROWS > 0) return std::max(1, std::min(c.gy, LSR_SCATTER_ROWS));
    return std::max(1, std::min(c.gy, LSR_SCATTER_LDS / (4 * c.gx)));
}

// Threads per (chunk, band) scatter block (and the chunk granule): 16 waves
// below 4M Gaussians, 8 waves from 4M up (16 measured slower at cfg5: scatter
// 0.98 -> 1.11 ms).  The count runs 8-wave blocks at every size (r05; in r02
// 16 waves had been faster for the count at cfg3 with 34-row bands).
int bin_block(int P) { return P >= (4 << 20) ? 512 : 1024; }

int bin_blocks(int P, const Cam& c, int& chunk)
{
    // ~512 (chunk x band) blocks, 2 per CU, of >= 1024 Gaussians; fewer
    // chunks when there are several bands keeps the B x T table small
    const int rows = bin_band_rows(c, P);
    const int S = (c.gy + rows - 1) / rows;
    // twice the blocks from 4M Gaussians up: cfg5 (5M) bin_scatter 1.20 ->
    // 1.02 ms; at cfg3 (1M) 1024 blocks make the count + table pass slower
    const int total = P >= (4 << 20) ? 2 * LSR_BIN_TARGET : LSR_BIN_TARGET;
    const int target = std::max(64, total / S);
    chunk = max(1024, (P + target - 1) / target);
    const int bb = bin_block(P);
    chunk = (chunk + bb - 1) / bb * bb;
    return (P + chunk - 1) / chunk;
}

// The privatised path needs one band row of tiles to fit LDS and a B x T
// table of moderate size.
bool bin_privatised_ok(const Cam& c) { return (size_t)c.gx * 4 <= LSR_BAND_LDS && (size_t)c.gx * c.gy <= (1u << 20); }

hipError_t launch_bin_count(const Cam& c, int P, int chunk, int B, const uint8_t* geom, const int32_t* radii,
                            uint32_t* table, uint32_t* tile_cnt, uint32_t* tile_start, uint64_t* tpart,
                            uint32_t* cls_cnt, uint32_t* cls_list, uint64_t* host_slot, uint32_t seq, hipStream_t st)
{
    const int T = c.gx * c.gy;
    const int rows = bin_band_rows(c, P);
    const int S = (c.gy + rows - 1) / rows;
    const dim3 grid(LSR_COUNT_XCD ? B * S : B, LSR_COUNT_XCD ? 1 : S);
    const size_t lds = (size_t)rows * c.gx * 4;
    if (lds > 65536) {
        (void)hipFuncSetAttribute((const void*)k_bin_count<512>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        (void)hipFuncSetAttribute((const void*)k_bin_scatter<512>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        (void)hipFuncSetAttribute((const void*)k_bin_scatter<1024>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    }
    if (B > 0) {
        // 8-wave count blocks at every size (r05, with the 68-row bands and the
        // colour pass beside it: cfg3 bin_count 0.104 -> 0.077 ms, step -1.3 / -1.7 %
        // in both A/B orders, profiles/r05s3_ab_tune{2,3}_cfg3.txt); the scatter keeps
        // bin_block's 16 waves below 4M
        if ((size_t)grid.x * grid.y >= (1u << 20)) return hipErrorInvalidValue;   // arrivals field (bits 44+)
        k_bin_count<512><<<grid, 512, lds, st>>>(c, P, chunk, rows, S, geom, radii, table, cls_cnt, host_slot, seq);
        BinPublish pb{tpart, cls_cnt + LSR_TICKET_WORD, tile_start + T, host_slot + LSR_CLS_SLOT, seq};
        const int G = (T + TBL_TILES - 1) / TBL_TILES, Tp = table_stride(T);
        if (B <= 16 * TBL_RPT)
            k_bin_table<16><<<G, 256, 0, st>>>(T, Tp, B, table, tile_cnt, cls_cnt, cls_list, pb);
        else if (B <= 32 * TBL_RPT)
            k_bin_table<32><<<G, 512, 0, st>>>(T, Tp, B, table, tile_cnt, cls_cnt, cls_list, pb);
        else if (B <= 64 * TBL_RPT)
            k_bin_table<64><<<G, 1024, 0, st>>>(T, Tp, B, table, tile_cnt, cls_cnt, cls_list, pb);
        else
            return hipErrorInvalidValue;   // bin_blocks keeps B <= 2 * LSR_BIN_TARGET
    } else {
        (void)hipMemsetAsync(tile_cnt, 0, (size_t)T * 4, st);
        (void)hipMemsetAsync(cls_cnt, 0, SORT_NCLS * 4, st);
        (void)launch_scan_u32(tile_cnt, tile_start, tpart, (size_t)T, true, st);
        (void)launch_publish_total(tpart + (scan_partials((size_t)T) - 1), tile_start + T, host_slot, seq, cls_cnt, st);
    }
    return hipGetLastError();
}

hipError_t launch_tile_start_apply(int T, int B, const uint32_t* tile_cnt, const uint64_t* tpart, uint32_t* tile_start,
                                   hipStream_t st)
{
    if (B > 0 && T > 0) k_tile_start_apply<<<(T + 255) / 256, 256, 0, st>>>(T, tile_cnt, tpart, tile_start);
    return hipGetLastError();
}

hipError_t launch_bin_scatter(const Cam& c, int P, int chunk, int B, const uint8_t* geom, const int32_t* radii,
                              const uint32_t* table, const uint32_t* tile_start, uint64_t* keys, hipStream_t st)
{
    const int rows = bin_scatter_rows(c);
    const int S = (c.gy + rows - 1) / rows;
    const size_t lds = (size_t)rows * c.gx * 4;
    if (lds > 65536) {
        (void)hipFuncSetAttribute((const void*)k_bin_scatter<512>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        (void)hipFuncSetAttribute((const void*)k_bin_scatter<1024>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    }
    const int km = scatter_merge(P), Bs = (B + km - 1) / km;
    if (B > 0 && bin_block(P) == 1024)
        k_bin_scatter<1024><<<Bs * S, 1024, lds, st>>>(c, P, chunk, km, rows, S, geom, radii, table, tile_start, keys);
    else if (B > 0)
        k_bin_scatter<512><<<Bs * S, 512, lds, st>>>(c, P, chunk, km, rows, S, geom, radii, table, tile_start, keys);
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

// Tiles of class 5 (n > 8192): one workgroup per tile (grid-stride over the
// class list), chunk-local bitonic stages in LDS, cross-chunk stages in
// global memory.
__device__ void tile_sort_big(int t, const uint32_t* __restrict__ tile_start, uint64_t* __restrict__ keys,
                              uint32_t* __restrict__ point_list, uint64_t* buf)
{
    const uint32_t s0 = tile_start[t], s1 = tile_start[t + 1];
    const int n = (int)(s1 - s0);
    uint64_t* g = keys + s0;
    if (n <= SORT_CHUNK) {
        for (int k = threadIdx.x; k < n; k += SORT_BLOCK) buf[k] = g[k];
        __syncthreads();
        bitonic_lds(buf, n, next_pow2(n));
        for (int k = threadIdx.x; k < n; k += SORT_BLOCK) point_list[s0 + k] = (uint32_t)buf[k];
        __syncthreads();
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
    __syncthreads();
}

__global__ void __launch_bounds__(SORT_BLOCK) k_tile_sort_big(int T, const uint32_t* __restrict__ tile_start,
                                                              uint64_t* __restrict__ keys,
                                                              uint32_t* __restrict__ point_list,
                                                              const uint32_t* __restrict__ cls_cnt,
                                                              const uint32_t* __restrict__ cls_list)
{
    __shared__ uint64_t buf[SORT_CHUNK];
    const uint32_t cnt = cls_cnt[5];
    for (uint32_t i = blockIdx.x; i < cnt; i += gridDim.x)
        tile_sort_big((int)cls_list[(size_t)5 * T + i], tile_start, keys, point_list, buf);
}

// Wave-level register bitonic sort for tiles of n <= 64*KPL keys: lane l
// holds elements [l*KPL, l*KPL + KPL) (padding = UINT64_MAX).  Steps whose
// partner distance j < KPL run inside the lane's registers; the others pair
// lane l with lane l ^ (j / KPL) through shuffles.  No LDS, no barriers.
__device__ __forceinline__ uint64_t shfl_xor_u64(uint64_t v, int m)
{
    const uint32_t lo = __shfl_xor((uint32_t)v, m, 64);
    const uint32_t hi = __shfl_xor((uint32_t)(v >> 32), m, 64);
    return ((uint64_t)hi << 32) | lo;
}

#ifndef LSR_SORT_XBATCH
#define LSR_SORT_XBATCH 1
#endif
// xor_lane_u32 (the register-path lane exchange) lives in lsr_device.h, where
// tests/micro/micro_checks.hip checks it against __shfl_xor on the GPU.
template <int M>
__device__ __forceinline__ uint64_t xor_lane_u64(uint64_t v)
{
#if LSR_SORT_DPP
    const uint32_t lo = xor_lane_u32<M>((uint32_t)v);
    const uint32_t hi = xor_lane_u32<M>((uint32_t)(v >> 32));
    return ((uint64_t)hi << 32) | lo;
#else
    return shfl_xor_u64(v, M);
#endif
}

template <int KPL, int K, int J>
__device__ __forceinline__ void wave_sort_xstep(uint64_t (&v)[KPL])
{
    constexpr int M = J / KPL;
    const int lane = threadIdx.x & 63;
    // K >= 2J >= 2 KPL: the direction bit of element lane*KPL + r is the
    // lane's alone, so one flag serves all KPL elements
    const bool take_min = ((lane & M) == 0) == (((lane * KPL) & K) == 0);
#if LSR_SORT_XBATCH
    // every partner first, then every select: the lane exchanges (DPP /
    // permlane) read registers the previous step wrote long before, so no
    // hazard wait states sit between a select and the exchange that needs it
    uint64_t o[KPL];
#pragma unroll
    for (int r = 0; r < KPL; r++) o[r] = xor_lane_u64<M>(v[r]);
#pragma unroll
    for (int r = 0; r < KPL; r++) v[r] = ((v[r] < o[r]) == take_min) ? v[r] : o[r];
#else
#pragma unroll
    for (int r = 0; r < KPL; r++) {
        const uint64_t o = xor_lane_u64<M>(v[r]);
        v[r] = ((v[r] < o) == take_min) ? v[r] : o;   // keep own value iff it is the wanted one
    }
#endif
}

template <int KPL, int K, int J>
__device__ __forceinline__ void wave_sort_steps(uint64_t (&v)[KPL])
{
    if constexpr (J >= 1) {
        if constexpr (J < KPL) {
            const int lane = threadIdx.x & 63;
            // direction of element lane*KPL + r: from r alone while K < KPL
            // (compile time), from the lane alone once K >= KPL (r < KPL <= K
            // never reaches bit K): one compare + one mask XOR per pair
            const bool desc_lane = ((lane * KPL) & K) != 0;
#pragma unroll
            for (int r = 0; r < KPL; r++) {
                if (r & J) continue;
                const uint64_t a = v[r], b = v[r | J];
                bool sw;
                if constexpr (K < KPL) sw = (r & K) ? (a < b) : (a > b);
                else sw = (a > b) != desc_lane;
                v[r] = sw ? b : a;
                v[r | J] = sw ? a : b;
            }
        } else {
            wave_sort_xstep<KPL, K, J>(v);
        }
        wave_sort_steps<KPL, K, J / 2>(v);
    }
}

template <int KPL, int K>
__device__ __forceinline__ void wave_sort_stages(uint64_t (&v)[KPL])
{
    if constexpr (K <= 64 * KPL) {
        wave_sort_steps<KPL, K, K / 2>(v);
        wave_sort_stages<KPL, 2 * K>(v);
    }
}

template <int KPL>
__device__ __forceinline__ void wave_sort_tile(const uint64_t* __restrict__ g, uint32_t* __restrict__ out, int n)
{
    const int lane = threadIdx.x & 63;
    uint64_t v[KPL];
#pragma unroll
    for (int r = 0; r < KPL; r++) {
        const int e = lane * KPL + r;
        v[r] = e < n ? g[e] : ~0ull;
    }
    wave_sort_stages<KPL, 2>(v);
#pragma unroll
    for (int r = 0; r < KPL; r++) {
        const int e = lane * KPL + r;
        if (e < n) out[e] = (uint32_t)v[r];
    }
}

// LDS slot of logical element e of a block sort: one u64 of padding every 16
// keys, so the lane-major run reads (lane stride KPL*8 bytes) spread over
// the banks instead of piling onto a few.
__device__ __forceinline__ int lpad(int e) { return e + (e >> 4); }

// Merge-path co-rank: how many of the first d outputs of merge(A, B) come
// from A, A = lds[a0, a0+na), B = lds[b0, b0+nb) (logical indices; keys are
// unique, so ties never occur).
__device__ __forceinline__ int merge_corank(const uint64_t* lds, int a0, int na, int b0, int nb, int d)
{
    int lo = max(0, d - nb), hi = min(d, na);
    while (lo < hi) {
        const int m = (lo + hi) >> 1;
        if (lds[lpad(a0 + m)] < lds[lpad(b0 + d - 1 - m)]) lo = m + 1;
        else hi = m;
    }
    return lo;
}

// KPL consecutive outputs of merge(A, B) starting at output d, into v.
template <int KPL>
__device__ __forceinline__ void merge_run(const uint64_t* lds, int a0, int na, int b0, int nb, int d,
                                          uint64_t (&v)[KPL])
{
    int i = merge_corank(lds, a0, na, b0, nb, d), j = d - i;
    uint64_t a = i < na ? lds[lpad(a0 + i)] : ~0ull, b = j < nb ? lds[lpad(b0 + j)] : ~0ull;
#pragma unroll
    for (int k = 0; k < KPL; k++) {
        const bool ta = a < b;
        v[k] = ta ? a : b;
        i += ta ? 1 : 0;
        j += ta ? 0 : 1;
        const bool ok = ta ? (i < na) : (j < nb);
        const uint64_t nx = ok ? lds[lpad(ta ? a0 + i : b0 + j)] : ~0ull;
        a = ta ? nx : a;
        b = ta ? b : nx;
    }
}

// One 4-wave workgroup per tile of 128*KPL < n <= 256*KPL keys.  The bucket
// is staged into LDS with coalesced loads (+inf padding), each wave sorts a
// 64*KPL run in registers (the wave bitonic network above), two merge-path
// rounds (every thread producing KPL consecutive outputs after a binary
// co-rank search) finish the order, and the ids leave through LDS with
// coalesced stores.
template <int KPL>
__device__ __forceinline__ void block_sort_tile(const uint64_t* __restrict__ g, uint32_t* __restrict__ out, int n,
                                                uint64_t* lds)
{
    constexpr int R = 64 * KPL;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    // batches of 8 loads in flight per thread (a full unroll would hold all
    // 4*KPL keys in VGPRs and collapse occupancy)
#pragma unroll 1
    for (int k0 = 0; k0 < 4 * KPL; k0 += 8) {
        uint64_t x[8];
#pragma unroll
        for (int k = 0; k < 8; k++) {
            const int e = (k0 + k) * 256 + tid;
            x[k] = e < n ? g[e] : ~0ull;
        }
#pragma unroll
        for (int k = 0; k < 8; k++) lds[lpad((k0 + k) * 256 + tid)] = x[k];
    }
    __syncthreads();
    uint64_t v[KPL];
#pragma unroll
    for (int r = 0; r < KPL; r++) v[r] = lds[lpad(w * R + lane * KPL + r)];
    wave_sort_stages<KPL, 2>(v);
#pragma unroll
    for (int r = 0; r < KPL; r++) lds[lpad(w * R + lane * KPL + r)] = v[r];
    __syncthreads();
    {
        const int p0 = (tid >> 7) * 2 * R, d = (tid & 127) * KPL;
        merge_run<KPL>(lds, p0, R, p0 + R, R, d, v);
        __syncthreads();
#pragma unroll
        for (int k = 0; k < KPL; k++) lds[lpad(p0 + d + k)] = v[k];
    }
    __syncthreads();
    const int d = tid * KPL;
    merge_run<KPL>(lds, 0, 2 * R, 2 * R, 2 * R, d, v);
    __syncthreads();
    uint32_t* l32 = (uint32_t*)lds;
#pragma unroll
    for (int k = 0; k < KPL; k++) l32[d + k + ((d + k) >> 5)] = (uint32_t)v[k];
    __syncthreads();
#pragma unroll 8
    for (int e = tid; e < n; e += 256) out[e] = l32[e + (e >> 5)];
    __syncthreads();
}

// Class c = 1..4 (KPL = 4 << (c - 1)): one workgroup per listed tile.
template <int KPL>
__global__ void __launch_bounds__(256) k_tile_sort_blk(int T, const uint32_t* __restrict__ tile_start,
                                                       const uint64_t* __restrict__ keys,
                                                       uint32_t* __restrict__ point_list,
                                                       const uint32_t* __restrict__ cls_cnt,
                                                       const uint32_t* __restrict__ cls_list, int cls)
{
    __shared__ uint64_t lds[(4 * 64 * KPL) * 17 / 16];
    const uint32_t cnt = cls_cnt[cls];
    for (uint32_t i = blockIdx.x; i < cnt; i += gridDim.x) {
        const int t = (int)cls_list[(size_t)cls * T + i];
        const uint32_t s0 = tile_start[t];
        block_sort_tile<KPL>(keys + s0, point_list + s0, (int)(tile_start[t + 1] - s0), lds);
    }
}

// Class 0 (n <= 512): one wave per listed tile, four per workgroup.
__global__ void __launch_bounds__(256) k_tile_sort_wave(int T, const uint32_t* __restrict__ tile_start,
                                                        const uint64_t* __restrict__ keys,
                                                        uint32_t* __restrict__ point_list,
                                                        const uint32_t* __restrict__ cls_cnt,
                                                        const uint32_t* __restrict__ cls_list)
{
    const uint32_t cnt = cls_cnt[0];
    for (uint32_t i = blockIdx.x * 4 + (threadIdx.x >> 6); i < cnt; i += gridDim.x * 4) {
        const int t = (int)cls_list[i];
        const uint32_t s0 = tile_start[t];
        const int n = (int)(tile_start[t + 1] - s0);
        const uint64_t* g = keys + s0;
        uint32_t* o = point_list + s0;
        if (n == 1) {
            if ((threadIdx.x & 63) == 0) o[0] = (uint32_t)g[0];
        } else if (n <= 64) wave_sort_tile<1>(g, o, n);
        else if (n <= 128) wave_sort_tile<2>(g, o, n);
        else if (n <= 256) wave_sort_tile<4>(g, o, n);
        else if (LSR_SORT_WAVE_MAX <= 512 || n <= 512) wave_sort_tile<8>(g, o, n);
        else if (LSR_SORT_WAVE_MAX <= 1024 || n <= 1024) wave_sort_tile<16>(g, o, n);
        else wave_sort_tile<32>(g, o, n);
    }
}

// host_cnt: the per-class tile counts when the host already has them (the
// privatised binning path publishes them with M); null = unknown, the lists
// are built here and every class runs a persistent grid.
hipError_t launch_tile_sort(int T, const uint32_t* tile_start, uint64_t* keys, uint32_t* point_list,
                            uint32_t* cls_cnt, uint32_t* cls_list, const uint32_t* host_cnt, hipStream_t st)
{
    if (T == 0) return hipSuccess;
    uint32_t cnt[SORT_NCLS];
    if (host_cnt) {
        for (int k = 0; k < SORT_NCLS; k++) cnt[k] = host_cnt[k];
    } else {
        (void)hipMemsetAsync(cls_cnt, 0, SORT_NCLS * 4, st);
        k_tile_classify<<<(T + 255) / 256, 256, 0, st>>>(T, tile_start, cls_cnt, cls_list);
        // persistent grids: enough workgroups to fill the chip, or the tiles
        const uint32_t fill[SORT_NCLS] = {256 * 8, 256 * 8, 256 * 8, 256 * 4, 256 * 2, 256 * 2};
        for (int k = 0; k < SORT_NCLS; k++) cnt[k] = std::min<uint32_t>((uint32_t)T, fill[k] * (k == 0 ? 4 : 1));
    }
    const uint32_t* cc = cls_cnt;
    const uint32_t* cl = cls_list;
    if (cnt[0]) k_tile_sort_wave<<<(cnt[0] + 3) / 4, 256, 0, st>>>(T, tile_start, keys, point_list, cc, cl);
    if (cnt[1]) k_tile_sort_blk<4><<<cnt[1], 256, 0, st>>>(T, tile_start, keys, point_list, cc, cl, 1);
    if (cnt[2]) k_tile_sort_blk<8><<<cnt[2], 256, 0, st>>>(T, tile_start, keys, point_list, cc, cl, 2);
    if (cnt[3]) k_tile_sort_blk<16><<<cnt[3], 256, 0, st>>>(T, tile_start, keys, point_list, cc, cl, 3);
    if (cnt[4]) k_tile_sort_blk<32><<<cnt[4], 256, 0, st>>>(T, tile_start, keys, point_list, cc, cl, 4);
    if (cnt[5]) k_tile_sort_big<<<cnt[5], SORT_BLOCK, 0, st>>>(T, tile_start, keys, point_list, cc, cl);
    return hipGetLastError();
}

}  // namespace lsr
