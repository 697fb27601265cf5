// order.hip — depth-ordered tile binning (the "ordered" binning mode).
//
// The reference's order of a tile's instances is (depth bits, Gaussian id)
// ascending (its stable radix sort over (tile | depth) keys emitted in
// Gaussian order: cuda_rasterizer/rasterizer_impl.cu duplicateWithKeys +
// cub::DeviceRadixSort::SortPairs).  The sorted-tiles mode (binning.hip)
// scatters (depth, id) keys into the tile buckets in arbitrary order and sorts
// every bucket.  This mode sorts the Gaussians instead — one stable LSD radix
// sort of P 32-bit depth keys, ~12x fewer keys than instances at 4K — and then
// places every tile's instances in that order, so the buckets come out sorted
// and the scatter writes the 4-B ids of point_list directly:
//
//  1. k_rs_hist / k_rs_scatter: 4 passes of 8 bits over the depth bits of the
//     visible Gaussians (invisible ones get the key 0xffffffff and sort last).
//     Stable: a block's items are ranked in index order (per wave: ballot
//     match of the digit, rank among lower lanes + the wave's running digit
//     count; waves and blocks in order through prefix sums), then written
//     through an LDS reorder so each digit's run leaves as one contiguous
//     segment.  Equal depths keep Gaussian-id order, as in the reference.
//  2. k_bin_count (binning.hip) over chunks of the SORTED order (records
//     gathered through the order), the B x T table scan and tile starts as in
//     the sorted-tiles mode.
//  3. k_bin_scatter_ord: block (chunk, band) as in k_bin_scatter, but every
//     wave owns the band's tile rows r with r % waves == wave (no two waves
//     share a tile), walks ALL the block's Gaussians in sorted order, and
//     places its instances in enumeration order: within one step the lanes
//     hitting the same tile are ranked by a ballot match of the tile index
//     and the group's highest lane advances the tile's LDS base (plain LDS
//     read / write, no atomics: deterministic).  A tile's run from one chunk
//     is therefore in sorted order, and the runs are in chunk order.
// No per-tile sort, no 8-B key buffer.
#include "bin_common.h"

namespace lsr {

#define RS_BLOCK 256                    // threads of a radix block = digits
#define RS_ITEMS 16                     // items per thread
#define RS_TILE (RS_BLOCK * RS_ITEMS)   // items per block
#define RS_WAVES (RS_BLOCK / 64)
#define RS_WAVE_ITEMS (RS_TILE / RS_WAVES)

#define LSR_RET(expr)                       \
    do {                                    \
        const hipError_t e_ = (expr);       \
        if (e_ != hipSuccess) return e_;    \
    } while (0)

static int rs_blocks(int n) { return (n + RS_TILE - 1) / RS_TILE; }

// Workspace of launch_depth_order: keys and ids twice (ping-pong), the
// per-pass digit x block histogram and its scan partials.
DepthOrderLayout depth_order_layout(int P)
{
    DepthOrderLayout L;
    const size_t n = (size_t)(P > 0 ? P : 1);
    const size_t nh = (size_t)256 * rs_blocks(P > 0 ? P : 1);
    size_t o = 0;
    L.kA = o;   o += align256(n * 4);
    L.kB = o;   o += align256(n * 4);
    L.vA = o;   o += align256(n * 4);
    L.vB = o;   o += align256(n * 4);
    L.hist = o; o += align256(nh * 4);
    L.part = o; o += align256((scan_partials(nh) + 1) * 8);
    L.total = o;
    return L;
}

// First-pass key of Gaussian i: the depth bits of a visible Gaussian (depth >
// 0 past the near plane, so the bits order like the floats), 0xffffffff for an
// invisible one (radius 0: never binned).
__device__ __forceinline__ uint32_t depth_key(const float* __restrict__ depth, const int32_t* __restrict__ radii, int i)
{
    return radii[i] > 0 ? __float_as_uint(depth[i]) : 0xffffffffu;
}

// Per-block digit histogram of pass `shift`: hist[d * nblk + block].
template <bool FIRST>
__global__ void __launch_bounds__(RS_BLOCK) k_rs_hist(int n, int shift, const uint32_t* __restrict__ kin,
                                                      const float* __restrict__ depth, const int32_t* __restrict__ radii,
                                                      uint32_t* __restrict__ hist, int nblk)
{
    __shared__ uint32_t h[RS_WAVES][256];
    for (int k = threadIdx.x; k < RS_WAVES * 256; k += RS_BLOCK) (&h[0][0])[k] = 0u;
    __syncthreads();
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int base = blockIdx.x * RS_TILE + w * RS_WAVE_ITEMS;
    uint32_t key[RS_ITEMS];
#pragma unroll
    for (int k = 0; k < RS_ITEMS; k++) {
        const int i = base + k * 64 + lane;
        key[k] = i < n ? (FIRST ? depth_key(depth, radii, i) : kin[i]) : 0u;
    }
#pragma unroll
    for (int k = 0; k < RS_ITEMS; k++)
        if (base + k * 64 + lane < n) atomicAdd(&h[w][(key[k] >> shift) & 255u], 1u);
    __syncthreads();
    uint32_t s = 0;
#pragma unroll
    for (int q = 0; q < RS_WAVES; q++) s += h[q][threadIdx.x];
    hist[(size_t)threadIdx.x * nblk + blockIdx.x] = s;
}

// Stable scatter of pass `shift` (hist_ex: the exclusive scan of hist in
// digit-major order = each (digit, block) run's global start).  FIRST: keys
// from the depths, ids = indices.  LAST: only the ids are written.
template <bool FIRST, bool LAST>
__global__ void __launch_bounds__(RS_BLOCK) k_rs_scatter(int n, int shift, const uint32_t* __restrict__ kin,
                                                         const uint32_t* __restrict__ vin,
                                                         const float* __restrict__ depth,
                                                         const int32_t* __restrict__ radii,
                                                         const uint32_t* __restrict__ hist_ex, int nblk,
                                                         uint32_t* __restrict__ kout, uint32_t* __restrict__ vout)
{
    __shared__ uint32_t wc[RS_WAVES][256];   // per-wave digit counts -> the wave's prefix per digit
    __shared__ uint32_t bex[256];            // block-local start of each digit
    __shared__ uint32_t goff[256];           // global start of the block's run of each digit
    __shared__ uint32_t wsum[RS_WAVES];
    __shared__ uint32_t sk[RS_TILE];         // the block's items in digit order
    __shared__ uint32_t sv[RS_TILE];
    const int t = threadIdx.x;
    for (int k = t; k < RS_WAVES * 256; k += RS_BLOCK) (&wc[0][0])[k] = 0u;
    goff[t] = hist_ex[(size_t)t * nblk + blockIdx.x];
    const int w = t >> 6, lane = t & 63;
    const int base = blockIdx.x * RS_TILE + w * RS_WAVE_ITEMS;
    uint32_t key[RS_ITEMS], val[RS_ITEMS], rk[RS_ITEMS];
#pragma unroll
    for (int k = 0; k < RS_ITEMS; k++) {
        const int i = base + k * 64 + lane;
        const bool ok = i < n;
        key[k] = ok ? (FIRST ? depth_key(depth, radii, i) : kin[i]) : 0xffffffffu;
        val[k] = FIRST ? (uint32_t)i : (ok ? vin[i] : 0u);
    }
    __syncthreads();
    const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
#pragma unroll
    for (int k = 0; k < RS_ITEMS; k++) {
        const bool ok = base + k * 64 + lane < n;
        const uint32_t d = (key[k] >> shift) & 255u;
        uint64_t peers = __ballot(ok);
#pragma unroll
        for (int b = 0; b < 8; b++) {
            const bool bit = (d >> b) & 1u;
            const uint64_t m = __ballot(bit);
            peers &= bit ? m : ~m;
        }
        // lanes of this round with digit d rank after the wave's earlier ones;
        // the group's highest lane advances the count (reads precede the write)
        const uint32_t old = wc[w][d];
        rk[k] = old + (uint32_t)__popcll(peers & lt);
        if (ok && (peers >> lane) == 1ull) wc[w][d] = old + (uint32_t)__popcll(peers);
    }
    __syncthreads();
    // digit t: the waves' prefixes, then the block's exclusive scan over digits
    uint32_t run = 0;
#pragma unroll
    for (int q = 0; q < RS_WAVES; q++) {
        const uint32_t x = wc[q][t];
        wc[q][t] = run;
        run += x;
    }
    uint32_t incl = run;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(incl, d, 64);
        if (lane >= d) incl += y;
    }
    if (lane == 63) wsum[w] = incl;
    __syncthreads();
    uint32_t wofs = 0;
#pragma unroll
    for (int q = 0; q < RS_WAVES; q++) wofs += q < w ? wsum[q] : 0u;
    bex[t] = wofs + incl - run;
    __syncthreads();
#pragma unroll
    for (int k = 0; k < RS_ITEMS; k++) {
        if (base + k * 64 + lane < n) {
            const uint32_t d = (key[k] >> shift) & 255u;
            const uint32_t li = bex[d] + wc[w][d] + rk[k];
            sk[li] = key[k];
            sv[li] = val[k];
        }
    }
    __syncthreads();
    const int cnt = min(RS_TILE, n - (int)blockIdx.x * RS_TILE);
    for (int j = t; j < cnt; j += RS_BLOCK) {
        const uint32_t kk = sk[j];
        const uint32_t d = (kk >> shift) & 255u;
        const uint32_t pos = goff[d] + ((uint32_t)j - bex[d]);
        if (!LAST) kout[pos] = kk;
        vout[pos] = sv[j];
    }
}

hipError_t launch_depth_order(int P, const uint8_t* geom, const int32_t* radii, uint8_t* ws, const uint32_t** order,
                              hipStream_t st)
{
    const DepthOrderLayout L = depth_order_layout(P);
    uint32_t* kA = (uint32_t*)(ws + L.kA);
    uint32_t* kB = (uint32_t*)(ws + L.kB);
    uint32_t* vA = (uint32_t*)(ws + L.vA);
    uint32_t* vB = (uint32_t*)(ws + L.vB);
    uint32_t* hist = (uint32_t*)(ws + L.hist);
    uint64_t* part = (uint64_t*)(ws + L.part);
    *order = vA;
    if (P <= 0) return hipSuccess;
    const GeomLayout GL = geom_layout((size_t)P);
    const float* depth = (const float*)(geom + GL.depth);
    const int nblk = rs_blocks(P);
    const size_t nh = (size_t)256 * nblk;
    // pass 0: depths -> (kB, vB); 1: -> (kA, vA); 2: -> (kB, vB); 3: ids -> vA
    k_rs_hist<true><<<nblk, RS_BLOCK, 0, st>>>(P, 0, nullptr, depth, radii, hist, nblk);
    LSR_RET(launch_scan_u32(hist, hist, part, nh, true, st));
    k_rs_scatter<true, false><<<nblk, RS_BLOCK, 0, st>>>(P, 0, nullptr, nullptr, depth, radii, hist, nblk, kB, vB);
    k_rs_hist<false><<<nblk, RS_BLOCK, 0, st>>>(P, 8, kB, nullptr, nullptr, hist, nblk);
    LSR_RET(launch_scan_u32(hist, hist, part, nh, true, st));
    k_rs_scatter<false, false><<<nblk, RS_BLOCK, 0, st>>>(P, 8, kB, vB, nullptr, nullptr, hist, nblk, kA, vA);
    k_rs_hist<false><<<nblk, RS_BLOCK, 0, st>>>(P, 16, kA, nullptr, nullptr, hist, nblk);
    LSR_RET(launch_scan_u32(hist, hist, part, nh, true, st));
    k_rs_scatter<false, false><<<nblk, RS_BLOCK, 0, st>>>(P, 16, kA, vA, nullptr, nullptr, hist, nblk, kB, vB);
    k_rs_hist<false><<<nblk, RS_BLOCK, 0, st>>>(P, 24, kB, nullptr, nullptr, hist, nblk);
    LSR_RET(launch_scan_u32(hist, hist, part, nh, true, st));
    k_rs_scatter<false, true><<<nblk, RS_BLOCK, 0, st>>>(P, 24, kB, vB, nullptr, nullptr, hist, nblk, nullptr, vA);
    return hipGetLastError();
}

// ------------------------------------------------------- ordered scatter ---
// The block's staged Gaussians (one per thread, in sorted order): span prep,
// box columns, band-relative rows [y0, y1) (empty: y0 = y1), id.
template <int BB>
struct OrdStage {
    float4 P0[BB];   // x, y, vm, vr
    float4 P1[BB];   // cb, det, tca, ica
    float me[BB];
    int box[BB];     // bx0 | bx1 << 16
    int yy[BB];      // y0 | y1 << 16
    uint32_t id[BB];
};
// A wave's row entries of one round: owner (staged index), first kept column |
// band row << 16, the scans of the owners' row counts and of the widths.
struct OrdWave {
    int rpre[65];
    int epre[65];
    int ex[64];
    int eo[64];
};

template <int BB>
__global__ void __launch_bounds__(BB) k_bin_scatter_ord(Cam c, int P, int chunk, int km, int rows, int S,
                                                        const uint8_t* __restrict__ geom,
                                                        const int32_t* __restrict__ radii,
                                                        const uint32_t* __restrict__ order,
                                                        const uint32_t* __restrict__ table,
                                                        const uint32_t* __restrict__ tile_start,
                                                        uint32_t* __restrict__ point_list)
{
    constexpr int NW = BB / 64;
    extern __shared__ uint32_t base[];
    __shared__ OrdStage<BB> sg;
    __shared__ OrdWave wvs[NW];
    const int T = c.gx * c.gy;
    const int o = xcd_remap(blockIdx.x, gridDim.x);
    const int blk = (o / S) * km;
    const Band bd(c, rows, o - (o / S) * S);
    const uint32_t* row = table + (size_t)blk * table_stride(T) + bd.t0;
    for (int k = threadIdx.x; k < bd.nt; k += BB) base[k] = tile_start[bd.t0 + k] + row[k];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    OrdWave& ws = wvs[w];
    const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
    // tile-index bits the match needs (uniform)
    const int nbits = bd.nt > 1 ? 32 - __clz(bd.nt - 1) : 0;
    const int g0 = blk * chunk, g1 = min(P, g0 + km * chunk);
    BinRec nx;
    if (g0 < g1) nx.load(geom, P, g1, radii, g0 + (int)threadIdx.x, false, order);
    for (int i0 = g0; i0 < g1; i0 += BB) {
        const BinRec cur = nx;
        __syncthreads();   // the previous step's staging is consumed (and base is ready)
        {
            int x0, x1, y0;
            const int h = band_box(c, bd, cur, x0, x1, y0);
            const SpanPrep sp = span_prep(cur.A, cur.B);
            sg.P0[threadIdx.x] = make_float4(sp.x, sp.y, sp.vm, sp.vr);
            sg.P1[threadIdx.x] = make_float4(sp.cb, sp.det, sp.tca, sp.ica);
            sg.me[threadIdx.x] = sp.me;
            sg.box[threadIdx.x] = x0 | (x1 << 16);
            sg.yy[threadIdx.x] = h > 0 ? y0 | ((y0 + h) << 16) : 0;
            sg.id[threadIdx.x] = cur.id;
        }
        nx.load(geom, P, g1, radii, i0 + BB + (int)threadIdx.x, false, order);
        __syncthreads();
        for (int s = 0; s < BB; s += 64) {
            // this wave's rows r (r % NW == w) of staged Gaussian s + lane
            const int q = s + lane;
            const int yy = sg.yy[q];
            const int y0 = yy & 0xffff, y1 = yy >> 16;
            const int fr = y0 + ((w - y0 % NW) + NW) % NW;
            const int h = fr < y1 ? (y1 - 1 - fr) / NW + 1 : 0;
            int sc = h;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const int y = __shfl_up(sc, d, 64);
                if (lane >= d) sc += y;
            }
            const int R = __shfl(sc, 63, 64);
            if (R == 0) continue;
            ws.rpre[lane] = sc - h;
            if (lane == 63) ws.rpre[64] = sc;
            wave_lds_fence();
            for (int r0 = 0; r0 < R; r0 += 64) {
                const int e = r0 + lane;
                int wd = 0;
                if (e < R) {
                    const int ol = wave_search(ws.rpre, e);
                    const int oq = s + ol;
                    const int oy0 = sg.yy[oq] & 0xffff;
                    const int ofr = oy0 + ((w - oy0 % NW) + NW) % NW;
                    const int yr = ofr + NW * (e - ws.rpre[ol]);
                    const float4 p0 = sg.P0[oq], p1 = sg.P1[oq];
                    const SpanPrep sp{p0.x, p0.y, p0.z, p0.w, p1.x, p1.y, p1.z, p1.w, sg.me[oq]};
                    const int bx = sg.box[oq];
                    int sx0, sx1;
                    row_span(sp, yr + bd.ty0, bx & 0xffff, bx >> 16, sx0, sx1);
                    wd = sx1 - sx0;
                    ws.ex[lane] = sx0 | (yr << 16);
                    ws.eo[lane] = oq;
                }
                int es = wd;
#pragma unroll
                for (int d = 1; d < 64; d <<= 1) {
                    const int y = __shfl_up(es, d, 64);
                    if (lane >= d) es += y;
                }
                ws.epre[lane] = es - wd;
                if (lane == 63) ws.epre[64] = es;
                wave_lds_fence();
                const int K = __shfl(es, 63, 64);
                for (int k0 = 0; k0 < K; k0 += 64) {
                    const int k = k0 + lane;
                    const bool ok = k < K;
                    int tl = 0;
                    uint32_t id = 0u;
                    if (ok) {
                        const int j = wave_search(ws.epre, k);
                        const int ex = ws.ex[j];
                        tl = (ex >> 16) * c.gx + (ex & 0xffff) + (k - ws.epre[j]);
                        id = sg.id[ws.eo[j]];
                    }
                    // lanes of this step on the same tile, ranked by lane (= enumeration) order
                    uint64_t peers = __ballot(ok);
                    for (int b = 0; b < nbits; b++) {
                        const bool bit = (tl >> b) & 1;
                        const uint64_t m = __ballot(bit);
                        peers &= bit ? m : ~m;
                    }
                    if (ok) {
                        const uint32_t old = base[tl];
                        point_list[old + (uint32_t)__popcll(peers & lt)] = id;
                        if ((peers >> lane) == 1ull) base[tl] = old + (uint32_t)__popcll(peers);
                    }
                    wave_lds_fence();
                }
            }
        }
    }
}

hipError_t launch_bin_scatter_ord(const Cam& c, int P, int chunk, int B, const uint8_t* geom, const int32_t* radii,
                                  const uint32_t* order, const uint32_t* table, const uint32_t* tile_start,
                                  uint32_t* point_list, hipStream_t st)
{
    const int rows = bin_scatter_rows(c);
    const int S = (c.gy + rows - 1) / rows;
    const size_t lds = (size_t)rows * c.gx * 4;
    const int km = scatter_merge(P), Bs = (B + km - 1) / km;
    if (B <= 0) return hipSuccess;
    static const bool attr = [] {
        (void)hipFuncSetAttribute((const void*)k_bin_scatter_ord<1024>, hipFuncAttributeMaxDynamicSharedMemorySize, 65536);
        (void)hipFuncSetAttribute((const void*)k_bin_scatter_ord<512>, hipFuncAttributeMaxDynamicSharedMemorySize, 65536);
        return true;
    }();
    (void)attr;
    if (bin_block(P) == 1024) {
        k_bin_scatter_ord<1024><<<Bs * S, 1024, lds, st>>>(c, P, chunk, km, rows, S, geom, radii, order, table,
                                                           tile_start, point_list);
    } else {
        k_bin_scatter_ord<512><<<Bs * S, 512, lds, st>>>(c, P, chunk, km, rows, S, geom, radii, order, table, tile_start,
                                                         point_list);
    }
    return hipGetLastError();
}

}  // namespace lsr
