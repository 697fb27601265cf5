// render.hip — per-pixel alpha blending over the per-tile depth-ordered
// Gaussian lists and its reverse replay (A.4).
//
// Work decomposition (both directions): one 64-thread workgroup = ONE wave
// per 8x8 pixel block, four blocks per 16x16 tile, 4T workgroups.  Waves of
// a tile never synchronise with each other (no __syncthreads anywhere), so a
// wave whose pixels saturate retires immediately instead of idling at a block
// barrier; the four blocks of a tile are placed consecutively inside one
// XCD's dispatch range (WaveTile / xcd_remap) so they share that XCD's L2.
//
// Per chunk of 64 tile instances a wave loads the ids (prefetched one chunk
// ahead), the 32-B splat records and feature rows, tests each against its
// 8x8 block with the per-Gaussian cut ellipse (block_overlap), and compacts
// the survivors in order with __ballot + mbcnt into its private LDS stage.
// The per-pixel blend recurrence (alpha, transmittance, early termination)
// is serial and stays on the VALU, two candidates per step (two independent
// exp chains in flight).  For D > 8 the language channels accumulate on the
// matrix cores (the ML form of k_render_fwd: per 4 candidates the 4 x 64
// weights aT are transposed in registers into the B operand of
// v_mfma_f32_16x16x4_f32, bitwise the sequential fmaf chain); the quick path
// adds its sparse codes into register-resident accumulators.
//
// Backward (k_render_bwd_mf): same mapping, instances replayed back to front
// from the wave's largest n_contrib in groups of 16 candidates: alpha/G per
// candidate (phase 1), the serial transmittance recurrence (phase 2), then
// every per-Gaussian pixel sum as a contraction — language on exact-f32 MFMA
// (v_mfma_f32_16x16x4_f32), colour and the six geometry moments on the VALU —
// added with line-coalesced buffer atomics (see the comment at the kernel).
#include "lsr_internal.h"

#include <type_traits>

#ifndef LSR_BWD_SPLAT_PF
#define LSR_BWD_SPLAT_PF 1  // bwd: chunk records loaded one chunk ahead (ids two ahead), D <= 32
#endif
#ifndef LSR_BWD_LO_RREG
#define LSR_BWD_LO_RREG 1   // language-only bwd: atomics straight from the MFMA accumulators (no LDS row tile)
#endif
#ifndef LSR_BWD16_WAVES
#define LSR_BWD16_WAVES 4  // the headline D = 16 list-driven backward: waves per SIMD it is compiled for
#endif
#ifndef LSR_MF_WAVES
#define LSR_MF_WAVES 2      // MFMA render kernels: min waves per SIMD (caps VGPRs at 256)
#endif
#define LSR_QUICK_KMAX 12   // quick path: (weight, code) pairs per Gaussian staged with the record

namespace lsr {

// ----------------------------------------------------------- reductions --
__device__ __forceinline__ int wave_max_i(int v)
{
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v = max(v, __shfl_xor(v, d, 64));
    return v;
}

__device__ __forceinline__ float wave_max_f(float v)
{
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v = fmaxf(v, __shfl_xor(v, d, 64));
    return v;
}

// ---------------------------------------------------------- forward -------
// Lane -> pixel mapping: wave w of the tile owns the 8x8 block
// (w & 1, w >> 1); lane l owns pixel (l & 7, l >> 3) of it.
struct PixMap {
    int bx, by, px, py;
    __device__ PixMap(const Cam& c, int tile, int t)
    {
        const int tx = tile % c.gx, ty = tile / c.gx;
        const int w = t >> 6, l = t & 63;
        bx = tx * LSR_TILE + (w & 1) * 8;
        by = ty * LSR_TILE + (w >> 1) * 8;
        px = bx + (l & 7);
        py = by + (l >> 3);
    }
};

// Stage one instance's feature row (rgb + dense language) into LDS.
template <int NL, int F4>
__device__ __forceinline__ void stage_features(float4* dst, const float* rgb, const float* lang, int D, uint32_t gid)
{
    float row[F4 * 4];
    row[0] = rgb[3 * gid];
    row[1] = rgb[3 * gid + 1];
    row[2] = rgb[3 * gid + 2];
    if (NL > 0 && D == NL && (NL % 4) == 0) {
        const float4* src = reinterpret_cast<const float4*>(lang + (size_t)gid * NL);
#pragma unroll
        for (int q = 0; q < NL / 4; q++) {
            const float4 v = src[q];
            row[3 + 4 * q] = v.x; row[4 + 4 * q] = v.y; row[5 + 4 * q] = v.z; row[6 + 4 * q] = v.w;
        }
    } else {
#pragma unroll
        for (int k = 0; k < NL; k++) row[3 + k] = (k < D) ? lang[(size_t)gid * D + k] : 0.f;
    }
#pragma unroll
    for (int k = 3 + NL; k < F4 * 4; k++) row[k] = 0.f;
#pragma unroll
    for (int q = 0; q < F4; q++) dst[q] = make_float4(row[4 * q], row[4 * q + 1], row[4 * q + 2], row[4 * q + 3]);
}

// Work-item mapping for the wave-independent render kernels: one 64-thread
// workgroup (one wave) per 8x8 block; the four blocks of a tile get
// consecutive indices inside one XCD's range (xcd_remap), so they share an L2.
//
// Inside its range an XCD walks the tiles in band order (band_tile): bands of
// LSR_BAND tile rows, column by column inside a band.  A Gaussian's tiles are
// then visited close together in time, so the lines its blocks read (records,
// feature rows) and the backward's gradient lines its atomics update are
// still in that XCD's L2 (row-major order revisits them a whole tile row
// later, after ~6 MB of other lines have passed through the 4 MB L2).
#ifndef LSR_BAND
#define LSR_BAND 4          // tile rows per band; 0 = row-major tile order (cfg3 sum 1.487 -> 1.479 ms, cfg5 fwd 1.93 -> 1.88)
#endif
__device__ __forceinline__ int band_tile(int t, int gx, int gy)
{
    if (LSR_BAND <= 0) return t;
    const int per = gx * LSR_BAND;
    const int b = t / per, r = t - b * per;
    const int rows = min(LSR_BAND, gy - b * LSR_BAND);
    const int col = r / rows;
    return (b * LSR_BAND + (r - col * rows)) * gx + col;
}
struct WaveTile {
    int tile, sub;
    // with an order: the block's tile range and list count from the same entry
    // (one load before the wave can start its list DMA and fragment loads)
    uint32_t rs = 0u, re = 0u, lc = 0u;
    bool ent = false;
    // order (the backward's RenderArgs::border): dispatch slot -> block 4 tile + sub
    __device__ WaveTile(const RenderArgs& a, const uint4* order = nullptr)
    {
        const int o = xcd_remap(blockIdx.x, gridDim.x);
        if (order) {
            const uint4 e = order[o];
            tile = (int)(e.x >> 2);
            sub = (int)(e.x & 3u);
            rs = e.y;
            re = e.z;
            lc = e.w;
            ent = true;
        } else {
            tile = band_tile(o >> 2, a.cam.gx, a.cam.gy);
            sub = o & 3;
        }
    }
};

// The list-driven backward's dispatch order.  A backward wave lasts about
// 5-8 us per 16-candidate group of its block list at cfg3, and with the
// blocks in band order the last waves to be dispatched are as heavy as any:
// the launch ended in a ~70 us drain with the machine less and less occupied
// (profiles/r06s_wtl.json: 86 % of the wave slots busy over the launch).
// XCD x's dispatch range (xcd_remap) now holds the blocks with the same
// range of NATURAL indices 4 tile + sub (a horizontal strip of tiles, so a
// tile's four blocks and most of a Gaussian's tiles still share that XCD's
// L2), in descending order of their list length in 16-candidate groups (the
// forward's lcount): the drain is made of the lightest blocks.  One
// workgroup per XCD range, an LDS counting sort, launched right after the
// forward render.  Speed only: every block is still processed exactly once.
// The sort costs L2 reuse (PMC fetch 344 -> 722 MB per launch) and still
// wins: a stable partition that keeps band order for all but the lightest
// quarter (moved to the end) fetched 462 MB and measured 0.457 ms against the
// sort's 0.450 (band order 0.470; profiles/r06za_ab_bwd_partition.txt).
// Keyed by the tile's instance count instead -- known before the render, so
// the sort could run on the colour stream during the binning -- it gained
// nothing: a block's list length does not follow its tile's count.
#define LSR_ORD_NB 64
#ifndef LSR_ORD_THREADS
#define LSR_ORD_THREADS 1024
#endif
#define LSR_ORD_KPT 16   // keys held per thread (ranges up to 16 x LSR_ORD_THREADS blocks in one pass)
__global__ void __launch_bounds__(LSR_ORD_THREADS) k_bwd_order(const uint32_t* __restrict__ lcount,
                                                    const uint32_t* __restrict__ tile_start, int n,
                                                    uint4* __restrict__ border)
{
    __shared__ uint32_t cnt[LSR_ORD_NB];
    const int q = n / 8, r = n % 8, x = blockIdx.x;
    const int lo = x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q;
    const int len = q + (x < r ? 1 : 0);
    const int tid = threadIdx.x;
    if (tid < LSR_ORD_NB) cnt[tid] = 0u;
    __syncthreads();
    auto key = [&](int i) { return min((int)((lcount[lo + i] + 15u) >> 4), LSR_ORD_NB - 1); };
    constexpr int STEP = LSR_ORD_THREADS * LSR_ORD_KPT;
    int kr[LSR_ORD_KPT];
    for (int c = 0; c < len; c += STEP) {
#pragma unroll
        for (int j = 0; j < LSR_ORD_KPT; j++) {
            const int i = c + tid + LSR_ORD_THREADS * j;
            kr[j] = i < len ? key(i) : -1;
        }
#pragma unroll
        for (int j = 0; j < LSR_ORD_KPT; j++)
            if (kr[j] >= 0) atomicAdd(&cnt[kr[j]], 1u);
    }
    __syncthreads();
    if (tid < 64) {   // range offsets, heaviest bucket first: one wave's prefix sum (lane k: bucket 63 - k)
        static_assert(LSR_ORD_NB == 64, "one bucket per lane");
        const uint32_t v = cnt[63 - tid];
        uint32_t incl = v;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t u = __shfl_up(incl, d, 64);
            if (tid >= d) incl += u;
        }
        cnt[63 - tid] = (uint32_t)lo + incl - v;
    }
    __syncthreads();
    for (int c = 0; c < len; c += STEP) {
        if (len > STEP) {   // (one pass holds the whole range otherwise)
#pragma unroll
            for (int j = 0; j < LSR_ORD_KPT; j++) {
                const int i = c + tid + LSR_ORD_THREADS * j;
                kr[j] = i < len ? key(i) : -1;
            }
        }
#pragma unroll
        for (int j = 0; j < LSR_ORD_KPT; j++)
            if (kr[j] >= 0) {
                const uint32_t blk = (uint32_t)(lo + c + tid + LSR_ORD_THREADS * j);
                border[atomicAdd(&cnt[kr[j]], 1u)] =
                    make_uint4(blk, tile_start[blk >> 2], tile_start[(blk >> 2) + 1], lcount[blk]);
            }
    }
}

hipError_t launch_bwd_order(const RenderArgs& a, uint4* border, hipStream_t st)
{
    const int n = 4 * a.cam.gx * a.cam.gy;
    if (n == 0) return hipSuccess;
    k_bwd_order<<<8, LSR_ORD_THREADS, 0, st>>>(a.lcount, a.tile_start, n, border);
    return hipGetLastError();
}


typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// Forward staging with the candidates' geometry pair-interleaved: entry
// j >> 1, component j & 1, so the blend loop reads candidates (2i, 2i+1) of
// each field with one ds_read_b64 and evaluates both exponents with packed
// f32 instructions (bitwise identical to the scalar ones).
#ifndef LSR_FWD_SFEAT
#define LSR_FWD_SFEAT 16    // fwd: from this many language channels up, feature rows are not staged in LDS:
                            // the ML form gathers the candidates' language slices as MFMA operands and
                            // stages only their RGB
#endif
template <int NL>
constexpr bool fwd_sfeat() { return LSR_FWD_SFEAT > 0 && NL >= LSR_FWD_SFEAT; }
// SF (the ML form) holds NE = 68 entries: up to 3 candidates of a partial
// group carried over from the previous chunk + 64 (with their list positions).
template <int F4, bool SF>
struct WaveStageP {
    static constexpr int NE = SF ? 68 : 64;
    f32x2 X[NE / 2], Y[NE / 2], CA[NE / 2], CB[NE / 2], CC[NE / 2], OP[NE / 2];
    float4 F[SF ? 1 : 64 * F4];
    uint32_t gid[SF ? NE : 1];
    float4 R[SF ? NE : 1];   // SF: the candidates' RGB (read by the ML blend as one broadcast line)
    uint32_t pos[SF ? NE : 1];   // SF: the entry's 1-based list position
    uint8_t src[SF ? 1 : 64];    // !SF: the staging lane (position = chunk base + src + 1)
};

// The backward's per-block candidate list (RenderArgs::listA/B): with LST the
// staged candidates are also written to list entries [lpos, lpos + cnt) in
// staging order (increasing tile-list position), B as {conic.c, opacity, id,
// 0-based position}; *mo receives the chunk's staging mask.
struct ListSink {
    float4* A = nullptr;
    float4* B = nullptr;
    uint32_t pos = 0;
};

template <int NL, int F4, bool LST = false>
__device__ __forceinline__ int stage_candidates_p_rec(WaveStageP<F4, fwd_sfeat<NL>()>& st, bool valid, uint32_t gid,
                                                      int pos, int bx, int by, float4 A, float4 B,
                                                      const float* __restrict__ rgb, const float* __restrict__ lang,
                                                      int D, const ListSink& ls = ListSink(), uint64_t* mo = nullptr,
                                                      int off = 0)
{
    constexpr bool SF = fwd_sfeat<NL>();
    constexpr int NE = WaveStageP<F4, SF>::NE;
    const bool ok = valid && block_overlap(A.x, A.y, __float_as_uint(B.w), bx, by) &&
                    block_overlap_exact(A.x, A.y, A.z, A.w, B.x, B.z, bx, by);
    const uint64_t m = wave_ballot(ok);
    const int cnt = __popcll(m);
    if constexpr (LST) *mo = m;
    if (ok) {
        const int r = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
        if constexpr (LST) {
            if (ls.A) {
                ls.A[ls.pos + r] = A;
                ls.B[ls.pos + r] = make_float4(B.x, B.y, __uint_as_float(gid), __int_as_float(pos - 1));
            }
        }
        // entry i = off + r (SF: after the carried entries)
        const int i = off + r;
        float* base = reinterpret_cast<float*>(&st) + (i & 1);
        const int e = (i >> 1) * 2;
        base[0 * NE + e] = A.x;
        base[1 * NE + e] = A.y;
        base[2 * NE + e] = A.z;
        base[3 * NE + e] = A.w;
        base[4 * NE + e] = B.x;
        base[5 * NE + e] = B.y;
        if constexpr (SF) {
            st.pos[i] = (uint32_t)pos;
            st.gid[i] = gid;
            st.R[i] = make_float4(rgb[3 * (size_t)gid], rgb[3 * (size_t)gid + 1], rgb[3 * (size_t)gid + 2], 0.f);
        } else {
            st.src[r] = (uint8_t)(threadIdx.x & 63);
        }
        if constexpr (!SF)
            stage_features<NL, F4>(&st.F[r * F4], rgb, lang, D, gid);
    }
    wave_lds_fence();
    return cnt;
}

template <int NL, int F4, bool LST = false>
__device__ __forceinline__ int stage_candidates_p(WaveStageP<F4, fwd_sfeat<NL>()>& st, bool valid, uint32_t gid, int pos, int bx,
                                                  int by, const float4* __restrict__ splatA,
                                                  const float4* __restrict__ splatB, const float* __restrict__ rgb,
                                                  const float* __restrict__ lang, int D, const ListSink& ls = ListSink(),
                                                  uint64_t* mo = nullptr, int off = 0)
{
    float4 A = make_float4(0.f, 0.f, 0.f, 0.f), B = A;
    if (valid) {
        A = splatA[gid];
        B = splatB[gid];
    }
    return stage_candidates_p_rec<NL, F4, LST>(st, valid, gid, pos, bx, by, A, B, rgb, lang, D, ls, mo, off);
}

// The backward's accumulators (RenderArgs::zero; lsr_fwd_out.grad_ws): a
// grid-strided share per wave, non-temporal 16-B stores, issued first so no
// early exit skips them.  The render is VALU / LDS bound; these writes replace
// the backward's two memset launches.
__device__ __forceinline__ void zero_backward_accumulators(const RenderArgs& a)
{
    typedef float v4f __attribute__((ext_vector_type(4)));
    const size_t stride = (size_t)gridDim.x * 64;
    if (a.zero) {
        v4f* const z = reinterpret_cast<v4f*>(a.zero);
        for (size_t i = (size_t)blockIdx.x * 64 + threadIdx.x; i < a.zero_n16; i += stride)
            __builtin_nontemporal_store(v4f{0.f, 0.f, 0.f, 0.f}, z + i);
    }
    if (a.zero2) {
        v4f* const z = reinterpret_cast<v4f*>(a.zero2);
        for (size_t i = (size_t)blockIdx.x * 64 + threadIdx.x; i < a.zero2_n16; i += stride)
            __builtin_nontemporal_store(v4f{0.f, 0.f, 0.f, 0.f}, z + i);
    }
}

// ZERO: this launch also clears the backward's accumulators (a.zero set);
// a separate instantiation, so a forward without a pending backward runs the
// unchanged kernel (the clearing loop alone moved cfg5's D = 32 render by +2 %)
// ML (D > 16): the language channels accumulate on the matrix
// cores instead of the VALU.  Per 4 staged candidates the blend (alpha, the
// serial transmittance / termination recurrence, the RGB sums) runs per pixel
// lane as below; the 4 x 64 weights aT are transposed in registers (two
// permlane swaps per pair of rows: lane group <-> candidate) into the B
// operand of v_mfma_f32_16x16x4_f32, whose A operand is each 16-channel
// block of the 4 candidates' language rows (gathered per lane; their RGB is
// staged in LDS with the candidate).  The MFMA is bitwise a fmaf chain over
// its 4 K terms in order (tools/micro/mfma_order.hip) and a skipped pair has
// aT = 0, so the outputs are bit-identical to the per-lane sequential blend;
// the VALU no longer issues the 2 x D language FMAs per candidate pair, which
// run on the otherwise idle matrix pipe.  (The LDS-staged-row form, D = 16,
// measured slower than the VALU blend and is not launched.)
// MLM (with ML): D below the language set's width NL (masked channels);
// otherwise D == NL is a compile-time constant (fewer registers).
// the D = 16 ML form at 6 waves / SIMD (80 VGPRs): its blend is latency bound
template <int NL, bool ML>
constexpr int fwd_waves() { return (ML && NL == 16) ? 6 : 1; }
template <int NL, bool ZERO = false, bool ML = false, bool MLM = false>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(fwd_waves<NL, ML>()))) k_render_fwd(RenderArgs a)
{
    if constexpr (ZERO) zero_backward_accumulators(a);
    constexpr int C = 3 + NL;
    constexpr int F4 = (C + 3) / 4;  // float4 per feature row
    constexpr bool SF = fwd_sfeat<NL>();
    static_assert(!ML || NL == 16 || NL == 32 || NL == 64, "ML: whole 16-channel language blocks");
    static_assert(ML || !SF, "scalar feature rows (D >= LSR_FWD_SFEAT) feed the ML form only");
    // the ML form's carried partial groups and `last` are kept in the SF stage
    // (st.pos / st.gid / st.R); a build with ML but LDS-staged rows would drop them
    static_assert(!ML || SF, "the ML carry logic needs the SF stage (LSR_FWD_SFEAT <= 16)");
    constexpr int MLB = ML ? NL / 16 : 1;   // ML: 16-channel output blocks
    __shared__ WaveStageP<F4, SF> st;

    const Cam& c = a.cam;
    const WaveTile wt(a);
    const int lane = threadIdx.x;
    const PixMap pm(c, wt.tile, lane + (wt.sub << 6));
    const bool inside = pm.px < c.W && pm.py < c.H;
    const float pfx = (float)pm.px, pfy = (float)pm.py;
    const uint32_t rs = a.tile_start[wt.tile], re = a.tile_start[wt.tile + 1];
    const int D = (ML && !MLM) ? NL : a.D;

    float T = 1.0f;
    bool done = !inside;
    float acc[F4 * 4];
#pragma unroll
    for (int k = 0; k < F4 * 4; k++) acc[k] = 0.f;
    f32x4 mlacc[MLB][4];   // ML: lane (li, lg) holds language channels 16 nb + 4 lg + r of block pixel 16 pb + li
#pragma unroll
    for (int nb = 0; nb < MLB; nb++)
#pragma unroll
        for (int pb = 0; pb < 4; pb++) mlacc[nb][pb] = f32x4{0.f, 0.f, 0.f, 0.f};
    uint32_t last = 0;

    // ZERO (a backward is pending): the staged candidates also go to this
    // block's list for the backward (RenderArgs::listA), nst entries so far;
    // (mlast, nlast, blast): the last chunk's mask, entries before it, its start
    ListSink ls;
    uint32_t nst = 0, nlast = 0, blast = rs;
    uint64_t mlast = 0;
    if constexpr (ZERO) {
        if (a.listA) {
            ls.A = a.listA + (size_t)4 * rs + (size_t)wt.sub * (re - rs);
            ls.B = a.listB + (size_t)4 * rs + (size_t)wt.sub * (re - rs);
        }
    }
    uint32_t next_gid = (rs + lane < re) ? a.point_list[rs + lane] : 0u;
    // SPF: a chunk's ids are loaded two chunks ahead and its records one chunk
    // ahead, issued after the current chunk's feature loads: the staging then
    // waits for one dependent gather (the feature rows) instead of two.
    // Positions past the list read gid 0 (a valid record, never staged).
    // (not with scalar feature rows, D >= LSR_FWD_SFEAT: cfg5 1.73 -> 1.82 ms)
    constexpr bool FSPF = !SF;
    uint32_t next_gid2 = 0u;
    float4 A1 = make_float4(0.f, 0.f, 0.f, 0.f), B1 = A1;
    if (FSPF && rs < re) {
        next_gid2 = (rs + 64 + lane < re) ? a.point_list[rs + 64 + lane] : 0u;
        A1 = a.splatA[next_gid];
        B1 = a.splatB[next_gid];
    }
    // ML: a partial group (carry < 4 entries) waits in the stage for the next
    // chunk's candidates, so every group but the list's last is full: the
    // blend's per-group work is paid per 4 candidates, not per chunk remainder.
    // The blend is per candidate in list order either way (bit-identical).
    int carry = 0;
    for (uint32_t base = rs; base < re; base += 64) {
        if (wave_ballot(!done) == 0) break;
        const uint32_t idx = base + lane;
        const bool valid = idx < re;
        const uint32_t gid = next_gid;
        int n;
        uint64_t mchunk = 0;
        ls.pos = nst;
        if constexpr (FSPF) {
            const float4 Ac = A1, Bc = B1;
            n = stage_candidates_p_rec<NL, F4, ZERO>(st, valid, gid, (int)(idx - rs) + 1, pm.bx, pm.by, Ac, Bc, a.rgb,
                                                     a.lang, D, ls, &mchunk, ML ? carry : 0);
            next_gid = next_gid2;
            A1 = a.splatA[next_gid];
            B1 = a.splatB[next_gid];
            const uint32_t q = min(idx + 128, re - 1);   // re > base: a valid position
            const uint32_t v = a.point_list[q];
            next_gid2 = idx + 128 < re ? v : 0u;
        } else {
            next_gid = (idx + 64 < re) ? a.point_list[idx + 64] : 0u;
            n = stage_candidates_p<NL, F4, ZERO>(st, valid, gid, (int)(idx - rs) + 1, pm.bx, pm.by, a.splatA,
                                                 a.splatB, a.rgb, a.lang, D, ls, &mchunk, ML ? carry : 0);
        }
        if constexpr (ZERO) {
            mlast = mchunk;
            nlast = nst;
            blast = base;
            nst += (uint32_t)n;
        }
        // Two instances per iteration, branch-free per lane: a lane that
        // skips an instance (exponent cut, alpha < 1/255, saturated or done)
        // blends it with weight 0 and keeps T.  The two exp chains are
        // independent (ILP); T carries from the first to the second exactly
        // as in the sequential per-pixel order.
        int lastj = -1;   // LASTJ: staged index of the chunk's last contributor
        if constexpr (ML) {
            const int lg = lane >> 4, li = lane & 15;
            const float* const Fs = reinterpret_cast<const float*>(st.F);
            n += carry;   // the stage's entries: carried + this chunk's
            // full groups only, except in the list's last chunk
            const int nproc = (base + 64 >= re) ? n : (n & ~3);
            int q0 = 0;
            for (; q0 < nproc; q0 += 4) {
                if (wave_ballot(!done) == 0) break;
                // A operand: language channel 16 nb + li of candidate q0 + lg
                // (0 past the chunk) -- from the staged rows, or (SF) gathered
                float av[MLB];
#pragma unroll
                for (int nb = 0; nb < MLB; nb++) {
                    // MLM: channels past D (a language set wider than D) read 0
                    const int ch = 16 * nb + li;
                    float fa;
                    if constexpr (SF)
                        fa = a.lang[(size_t)st.gid[min(q0 + lg, n - 1)] * D + (MLM ? min(ch, D - 1) : ch)];
                    else
                        fa = Fs[(q0 + lg) * (F4 * 4) + 3 + ch];
                    av[nb] = ((q0 + lg < n) & (!MLM || ch < D)) ? fa : 0.f;
                }
                // al[k]: the pair's alpha where it is blended (the lane not done,
                // exponent <= 0, alpha >= 1/255), else 0; cm[k] the lanes of al != 0
                float al[4];
                bool cm[4];
#pragma unroll
                for (int h = 0; h < 2; h++) {
                    const int j0 = q0 + 2 * h, e = j0 >> 1;
                    const f32x2 sX = st.X[e], sY = st.Y[e], sCA = st.CA[e], sCB = st.CB[e], sCC = st.CC[e];
                    const f32x2 OP = st.OP[e];
                    const f32x2 dx = sX - f32x2{pfx, pfx}, dy = sY - f32x2{pfy, pfy};
                    const f32x2 P = __builtin_elementwise_fma(f32x2{-0.5f, -0.5f},
                                                              __builtin_elementwise_fma(sCA * dx, dx, (sCC * dy) * dy),
                                                              -((sCB * dx) * dy));
                    const f32x2 EX = expf_det2(P);
                    const float a0 = fminf(0.99f, OP.x * EX.x), a1 = fminf(0.99f, OP.y * EX.y);
                    // no exponent-cut test: below the cut the 1/255 test rejects the pair
                    const bool c0 = (j0 < n) & !done & !(P.x > 0.0f) & !(a0 < 1.0f / 255.0f);
                    const bool c1 = (j0 + 1 < n) & !done & !(P.y > 0.0f) & !(a1 < 1.0f / 255.0f);
                    al[2 * h] = c0 ? a0 : 0.f;
                    al[2 * h + 1] = c1 ? a1 : 0.f;
                    cm[2 * h] = c0;
                    cm[2 * h + 1] = c1;
                }
                // the serial recurrence.  T never increases, so if no lane's
                // transmittance after the 4 candidates (computed as if none
                // terminated) is below 1e-4, none terminated: then a lane with
                // al = 0 gets aT = 0 and T unchanged with no selects and no
                // termination tests.  Otherwise (rare) the group runs the legacy
                // ok0 / term / ok logic.  Bitwise the legacy result either way.
                float s4[4];
                // candidate k's rgb (past the chunk a staged row's: aT = 0 there)
                auto rgb_of = [&](int k) -> float3 {
                    const int kk = min(q0 + k, n - 1);
                    if constexpr (SF) {   // the line staged with the candidate
                        const float4 f = st.R[kk];
                        return make_float3(f.x, f.y, f.z);
                    } else {
                        const float4 f = st.F[kk * F4];
                        return make_float3(f.x, f.y, f.z);
                    }
                };
                // transmittance before each candidate, assuming no termination
                float Tk[5];
                Tk[0] = T;
#pragma unroll
                for (int k = 0; k < 4; k++) Tk[k + 1] = Tk[k] * (1.0f - al[k]);
                if (wave_ballot(Tk[4] < 0.0001f) == 0u) {
#pragma unroll
                    for (int k = 0; k < 4; k++) {
                        const float aT = al[k] * Tk[k];
                        const float3 f = rgb_of(k);
                        acc[0] = fmaf(f.x, aT, acc[0]);
                        acc[1] = fmaf(f.y, aT, acc[1]);
                        acc[2] = fmaf(f.z, aT, acc[2]);
                        lastj = cm[k] ? q0 + k : lastj;
                        s4[k] = aT;
                    }
                    T = Tk[4];
                } else {
#pragma unroll
                    for (int k = 0; k < 4; k++) {
                        const float alk = al[k];
                        const float test_T = T * (1.0f - alk);
                        const bool ok0 = (alk != 0.f) & !done;
                        const bool term = ok0 & (test_T < 0.0001f);
                        done = done | term;
                        const bool ok = ok0 & !term;
                        const float aT = ok ? alk * T : 0.f;
                        const float3 f = rgb_of(k);
                        acc[0] = fmaf(f.x, aT, acc[0]);
                        acc[1] = fmaf(f.y, aT, acc[1]);
                        acc[2] = fmaf(f.z, aT, acc[2]);
                        T = ok ? test_T : T;
                        lastj = ok ? q0 + k : lastj;
                        s4[k] = aT;
                    }
                }
                // transpose (lane group, candidate): lane (li, lg) then holds
                // candidate lg's aT at block pixel 16 pb + li in s4[pb]
                {
                    auto sw32 = [](float& x, float& y) {
                        const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(y), false, false);
                        x = __uint_as_float(r[0]);
                        y = __uint_as_float(r[1]);
                    };
                    auto sw16 = [](float& x, float& y) {
                        const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(y), false, false);
                        x = __uint_as_float(r[0]);
                        y = __uint_as_float(r[1]);
                    };
                    sw32(s4[0], s4[2]);
                    sw32(s4[1], s4[3]);
                    sw16(s4[0], s4[1]);
                    sw16(s4[2], s4[3]);
                }
#pragma unroll
                for (int pb = 0; pb < 4; pb++)
#pragma unroll
                    for (int nb = 0; nb < MLB; nb++)
                        mlacc[nb][pb] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[nb], s4[pb], mlacc[nb][pb], 0, 0, 0);
            }
            if constexpr (SF) {
                if (lastj >= 0) last = st.pos[lastj];
                lastj = -1;
                // the partial group's entries [q0, n) -> [0, carry) (q0 >= 4 when
                // they move: no overlap; a wave's LDS accesses complete in order)
                carry = n - q0;
                if (q0 > 0 && carry > 0) {
                    if (lane < carry) {
                        const int i = q0 + lane;
                        float* fb = reinterpret_cast<float*>(&st);
                        constexpr int NE = WaveStageP<F4, SF>::NE;
                        float v[6];
#pragma unroll
                        for (int f = 0; f < 6; f++) v[f] = fb[f * NE + i];
                        const uint32_t pv = st.pos[i], gv = st.gid[i];
                        const float4 rv = st.R[i];
#pragma unroll
                        for (int f = 0; f < 6; f++) fb[f * NE + lane] = v[f];
                        st.pos[lane] = pv;
                        st.gid[lane] = gv;
                        st.R[lane] = rv;
                    }
                }
            }
        } else
        for (int j0 = 0; j0 < n; j0 += 2) {
            if (wave_ballot(!done) == 0) break;
            const bool two = j0 + 1 < n;
            const int j1 = two ? j0 + 1 : j0;
            // both candidates' exponents at once (splat_power, lane-wise);
            // a missing second candidate reads a stale slot: ok1 masks it
            const int e = j0 >> 1;
            const f32x2 sX = st.X[e], sY = st.Y[e], sCA = st.CA[e], sCB = st.CB[e], sCC = st.CC[e];
            const f32x2 OP = st.OP[e];
            const f32x2 dx = sX - f32x2{pfx, pfx}, dy = sY - f32x2{pfy, pfy};
            const f32x2 P = __builtin_elementwise_fma(f32x2{-0.5f, -0.5f},
                                                      __builtin_elementwise_fma(sCA * dx, dx, (sCC * dy) * dy),
                                                      -((sCB * dx) * dy));
            const float p0 = P.x, p1 = P.y;
            // no exponent-cut test: below the cut alpha < e^-0.02 / 255, so the
            // 1/255 test below rejects the pair anyway (exact)
            bool ok0 = !done && !(p0 > 0.0f);
            bool ok1 = two && !done && !(p1 > 0.0f);
            const f32x2 EX = expf_det2(P);   // both exponents packed (bitwise = expf_det)
            const float al0 = fminf(0.99f, OP.x * EX.x);
            const float al1 = fminf(0.99f, OP.y * EX.y);
            ok0 = ok0 && !(al0 < 1.0f / 255.0f);
            ok1 = ok1 && !(al1 < 1.0f / 255.0f);
            {
                const float test_T = T * (1.0f - al0);
                const bool term = ok0 && (test_T < 0.0001f);
                done = done || term;
                ok0 = ok0 && !term;
                ok1 = ok1 && !term;
                const float aT = ok0 ? al0 * T : 0.f;
                {
#pragma unroll
                    for (int f = 0; f < F4; f++) {
                        const float4 v = st.F[j0 * F4 + f];
                        // the row's zero padding past channel C is not accumulated
                        if (4 * f + 0 < C) acc[4 * f + 0] = fmaf(v.x, aT, acc[4 * f + 0]);
                        if (4 * f + 1 < C) acc[4 * f + 1] = fmaf(v.y, aT, acc[4 * f + 1]);
                        if (4 * f + 2 < C) acc[4 * f + 2] = fmaf(v.z, aT, acc[4 * f + 2]);
                        if (4 * f + 3 < C) acc[4 * f + 3] = fmaf(v.w, aT, acc[4 * f + 3]);
                        // keep the 16-B read (ds_read_b128: 4 LDS cycles; the b96 the
                        // compiler would narrow it to costs 8)
                        else asm volatile("" ::"v"(v.w));
                    }
                }
                T = ok0 ? test_T : T;
                lastj = ok0 ? j0 : lastj;
            }
            {
                const float test_T = T * (1.0f - al1);
                const bool term = ok1 && (test_T < 0.0001f);
                done = done || term;
                ok1 = ok1 && !term;
                const float aT = ok1 ? al1 * T : 0.f;
                {
#pragma unroll
                    for (int f = 0; f < F4; f++) {
                        const float4 v = st.F[j1 * F4 + f];
                        // the row's zero padding past channel C is not accumulated
                        if (4 * f + 0 < C) acc[4 * f + 0] = fmaf(v.x, aT, acc[4 * f + 0]);
                        if (4 * f + 1 < C) acc[4 * f + 1] = fmaf(v.y, aT, acc[4 * f + 1]);
                        if (4 * f + 2 < C) acc[4 * f + 2] = fmaf(v.z, aT, acc[4 * f + 2]);
                        if (4 * f + 3 < C) acc[4 * f + 3] = fmaf(v.w, aT, acc[4 * f + 3]);
                        // keep the 16-B read (ds_read_b128: 4 LDS cycles; the b96 the
                        // compiler would narrow it to costs 8)
                        else asm volatile("" ::"v"(v.w));
                    }
                }
                T = ok1 ? test_T : T;
                lastj = ok1 ? j1 : lastj;
            }
        }
        if constexpr (!ML) {
            if (lastj >= 0) last = (uint32_t)(base - rs) + 1u + st.src[lastj];
        }
        wave_lds_fence();
    }
    if constexpr (ZERO) {
        if (a.listA) {
            // entries the backward needs: 0-based position < wmax (the block's largest
            // n_contrib).  Exact when wmax falls in the last staged chunk (the usual
            // case); otherwise every entry before that chunk (the extra ones have
            // position >= every pixel's n_contrib: the backward evaluates them to 0)
            const int wmax = wave_max_i(inside ? (int)last : 0);
            const int off = wmax - (int)(blast - rs);
            uint32_t cnt = nlast;
            if (off > 0) cnt += (uint32_t)__popcll(off >= 64 ? mlast : (mlast & ((1ull << off) - 1ull)));
            if (lane == 0) a.lcount[4 * wt.tile + wt.sub] = cnt;
        }
    }
    if (inside) {
        const size_t HW = (size_t)c.H * c.W;
        const size_t pix = (size_t)pm.py * c.W + pm.px;
        a.final_T[pix] = T;
        a.n_contrib[pix] = last;
#pragma unroll
        for (int ch = 0; ch < 3; ch++) a.out_color[ch * HW + pix] = fmaf(T, c.bg[ch], acc[ch]);
        if constexpr (!ML) {
#pragma unroll
            for (int k = 0; k < NL; k++)
                if (k < D) a.out_lang[k * HW + pix] = acc[3 + k];
        }
    }
    if constexpr (ML) {
        const size_t HW = (size_t)c.H * c.W;
        const int lg = lane >> 4, li = lane & 15;
#pragma unroll
        for (int pb = 0; pb < 4; pb++) {
            const int q = pb * 16 + li;
            const int qx = pm.bx + (q & 7), qy = pm.by + (q >> 3);
            if (qx < c.W && qy < c.H) {
                const size_t pix = (size_t)qy * c.W + qx;
#pragma unroll
                for (int nb = 0; nb < MLB; nb++)
#pragma unroll
                    for (int r = 0; r < 4; r++)
                        if (16 * nb + 4 * lg + r < D) a.out_lang[(size_t)(16 * nb + 4 * lg + r) * HW + pix] = mlacc[nb][pb][r];
            }
        }
    }
}

// Sparse "quick" language path: Dq output channels, K (weight, index) pairs
// per Gaussian.  One wave per 8x8 pixel block; per-pixel accumulators in LDS
// laid out [channel][lane] (conflict-free: the channel index is wave-uniform
// because every lane processes the same Gaussian).
__global__ void __launch_bounds__(64) k_render_fwd_quick(RenderArgs a)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int K = a.K, Dq = a.Dq;
    float* acc = (float*)smem;                                    // Dq * 64
    float4* sA = (float4*)(smem + (size_t)Dq * 64 * 4);           // 64
    float4* sB = sA + 64;                                         // 64
    float* sRGB = (float*)(sB + 64);                              // 64 * 3
    float* sW = sRGB + 64 * 3;                                    // 64 * K
    int* sI = (int*)(sW + 64 * K);                                // 64 * K

    const Cam& c = a.cam;
    const int tile = band_tile(xcd_remap(blockIdx.x >> 2, gridDim.x >> 2), c.gx, c.gy);
    const int t = threadIdx.x;
    const PixMap pm(c, tile, t + ((blockIdx.x & 3) << 6));
    const bool inside = pm.px < c.W && pm.py < c.H;
    const float pfx = (float)pm.px, pfy = (float)pm.py;
    const uint32_t rs = a.tile_start[tile], re = a.tile_start[tile + 1];
    for (int q = 0; q < Dq; q++) acc[q * 64 + t] = 0.f;

    float T = 1.0f, cr = 0.f, cg = 0.f, cb = 0.f;
    uint32_t last = 0;
    bool done = !inside;
    for (uint32_t base = rs; base < re; base += 64) {
        if (__syncthreads_count(done) == 64) break;
        const uint32_t idx = base + t;
        if (idx < re) {
            const uint32_t gid = a.point_list[idx];
            sA[t] = a.splatA[gid];
            sB[t] = a.splatB[gid];
            sRGB[3 * t] = a.rgb[3 * gid];
            sRGB[3 * t + 1] = a.rgb[3 * gid + 1];
            sRGB[3 * t + 2] = a.rgb[3 * gid + 2];
            for (int k = 0; k < K; k++) {
                sW[t * K + k] = a.qw[(size_t)gid * K + k];
                const int q = quick_index(a.qi, a.qidx_dtype, (size_t)gid * K + k);
                sI[t * K + k] = (q >= 0 && q < Dq) ? q : -1;
            }
        }
        __syncthreads();
        const int n = (int)min(64u, re - base);
        const uint32_t pos0 = base - rs + 1;
        bool ok = false;
        if (t < n) ok = block_overlap(sA[t].x, sA[t].y, __float_as_uint(sB[t].w), pm.bx, pm.by);
        uint64_t bits = wave_ballot(ok);
        while (bits) {
            if (wave_ballot(!done) == 0) break;
            const int j = __builtin_ctzll(bits);
            bits &= bits - 1;
            if (done) continue;
            const float4 A = sA[j];
            const float4 B = sB[j];
            const float dx = A.x - pfx, dy = A.y - pfy;
            const float power = splat_power(A.z, A.w, B.x, dx, dy);
            if (power > 0.0f || power < B.z) continue;
            const float G = expf_det(power);
            const float alpha = fminf(0.99f, B.y * G);
            if (alpha < 1.0f / 255.0f) continue;
            const float test_T = T * (1.0f - alpha);
            if (test_T < 0.0001f) {
                done = true;
                continue;
            }
            const float aT = alpha * T;
            cr = fmaf(sRGB[3 * j], aT, cr);
            cg = fmaf(sRGB[3 * j + 1], aT, cg);
            cb = fmaf(sRGB[3 * j + 2], aT, cb);
            for (int k = 0; k < K; k++) {
                const int q = sI[j * K + k];
                if (q >= 0) acc[q * 64 + t] = fmaf(sW[j * K + k], aT, acc[q * 64 + t]);
            }
            T = test_T;
            last = pos0 + j;
        }
    }
    if (inside) {
        const size_t HW = (size_t)c.H * c.W;
        const size_t pix = (size_t)pm.py * c.W + pm.px;
        a.final_T[pix] = T;
        a.n_contrib[pix] = last;
        a.out_color[pix] = fmaf(T, c.bg[0], cr);
        a.out_color[HW + pix] = fmaf(T, c.bg[1], cg);
        a.out_color[2 * HW + pix] = fmaf(T, c.bg[2], cb);
        for (int q = 0; q < Dq; q++) a.out_lang[q * HW + pix] = acc[q * 64 + t];
    }
}

// Quick path, sparse accumulation in registers (default for Dq <= 192, K <= 12).
// The dense-slab kernels above scatter each group's (weight, code) pairs into a
// 16 x Dq tile and accumulate it on MFMA: 16x the arithmetic the 12 non-zero
// codes need, plus barriers between the blend wave and the slab waves.  Here
// one wave per 8x8 block keeps each pixel's Dq accumulators in VGPRs (NP
// vectors of 32) and, per contributing candidate, adds only its K pairs:
// the code is wave-uniform, so acc[code] is a register indexed by M0 (movrel)
// and each pair costs one FMA plus two register moves.  Same per-pixel
// recurrence, same fmaf(w, alpha T, acc) in candidate order as the oracle:
// bit-exact.  Staged per candidate in LDS: the splat record, rgb, the K
// weights and the codes as bytes (0xFF = outside [0, Dq)).
typedef float lsr_f32x32 __attribute__((ext_vector_type(32)));
struct WaveStageV {
    float4 A[64];
    float4 B[64];          // .w = 1-based tile-list position (int bits)
    float4 C[64];          // rgb
    float4 Wt[64][3];      // weights 0..11
    uint4 Q[64];           // codes 0..11 as bytes
};

// The Dq <= 192 accumulators live in v64..v255, outside the compiler's
// allocation (amdgpu_num_vgpr(63): compiled code uses v0..v62; an asm clobber
// of v255 makes the kernel descriptor allocate all 256).  A candidate's K <= 12
// updates run in one asm block in VGPR index mode with SRC2 and DST indexed
// from v63: code q is stored as index q + 1, so v_fma_f32 v63, w, aT, v63
// updates v[64 + q] in one VALU instruction, and an invalid code (index 0)
// lands in the junk register v63.  M0 (the index) is saved and restored.
// (s_set_gpr_idx_idx reads only bits [7:0], so byte k of a code word is
// selected by a shift.)
// The index needs one wait state before the VALU that uses it: the shift
// forming the NEXT code's index (into the other of two SGPRs) fills it, so only
// the word's last code takes an s_nop (3 per candidate instead of 12).
#define LSR_QV_WORD(word, w0, w1, w2, w3)                                               \
    "s_set_gpr_idx_idx %[" #word "]\n\t"                                                \
    "s_lshr_b32 %[ia], %[" #word "], 8\n\t"                                             \
    "v_fma_f32 v63, %[" #w0 "], %[aT], v63\n\t"                                         \
    "s_set_gpr_idx_idx %[ia]\n\t"                                                       \
    "s_lshr_b32 %[ib], %[" #word "], 16\n\t"                                            \
    "v_fma_f32 v63, %[" #w1 "], %[aT], v63\n\t"                                         \
    "s_set_gpr_idx_idx %[ib]\n\t"                                                       \
    "s_lshr_b32 %[ia], %[" #word "], 24\n\t"                                            \
    "v_fma_f32 v63, %[" #w2 "], %[aT], v63\n\t"                                         \
    "s_set_gpr_idx_idx %[ia]\n\t"                                                       \
    "s_nop 0\n\t"                                                                       \
    "v_fma_f32 v63, %[" #w3 "], %[aT], v63\n\t"
// one candidate's K <= 12 pairs (codes in three words q0..q2, weights w0..w11)
#define LSR_QV_UPDATE(aT_, Q_, W0_, W1_, W2_)                                                                   \
    do {                                                                                                        \
        const uint32_t qw0 = __builtin_amdgcn_readfirstlane((Q_).x), qw1 = __builtin_amdgcn_readfirstlane((Q_).y), \
                       qw2 = __builtin_amdgcn_readfirstlane((Q_).z);                                            \
        uint32_t ia, ib, sv;                                                                                    \
        asm volatile("s_mov_b32 %[sv], m0\n\t"                                                                  \
                     "s_set_gpr_idx_on 0, gpr_idx(SRC2,DST)\n\t"                                                \
                     LSR_QV_WORD(q0, w0, w1, w2, w3) LSR_QV_WORD(q1, w4, w5, w6, w7)                            \
                     LSR_QV_WORD(q2, w8, w9, w10, w11)                                                          \
                     "s_set_gpr_idx_off\n\t"                                                                    \
                     "s_mov_b32 m0, %[sv]"                                                                      \
                     : [ia] "=&s"(ia), [ib] "=&s"(ib), [sv] "=&s"(sv)                                           \
                     : [q0] "s"(qw0), [q1] "s"(qw1), [q2] "s"(qw2), [aT] "v"(aT_), [w0] "v"((W0_).x),           \
                       [w1] "v"((W0_).y), [w2] "v"((W0_).z), [w3] "v"((W0_).w), [w4] "v"((W1_).x),              \
                       [w5] "v"((W1_).y), [w6] "v"((W1_).z), [w7] "v"((W1_).w), [w8] "v"((W2_).x),              \
                       [w9] "v"((W2_).y), [w10] "v"((W2_).z), [w11] "v"((W2_).w)                                \
                     : "scc");                                                                                  \
    } while (0)

#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"   // the v255 clobber is the point: it sizes the allocation
template <int NP>
__global__ void __launch_bounds__(64, 2) __attribute__((amdgpu_num_vgpr(63))) k_render_fwd_quick_v(RenderArgs a)
{
    static_assert(NP >= 1 && NP <= 6, "up to 192 quick channels");
    __shared__ WaveStageV st;
    const Cam& c = a.cam;
    const WaveTile wt(a);
    const int lane = threadIdx.x;
    const PixMap pm(c, wt.tile, lane + (wt.sub << 6));
    const bool inside = pm.px < c.W && pm.py < c.H;
    const float pfx = (float)pm.px, pfy = (float)pm.py;
    const uint32_t rs = a.tile_start[wt.tile], re = a.tile_start[wt.tile + 1];
    const int K = a.K, Dq = a.Dq;

    {   // zero v63 (junk) .. v255 (accumulators)
        uint32_t i, sv;
        asm volatile(
            "s_mov_b32 %[sv], m0\n\t"
            "s_mov_b32 %[i], 0\n\t"
            "s_set_gpr_idx_on 0, gpr_idx(DST)\n\t"
            "1:\n\t"
            "s_set_gpr_idx_idx %[i]\n\t"
            "s_nop 0\n\t"
            "v_mov_b32 v63, 0\n\t"
            "s_add_u32 %[i], %[i], 1\n\t"
            "s_cmp_lt_u32 %[i], 193\n\t"
            "s_cbranch_scc1 1b\n\t"
            "s_set_gpr_idx_off\n\t"
            "s_mov_b32 m0, %[sv]"
            : [i] "=&s"(i), [sv] "=&s"(sv)
            :
            : "scc", "v63", "v255", "memory");
    }
    float T = 1.0f, cr = 0.f, cg = 0.f, cbl = 0.f;
    uint32_t last = 0;
    bool done = !inside;
    uint32_t next_gid = (rs + lane < re) ? a.point_list[rs + lane] : 0u;
    for (uint32_t base = rs; base < re; base += 64) {
        if (wave_ballot(!done) == 0) break;
        const uint32_t idx = base + lane;
        const bool valid = idx < re;
        const uint32_t gid = next_gid;
        next_gid = (idx + 64 < re) ? a.point_list[idx + 64] : 0u;
        float4 A = make_float4(0.f, 0.f, 0.f, 0.f), B = A;
        if (valid) {
            A = a.splatA[gid];
            B = a.splatB[gid];
        }
        const bool ok = valid && block_overlap(A.x, A.y, __float_as_uint(B.w), pm.bx, pm.by) &&
                        block_overlap_exact(A.x, A.y, A.z, A.w, B.x, B.z, pm.bx, pm.by);
        const uint64_t m = wave_ballot(ok);
        if (ok) {
            const int r = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
            st.A[r] = A;
            st.B[r] = make_float4(B.x, B.y, B.z, __int_as_float((int)(idx - rs) + 1));
            st.C[r] = make_float4(a.rgb[3 * (size_t)gid], a.rgb[3 * (size_t)gid + 1], a.rgb[3 * (size_t)gid + 2], 0.f);
            float wv[12];
            uint32_t qv[3] = {0u, 0u, 0u};   // register index q + 1 per code; 0 = the junk register
#pragma unroll
            for (int k = 0; k < 12; k++) {
                wv[k] = 0.f;
                if (k < K) {
                    const size_t off = (size_t)gid * K + k;
                    wv[k] = a.qw[off];
                    const int q = quick_index(a.qi, a.qidx_dtype, off);
                    const uint32_t qb = (q >= 0 && q < Dq) ? (uint32_t)(q + 1) : 0u;
                    qv[k >> 2] |= qb << (8 * (k & 3));
                }
            }
            st.Wt[r][0] = make_float4(wv[0], wv[1], wv[2], wv[3]);
            st.Wt[r][1] = make_float4(wv[4], wv[5], wv[6], wv[7]);
            st.Wt[r][2] = make_float4(wv[8], wv[9], wv[10], wv[11]);
            st.Q[r] = make_uint4(qv[0], qv[1], qv[2], 0u);
        }
        wave_lds_fence();
        const int n = __popcll(m);
        // two candidates per step: their exponents on packed f32 (expf_det2,
        // bitwise = expf_det), then the per-pixel recurrence in order
        for (int j0 = 0; j0 < n; j0 += 2) {
            if (wave_ballot(!done) == 0) break;
            const bool two = j0 + 1 < n;
            const int j1 = two ? j0 + 1 : j0;
            const float4 A0 = st.A[j0], B0 = st.B[j0];
            const float4 A1 = st.A[j1], B1 = st.B[j1];
            const float p0 = splat_power(A0.z, A0.w, B0.x, A0.x - pfx, A0.y - pfy);
            const float p1 = splat_power(A1.z, A1.w, B1.x, A1.x - pfx, A1.y - pfy);
            bool ok0 = !done && !(p0 > 0.0f || p0 < B0.z);
            bool ok1 = two && !done && !(p1 > 0.0f || p1 < B1.z);
            if (!wave_any(ok0 || ok1)) continue;
            const f32x2 EX = expf_det2(f32x2{p0, p1});
            const float al0 = fminf(0.99f, B0.y * EX.x);
            const float al1 = fminf(0.99f, B1.y * EX.y);
            ok0 = ok0 && !(al0 < 1.0f / 255.0f);
            ok1 = ok1 && !(al1 < 1.0f / 255.0f);
            float aT0, aT1;
            {
                const float test_T = T * (1.0f - al0);
                const bool term = ok0 && (test_T < 0.0001f);
                done = done || term;
                ok0 = ok0 && !term;
                ok1 = ok1 && !term;
                aT0 = ok0 ? al0 * T : 0.f;
                if (ok0) {
                    const float4 C0 = st.C[j0];
                    cr = fmaf(C0.x, aT0, cr);
                    cg = fmaf(C0.y, aT0, cg);
                    cbl = fmaf(C0.z, aT0, cbl);
                    T = test_T;
                    last = (uint32_t)__float_as_int(B0.w);
                }
            }
            {
                const float test_T = T * (1.0f - al1);
                const bool term = ok1 && (test_T < 0.0001f);
                done = done || term;
                ok1 = ok1 && !term;
                aT1 = ok1 ? al1 * T : 0.f;
                if (ok1) {
                    const float4 C1 = st.C[j1];
                    cr = fmaf(C1.x, aT1, cr);
                    cg = fmaf(C1.y, aT1, cg);
                    cbl = fmaf(C1.z, aT1, cbl);
                    T = test_T;
                    last = (uint32_t)__float_as_int(B1.w);
                }
            }
            if (wave_any(ok0)) LSR_QV_UPDATE(aT0, st.Q[j0], st.Wt[j0][0], st.Wt[j0][1], st.Wt[j0][2]);
            if (wave_any(ok1)) LSR_QV_UPDATE(aT1, st.Q[j1], st.Wt[j1][0], st.Wt[j1][1], st.Wt[j1][2]);
        }
        wave_lds_fence();
    }
    const size_t HW = (size_t)c.H * c.W;
    if (inside) {
        const size_t pix = (size_t)pm.py * c.W + pm.px;
        a.final_T[pix] = T;
        a.n_contrib[pix] = last;
        a.out_color[pix] = fmaf(T, c.bg[0], cr);
        a.out_color[HW + pix] = fmaf(T, c.bg[1], cg);
        a.out_color[2 * HW + pix] = fmaf(T, c.bg[2], cbl);
        float* const o = a.out_lang + pix;
        for (int q = 0; q < Dq; q++) {
            float v;
            uint32_t sv;
            asm volatile(
                "s_mov_b32 %[sv], m0\n\t"
                "s_set_gpr_idx_on %[q], gpr_idx(SRC0)\n\t"
                "s_nop 0\n\t"
                "v_mov_b32 %[v], v64\n\t"
                "s_set_gpr_idx_off\n\t"
                "s_mov_b32 m0, %[sv]"
                : [v] "=v"(v), [sv] "=&s"(sv)
                : [q] "s"(q)
                : "memory");
            o[(size_t)q * HW] = v;
        }
    }
}

// Quick path with the chunk records prefetched by LDS-DMA (default when the
// sparse rows allow 16-B copies: K % 4 == 0, 16-B aligned weights/indices).
// k_render_fwd_quick_v gathers each chunk's records, rgb, 12 weights and 12
// indices into VGPRs when it reaches the chunk, so every chunk waits for two
// dependent global round trips, and at 2 waves/SIMD (the 192 accumulators take
// the register file) nothing hides them (r03 PMC: waves parked in s_waitcnt
// 59 % of their cycles).  Here the NEXT chunk's raw rows are copied straight
// into a per-wave LDS buffer by global_load_lds (no VGPR destination, ids
// loaded two chunks ahead) while the current chunk blends; staging then reads
// LDS.  Blend, accumulation and outputs are k_render_fwd_quick_v's, bit for bit.
// NQ = 16-B parts of an index row: 3 (fp32 / int32), 6 (int64), 1 (packed)
template <int NQ>
struct WaveRawQ {
    float4 A[64];
    float4 B[64];
    float rgb[3][64];                   // channel c of lane l (three 4-B DMAs)
    float4 W[3][64];                    // weight row part p (4 weights) of lane l
    uint4 Q[NQ][64];                    // index row bytes [16 p, 16 p + 16) of lane l
    uint32_t nid[64];                   // the point-list ids of the chunk after next
};
template <int DT>
constexpr int quick_nq() { return DT == 2 ? 6 : DT == 3 ? 1 : 3; }

template <int DT>
__device__ __forceinline__ int quick_code_raw(const WaveRawQ<quick_nq<DT>()>& raw, int lane, int k)
{
    if constexpr (DT == 2) {
        const uint4 q = raw.Q[k >> 1][lane];
        const uint32_t lo = (k & 1) ? q.z : q.x, hi = (k & 1) ? q.w : q.y;
        return hi != 0u || lo > 0x7fffffffu ? -1 : (int)lo;
    } else {
        const uint4 q = raw.Q[k >> 2][lane];
        const uint32_t v = (k & 3) == 0 ? q.x : (k & 3) == 1 ? q.y : (k & 3) == 2 ? q.z : q.w;
        return DT == 0 ? quick_code_f32(__uint_as_float(v)) : (int)v;
    }
}

// One chunk's rows -> raw by LDS-DMA (K = 12 codes per Gaussian): lane l's
// record, rgb, weight row and index row land at slot l of each array (an LDS-
// DMA writes wave-uniform M0 + lane x size).  One asm block walks M0 through
// the arrays (raw's layout is fixed by the static_asserts below); the weight
// and index row parts are the immediate offsets of one address each; the same
// asm block also copies the point-list ids two chunks ahead into raw.nid, so
// no VGPR-destination load is ever in flight behind the DMAs (a compiler-
// inserted wait for such a load is a vmcnt(N) that the compiler computes
// without the asm's DMAs, and drained them: every chunk's first pair waited
// for the prefetch just issued).  The
// immediate offset applies to the LDS destination as well (M0 + offset + 16
// lane), so M0 steps to each array's base minus that offset.  The colour
// goes as three 4-B DMAs (one channel plane each): a dwordx3 LDS-DMA does not
// land at 12 x lane (measured: wrong colours with the 12-B layout).  (The
// __builtin_amdgcn_global_load_lds form crashes ROCm 7.2's SIFixSGPRCopies in
// this kernel, and per-call M0 constants spilled SGPRs.)  The caller waits with
// s_waitcnt vmcnt before reading raw.
#define LSR_GLDS(step, insn) "s_add_u32 m0, m0, " #step "\n\ts_nop 0\n\t" insn "\n\t"
template <int NQ>
__device__ __forceinline__ void quick_dma12(WaveRawQ<NQ>& raw, const RenderArgs& a, uint32_t g, const uint32_t* pI)
{
    static_assert(offsetof(WaveRawQ<NQ>, B) == 1024 && offsetof(WaveRawQ<NQ>, rgb) == 2048 &&
                  offsetof(WaveRawQ<NQ>, W) == 2816 && offsetof(WaveRawQ<NQ>, Q) == 5888 &&
                  offsetof(WaveRawQ<NQ>, nid) == 5888 + 1024 * NQ, "raw layout");
    const uint32_t base = (uint32_t)(uintptr_t)&raw;   // the LDS byte address (low half of the flat address)
    const float4* pA = a.splatA + g;
    const float4* pB = a.splatB + g;
    const float* pR = a.rgb + 3 * (size_t)g;
    const float* pW = a.qw + 12 * (size_t)g;
    const char* pQ = reinterpret_cast<const char*>(a.qi) + (size_t)g * (16 * NQ);
    uint32_t keep;
    if constexpr (NQ == 1) {
        asm volatile("s_mov_b32 %[keep], m0\n\t"
                     "s_mov_b32 m0, %[base]\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %[pA], off\n\t"
                     LSR_GLDS(1024, "global_load_lds_dwordx4 %[pB], off")
                     LSR_GLDS(1024, "global_load_lds_dword %[pR], off")
                     LSR_GLDS(252, "global_load_lds_dword %[pR], off offset:4")
                     LSR_GLDS(252, "global_load_lds_dword %[pR], off offset:8")
                     LSR_GLDS(264, "global_load_lds_dwordx4 %[pW], off")
                     LSR_GLDS(1008, "global_load_lds_dwordx4 %[pW], off offset:16")
                     LSR_GLDS(1008, "global_load_lds_dwordx4 %[pW], off offset:32")
                     LSR_GLDS(1056, "global_load_lds_dwordx4 %[pQ], off")
                     LSR_GLDS(1024, "global_load_lds_dword %[pI], off")
                     "s_mov_b32 m0, %[keep]"
                     : [keep] "=&s"(keep)
                     : [base] "s"(base), [pA] "v"(pA), [pB] "v"(pB), [pR] "v"(pR), [pW] "v"(pW), [pQ] "v"(pQ),
                       [pI] "v"(pI)
                     : "memory", "scc");
    } else if constexpr (NQ == 3) {
        asm volatile("s_mov_b32 %[keep], m0\n\t"
                     "s_mov_b32 m0, %[base]\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %[pA], off\n\t"
                     LSR_GLDS(1024, "global_load_lds_dwordx4 %[pB], off")
                     LSR_GLDS(1024, "global_load_lds_dword %[pR], off")
                     LSR_GLDS(252, "global_load_lds_dword %[pR], off offset:4")
                     LSR_GLDS(252, "global_load_lds_dword %[pR], off offset:8")
                     LSR_GLDS(264, "global_load_lds_dwordx4 %[pW], off")
                     LSR_GLDS(1008, "global_load_lds_dwordx4 %[pW], off offset:16")
                     LSR_GLDS(1008, "global_load_lds_dwordx4 %[pW], off offset:32")
                     LSR_GLDS(1056, "global_load_lds_dwordx4 %[pQ], off")
                     LSR_GLDS(1008, "global_load_lds_dwordx4 %[pQ], off offset:16")
                     LSR_GLDS(1008, "global_load_lds_dwordx4 %[pQ], off offset:32")
                     LSR_GLDS(1056, "global_load_lds_dword %[pI], off")
                     "s_mov_b32 m0, %[keep]"
                     : [keep] "=&s"(keep)
                     : [base] "s"(base), [pA] "v"(pA), [pB] "v"(pB), [pR] "v"(pR), [pW] "v"(pW), [pQ] "v"(pQ),
                       [pI] "v"(pI)
                     : "memory", "scc");
    } else {
        asm volatile("s_mov_b32 %[keep], m0\n\t"
                     "s_mov_b32 m0, %[base]\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %[pA], off\n\t"
                     LSR_GLDS(1024, "global_load_lds_dwordx4 %[pB], off")
                     LSR_GLDS(1024, "global_load_lds_dword %[pR], off")
                     LSR_GLDS(252, "global_load_lds_dword %[pR], off offset:4")
                     LSR_GLDS(252, "global_load_lds_dword %[pR], off offset:8")
                     LSR_GLDS(264, "global_load_lds_dwordx4 %[pW], off")
                     LSR_GLDS(1008, "global_load_lds_dwordx4 %[pW], off offset:16")
                     LSR_GLDS(1008, "global_load_lds_dwordx4 %[pW], off offset:32")
                     LSR_GLDS(1056, "global_load_lds_dwordx4 %[pQ], off")
                     LSR_GLDS(1008, "global_load_lds_dwordx4 %[pQ], off offset:16")
                     LSR_GLDS(1008, "global_load_lds_dwordx4 %[pQ], off offset:32")
                     LSR_GLDS(1008, "global_load_lds_dwordx4 %[pQ], off offset:48")
                     LSR_GLDS(1008, "global_load_lds_dwordx4 %[pQ], off offset:64")
                     LSR_GLDS(1008, "global_load_lds_dwordx4 %[pQ], off offset:80")
                     LSR_GLDS(1104, "global_load_lds_dword %[pI], off")
                     "s_mov_b32 m0, %[keep]"
                     : [keep] "=&s"(keep)
                     : [base] "s"(base), [pA] "v"(pA), [pB] "v"(pB), [pR] "v"(pR), [pW] "v"(pW), [pQ] "v"(pQ),
                       [pI] "v"(pI)
                     : "memory", "scc");
    }
}
#undef LSR_GLDS

#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"   // the v255 clobber is the point: it sizes the allocation
// Pixel-major epilogue (LSR_LAYOUT_HWC): the pixel's 192 weights, v64..v255, as 48
// 16-B stores into its 768-B row (immediate offsets from one address).
#define LSR_QHWC(a, b, off) "global_store_dwordx4 %[p], v[" #a ":" #b "], off offset:" #off "\n\t"
#define LSR_QHWC_ALL \
    LSR_QHWC(64, 67, 0) LSR_QHWC(68, 71, 16) LSR_QHWC(72, 75, 32) LSR_QHWC(76, 79, 48) \
    LSR_QHWC(80, 83, 64) LSR_QHWC(84, 87, 80) LSR_QHWC(88, 91, 96) LSR_QHWC(92, 95, 112) \
    LSR_QHWC(96, 99, 128) LSR_QHWC(100, 103, 144) LSR_QHWC(104, 107, 160) LSR_QHWC(108, 111, 176) \
    LSR_QHWC(112, 115, 192) LSR_QHWC(116, 119, 208) LSR_QHWC(120, 123, 224) LSR_QHWC(124, 127, 240) \
    LSR_QHWC(128, 131, 256) LSR_QHWC(132, 135, 272) LSR_QHWC(136, 139, 288) LSR_QHWC(140, 143, 304) \
    LSR_QHWC(144, 147, 320) LSR_QHWC(148, 151, 336) LSR_QHWC(152, 155, 352) LSR_QHWC(156, 159, 368) \
    LSR_QHWC(160, 163, 384) LSR_QHWC(164, 167, 400) LSR_QHWC(168, 171, 416) LSR_QHWC(172, 175, 432) \
    LSR_QHWC(176, 179, 448) LSR_QHWC(180, 183, 464) LSR_QHWC(184, 187, 480) LSR_QHWC(188, 191, 496) \
    LSR_QHWC(192, 195, 512) LSR_QHWC(196, 199, 528) LSR_QHWC(200, 203, 544) LSR_QHWC(204, 207, 560) \
    LSR_QHWC(208, 211, 576) LSR_QHWC(212, 215, 592) LSR_QHWC(216, 219, 608) LSR_QHWC(220, 223, 624) \
    LSR_QHWC(224, 227, 640) LSR_QHWC(228, 231, 656) LSR_QHWC(232, 235, 672) LSR_QHWC(236, 239, 688) \
    LSR_QHWC(240, 243, 704) LSR_QHWC(244, 247, 720) LSR_QHWC(248, 251, 736) LSR_QHWC(252, 255, 752)
// Epilogue of the 192-channel quick kernel: channel q = N - 64 is register vN.
#define LSR_QEPI(N) "buffer_store_dword v" #N ", %[vo], %[rs], %[so] offen\n\ts_add_u32 %[so], %[so], %[hw4]\n\t"
#define LSR_QEPI10(h) LSR_QEPI(h##0) LSR_QEPI(h##1) LSR_QEPI(h##2) LSR_QEPI(h##3) LSR_QEPI(h##4) \
                      LSR_QEPI(h##5) LSR_QEPI(h##6) LSR_QEPI(h##7) LSR_QEPI(h##8) LSR_QEPI(h##9)
#define LSR_QEPI_ALL                                                                                     \
    LSR_QEPI(64) LSR_QEPI(65) LSR_QEPI(66) LSR_QEPI(67) LSR_QEPI(68) LSR_QEPI(69)                        \
    LSR_QEPI10(7) LSR_QEPI10(8) LSR_QEPI10(9) LSR_QEPI10(10) LSR_QEPI10(11) LSR_QEPI10(12) LSR_QEPI10(13) \
    LSR_QEPI10(14) LSR_QEPI10(15) LSR_QEPI10(16) LSR_QEPI10(17) LSR_QEPI10(18) LSR_QEPI10(19)             \
    LSR_QEPI10(20) LSR_QEPI10(21) LSR_QEPI10(22) LSR_QEPI10(23) LSR_QEPI10(24)                           \
    LSR_QEPI(250) LSR_QEPI(251) LSR_QEPI(252) LSR_QEPI(253) LSR_QEPI(254) LSR_QEPI(255)
// BAND: one wave per 16x4 band of the tile (the channel-major map: each of the
// 192 channel stores then writes 64-B row pieces instead of 32-B ones, render
// -2.5 %); else one wave per 8x8 block (the pixel-major map, whose stores are
// per-pixel rows: the tighter block cull wins, -5.6 %)
template <int DT, bool BAND>
__global__ void __launch_bounds__(64, 2) __attribute__((amdgpu_num_vgpr(63))) k_render_fwd_quick_d(RenderArgs a)
{
    constexpr int NQ = quick_nq<DT>();
    __shared__ WaveStageV st;
    __shared__ WaveRawQ<NQ> raw;
    const Cam& c = a.cam;
    const WaveTile wt(a);
    const int lane = threadIdx.x;
    constexpr int BW = BAND ? 16 : 8, BH = 64 / BW;
    PixMap pm(c, wt.tile, lane + (wt.sub << 6));
    if constexpr (BAND) {
        pm.bx = (wt.tile % c.gx) * LSR_TILE;
        pm.by = (wt.tile / c.gx) * LSR_TILE + wt.sub * BH;
        pm.px = pm.bx + (lane & (BW - 1));
        pm.py = pm.by + lane / BW;
    }
    const bool inside = pm.px < c.W && pm.py < c.H;
    const float pfx = (float)pm.px, pfy = (float)pm.py;
    const uint32_t rs = a.tile_start[wt.tile], re = a.tile_start[wt.tile + 1];
    const int Dq = a.Dq;

    {   // zero v63 (junk) .. v255 (accumulators)
        uint32_t i, sv;
        asm volatile(
            "s_mov_b32 %[sv], m0\n\t"
            "s_mov_b32 %[i], 0\n\t"
            "s_set_gpr_idx_on 0, gpr_idx(DST)\n\t"
            "1:\n\t"
            "s_set_gpr_idx_idx %[i]\n\t"
            "s_nop 0\n\t"
            "v_mov_b32 v63, 0\n\t"
            "s_add_u32 %[i], %[i], 1\n\t"
            "s_cmp_lt_u32 %[i], 193\n\t"
            "s_cbranch_scc1 1b\n\t"
            "s_set_gpr_idx_off\n\t"
            "s_mov_b32 m0, %[sv]"
            : [i] "=&s"(i), [sv] "=&s"(sv)
            :
            : "scc", "v63", "v255", "memory");
    }
    float T = 1.0f, cr = 0.f, cg = 0.f, cbl = 0.f;
    uint32_t last = 0;
    bool done = !inside;
    // the first chunk's rows, and (in raw.nid) the ids of the chunk after it; positions
    // past the list read the list's last id, and gid 0 (a valid row, never staged) is used
    if (rs < re) quick_dma12<NQ>(raw, a, (rs + lane < re) ? a.point_list[rs + lane] : 0u,
                                 a.point_list + min(rs + 64 + lane, re - 1));
    for (uint32_t base = rs; base < re; base += 64) {
        if (wave_ballot(!done) == 0) break;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this chunk's rows have landed in raw
        const uint32_t idx = base + lane;
        const bool valid = idx < re;
        const float4 A = raw.A[lane], B = raw.B[lane];
        const bool ok = valid && rect_overlap(A.x, A.y, __float_as_uint(B.w), pm.bx, pm.by, BW - 1, BH - 1) &&
                        rect_overlap_exact(A.x, A.y, A.z, A.w, B.x, B.z, pm.bx, pm.by, (float)(BW - 1), (float)(BH - 1));
        const uint64_t m = wave_ballot(ok);
        if (ok) {
            const int r = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
            st.A[r] = A;
            st.B[r] = make_float4(B.x, B.y, B.z, __int_as_float((int)(idx - rs) + 1));
            st.C[r] = make_float4(raw.rgb[0][lane], raw.rgb[1][lane], raw.rgb[2][lane], 0.f);
            st.Wt[r][0] = raw.W[0][lane];
            st.Wt[r][1] = raw.W[1][lane];
            st.Wt[r][2] = raw.W[2][lane];
            uint32_t qv[3] = {0u, 0u, 0u};   // register index q + 1 per code; 0 = the junk register
            if constexpr (DT == 3) {
                // packed rows are register indices already; a byte above Dq (not
                // written by lsr_quick_pack_codes for this Dq) is dropped, so no
                // index can leave v64 .. v(63 + Dq)
                const uint4 p = raw.Q[0][lane];
                const uint32_t pw[3] = {p.x, p.y, p.z};
#pragma unroll
                for (int k = 0; k < 12; k++) {
                    const uint32_t b = (pw[k >> 2] >> (8 * (k & 3))) & 0xffu;
                    qv[k >> 2] |= (b <= (uint32_t)Dq ? b : 0u) << (8 * (k & 3));
                }
            } else {
#pragma unroll
                for (int k = 0; k < 12; k++) {   // K = 12 (quick_dma_ok)
                    const int q = quick_code_raw<DT>(raw, lane, k);
                    const uint32_t qb = (q >= 0 && q < Dq) ? (uint32_t)(q + 1) : 0u;
                    qv[k >> 2] |= qb << (8 * (k & 3));
                }
            }
            st.Q[r] = make_uint4(qv[0], qv[1], qv[2], 0u);
        }
        const uint32_t gid_n = idx + 64 < re ? raw.nid[lane] : 0u;
        wave_lds_fence();   // raw read, stage written: raw may be refilled
        if (base + 64 < re) quick_dma12<NQ>(raw, a, gid_n, a.point_list + min(idx + 128, re - 1));
        const int n = __popcll(m);
        // the blend of k_render_fwd_quick_v, unchanged
        for (int j0 = 0; j0 < n; j0 += 2) {
            if (wave_ballot(!done) == 0) break;
            const bool two = j0 + 1 < n;
            const int j1 = two ? j0 + 1 : j0;
            const float4 A0 = st.A[j0], B0 = st.B[j0];
            const float4 A1 = st.A[j1], B1 = st.B[j1];
            // the colours read with the geometry, and the blend below as selects
            // (the same fmaf on the same operands where a pixel takes the
            // candidate): no LDS round trip or exec-mask branch per candidate
            const float4 C0 = st.C[j0], C1 = st.C[j1];
            const float p0 = splat_power(A0.z, A0.w, B0.x, A0.x - pfx, A0.y - pfy);
            const float p1 = splat_power(A1.z, A1.w, B1.x, A1.x - pfx, A1.y - pfy);
            bool ok0 = !done && !(p0 > 0.0f || p0 < B0.z);
            bool ok1 = two && !done && !(p1 > 0.0f || p1 < B1.z);
            if (!wave_any(ok0 || ok1)) continue;
            const f32x2 EX = expf_det2(f32x2{p0, p1});
            const float al0 = fminf(0.99f, B0.y * EX.x);
            const float al1 = fminf(0.99f, B1.y * EX.y);
            ok0 = ok0 && !(al0 < 1.0f / 255.0f);
            ok1 = ok1 && !(al1 < 1.0f / 255.0f);
            float aT0, aT1;
            {
                const float test_T = T * (1.0f - al0);
                const bool term = ok0 && (test_T < 0.0001f);
                done = done || term;
                ok0 = ok0 && !term;
                ok1 = ok1 && !term;
                aT0 = ok0 ? al0 * T : 0.f;
                cr = ok0 ? fmaf(C0.x, aT0, cr) : cr;
                cg = ok0 ? fmaf(C0.y, aT0, cg) : cg;
                cbl = ok0 ? fmaf(C0.z, aT0, cbl) : cbl;
                T = ok0 ? test_T : T;
                last = ok0 ? (uint32_t)__float_as_int(B0.w) : last;
            }
            {
                const float test_T = T * (1.0f - al1);
                const bool term = ok1 && (test_T < 0.0001f);
                done = done || term;
                ok1 = ok1 && !term;
                aT1 = ok1 ? al1 * T : 0.f;
                cr = ok1 ? fmaf(C1.x, aT1, cr) : cr;
                cg = ok1 ? fmaf(C1.y, aT1, cg) : cg;
                cbl = ok1 ? fmaf(C1.z, aT1, cbl) : cbl;
                T = ok1 ? test_T : T;
                last = ok1 ? (uint32_t)__float_as_int(B1.w) : last;
            }
            if (wave_any(ok0)) LSR_QV_UPDATE(aT0, st.Q[j0], st.Wt[j0][0], st.Wt[j0][1], st.Wt[j0][2]);
            if (wave_any(ok1)) LSR_QV_UPDATE(aT1, st.Q[j1], st.Wt[j1][0], st.Wt[j1][1], st.Wt[j1][2]);
        }
        wave_lds_fence();
    }
    // no LDS-DMA may land after the wave (and its LDS) is gone
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const size_t HW = (size_t)c.H * c.W;
    if (inside) {
        const size_t pix = (size_t)pm.py * c.W + pm.px;
        a.final_T[pix] = T;
        a.n_contrib[pix] = last;
        a.out_color[pix] = fmaf(T, c.bg[0], cr);
        a.out_color[HW + pix] = fmaf(T, c.bg[1], cg);
        a.out_color[2 * HW + pix] = fmaf(T, c.bg[2], cbl);
        float* const o = a.out_lang + pix;
        if (a.quick_hwc) {   // Dq == 192 (lsr_api validate)
            float* const row = a.out_lang + pix * 192;
            asm volatile(LSR_QHWC_ALL : : [p] "v"(row) : "memory");
        } else if (Dq == 192 && (uint64_t)HW * 192u * 4u < 0x80000000ull) {
            // all 192 channels straight from v64..v255 by buffer stores, the channel
            // plane's byte offset in an SGPR stepped by HW * 4: two instructions per
            // channel instead of the index-mode read, the M0 save / restore and a
            // 64-bit address per store
            const __amdgpu_buffer_rsrc_t ro =
                __builtin_amdgcn_make_buffer_rsrc(a.out_lang, 0, (int)(HW * 192u * 4u), 0x00020000);
            uint32_t so;
            asm volatile("s_mov_b32 %[so], 0\n\t"
                         LSR_QEPI_ALL
                         : [so] "=&s"(so)
                         : [vo] "v"((uint32_t)pix * 4u), [rs] "s"(ro), [hw4] "s"((uint32_t)HW * 4u)
                         : "memory", "scc");
        } else {
            for (int q = 0; q < Dq; q++) {
                float v;
                uint32_t sv;
                asm volatile(
                    "s_mov_b32 %[sv], m0\n\t"
                    "s_set_gpr_idx_on %[q], gpr_idx(SRC0)\n\t"
                    "s_nop 0\n\t"
                    "v_mov_b32 %[v], v64\n\t"
                    "s_set_gpr_idx_off\n\t"
                    "s_mov_b32 m0, %[sv]"
                    : [v] "=v"(v), [sv] "=&s"(sv)
                    : [q] "s"(q)
                    : "memory");
                o[(size_t)q * HW] = v;
            }
        }
    }
}
#pragma clang diagnostic pop

// the LDS-DMA quick kernel applies: 12 codes per Gaussian (3 levels x top-4), 16-B aligned rows
static bool quick_dma_ok(const RenderArgs& a)
{
    return a.K == 12 && a.Dq <= 192 && ((uintptr_t)a.qw % 16) == 0 && ((uintptr_t)a.qi % 16) == 0 &&
           ((uintptr_t)a.rgb % 4) == 0;
}

#pragma clang diagnostic pop

int lang_set_for(int D)
{
    if (D <= 0) return 0;
    if (D <= 4) return 4;
    if (D <= 8) return 8;
    if (D <= 16) return 16;
    if (D <= 32) return 32;
    if (D <= 64) return 64;
    return -1;
}

hipError_t launch_render_fwd(const RenderArgs& a, hipStream_t st)
{
    const int T = a.cam.gx * a.cam.gy;
    if (T == 0) return hipSuccess;
    if (a.qw) {
        if (a.quick_hwc && !(quick_dma_ok(a) && a.Dq == 192)) return hipErrorInvalidValue;
        if (a.qidx_dtype == LSR_INDEX_PACKED && !quick_dma_ok(a)) return hipErrorInvalidValue;
        if (quick_dma_ok(a)) {
            if (a.quick_hwc) {
                switch (a.qidx_dtype) {
                    case LSR_INDEX_F32: k_render_fwd_quick_d<0, false><<<T * 4, 64, 0, st>>>(a); break;
                    case LSR_INDEX_I32: k_render_fwd_quick_d<1, false><<<T * 4, 64, 0, st>>>(a); break;
                    case LSR_INDEX_PACKED: k_render_fwd_quick_d<3, false><<<T * 4, 64, 0, st>>>(a); break;
                    default: k_render_fwd_quick_d<2, false><<<T * 4, 64, 0, st>>>(a); break;
                }
            } else {
                switch (a.qidx_dtype) {
                    case LSR_INDEX_F32: k_render_fwd_quick_d<0, true><<<T * 4, 64, 0, st>>>(a); break;
                    case LSR_INDEX_I32: k_render_fwd_quick_d<1, true><<<T * 4, 64, 0, st>>>(a); break;
                    case LSR_INDEX_PACKED: k_render_fwd_quick_d<3, true><<<T * 4, 64, 0, st>>>(a); break;
                    default: k_render_fwd_quick_d<2, true><<<T * 4, 64, 0, st>>>(a); break;
                }
            }
            return hipGetLastError();
        }
        if (a.K <= 12 && a.Dq <= 192) {
            switch ((a.Dq + 31) / 32) {
                case 1: k_render_fwd_quick_v<1><<<T * 4, 64, 0, st>>>(a); break;
                case 2: k_render_fwd_quick_v<2><<<T * 4, 64, 0, st>>>(a); break;
                case 3: k_render_fwd_quick_v<3><<<T * 4, 64, 0, st>>>(a); break;
                case 4: k_render_fwd_quick_v<4><<<T * 4, 64, 0, st>>>(a); break;
                case 5: k_render_fwd_quick_v<5><<<T * 4, 64, 0, st>>>(a); break;
                default: k_render_fwd_quick_v<6><<<T * 4, 64, 0, st>>>(a); break;
            }
            return hipGetLastError();
        }
        const size_t sm = (size_t)a.Dq * 64 * 4 + 64 * 32 + 64 * 12 + (size_t)64 * a.K * 8;
        k_render_fwd_quick<<<T * 4, 64, sm, st>>>(a);
        return hipGetLastError();
    }
    switch (lang_set_for(a.D)) {
#define LSR_FWD_LAUNCH(K, NL) ((a.zero || a.zero2) ? K<NL, true><<<4 * T, 64, 0, st>>>(a) : K<NL, false><<<4 * T, 64, 0, st>>>(a))
        case 0: LSR_FWD_LAUNCH(k_render_fwd, 0); break;
        case 4: LSR_FWD_LAUNCH(k_render_fwd, 4); break;
        case 8: LSR_FWD_LAUNCH(k_render_fwd, 8); break;
        // D in (8, 16]: the ML form with gathered rows (cfg3 render_fwd 0.307 -> 0.299 ms against the
        // VALU blend; the ML form with LDS-staged rows measured +2.6 %)
        case 16:
            if constexpr (fwd_sfeat<16>()) {
                if (a.D == 16) {
                    if (a.zero || a.zero2) k_render_fwd<16, true, true><<<4 * T, 64, 0, st>>>(a);
                    else k_render_fwd<16, false, true><<<4 * T, 64, 0, st>>>(a);
                } else {
                    if (a.zero || a.zero2) k_render_fwd<16, true, true, true><<<4 * T, 64, 0, st>>>(a);
                    else k_render_fwd<16, false, true, true><<<4 * T, 64, 0, st>>>(a);
                }
            } else {
                LSR_FWD_LAUNCH(k_render_fwd, 16);
            }
            break;
        case 32:
            // D in (16, 32]: the ML form (cfg5 render_fwd 1.650 -> 1.266 ms against the VALU blend)
            if (a.D == 32) {
                if (a.zero || a.zero2) k_render_fwd<32, true, true><<<4 * T, 64, 0, st>>>(a);
                else k_render_fwd<32, false, true><<<4 * T, 64, 0, st>>>(a);
            } else {
                if (a.zero || a.zero2) k_render_fwd<32, true, true, true><<<4 * T, 64, 0, st>>>(a);
                else k_render_fwd<32, false, true, true><<<4 * T, 64, 0, st>>>(a);
            }
            break;
        case 64:
            // D = 64: always the ML form (measured 0.996 -> 0.688 ms against the
            // earlier 16-candidate-group MFMA kernel at cfg3 geometry; the
            // VALU-only blend is slower still)
            if (a.D == 64) {
                if (a.zero || a.zero2) k_render_fwd<64, true, true><<<4 * T, 64, 0, st>>>(a);
                else k_render_fwd<64, false, true><<<4 * T, 64, 0, st>>>(a);
            } else {
                if (a.zero || a.zero2) k_render_fwd<64, true, true, true><<<4 * T, 64, 0, st>>>(a);
                else k_render_fwd<64, false, true, true><<<4 * T, 64, 0, st>>>(a);
            }
            break;
#undef LSR_FWD_LAUNCH
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// --------------------------------------------------------- backward -------
// Gradient row width: the compiled channel set's value count, padded to the
// 32-value reduction groups.
int grad_row_width(int D)
{
    const int nl = lang_set_for(D);
    const int nv = LSR_GROW_LANG + (nl > 0 ? nl : 0);
    return (nv + 31) / 32 * 32;
}

// ------------------------------------------------ factorised backward ----
// Every per-(pixel, instance) gradient term is a product of a per-pair
// scalar and a per-pixel quantity, so the pixel sums of a wave are GEMMs:
//   colour / language:  g[j][c]  = sum_p aT[j][p] * dL/dout[c][p]
//   geometry:           with u = dL/dalpha * G, dx = X_j - lx_p (X_j, lx_p
//                       relative to the 8x8 block centre), the six values
//                       (mean2D x/y, conic a/b/c, opacity) are linear in the
//                       moments  sum_p u[j][p] * {1, lx, ly, lx^2, lx*ly, ly^2}
//   per-pair dot:       dot[j][p] = sum_c f[j][c] * dL/dout[c][p]
// All three run on exact-f32 MFMA (v_mfma_f32_16x16x4_f32) over groups of 16
// instances; the serial per-pixel recurrence (T recovery, rec) is the only
// per-pair VALU work left.  The B operands (dL/dout in two layouts and the
// pixel moments) are per-wave constants held in registers.
template <int NL>
struct BwdFrags {
    static constexpr int C = 3 + NL;
    static constexpr int KS = (C + 3) / 4;      // dot K-steps over channels
    static constexpr int NBC = (C + 15) / 16;   // channel blocks of the gradient product
    float dotB[KS][4];    // dL/dout[4t + (l>>4)][pb*16 + (l&15)]
    float chB[NBC][16];   // dL/dout[nb*16 + (l&15)][4t + (l>>4)]
    float momB[16];       // moment (l&15) of block pixel 4t + (l>>4)
};

template <int NL>
__device__ __forceinline__ float gd_at(const RenderBwdArgs& b, int c, int q, int bx, int by)
{
    const Cam& cm = b.f.cam;
    const int qx = bx + (q & 7), qy = by + (q >> 3);
    const bool ok = qx < cm.W && qy < cm.H && c < 3 + b.f.D;
    const size_t HW = (size_t)cm.H * cm.W;
    const size_t pix = (size_t)min(qy, cm.H - 1) * cm.W + min(qx, cm.W - 1);
    const float* src = c < 3 ? b.dout_color + (size_t)c * HW : b.dout_lang + (size_t)min(c - 3, max(b.f.D - 1, 0)) * HW;
    if (c >= 3 && b.f.D == 0) src = b.dout_color;
    const float v = src[pix];
    return ok ? v : 0.f;
}

#ifndef LSR_GRP_STRIDE
#define LSR_GRP_STRIDE 66   // dot/u and aT tiles: conflict-free A-fragment reads (li*66 mod 32 = 2 li)
#endif
#define LSR_BUF_OOB 0x7ffffffc  // a byte offset past every buffer the backward addresses this way
#define LSR_MOM9_STRIDE 12  // reduced moment + colour sums per candidate (16-B aligned rows)
#define LSR_LOG2E 1.4426950408889634f
#define LSR_MF_ATOMIC(ptr, v) atomicAdd((ptr), (v))

// Lane mask of |v| < bound, straight from the compare (the compiler otherwise
// round-trips a ballot's operand through a VGPR: two extra VALU per use).
__device__ __forceinline__ uint64_t lanes_abs_lt(float v, float bound)
{
    uint64_t m;
    asm("v_cmp_gt_f32_e64 %0, %1, |%2|" : "=s"(m) : "s"(bound), "v"(v));
    return m;
}

// Per-wave LDS staging of one chunk's candidate geometry (no feature rows).
// 80 entries: up to 15 candidates carried over from the previous chunk + 64.
// B.w holds the candidate's tile-list position (int bits) once staged: the
// cut extents it carried are only needed by the staging test itself.
struct WaveStageG {
    float4 A[80];
    float4 B[80];
    uint32_t gid[80];
};

// LST: the block's candidate list (written by the forward, RenderArgs::listA/B)
// copied into LDS by LDS-DMA, one 16-candidate group per chunk, two buffers
// (the next chunk lands while this one is processed).  B = {conic.c, opacity,
// id bits, 0-based position bits}.  16-entry chunks keep the D = 16 kernel's
// LDS at 10240 B, which with <= 128 VGPRs (amdgpu_waves_per_eu(4) below) lets
// 4 waves per SIMD reside instead of 3 (64-entry chunks: 12096 B): backward
// 0.503 -> 0.469 ms at cfg3.
#define LSR_LST_CHUNK 16
struct WaveStageL {
    float4 A[2 * LSR_LST_CHUNK];
    float4 B[2 * LSR_LST_CHUNK];
};
// waves per SIMD the MFMA backward is compiled for: 4 for the list-driven
// D = 16 kernel (the headline's), the launch-bounds floor otherwise
template <int NL, bool LD, bool LST, bool DET = false>
constexpr int bwd_waves() { return (LST && LD && NL == 16 && !DET) ? LSR_BWD16_WAVES : LSR_MF_WAVES; }

// LDS-DMA of one 16-B row part per lane: lane l's bytes land at lds + 16 l (an
// LDS-DMA writes wave-uniform M0 + lane x size).  Inline asm with M0 saved and
// restored (the builtin form crashed ROCm 7.2's SIFixSGPRCopies in the quick
// kernel); the caller waits with s_waitcnt vmcnt before reading lds.
__device__ __forceinline__ void glds16(const void* g, const void* lds)
{
    const uint32_t l = (uint32_t)(uintptr_t)lds;   // the LDS byte address (low half of the flat address)
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(g), "s"(l) : "memory");
}

// s_waitcnt vmcnt(N) only (gfx9 encoding: vmcnt[3:0] bits 3:0, [5:4] bits 15:14;
// expcnt and lgkmcnt at their maxima)
template <int N>
__device__ __forceinline__ void wait_vmcnt()
{
    static_assert(N >= 0 && N <= 63, "vmcnt is 6 bits");
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");   // also a compiler barrier for the LDS reads after it
}

// Appends this chunk's candidates after the `carry` entries already staged.
__device__ __forceinline__ int stage_candidates_geo(WaveStageG& st, int carry, bool valid, uint32_t gid, int pos,
                                                    int bx, int by, const float4* __restrict__ splatA,
                                                    const float4* __restrict__ splatB)
{
    float4 A = make_float4(0.f, 0.f, 0.f, 0.f), B = A;
    if (valid) {
        A = splatA[gid];
        B = splatB[gid];
    }
    const bool ok = valid && block_overlap(A.x, A.y, __float_as_uint(B.w), bx, by) &&
                    block_overlap_exact(A.x, A.y, A.z, A.w, B.x, B.z, bx, by);
    const uint64_t m = wave_ballot(ok);
    if (ok) {
        const int r = carry + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
        st.A[r] = A;
        st.B[r] = make_float4(B.x, B.y, B.z, __int_as_float(pos));
        st.gid[r] = gid;
    }
    wave_lds_fence();
    return __popcll(m);
}

// As stage_candidates_geo, with the chunk's records already loaded.
__device__ __forceinline__ int stage_candidates_geo_rec(WaveStageG& st, int carry, bool valid, uint32_t gid, int pos,
                                                        int bx, int by, float4 A, float4 B)
{
    const bool ok = valid && block_overlap(A.x, A.y, __float_as_uint(B.w), bx, by) &&
                    block_overlap_exact(A.x, A.y, A.z, A.w, B.x, B.z, bx, by);
    const uint64_t m = wave_ballot(ok);
    if (ok) {
        const int r = carry + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
        st.A[r] = A;
        st.B[r] = make_float4(B.x, B.y, B.z, __int_as_float(pos));
        st.gid[r] = gid;
    }
    wave_lds_fence();
    return __popcll(m);
}

// Feature c of Gaussian gid (rgb, then dense language; 0 past the channels).
template <int NL>
__device__ __forceinline__ float feature_at(const RenderArgs& a, uint32_t gid, int c)
{
    const bool ok = c < 3 + a.D;
    const float* src = c < 3 ? a.rgb + 3 * (size_t)gid + c
                             : (ok ? a.lang + (size_t)gid * a.D + (c - 3) : a.rgb + 3 * (size_t)gid);
    const float v = *src;
    return ok ? v : 0.f;
}

// Channel of the dot product's K-step t in lane group lg.  Default: channel
// 4t + lg.  VEC (whole 16-channel language rows, D = NL, rows 16-B aligned):
// the K order follows the rows' float4 layout, so a candidate's features are
// gathered with one 16-B load per 16-channel line and lane group (lane group
// lg takes float4 lg of each line: K-steps 4r..4r+3 are line r's channels
// 16r + 4lg + u) plus one load of its colour (the last K-step: channel lg,
// lane group 3 none).  The dot is the same sum over channels in another order.
template <int NL, bool VEC>
__device__ __forceinline__ int dot_channel(int t, int lg)
{
    if constexpr (VEC) {
        if (t < NL / 4) return 3 + 16 * (t >> 2) + 4 * lg + (t & 3);
        return lg < 3 ? lg : 3 + NL;   // past the channels: 0
    }
    return 4 * t + lg;
}

// The dot product's A fragments of candidate gid for lane group lg, in
// dot_channel order.
template <int NL, bool VEC, int KS>
__device__ __forceinline__ void dot_features(const RenderArgs& a, uint32_t gid, int lg, float (&af)[KS])
{
    if constexpr (VEC) {
        static_assert(NL % 16 == 0 && KS == NL / 4 + 1, "VEC: whole 16-channel lines");
        const float4* row = reinterpret_cast<const float4*>(a.lang) + (size_t)gid * (NL / 4) + lg;
#pragma unroll
        for (int r = 0; r < NL / 16; r++) {
            const float4 v = row[4 * r];
            af[4 * r + 0] = v.x;
            af[4 * r + 1] = v.y;
            af[4 * r + 2] = v.z;
            af[4 * r + 3] = v.w;
        }
        const float c = a.rgb[3 * (size_t)gid + min(lg, 2)];
        af[NL / 4] = lg < 3 ? c : 0.f;
    } else {
#pragma unroll
        for (int t = 0; t < KS; t++) af[t] = feature_at<NL>(a, gid, 4 * t + lg);
    }
}

#define BWD_MFMA(a, b_, c) __builtin_amdgcn_mfma_f32_16x16x4f32((a), (b_), (c), 0, 0, 0)

// ---------------------------------- deterministic backward (LSR_OPT_DETERMINISTIC)
// Every per-Gaussian gradient is a sum over the 8x8 blocks the Gaussian is
// staged in of a per-block partial (the block's 64 pixels summed in a fixed
// order by its wave); only the order in which the blocks' atomics land varies.
// DET adds the partials as 64-bit fixed-point integers instead (associative:
// the same bits in any order).  The exponent of (Gaussian i, column class) is
// chosen from an a-priori bound of the partials (64 pixels x the per-pixel
// bound) and of how many blocks can contribute (the radius rect, nb =
// (r/4 + 2)^2 blocks), so the sum cannot overflow:
//   class 0 colour / language  aT |dL/dout|                        <= Dm
//   class 1 opacity            G |dL/dalpha|                       <= Am
//   class 2 mean2D (NDC)       0.5 W o G |conic d| |dL/dalpha|     <= 0.554 max(W,H) Am
//                              (|conic| <= 1/0.3 from the 0.3 dilation; sup sqrt(q) e^(-q/2) = e^(-1/2))
//   class 3 conic              0.5 o G |d|^2 |dL/dalpha|           <= 0.041 r^2 Am
//                              (G |d|^2 <= (2/e) lambda_max(cov2D) <= (2/e) (r/3)^2)
// with Dm = max |dL/dout| and Am = (2 C Fm + |bg|_1) Dm >= |dL/dalpha|
// (|dot|, |S| <= C Fm Dm for Fm = max |feature|, T <= 1, T_final / (1 - alpha) <= T).
// s = 61 - e(nb) - e(bound): every partial and every sum stays below 2^61 in
// fixed units (frexp exponent e: x < 2^e); one rounding per partial, at 2^-s.
__device__ __forceinline__ int det_class_of(int f)
{
    return f < 2 ? 2 : (f < 5 ? 3 : (f == 5 ? 1 : 0));
}

__device__ __forceinline__ int det_shift(int cls, int r, float Dm, float Am, float WH)
{
    const float rr = (float)max(r, 1);
    const float q = fmaf(0.25f, rr, 2.f);
    const float B = cls == 0 ? 64.f * Dm : (cls == 1 ? 64.f * Am : (cls == 2 ? 40.f * WH * Am : 3.f * rr * rr * Am));
    int en = 0, eb = 0;
    (void)frexpf(q * q, &en);
    (void)frexpf(fmaxf(B, 1e-30f), &eb);
    return min(max(61 - en - eb, -100), 100);
}

// adds v at 2^s; a value outside the bound (never, by the analysis above) or a
// non-finite one flags the call instead (the conversion then writes NaN)
__device__ __forceinline__ void det_add(long long* p, float v, int s, uint32_t* flag)
{
    const float x = ldexpf(v, s);
    if (!(fabsf(x) < 0x1p61f)) {
        atomicOr(flag, 1u);
        return;
    }
    atomicAdd(reinterpret_cast<unsigned long long*>(p), (unsigned long long)__float2ll_rn(x));
}
// LO (language only): the autograd call needs dL/dlanguage alone (feature-mode
// training: geometry frozen, scene/gaussian_model.py:238-243, and means2D not
// requiring grad).  Then dL/dlang[j][c] = sum_p aT[j][p] dL/dout[c][p] is all
// that is left: no dot products, no dL/dalpha recurrence, no moments, and the
// rows go straight into the (N, D) output (b.grad_acc, b.VP = D).

// SP (with LO): the language input is the quick path's sparse (weights,
// codes) rows; the per-channel gradient rows are gathered at each Gaussian's
// codes into dL/dweights (b.qw_acc, (P, K)) instead of being added densely.
// LST: the candidates come from the forward's per-block list (RenderArgs::listA,
// lcount) instead of being re-staged from the tile list: no ids -> records
// gathers, no block tests, no compaction; the list chunks arrive by LDS-DMA one
// chunk ahead.  The same candidates in the same order: results unchanged.
template <int NL, bool LO = false, bool LD = false, bool SP = false, bool LST = false, bool DET = false>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(bwd_waves<NL, LD, LST, DET>()))) k_render_bwd_mf(RenderBwdArgs b)
{
    static_assert(!(LST && SP), "the sparse-input backward follows the quick forward (no lists)");
    static_assert(!(DET && SP), "the deterministic backward expands the sparse input (lsr_api backward_quick)");
    static_assert(!LO || NL > 0, "language-only backward needs D > 0");
    static_assert(!SP || LO, "the sparse-input gradient is a language-only backward");
    static_assert(!LD || (!LO && NL % 16 == 0), "direct dL/dlang needs whole 16-channel lines");
    using FR = BwdFrags<NL>;
    constexpr int KS = FR::KS;
    // LD implies D == NL (launch_render_bwd) and 16-B aligned rows (lsr_api)
    constexpr bool VEC = LD;
    // RREG (direct dL/dlang): the language lines' atomics take their values
    // straight from the MFMA accumulators, lane (li, lg) adding candidate
    // 4 lg + q's channel li (the C layout), so those rows skip LDS
    // (LO, not SP: every line is a language line, so all of them come
    // straight from the accumulators and the LDS row tile is not used)
    constexpr bool RREG = LD || (LO && !SP && LSR_BWD_LO_RREG);
    // MFMA channel blocks cover the language channels only; RGB (3) and the
    // six geometry moments are summed on the VALU (see phase 3)
    constexpr int NBC = (NL + 15) / 16;
    constexpr int NBA = NBC > 0 ? NBC : 1;
    __shared__ float2 sRG[64];        // dL/dout R, G of the block's pixels
    __shared__ float sBc[64];         // dL/dout B
    constexpr int GS = LSR_GRP_STRIDE;
    // the stage: re-staged tile-list candidates (!LST) or two list chunks (LST)
    __shared__ std::conditional_t<LST, WaveStageL, WaveStageG> stv;
    auto& st = stv;    // !LST
    auto& stl = stv;   // LST
    // first language column of a staged row; LD: the language lines start at
    // 16 and go to b.lang_acc, the first line (geometry + colour) to the row
    constexpr int GCOL0 = LO ? 0 : (LD ? 16 : LSR_GROW_LANG);
    constexpr int GRL = (GCOL0 + NL + 15) / 16;            // 16-float lines per gradient row
    constexpr int GRS = 16 * GRL + 4;                     // staged row stride
    // The gradient-row tile and the moments are written only after phase 3
    // has read dot/u and aT into registers (a wave's LDS operations complete
    // in order), so they share those buffers: 2.3-5.4 KB less LDS per wave,
    // 12 instead of 10 resident waves per CU at D = 16.
    constexpr int DUG = (16 * GS > 16 * GRS) ? 16 * GS : 16 * GRS;
    __shared__ float sDU[DUG];        // dot[k][p] -> u[k][p] -> the group's gradient rows
    __shared__ __attribute__((aligned(16))) float sAT[16 * GS];   // G[k][p] (phase 1) -> aT[k][p] (phase 2) -> moments
    static_assert(16 * LSR_MOM9_STRIDE <= 16 * GS, "moment rows must fit the aT tile");
    float* const sGr = sDU;
    float* const sMom = sAT;

    const RenderArgs& a = b.f;
    const Cam& c = a.cam;
    const WaveTile wt(a, LST ? a.border : nullptr);
    const int lane = threadIdx.x;
    const int lg = lane >> 4, li = lane & 15;
    const PixMap pm(c, wt.tile, lane + (wt.sub << 6));
    const bool inside = pm.px < c.W && pm.py < c.H;
    const float pfx = (float)pm.px, pfy = (float)pm.py;
    const float cx = (float)pm.bx + 3.5f, cy = (float)pm.by + 3.5f;
    const uint32_t rs = wt.ent ? wt.rs : a.tile_start[wt.tile];
    const size_t HW = (size_t)c.H * c.W;
    const size_t pix = (size_t)pm.py * c.W + pm.px;
    const int D = a.D;
    const int VP = b.VP;
    const float ddelx_dx = 0.5f * (float)c.W, ddely_dy = 0.5f * (float)c.H;
    // gradient rows (and LD: the language output) as raw buffers when every
    // byte offset fits 31 bits (uniform; otherwise 64-bit global atomics)
    const uint64_t nbg = (uint64_t)a.P * (uint64_t)VP * 4u;
    const uint64_t nbl = LD ? (uint64_t)a.P * (uint64_t)D * 4u : 0u;
    const bool buf_atom = nbg < (uint64_t)LSR_BUF_OOB && nbl < (uint64_t)LSR_BUF_OOB;
    const __amdgpu_buffer_rsrc_t rg =
        __builtin_amdgcn_make_buffer_rsrc(b.grad_acc, 0, (int)min(nbg, (uint64_t)LSR_BUF_OOB), 0x00020000);
    const __amdgpu_buffer_rsrc_t rl = __builtin_amdgcn_make_buffer_rsrc(
        LD ? b.lang_acc : b.grad_acc, 0, (int)min(LD ? nbl : nbg, (uint64_t)LSR_BUF_OOB), 0x00020000);

    const float T_final = inside ? a.final_T[pix] : 0.f;
    const int last = inside ? (int)a.n_contrib[pix] : 0;
    const int wmax = wave_max_i(last);
    if (wmax == 0) return;
    // Prologue order: the loads the first chunk's staging depends on (ids,
    // then records) are issued before the block's dL/dout fragments, so
    // waiting for them (vector-memory operations complete in issue order)
    // never waits for the 40 fragment loads; the lane's own RGB dL/dout is
    // loaded first among those, reaches LDS (sRG, sBc) just before the chunk
    // loop, and gives the background term without reloading it.
    // SPF: chunk c's ids are loaded two chunks ahead and its records one chunk
    // ahead, so staging never waits on a dependent gather (9 more VGPRs: off
    // for the widest language set, where they would spill)
    constexpr bool SPF = LSR_BWD_SPLAT_PF && NL <= 32;
    // tile-list position clamped to the range (wmax >= 1: position 0 exists), result selected
    auto pl_at = [&](int q) -> uint32_t { const uint32_t v = a.point_list[rs + max(q, 0)]; return q >= 0 ? v : 0u; };
    uint32_t gid1 = 0u, gid2 = 0u;
    float4 A1 = make_float4(0.f, 0.f, 0.f, 0.f), B1 = A1;
    // LST: entries [lbase, lbase + cnt) of the block's list, back to front
    const uint32_t lcnt = LST ? (wt.ent ? wt.lc : a.lcount[4 * wt.tile + wt.sub]) : 0u;
    const size_t lbase = LST ? (size_t)4 * rs + (size_t)wt.sub * ((wt.ent ? wt.re : a.tile_start[wt.tile + 1]) - rs) : 0;
    if constexpr (!LST) {
        gid1 = pl_at(wmax - 1 - lane);
        if constexpr (SPF) {
            gid2 = pl_at(wmax - 65 - lane);
            A1 = a.splatA[gid1];   // gid 0 for positions past the range: a valid record, never staged
            B1 = a.splatB[gid1];
        }
        // entries past a group's end are read unconditionally (immediate-offset
        // loads, no index clamps): keep them finite
        for (int e = lane; e < 80; e += 64) {
            st.A[e] = make_float4(0.f, 0.f, 0.f, 0.f);
            st.B[e] = make_float4(0.f, 0.f, 0.f, __int_as_float(0x7fffffff));
            st.gid[e] = 0u;
        }
    }
    // LST: chunk c0's entries lbase + lcnt - 1 - (c0 + lane) -> stl buffer `off`,
    // lanes < LSR_LST_CHUNK (lanes past the list copy entry 0: finite, and
    // past the group's end)
    auto list_dma = [&](int c0, int off) {
        const int e = (int)lcnt - 1 - (c0 + lane);
        const size_t src = lbase + (size_t)(e >= 0 ? e : 0);
        if (lane < LSR_LST_CHUNK) {
            glds16(a.listA + src, stl.A + off);
            glds16(a.listB + src, stl.B + off);
        }
    };

    float dr0 = 0.f, dr1 = 0.f, dr2 = 0.f;   // the lane's own pixel's RGB dL/dout (0 outside the image)
    if constexpr (!LO) {
        dr0 = gd_at<NL>(b, 0, lane, pm.bx, pm.by);
        dr1 = gd_at<NL>(b, 1, lane, pm.bx, pm.by);
        dr2 = gd_at<NL>(b, 2, lane, pm.bx, pm.by);
    }
    float dotB[KS][4], chB[NBA][16];
    // VEC: the dL/dout fragments through raw buffer descriptors when every
    // byte offset fits 31 bits (uniform): a fragment's offset is its
    // channel's plane plus the pixel's, and a pixel outside the image gets an
    // offset past both buffers (the load returns 0), so no clamps or selects
    const uint64_t HW4 = (uint64_t)HW * 4u;
    const bool gd_buf = VEC && HW4 * (uint64_t)(D > 3 ? D : 3) < 0x7fffffffull;
    if (VEC && gd_buf) {
        const __amdgpu_buffer_rsrc_t rcol = __builtin_amdgcn_make_buffer_rsrc((void*)b.dout_color, 0, (int)(HW4 * 3u), 0x00020000);
        const __amdgpu_buffer_rsrc_t rlng = __builtin_amdgcn_make_buffer_rsrc((void*)b.dout_lang, 0, (int)(HW4 * (uint64_t)D), 0x00020000);
        const uint32_t hw4 = (uint32_t)HW4;
        auto poff = [&](int q) -> uint32_t {
            const int qx = pm.bx + (q & 7), qy = pm.by + (q >> 3);
            return (qx < c.W && qy < c.H) ? (uint32_t)(qy * c.W + qx) * 4u : 0x80000000u;
        };
        auto ld = [&](__amdgpu_buffer_rsrc_t r, uint32_t off) {
            return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0));
        };
        uint32_t pa[4];
#pragma unroll
        for (int pb = 0; pb < 4; pb++) pa[pb] = poff(pb * 16 + li);
#pragma unroll
        for (int t = 0; t < KS; t++)
#pragma unroll
            for (int pb = 0; pb < 4; pb++) {
                if (t < NL / 4) {
                    const int chl = dot_channel<NL, VEC>(t, lg) - 3;   // a language channel
                    dotB[t][pb] = ld(rlng, (uint32_t)chl * hw4 + pa[pb]);
                } else {   // colour channel lg; lane group 3 none
                    dotB[t][pb] = ld(rcol, lg < 3 ? (uint32_t)lg * hw4 + pa[pb] : 0x80000000u);
                }
            }
#pragma unroll
        for (int nb = 0; nb < NBC; nb++)
#pragma unroll
            for (int t = 0; t < 16; t++) chB[nb][t] = ld(rlng, (uint32_t)(nb * 16 + li) * hw4 + poff(4 * t + lg));
    } else
    {
    if constexpr (!LO) {
#pragma unroll
        for (int t = 0; t < KS; t++)
#pragma unroll
            for (int pb = 0; pb < 4; pb++)
                dotB[t][pb] = gd_at<NL>(b, dot_channel<NL, VEC>(t, lg), pb * 16 + li, pm.bx, pm.by);
    }
#pragma unroll
    for (int nb = 0; nb < NBC; nb++)
#pragma unroll
        for (int t = 0; t < 16; t++)
            chB[nb][t] = gd_at<NL>(b, 3 + nb * 16 + li, 4 * t + lg, pm.bx, pm.by);
    }
    // block-centred x of the pixels this lane's fragments cover: columns lg
    // (even K-steps) and 4 + lg (odd K-steps)
    const float lxe = (float)lg - 3.5f, lxo = (float)lg + 0.5f;
    const float lxe2 = lxe * lxe, lxo2 = lxo * lxo;
    const float bg0 = c.bg[0], bg1 = c.bg[1], bg2 = c.bg[2];
    // dr* are the lane's own pixel's values (0 outside): 0 with a black
    // background, and the term below is then exact 0
    const float bg_dot = LO ? 0.f : bg0 * dr0 + bg1 * dr1 + bg2 * dr2;

    const bool has_bg = (bg0 != 0.f) || (bg1 != 0.f) || (bg2 != 0.f);   // uniform
    float T = T_final;
    float S = 0.f;

    // positions [0, wmax) back to front, 64 per chunk; candidates are processed
    // in groups of 16, a partial group carried into the next chunk
    int carry = 0;
    float af[KS];
    if constexpr (!LO) {
        sRG[lane] = make_float2(dr0, dr1);
        sBc[lane] = dr2;
    }
    // LST: a chunk's DMA is waited for with vmcnt(N), N = a lower bound of the
    // VMEM operations the previous (full, one-group) chunk issued after it --
    // its buffer atomics, GRL x 4 per group (unconditional, never merged; the
    // feature gathers are not counted) -- so the wait does not drain them
    // INVARIANT: the atomic loop below issues exactly GRL x 4
    // unconditional buffer atomics per group (masked lanes get an out-of-range
    // offset, never a branch), all after this chunk's DMA; the counted wait
    // relies on it.  Change that loop and this count together.
    constexpr int ATOMICS_PER_GROUP = GRL * 4;
    constexpr int OPG = ATOMICS_PER_GROUP;
    constexpr int CGR = LSR_LST_CHUNK / 16;   // groups per list chunk
    constexpr int CHUNK_OPS = CGR * OPG < 63 ? CGR * OPG : 63;
    constexpr int CH = LST ? LSR_LST_CHUNK : 64;   // candidates per chunk
    if constexpr (LST) list_dma(0, 0);
    const int cend = LST ? (int)lcnt : wmax;
    for (int c0 = 0; c0 < cend; c0 += CH) {
        int n, nfull;
        const float4* SA;
        const float4* SB;
        const uint32_t* SG;
        if constexpr (LST) {
            const int off = (c0 / CH & 1) * CH;
            // (DET: conditional 64-bit atomics, so no count of them: drain)
            if (c0 == 0 || !buf_atom || DET) wait_vmcnt<0>();
            else wait_vmcnt<CHUNK_OPS>();
            if (c0 + CH < cend) list_dma(c0 + CH, CH - off);
            n = nfull = min(CH, cend - c0);
            SA = stl.A + off;
            SB = stl.B + off;
            SG = reinterpret_cast<const uint32_t*>(stl.B + off) + 2;   // B.z, stride 4 words
        } else {
            const int p = wmax - 1 - (c0 + lane);
            const bool valid = p >= 0;
            if constexpr (SPF) {
                const uint32_t gid = gid1;
                const float4 Ac = A1, Bc = B1;
                gid1 = gid2;
                A1 = a.splatA[gid1];
                B1 = a.splatB[gid1];
                gid2 = pl_at(p - 128);
                n = carry + stage_candidates_geo_rec(st, carry, valid, gid, p, pm.bx, pm.by, Ac, Bc);
            } else {
                const uint32_t gid = gid1;
                gid1 = pl_at(p - 64);
                n = carry + stage_candidates_geo(st, carry, valid, gid, p, pm.bx, pm.by, a.splatA, a.splatB);
            }
            nfull = (c0 + 64 >= wmax) ? n : (n & ~15);
            SA = st.A;
            SB = st.B;
            SG = st.gid;
        }
        constexpr int SGS = LST ? 4 : 1;   // word stride of the id array

        for (int g0 = 0; g0 < nfull; g0 += 16) {
            const int kn = min(16, nfull - g0);
            // A fragments of the dot product: feature 4t+lg of candidate g0+li,
            // gathered now, consumed after phase 1
            if constexpr (!LO) {
                const uint32_t gi = SG[SGS * (g0 + (li < kn ? li : 0))];
                dot_features<NL, VEC>(a, gi, lg, af);
            }
            // phase 1: G of the 16 candidates (0 where the pair does not
            // contribute), independent across candidates; straight-line code.
            // The forward's exponent cut (power < B.z) needs no test here: below
            // it alpha < e^-0.02 / 255, far outside the fast exp's error band, so
            // the alpha test rejects those pairs.  Lanes in the band are collected
            // as a lane mask (scalar ORs), not per-lane flags.
            uint64_t near_m = 0u;
            const int kn_u = __builtin_amdgcn_readfirstlane(kn);   // uniform: scalar compares below
            // candidate li's opacity in lane li: phase 2 takes candidate k's
            // from lane k (v_readlane) instead of a broadcast LDS read per k
            const int opl = __float_as_int(SB[g0 + li].y);
#define BWD_OP(k) __int_as_float(__builtin_amdgcn_readlane(opl, (k)))
            // GREG: G stays in registers from phase 1 to phase 2 (no LDS round trip)
            float Gr[16];
            (void)Gr;
#pragma unroll
            for (int k = 0; k < 16; k++) {
                const float4 A = SA[g0 + k];
                const float4 B = SB[g0 + k];
                const float power = splat_power(A.z, A.w, B.x, A.x - pfx, A.y - pfy);
                const bool cj = (k < kn_u) && (__float_as_int(B.w) < last) && !(power > 0.0f);
                // G = 0 for a non-candidate pair: alpha - 1/255 is then far below the band
                const float G = cj ? __builtin_amdgcn_exp2f(power * LSR_LOG2E) : 0.f;
                const float d = fminf(0.99f, B.y * G) - (1.0f / 255.0f);
                near_m |= lanes_abs_lt(d, 2e-8f);
                Gr[k] = d >= 0.f ? G : 0.f;
            }
            if (near_m != 0u) {
                // the 1/255 decision must be the forward's: lanes inside the fast
                // exp's error band re-evaluate with the forward's exp (rare)
#pragma unroll
                for (int k = 0; k < 16; k++) {
                    if (k >= kn) break;
                    const int j = g0 + k;
                    const float4 A = SA[j];
                    const float4 B = SB[j];
                    const float power = splat_power(A.z, A.w, B.x, A.x - pfx, A.y - pfy);
                    const bool cj = (__float_as_int(B.w) < last) & !(power > 0.0f) & (LST || !(power < B.z));
                    const float af2 = fminf(0.99f, B.y * __builtin_amdgcn_exp2f(power * LSR_LOG2E));
                    if (cj & (fabsf(af2 - (1.0f / 255.0f)) < 2e-8f)) {
                        const float G = expf_det(power);
                        const float alpha = fminf(0.99f, B.y * G);
                        Gr[k] = !(alpha < 1.0f / 255.0f) ? G : 0.f;
                    }
                }
            }
            // dot[k][p] of the group's candidates on MFMA: (16 x C) . (C x 64)
            float dv[16];
            (void)dv;
            if constexpr (!LO) {
                f32x4 acc[4];
#pragma unroll
                for (int pb = 0; pb < 4; pb++) acc[pb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int t = 0; t < KS; t++)
#pragma unroll
                    for (int pb = 0; pb < 4; pb++)
                        acc[pb] = BWD_MFMA(af[t], dotB[t][pb], acc[pb]);
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    uint32_t x0 = __float_as_uint(acc[0][r]), x1 = __float_as_uint(acc[1][r]);
                    uint32_t x2 = __float_as_uint(acc[2][r]), x3 = __float_as_uint(acc[3][r]);
                    auto s02 = __builtin_amdgcn_permlane32_swap(x0, x2, false, false);
                    auto s13 = __builtin_amdgcn_permlane32_swap(x1, x3, false, false);
                    auto s01 = __builtin_amdgcn_permlane16_swap(s02[0], s13[0], false, false);
                    auto s23 = __builtin_amdgcn_permlane16_swap(s02[1], s13[1], false, false);
                    dv[0 + r] = __uint_as_float(s01[0]);
                    dv[4 + r] = __uint_as_float(s01[1]);
                    dv[8 + r] = __uint_as_float(s23[0]);
                    dv[12 + r] = __uint_as_float(s23[1]);
                }
            }
            wave_lds_fence();
            // phase 2: the serial back-to-front recurrence per pixel.  S is the
            // colour accumulated behind the current instance (the upstream
            // "accum_rec" once the last contributor is folded in):
            //   dL/dalpha_k = (dot_k - S) T_k,   S <- alpha_k dot_k + (1 - alpha_k) S
            // G = 0 marks a non-contributing pair: alpha = 0, rcp(1) = 1 and the
            // S update is an exact identity, so no selects are needed.
            if constexpr (LO) {
                // transmittance only: aT_k = alpha_k T_k (T_k recovered back to front)
#pragma unroll
                for (int k = 0; k < 16; k++) {
                    const float G = Gr[k];
                    const float al = fminf(0.99f, BWD_OP(k) * G);
                    T = T * __builtin_amdgcn_rcpf(1.f - al);
                    sAT[k * GS + lane] = al * T;
                }
            } else if (has_bg) {
#pragma unroll
                for (int k = 0; k < 16; k++) {
                    const float G = Gr[k];
                    const float dot = dv[k];
                    const float al = fminf(0.99f, BWD_OP(k) * G);
                    const float om = 1.f - al;
                    const float rcp = __builtin_amdgcn_rcpf(om);
                    T = T * rcp;
                    const float dL_dalpha = fmaf(-T_final * rcp, bg_dot, (dot - S) * T);
                    sDU[k * GS + lane] = dL_dalpha * G;
                    sAT[k * GS + lane] = al * T;
                    S = fmaf(al, dot, om * S);
                }
            } else {
#pragma unroll
                for (int k = 0; k < 16; k++) {
                    const float G = Gr[k];
                    const float dot = dv[k];
                    const float al = fminf(0.99f, BWD_OP(k) * G);
                    const float om = 1.f - al;
                    T = T * __builtin_amdgcn_rcpf(om);
                    sDU[k * GS + lane] = ((dot - S) * T) * G;
                    sAT[k * GS + lane] = al * T;
                    S = fmaf(al, dot, om * S);
                }
            }
            wave_lds_fence();
            // phase 3: language gradients on MFMA; RGB gradients and the six
            // pixel moments sum_p u {1, lx, ly, lx^2, lx ly, ly^2} on the VALU.
            // Lane (li, lg) reads candidate li's aT and u at pixel q = 4t + lg
            // (the MFMA A fragments) and keeps partial sums over its 16 pixels;
            // the four lane groups are then added.  Rows pair K-steps 2r
            // (columns lg) and 2r + 1 (columns 4 + lg) at ly = r - 3.5.
            f32x4 ch[NBA];
#pragma unroll
            for (int nb = 0; nb < NBA; nb++) ch[nb] = f32x4{0.f, 0.f, 0.f, 0.f};
            float M0 = 0.f, M1 = 0.f, M2 = 0.f, M3 = 0.f, M4 = 0.f, M5 = 0.f;
            float C0 = 0.f, C1 = 0.f, C2 = 0.f;
            float ue = 0.f;
            if constexpr (LO) {
#pragma unroll
                for (int t = 0; t < 16; t++) {
                    const float aa = sAT[li * GS + 4 * t + lg];
#pragma unroll
                    for (int nb = 0; nb < NBC; nb++) ch[nb] = BWD_MFMA(aa, chB[nb][t], ch[nb]);
                }
            } else {
#pragma unroll
            for (int t = 0; t < 16; t++) {
                const float au = sDU[li * GS + 4 * t + lg];
                const float aa = sAT[li * GS + 4 * t + lg];
#pragma unroll
                for (int nb = 0; nb < NBC; nb++) ch[nb] = BWD_MFMA(aa, chB[nb][t], ch[nb]);
                // (R, G) as one 8-B read + B as a 4-B read: 2 + 2 LDS cycles, where
                // the 12-B read of a float4's three used components (ds_read_b96) costs 8
                const float2 rg = sRG[4 * t + lg];
                const float4 d = make_float4(rg.x, rg.y, sBc[4 * t + lg], 0.f);
                C0 = fmaf(aa, d.x, C0);
                C1 = fmaf(aa, d.y, C1);
                C2 = fmaf(aa, d.z, C2);
                // lx is a lane constant per column parity (lxe even t, lxo odd t)
                // and ly a constant per t, so the six moments follow from the
                // column-parity sums of u, ly u and ly^2 u (3 VALU per t instead
                // of 11 per t pair; combined with lxe / lxo after the loop)
                const float ly = (float)(t >> 1) - 3.5f;
                if ((t & 1) == 0) {
                    M0 += au;
                    M2 = fmaf(ly, au, M2);
                    M5 = fmaf(ly * ly, au, M5);
                } else {
                    M1 += au;
                    M3 = fmaf(ly, au, M3);
                    M4 = fmaf(ly * ly, au, M4);
                }
            }
            {
                // (M0, M2, M5) = even-column sums of (u, ly u, ly^2 u); (M1, M3, M4) the odd columns'
                const float se = M0, so = M1, ye = M2, yo = M3, qe = M5, qo = M4;
                M0 = se + so;
                M1 = fmaf(lxe, se, lxo * so);
                M2 = ye + yo;
                M3 = fmaf(lxe2, se, lxo2 * so);
                M4 = fmaf(lxe, ye, lxo * yo);
                M5 = qe + qo;
            }
            // The nine partial sums over the four lane groups, reduced two at a
            // time: a permlane swap exchanges half of one value for half of
            // another, so swap + add halves two values' lane groups at once
            // (8 swaps + 8 adds instead of 18 xor-exchanges).  Row lg then holds
            // value slot s0(lg) of Y0 and 4 + s0(lg) of Y1 (slots: M0..M5, C0..C2);
            // the rows park them in the moment area (sAT is free once the loop
            // above has read it: a wave's LDS operations complete in order).
            {
                auto red32 = [](float x, float y) {
                    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(y), false, false);
                    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
                };
                auto red16 = [](float x, float y) {
                    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(y), false, false);
                    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
                };
                const float Y0 = red16(red32(M0, M1), red32(M2, M3));   // rows: M0 M2 M1 M3
                const float Y1 = red16(red32(M4, M5), red32(C0, C1));   // rows: M4 C0 M5 C1
                const float X4 = red32(C2, C2);
                const float Y2 = red16(X4, X4);                         // row 0: C2
                const int s0 = ((lg & 1) << 1) | (lg >> 1);
                float* const mr = sMom + li * LSR_MOM9_STRIDE;
                mr[s0] = Y0;
                mr[4 + s0] = Y1;
                if (lg == 0) mr[8] = Y2;
            }
            }
            // Gradient rows of the group staged in LDS (row layout of lsr_device.h:
            // [0..5] geometry, [6..8] colour, [12..) language), then added with
            // line-coalesced atomics: each 16-lane group covers one 64-B line of
            // one Gaussian's row.  Language: lane holds slot 4*lg+r, channel nb*16+li.
#pragma unroll
            for (int nb = 0; nb < (RREG ? 0 : NBC); nb++) {
                const int chn = nb * 16 + li;
                if (chn < NL) {
#pragma unroll
                    for (int r = 0; r < 4; r++) sGr[(4 * lg + r) * GRS + GCOL0 + chn] = ch[nb][r];
                }
            }
            if constexpr (!LO) wave_lds_fence();
            if (!LO && lane < kn) {   // lane = candidate li (lg = 0)
                const int j = g0 + lane;
                const float4 A = SA[j];
                const float4 B = SB[j];
                const float* const mr = sMom + lane * LSR_MOM9_STRIDE;
                const float4 m03 = *reinterpret_cast<const float4*>(mr);
                const float4 m47 = *reinterpret_cast<const float4*>(mr + 4);
                const float S0 = m03.x, S1 = m03.y, S2 = m03.z, S3 = m03.w, S4 = m47.x, S5 = m47.y;
                C0 = m47.z;
                C1 = m47.w;
                C2 = mr[8];
                const float X = A.x - cx, Y = A.y - cy;
                const float Sdx = fmaf(X, S0, -S1), Sdy = fmaf(Y, S0, -S2);
                const float Sdxx = fmaf(X, fmaf(X, S0, -2.f * S1), S3);
                const float Sdxy = fmaf(X, fmaf(Y, S0, -S2), fmaf(-Y, S1, S4));
                const float Sdyy = fmaf(Y, fmaf(Y, S0, -2.f * S2), S5);
                const float o = B.y;
                float* gr = sGr + lane * GRS;
                gr[0] = -o * ddelx_dx * fmaf(A.z, Sdx, A.w * Sdy);
                gr[1] = -o * ddely_dy * fmaf(B.x, Sdy, A.w * Sdx);
                gr[2] = -0.5f * o * Sdxx;
                gr[3] = -o * Sdxy;
                gr[4] = -0.5f * o * Sdyy;
                gr[5] = S0;
                gr[6] = C0;
                gr[7] = C1;
                gr[8] = C2;
            }
            wave_lds_fence();
            if constexpr (SP) {
                // (slot, code) pairs: dL/dw[gid][m] += row[slot][idx[gid][m]]
                const int K = a.K;
                for (int e = lane; e < 16 * K; e += 64) {
                    const int slot = e / K, m = e - slot * K;
                    if (slot < kn) {
                        const size_t off = (size_t)SG[SGS * (g0 + slot)] * K + m;
                        const int q = quick_index(a.qi, a.qidx_dtype, off);
                        if (q >= 0 && q < D) {
                            const float v = sGr[slot * GRS + GCOL0 + q];
                            if (v != 0.f) LSR_MF_ATOMIC(b.qw_acc + off, v);
                        }
                    }
                }
            } else {
                // every value and id the group's atomics need is read from LDS
                // first (one wait), then the atomics issue back to back
                uint32_t gq[4];
                float vq[GRL][4];
                // slot of the q-th atomic of this lane: 4q + lg, or (RREG) 4 lg + q
                auto slot_of = [&](int q) { return RREG ? 4 * lg + q : 4 * q + lg; };
#pragma unroll
                for (int q = 0; q < 4; q++) gq[q] = SG[SGS * (g0 + slot_of(q))];
#pragma unroll
                for (int h = 0; h < GRL; h++)
#pragma unroll
                    for (int q = 0; q < 4; q++) {
                        if (RREG && LO)
                            vq[h][q] = ch[h][q];
                        else if (RREG && h > 0)
                            vq[h][q] = ch[h - 1][q];
                        else
                            vq[h][q] = sGr[slot_of(q) * GRS + 16 * h + li];
                    }
                if constexpr (DET) {
                    // fixed-point twins of the rows (det_shift above): the same
                    // values, order-independent sums
                    uint32_t* const dflag = reinterpret_cast<uint32_t*>(b.det_bounds + 2);
                    uint32_t sq[4];
#pragma unroll
                    for (int q = 0; q < 4; q++) sq[q] = slot_of(q) < kn ? b.det_sh[gq[q]] : 0u;
#pragma unroll
                    for (int h = 0; h < GRL; h++) {
                        const int f = 16 * h + li;
                        const bool fcol = LO ? (f < D)
                                          : LD ? (h == 0 ? (f < 9) : (f - 16 < D))
                                               : ((f < 9) | ((f >= LSR_GROW_LANG) & (f < LSR_GROW_LANG + D)));
                        const int cls = LO ? 0 : ((LD && h > 0) ? 0 : det_class_of(f));
#pragma unroll
                        for (int q = 0; q < 4; q++) {
                            const float v = vq[h][q];
                            if (fcol & (slot_of(q) < kn) & (v != 0.f)) {
                                const int sh = (int)(int8_t)(sq[q] >> (8 * cls));
                                if (LD && h > 0)
                                    det_add(b.det_lang + (size_t)gq[q] * D + (f - 16), v, sh, dflag);
                                else
                                    det_add(b.det_rows + (size_t)gq[q] * VP + f, v, sh, dflag);
                            }
                        }
                    }
                } else if (buf_atom) {
                    // buffer atomics: 32-bit offsets, and a lane with nothing
                    // to add gets an offset past the buffer (the range check
                    // drops it: tools/micro/buf_oob_atomic.hip) instead of an
                    // exec-masked branch per atomic.  INVARIANT: exactly
                    // ATOMICS_PER_GROUP = GRL x 4 of them, unconditionally (the
                    // LST chunk wait above counts them as vmcnt operations)
                    static_assert(ATOMICS_PER_GROUP == GRL * 4, "the LST wait counts these atomics");
#pragma unroll
                    for (int h = 0; h < GRL; h++) {
                        const int f = 16 * h + li;
                        const bool fcol = LO ? (f < D)
                                          : LD ? (h == 0 ? (f < 9) : (f - 16 < D))
                                               : ((f < 9) | ((f >= LSR_GROW_LANG) & (f < LSR_GROW_LANG + D)));
#pragma unroll
                        for (int q = 0; q < 4; q++) {
                            const float v = vq[h][q];
                            const bool on = fcol & (slot_of(q) < kn) & (v != 0.f);
                            if (LD && h > 0) {
                                const int off = (int)(gq[q] * (uint32_t)D + (uint32_t)(f - 16)) * 4;
                                __builtin_amdgcn_raw_ptr_buffer_atomic_fadd_f32(v, rl, on ? off : LSR_BUF_OOB, 0, 0);
                            } else {
                                const int off = (int)(gq[q] * (uint32_t)VP + (uint32_t)f) * 4;
                                __builtin_amdgcn_raw_ptr_buffer_atomic_fadd_f32(v, rg, on ? off : LSR_BUF_OOB, 0, 0);
                            }
                        }
                    }
                } else
#pragma unroll
                for (int h = 0; h < GRL; h++) {
                    const int f = 16 * h + li;
                    const bool fcol = LO ? (f < D)
                                      : LD ? (h == 0 ? (f < 9) : (f - 16 < D))
                                           : ((f < 9) | ((f >= LSR_GROW_LANG) & (f < LSR_GROW_LANG + D)));
#pragma unroll
                    for (int q = 0; q < 4; q++) {
                        const float v = vq[h][q];
                        if (fcol & (slot_of(q) < kn) & (v != 0.f)) {
                            if (LD && h > 0)
                                LSR_MF_ATOMIC(b.lang_acc + (size_t)gq[q] * D + (f - 16), v);
                            else
                                LSR_MF_ATOMIC(b.grad_acc + (size_t)gq[q] * VP + f, v);
                        }
                    }
                }
            }
            wave_lds_fence();
        }
        // carry the partial group to the front of the stage
        if constexpr (!LST) {
            carry = n - nfull;
            if (nfull > 0 && lane < carry) {   // source >= 16 > destination: no overlap
                st.A[lane] = st.A[nfull + lane];
                st.B[lane] = st.B[nfull + lane];
                st.gid[lane] = st.gid[nfull + lane];
            }
        }
        wave_lds_fence();
    }
}


hipError_t launch_render_bwd_lang(const RenderBwdArgs& b, hipStream_t st)
{
    const int T = b.f.cam.gx * b.f.cam.gy;
    if (T == 0) return hipSuccess;
    if (b.det_rows && (!b.det_bounds || !b.det_sh)) return hipErrorInvalidValue;
    // LST: the forward's per-block candidate lists (RenderArgs::listA); DET: fixed-point sums
#define LSR_BWD_LO(NL)                                                                                           \
    (b.det_rows ? (b.f.listA ? k_render_bwd_mf<NL, true, false, false, true, true><<<4 * T, 64, 0, st>>>(b)     \
                             : k_render_bwd_mf<NL, true, false, false, false, true><<<4 * T, 64, 0, st>>>(b))   \
                : (b.f.listA ? k_render_bwd_mf<NL, true, false, false, true><<<4 * T, 64, 0, st>>>(b)           \
                             : k_render_bwd_mf<NL, true><<<4 * T, 64, 0, st>>>(b)))
    switch (lang_set_for(b.f.D)) {
        case 4: LSR_BWD_LO(4); break;
        case 8: LSR_BWD_LO(8); break;
        case 16: LSR_BWD_LO(16); break;
        case 32: LSR_BWD_LO(32); break;
        case 64: LSR_BWD_LO(64); break;
        default: return hipErrorInvalidValue;
    }
#undef LSR_BWD_LO
    return hipGetLastError();
}

hipError_t launch_render_bwd_lang_sparse(const RenderBwdArgs& b, hipStream_t st)
{
    const int T = b.f.cam.gx * b.f.cam.gy;
    if (T == 0) return hipSuccess;
    if (!b.qw_acc || !b.f.qi || b.f.K <= 0) return hipErrorInvalidValue;
    switch (lang_set_for(b.f.D)) {
        case 4: k_render_bwd_mf<4, true, false, true><<<4 * T, 64, 0, st>>>(b); break;
        case 8: k_render_bwd_mf<8, true, false, true><<<4 * T, 64, 0, st>>>(b); break;
        case 16: k_render_bwd_mf<16, true, false, true><<<4 * T, 64, 0, st>>>(b); break;
        case 32: k_render_bwd_mf<32, true, false, true><<<4 * T, 64, 0, st>>>(b); break;
        case 64: k_render_bwd_mf<64, true, false, true><<<4 * T, 64, 0, st>>>(b); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}


bool bwd_lang_direct(int D)
{
    return D == 16 || D == 32;
}

hipError_t launch_render_bwd(const RenderBwdArgs& b, hipStream_t st)
{
    const int T = b.f.cam.gx * b.f.cam.gy;
    if (T == 0) return hipSuccess;
    // LST: the forward's per-block candidate lists (RenderArgs::listA)
    const bool lst = b.f.listA != nullptr;
    const bool det = b.det_rows != nullptr;
    if (det && (!b.det_bounds || !b.det_sh || ((b.lang_acc != nullptr) != (b.det_lang != nullptr))))
        return hipErrorInvalidValue;
    if (b.lang_acc) {
        if (!bwd_lang_direct(b.f.D) || (uintptr_t)b.f.lang % 16 != 0) return hipErrorInvalidValue;
        if (b.f.D == 16) {
            if (det) {
                if (lst) k_render_bwd_mf<16, false, true, false, true, true><<<4 * T, 64, 0, st>>>(b);
                else k_render_bwd_mf<16, false, true, false, false, true><<<4 * T, 64, 0, st>>>(b);
            } else if (lst) k_render_bwd_mf<16, false, true, false, true><<<4 * T, 64, 0, st>>>(b);
            else k_render_bwd_mf<16, false, true><<<4 * T, 64, 0, st>>>(b);
        } else {
            if (det) {
                if (lst) k_render_bwd_mf<32, false, true, false, true, true><<<4 * T, 64, 0, st>>>(b);
                else k_render_bwd_mf<32, false, true, false, false, true><<<4 * T, 64, 0, st>>>(b);
            } else if (lst) k_render_bwd_mf<32, false, true, false, true><<<4 * T, 64, 0, st>>>(b);
            else k_render_bwd_mf<32, false, true><<<4 * T, 64, 0, st>>>(b);
        }
        return hipGetLastError();
    }
#define LSR_BWD_FULL(NL)                                                                                 \
    (det ? (lst ? k_render_bwd_mf<NL, false, false, false, true, true><<<4 * T, 64, 0, st>>>(b)          \
                : k_render_bwd_mf<NL, false, false, false, false, true><<<4 * T, 64, 0, st>>>(b))        \
         : (lst ? k_render_bwd_mf<NL, false, false, false, true><<<4 * T, 64, 0, st>>>(b)                \
                : k_render_bwd_mf<NL><<<4 * T, 64, 0, st>>>(b)))
    switch (lang_set_for(b.f.D)) {
        case 0: LSR_BWD_FULL(0); break;
        case 4: LSR_BWD_FULL(4); break;
        case 8: LSR_BWD_FULL(8); break;
        case 16: LSR_BWD_FULL(16); break;
        case 32: LSR_BWD_FULL(32); break;
        case 64: LSR_BWD_FULL(64); break;
        default: return hipErrorInvalidValue;
    }
#undef LSR_BWD_FULL
    return hipGetLastError();
}


// ------------------------------------------ deterministic backward: bounds
// max |dL/dout| over the 3 + D upstream planes and max |feature| over the
// visible Gaussians' colours and the dense language input (order-independent);
// bit 0 of word 2 flags a non-finite value.  Blocks [0, nbd) read the three
// arrays as one float4 index space, 8 loads in flight per lane (a strided loop
// per array left a chain of dependent rounds); blocks below gridDim - nbd take
// one visible Gaussian's row per thread.
__device__ __forceinline__ void det_max4(float4 v, float& m, bool& bad)
{
    bad |= !(isfinite(v.x) && isfinite(v.y) && isfinite(v.z) && isfinite(v.w));
    m = fmaxf(m, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
}

__global__ void __launch_bounds__(256) k_det_bounds(const float* __restrict__ dc, const float* __restrict__ dl,
                                                    uint32_t ncol, uint32_t nlang, int nbd,
                                                    const float* __restrict__ lang, uint32_t nfeat,
                                                    const float* __restrict__ rgb, const int32_t* __restrict__ radii,
                                                    int P, float* bounds)
{
    float md = 0.f, mf = 0.f;
    bool bad = false;
    // the colour blocks first (their dependent radius -> colour loads then
    // overlap the stream instead of trailing it)
    const int nbf = (int)gridDim.x - nbd;
    const int blk = (int)blockIdx.x - nbf;
    if (blk >= 0) {
        // float4 parts of the aligned arrays: [colour planes | language planes | language input]
        auto n4 = [](const float* p, uint32_t n) { return (p && ((uintptr_t)p & 15u) == 0) ? n / 4 : 0u; };
        const uint32_t N1 = n4(dc, ncol), N2 = N1 + n4(dl, nlang), N3 = N2 + n4(lang, nfeat);
        const float4* c4 = reinterpret_cast<const float4*>(dc);
        const float4* l4 = reinterpret_cast<const float4*>(dl);
        const float4* f4 = reinterpret_cast<const float4*>(lang);
        // block chunks of 4 x 256 consecutive float4 (a copy's access pattern)
        const uint32_t nch = (N3 + 1023) / 1024;
        for (uint32_t ch = (uint32_t)blk; ch < nch; ch += (uint32_t)nbd) {
            float4 v[4];
            uint32_t ec[4];
#pragma unroll
            for (int k = 0; k < 4; k++) {
                // branch-free: past the end, lanes re-read the last element (a
                // real one, counted where it belongs)
                ec[k] = min(ch * 1024u + (uint32_t)k * 256u + threadIdx.x, N3 - 1);
                const float4* q = ec[k] < N1 ? c4 + ec[k] : (ec[k] < N2 ? l4 + (ec[k] - N1) : f4 + (ec[k] - N2));
                v[k] = *q;
            }
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const bool isd = ec[k] < N2;
                float m = isd ? md : mf;
                det_max4(v[k], m, bad);
                md = isd ? m : md;
                mf = isd ? mf : m;
            }
        }
        const uint32_t stride = (uint32_t)nbd * blockDim.x, b0 = (uint32_t)blk * blockDim.x + threadIdx.x;
        // the scalar rest: tails past the float4 parts, or a whole misaligned array
        auto rest = [&](const float* p, uint32_t n, float& m) {
            if (!p) return;
            for (uint32_t e = 4 * n4(p, n) + b0; e < n; e += stride) {
                const float x = p[e];
                bad |= !isfinite(x);
                m = fmaxf(m, fabsf(x));
            }
        };
        rest(dc, ncol, md);
        rest(dl, nlang, md);
        rest(lang, nfeat, mf);
    } else {
        // the colours of the visible Gaussians (a culled Gaussian's colour is never written)
        const int stride = nbf * (int)blockDim.x;
        for (int i = (int)blockIdx.x * (int)blockDim.x + (int)threadIdx.x; i < P; i += stride) {
            if (radii[i] <= 0) continue;
            for (int c = 0; c < 3; c++) {
                const float v = rgb[3 * (size_t)i + c];
                bad |= !isfinite(v);
                mf = fmaxf(mf, fabsf(v));
            }
        }
    }
    // the block's partial to its own slot (same-address atomics serialise: one
    // per wave over ~6 K blocks cost 0.3 ms, one per block over 1.3 K 0.05 ms);
    // k_det_reduce folds the slots
    __shared__ float smd[4], smf[4];
    __shared__ uint32_t sbad[4];
    md = wave_max_f(md);
    mf = wave_max_f(mf);
    const bool wbad = wave_ballot(bad) != 0u;
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        smd[w] = md;
        smf[w] = mf;
        sbad[w] = wbad ? 1u : 0u;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        float* part = bounds + 64;
        part[blockIdx.x] = fmaxf(fmaxf(smd[0], smd[1]), fmaxf(smd[2], smd[3]));
        part[LSR_DET_BLOCKS + blockIdx.x] = fmaxf(fmaxf(smf[0], smf[1]), fmaxf(smf[2], smf[3]));
        reinterpret_cast<uint32_t*>(part)[2 * LSR_DET_BLOCKS + blockIdx.x] = sbad[0] | sbad[1] | sbad[2] | sbad[3];
    }
}

// per Gaussian, det_shift of the four column classes as signed bytes (the
// adds and the conversion read the same table, so their exponents agree by
// construction)
__global__ void __launch_bounds__(256) k_det_shifts(const int32_t* __restrict__ radii, const float* __restrict__ bounds,
                                                    int P, int D, const float* __restrict__ bg, float WH,
                                                    uint32_t* __restrict__ sh)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P) return;
    const float Dm = bounds[0];
    const float Am = (2.f * (float)(3 + D) * bounds[1] + (fabsf(bg[0]) + fabsf(bg[1]) + fabsf(bg[2]))) * Dm;
    const int r = radii[i];
    uint32_t w = 0u;
#pragma unroll
    for (int cls = 0; cls < 4; cls++) w |= ((uint32_t)det_shift(cls, r, Dm, Am, WH) & 0xffu) << (8 * cls);
    sh[i] = w;
}

// one block: the nb partials -> bounds[0..2]
__global__ void __launch_bounds__(1024) k_det_reduce(float* bounds, int nb)
{
    const float* part = bounds + 64;
    float md = 0.f, mf = 0.f;
    uint32_t bad = 0u;
    for (int i = threadIdx.x; i < nb; i += blockDim.x) {
        md = fmaxf(md, part[i]);
        mf = fmaxf(mf, part[LSR_DET_BLOCKS + i]);
        bad |= reinterpret_cast<const uint32_t*>(part)[2 * LSR_DET_BLOCKS + i];
    }
    __shared__ float smd[16], smf[16];
    __shared__ uint32_t sbad[16];
    md = wave_max_f(md);
    mf = wave_max_f(mf);
    const bool wbad = wave_ballot(bad != 0u) != 0u;
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        smd[w] = md;
        smf[w] = mf;
        sbad[w] = wbad ? 1u : 0u;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        const int nw = (int)(blockDim.x + 63) / 64;
        for (int k = 1; k < nw; k++) {
            md = fmaxf(md, smd[k]);
            mf = fmaxf(mf, smf[k]);
            sbad[0] |= sbad[k];
        }
        bounds[0] = md;
        bounds[1] = mf;
        reinterpret_cast<uint32_t*>(bounds)[2] = sbad[0];
    }
}

hipError_t launch_det_bounds(const RenderBwdArgs& b, float* bounds, hipStream_t st)
{
    const size_t HW = (size_t)b.f.cam.W * b.f.cam.H;
    const int D = b.f.D;
    if (D > 0 && (!b.dout_lang || !b.f.lang)) return hipErrorInvalidValue;
    if (!b.det_sh || !b.radii) return hipErrorInvalidValue;
    const size_t nf = (size_t)b.f.P * (size_t)(D > 0 ? D : 0);
    if (3 * HW >= (1ull << 32) || (size_t)D * HW >= (1ull << 32) || nf >= (1ull << 32)) return hipErrorInvalidValue;
    // one 16-KB chunk per scan block; one Gaussian per colour thread
    const size_t n4 = (3 * HW + (size_t)D * HW + nf) / 4;
    const int nbd = (int)std::max<size_t>(1, std::min<size_t>((n4 + 1023) / 1024, LSR_DET_BLOCKS - LSR_DET_BLOCKS / 4));
    const int nbf = std::max(1, std::min((b.f.P + 255) / 256, LSR_DET_BLOCKS / 4));
    k_det_bounds<<<nbd + nbf, 256, 0, st>>>(b.dout_color, D > 0 ? b.dout_lang : nullptr, (uint32_t)(3 * HW),
                                            (uint32_t)((size_t)D * HW), nbd, D > 0 ? b.f.lang : nullptr,
                                            (uint32_t)nf, b.f.rgb, b.radii, b.f.P, bounds);
    k_det_reduce<<<1, 1024, 0, st>>>(bounds, nbd + nbf);
    if (b.f.P > 0)
        k_det_shifts<<<(b.f.P + 255) / 256, 256, 0, st>>>(b.radii, bounds, b.f.P, D, b.f.cam.bg,
                                                          (float)std::max(b.f.cam.W, b.f.cam.H), b.det_sh);
    return hipGetLastError();
}

// ---------------------------------------- deterministic backward: to fp32
// mode 0: rows (P, VP) generic layout ([0..8] geometry + colour, [12, 12 + D)
// language) -> gout; mode 1 (lang_direct): rows (P, 16) -> gout, lang (P, D)
// -> lout; mode 2 (language only): rows (P, D) -> lout.  Every element of the
// outputs is written (unused row slots 0).  One thread per (Gaussian, 4
// columns), 32-bit index arithmetic.
__device__ __forceinline__ float det_value(long long acc, int s)
{
    return acc != 0 ? (float)ldexp((double)acc, -s) : 0.f;
}

__global__ void __launch_bounds__(256) k_det_finish(const long long* __restrict__ rows,
                                                    const long long* __restrict__ lang,
                                                    const uint32_t* __restrict__ shifts,
                                                    const float* __restrict__ bounds, int P, int VP, int D, int mode,
                                                    float* __restrict__ gout, float* __restrict__ lout)
{
    // column quads per Gaussian: the row part, then (mode 1) the language part
    const int wr = mode == 2 ? D : VP;
    const int qr = (wr + 3) / 4;
    const int ql = mode == 1 ? (D + 3) / 4 : 0;
    const int qn = qr + ql;
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t i = t / (uint32_t)qn;
    if (i >= (uint32_t)P) return;
    const int q = (int)(t - i * (uint32_t)qn);
    const bool bad = (__float_as_uint(bounds[2]) & 1u) != 0u;
    const uint32_t sw = shifts[i];   // the exponents the adds used
    const bool in_rows = q < qr;
    const int c0 = 4 * (in_rows ? q : q - qr);
    const int w = in_rows ? wr : D;
    const long long* src = (in_rows ? rows : lang) + (size_t)i * w;
    float* dst = (in_rows && mode != 2 ? gout : lout) + (size_t)i * w;
    float v[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int col = c0 + k;
        int cls = 0;
        bool used = col < w;
        if (in_rows && mode != 2) {
            used = used && (col < 9 || (mode == 0 && col >= LSR_GROW_LANG && col < LSR_GROW_LANG + D));
            cls = det_class_of(col);
        }
        const long long acc = used ? src[col] : 0;
        v[k] = bad ? __builtin_nanf("") : det_value(acc, (int)(int8_t)(sw >> (8 * cls)));
    }
    if (c0 + 4 <= w && ((uintptr_t)(dst + c0) & 15u) == 0) {
        *reinterpret_cast<float4*>(dst + c0) = make_float4(v[0], v[1], v[2], v[3]);
    } else {
#pragma unroll
        for (int k = 0; k < 4; k++)
            if (c0 + k < w) dst[c0 + k] = v[k];
    }
}

hipError_t launch_det_finish(const RenderBwdArgs& b, bool lang_only, float* grad_out, float* lang_out, hipStream_t st)
{
    const int P = b.f.P, D = b.f.D;
    const int mode = lang_only ? 2 : (b.det_lang ? 1 : 0);
    if (!b.det_rows || !b.det_bounds || !b.det_sh || (mode == 0 && !grad_out) || (mode != 0 && !lang_out) ||
        (mode == 1 && !grad_out))
        return hipErrorInvalidValue;
    const int wr = mode == 2 ? D : b.VP;
    const int qn = (wr + 3) / 4 + (mode == 1 ? (D + 3) / 4 : 0);
    const size_t n = (size_t)P * (size_t)qn;
    if (n == 0) return hipSuccess;
    if (n >= (1ull << 32)) return hipErrorInvalidValue;
    k_det_finish<<<(unsigned)((n + 255) / 256), 256, 0, st>>>(b.det_rows, b.det_lang, b.det_sh, b.det_bounds, P, b.VP,
                                                              D, mode, grad_out, lang_out);
    return hipGetLastError();
}
}  // namespace lsr
