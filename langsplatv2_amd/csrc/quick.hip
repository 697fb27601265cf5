// quick.hip — codebook decode of the sparse "quick" language map
// (SURVEY.md §8f rank 1).  Replaces, after render(), the reference's
//   W = weight_map.view(L, K, H*W)
//   F = einsum('ldk,lkn->ldn', codebooks.permute(0, 2, 1), W)   (L, Df, H*W)
//   F = F / (F.norm(dim=1, keepdim=True) + 1e-10)
// (eval_lerf.py:210-220, backend_renderer.py:16-36) and, with L = 1 and no
// normalisation, compute_final_feature_map (scene/gaussian_model.py:545-550).
//
// The decode is a dense f32 GEMM (Df x K) . (K x pixels) per level and runs on
// v_mfma_f32_16x16x4_f32.  One wave owns a 16x4-pixel block (each output row
// segment is a full 64-B line) and holds the block's K x 64 weight tile in
// registers in the MFMA output layout; the K-order of every contraction is
// chosen so that the same registers serve as the B operand of both products:
//   norm^2[p] = w_p^T G w_p with G = CB CB^T (K x K, one small GEMM per call):
//               H = G W on MFMA, then an elementwise product with W and a
//               reduction over the four lane groups — 1/8 of the decode's MFMAs,
//               so each output is written exactly once, already normalised;
//   F = CB^T W: 16 K-steps x 4 pixel blocks per 16 output dims.
#include "lsr_internal.h"

namespace lsr {

typedef float f32x4q __attribute__((ext_vector_type(4)));

// G[l][k][k2] = sum_d CB[l][k][d] * CB[l][k2][d]
__global__ void __launch_bounds__(256) k_codebook_gram(const float* __restrict__ cb, int K, int Df,
                                                       float* __restrict__ G)
{
    const int l = blockIdx.y;
    const int idx = blockIdx.x * 256 + threadIdx.x;
    if (idx >= K * K) return;
    const int k = idx / K, k2 = idx % K;
    const float* a = cb + ((size_t)l * K + k) * Df;
    const float* b = cb + ((size_t)l * K + k2) * Df;
    float s = 0.f;
    for (int d = 0; d < Df; d++) s = fmaf(a[d], b[d], s);
    G[(size_t)l * K * K + idx] = s;
}

template <int K>
__global__ void __launch_bounds__(64) k_quick_decode(const float* __restrict__ wmap, int L, int Df, int W, int H,
                                                     const float* __restrict__ cb, const float* __restrict__ G,
                                                     float* __restrict__ out, float eps, int normalize)
{
    constexpr int KB = K / 16;
    const int lane = threadIdx.x, lg = lane >> 4, li = lane & 15;
    const int nbx = (W + 15) / 16;
    const int bx = (int)(blockIdx.x % nbx) * 16, by = (int)(blockIdx.x / nbx) * 4;
    const size_t HW = (size_t)W * H;
    bool inp[4];
    size_t pixo[4];
#pragma unroll
    for (int pb = 0; pb < 4; pb++) {
        const int x = bx + li, y = by + pb;
        inp[pb] = x < W && y < H;
        pixo[pb] = inp[pb] ? (size_t)y * W + x : 0;
    }
    for (int l = 0; l < L; l++) {
        // weight tile, MFMA output layout: Wt[kb][r][pb] = w[l*K + kb*16 + 4*lg + r][pixel (pb, li)]
        float Wt[KB][4][4];
#pragma unroll
        for (int kb = 0; kb < KB; kb++)
#pragma unroll
            for (int r = 0; r < 4; r++)
#pragma unroll
                for (int pb = 0; pb < 4; pb++)
                    Wt[kb][r][pb] = inp[pb] ? wmap[(size_t)(l * K + kb * 16 + 4 * lg + r) * HW + pixo[pb]] : 0.f;
        float inv[4] = {1.f, 1.f, 1.f, 1.f};
        if (normalize) {
            const float* Gl = G + (size_t)l * K * K;
            float part[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int kb = 0; kb < KB; kb++) {
                f32x4q h[4];
#pragma unroll
                for (int pb = 0; pb < 4; pb++) h[pb] = f32x4q{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int kb2 = 0; kb2 < KB; kb2++)
#pragma unroll
                    for (int r2 = 0; r2 < 4; r2++) {
                        const float a = Gl[(kb * 16 + li) * K + kb2 * 16 + 4 * lg + r2];
#pragma unroll
                        for (int pb = 0; pb < 4; pb++)
                            h[pb] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, Wt[kb2][r2][pb], h[pb], 0, 0, 0);
                    }
#pragma unroll
                for (int pb = 0; pb < 4; pb++)
#pragma unroll
                    for (int r = 0; r < 4; r++) part[pb] = fmaf(Wt[kb][r][pb], h[pb][r], part[pb]);
            }
            // sum over the four lane groups (lanes li, li+16, li+32, li+48)
#pragma unroll
            for (int pb = 0; pb < 4; pb++) {
                float v = part[pb];
                v += __shfl_xor(v, 16, 64);
                v += __shfl_xor(v, 32, 64);
                inv[pb] = 1.f / (sqrtf(fmaxf(v, 0.f)) + eps);
            }
        }
        // F[d][p] = sum_k CB[l][k][d] W[k][p], 16 output dims per pass
        const float* CBl = cb + (size_t)l * K * Df;
        float an[KB][4];
#pragma unroll
        for (int kb = 0; kb < KB; kb++)
#pragma unroll
            for (int r = 0; r < 4; r++) an[kb][r] = CBl[(size_t)(kb * 16 + 4 * lg + r) * Df + li];
        for (int rb = 0; rb < Df / 16; rb++) {
            float ac[KB][4];
#pragma unroll
            for (int kb = 0; kb < KB; kb++)
#pragma unroll
                for (int r = 0; r < 4; r++) ac[kb][r] = an[kb][r];
            if (rb + 1 < Df / 16) {   // prefetch the next 16 dims' A fragments
#pragma unroll
                for (int kb = 0; kb < KB; kb++)
#pragma unroll
                    for (int r = 0; r < 4; r++) an[kb][r] = CBl[(size_t)(kb * 16 + 4 * lg + r) * Df + (rb + 1) * 16 + li];
            }
            f32x4q f[4];
#pragma unroll
            for (int pb = 0; pb < 4; pb++) f[pb] = f32x4q{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int kb = 0; kb < KB; kb++)
#pragma unroll
                for (int r = 0; r < 4; r++)
#pragma unroll
                    for (int pb = 0; pb < 4; pb++)
                        f[pb] = __builtin_amdgcn_mfma_f32_16x16x4f32(ac[kb][r], Wt[kb][r][pb], f[pb], 0, 0, 0);
            // lane holds F[rb*16 + 4*lg + r][pixel (pb, li)]
#pragma unroll
            for (int pb = 0; pb < 4; pb++)
                if (inp[pb]) {
#pragma unroll
                    for (int r = 0; r < 4; r++)
                        out[(size_t)(l * Df + rb * 16 + 4 * lg + r) * HW + pixo[pb]] = f[pb][r] * inv[pb];
                }
        }
    }
}

// ---------------------------------------------------------------------------
// Split-f16 decode (default).  The f32 MFMA above runs at 1/16 of the f16 rate
// and made the decode matrix-core bound (3.7 ms at 1 Mpix, 3 levels; the
// output is 6.3 GB, 1.05 ms at 6 TB/s).  Here every f32 operand x is split
// into x_hi = f16(x), x_lo = f16(x - x_hi) (22 significant bits together) and
//   F = W_hi C_hi + W_hi C_lo + W_lo C_hi
// runs on v_mfma_f32_16x16x32_f16 with f32 accumulation: the products are
// exact in f32, the dropped W_lo C_lo term is <= 2^-22 |W||C|, i.e. within a
// few f32 ulps of the exact-f32 decode.  The codebook is scaled per level by a
// power of two into [0.5, 1) before the split (f16 range; exact) and the
// scale is applied to the results.
//
// Orientation: A = W^T (rows = 16 pixels along x, K = codes), B = codebook
// (K = codes, cols = 16 output dims), so a lane's result is 4 CONSECUTIVE
// pixels of one output dim: one 16-B store per lane, each store instruction a
// full 64-B segment per dim.  The L2 norm needs |F_p| before any dim of pixel
// p is written: |F_p|^2 = w_p^T G w_p with the level's Gram matrix
// G = CB CB^T (64 x 64, exact f32, k_codebook_gram), H^T = W^T G on the same
// split-f16 MFMA with the same A fragments (1/8 of the decode's matrix work),
// then sum_m W[m][p] H[m][p] with W re-read as 16-B rows and a 16-lane sum.
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
#ifndef LSR_DEC_PB
#define LSR_DEC_PB 4      // 16-pixel blocks whose A fragments stay in registers across the dim blocks
#endif
#ifndef LSR_DEC_WAVES
#define LSR_DEC_WAVES 2   // min waves per SIMD (caps VGPRs at 256; 176 used); uncapped it took 214 = 1 wave
#endif

// Fragments: frag[(((l * NDB + db) * 2 + s) * 64 + lane) * 2 + {0: hi, 1: lo}] holds, for lane
// (li = lane & 15, lg = lane >> 4), B[k = 8 lg + j][col li] of K-step s and dim block db:
// scale_l * CB[l][32 s + 8 lg + j][16 db + li], j = 0..7, split into f16 hi / lo.
// scales[l] = 1 / scale_l.  One workgroup per level.
__global__ void __launch_bounds__(256) k_codebook_frag(const float* __restrict__ cb, int K, int Df,
                                                       uint4* __restrict__ frag, float* __restrict__ scales)
{
    const int l = blockIdx.x;
    const float* c = cb + (size_t)l * K * Df;
    __shared__ float red[256];
    float m = 0.f;
    for (int i = threadIdx.x; i < K * Df; i += 256) m = fmaxf(m, fabsf(c[i]));
    red[threadIdx.x] = m;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) red[threadIdx.x] = fmaxf(red[threadIdx.x], red[threadIdx.x + w]);
        __syncthreads();
    }
    const float mx = red[0];
    int e = 0;
    if (mx > 0.f && mx < 3.0e38f) (void)frexpf(mx, &e);   // mx = f 2^e, f in [0.5, 1)
    const float scale = ldexpf(1.f, -e);
    if (threadIdx.x == 0) scales[l] = ldexpf(1.f, e);
    const int NDB = Df / 16;
    for (int idx = threadIdx.x; idx < NDB * 128; idx += 256) {
        const int lane = idx & 63, s = (idx >> 6) & 1, db = idx >> 7;
        const int li = lane & 15, lg = lane >> 4;
        h8 hi, lo;
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const float v = c[(size_t)(32 * s + 8 * lg + j) * Df + 16 * db + li] * scale;
            const _Float16 h = (_Float16)v;
            hi[j] = h;
            lo[j] = (_Float16)(v - (float)h);
        }
        uint4* dst = frag + ((((size_t)l * NDB + db) * 2 + s) * 64 + lane) * 2;
        dst[0] = __builtin_bit_cast(uint4, hi);
        dst[1] = __builtin_bit_cast(uint4, lo);
    }
}

// 16-lane sum (every lane of each 16-lane row gets its row's total)
__device__ __forceinline__ float row16_sum(float v)
{
    v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, false));   // quad [1,0,3,2]
    v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xF, 0xF, false));   // quad [2,3,0,1]
    v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x141, 0xF, 0xF, false));  // row_half_mirror
    v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x140, 0xF, 0xF, false));  // row_mirror
    return v;
}

// F tile of pixel row pb for one 16-dim block: the split product, small terms first
#define LSR_DEC_MFMA6(acc, pb)                                                                  \
    do {                                                                                        \
        acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(Wl[pb][0], c0h, acc, 0, 0, 0);             \
        acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(Wh[pb][0], c0l, acc, 0, 0, 0);             \
        acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(Wl[pb][1], c1h, acc, 0, 0, 0);             \
        acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(Wh[pb][1], c1l, acc, 0, 0, 0);             \
        acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(Wh[pb][0], c0h, acc, 0, 0, 0);             \
        acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(Wh[pb][1], c1h, acc, 0, 0, 0);             \
    } while (0)

template <bool NORM, bool VEC>
__global__ void __launch_bounds__(64, LSR_DEC_WAVES) k_quick_decode_h(const float* __restrict__ wmap, int L, int Df,
                                                                      int W, int H, const uint4* __restrict__ frag,
                                                                      const float* __restrict__ scales,
                                                                      const uint4* __restrict__ gfrag,
                                                                      const float* __restrict__ gscales,
                                                                      float* __restrict__ out, float eps)
{
    const int lane = threadIdx.x, lg = lane >> 4, li = lane & 15;
    // one wave = 64 consecutive pixels of one image row, in two halves of two 16-pixel
    // blocks (PB) whose A fragments (hi + lo, 32 VGPRs) stay in registers across every
    // dim block; each dim's 64-B output pieces of a half are adjacent (whole lines)
    constexpr int PB = LSR_DEC_PB;
    const int nbx = (W + 63) / 64;
    const int bx0 = (int)(blockIdx.x % nbx) * 64, y = (int)(blockIdx.x / nbx);
    const size_t HW = (size_t)W * H;
    const int NDB = Df / 16;
    for (int l = 0; l < L; l++) {
        const float sc = scales[l];
        const uint4* fl = frag + (size_t)l * NDB * 256;   // per dim block: 2 K-steps x 64 lanes x (hi, lo)
        for (int half = 0; half < 4 / PB; half++) {
            const int bx = bx0 + 16 * PB * half;
            if (bx >= W) break;
            // A = W^T: lane (li, lg) holds W[32 s + 8 lg + j][x = bx + 16 pb + li]
            h8 Wh[PB][2], Wl[PB][2];
#pragma unroll
            for (int pb = 0; pb < PB; pb++) {
                const int xa = bx + 16 * pb + li;
                const size_t pa = (size_t)y * W + min(xa, W - 1);
#pragma unroll
                for (int s = 0; s < 2; s++)
#pragma unroll
                    for (int j = 0; j < 8; j++) {
                        const float w = wmap[(size_t)(l * 64 + 32 * s + 8 * lg + j) * HW + pa];
                        const float v = xa < W ? w : 0.f;
                        const _Float16 h = (_Float16)v;
                        Wh[pb][s][j] = h;
                        Wl[pb][s][j] = (_Float16)(v - (float)h);
                    }
            }
            float mul[PB][4];
#pragma unroll
            for (int pb = 0; pb < PB; pb++)
#pragma unroll
                for (int r = 0; r < 4; r++) mul[pb][r] = sc;
            if constexpr (NORM) {
                // |F_p|^2 = sum_m W[m][p] (G W)[m][p]; lane (m = 16 mb + li, lg) gets (G W)[m] at x = 4 lg + r
                float sq[PB][4];
#pragma unroll
                for (int pb = 0; pb < PB; pb++)
#pragma unroll
                    for (int r = 0; r < 4; r++) sq[pb][r] = 0.f;
                const uint4* gl = gfrag + (size_t)l * 4 * 256;
#pragma unroll 1
                for (int mb = 0; mb < 4; mb++) {
                    const uint4* f = gl + (size_t)mb * 256 + lane * 2;
                    const h8 c0h = __builtin_bit_cast(h8, f[0]), c0l = __builtin_bit_cast(h8, f[1]);
                    const h8 c1h = __builtin_bit_cast(h8, f[128]), c1l = __builtin_bit_cast(h8, f[129]);
                    const float* wm = wmap + (size_t)(l * 64 + mb * 16 + li) * HW + (size_t)y * W;
#pragma unroll
                    for (int pb = 0; pb < PB; pb++) {
                        f32x4q acc = {0.f, 0.f, 0.f, 0.f};
                        LSR_DEC_MFMA6(acc, pb);
                        const int xo = bx + 16 * pb + 4 * lg;
                        float wv[4] = {0.f, 0.f, 0.f, 0.f};
                        if (VEC && xo + 3 < W) {
                            const float4 v = *reinterpret_cast<const float4*>(wm + xo);
                            wv[0] = v.x; wv[1] = v.y; wv[2] = v.z; wv[3] = v.w;
                        } else {
#pragma unroll
                            for (int r = 0; r < 4; r++)
                                if (xo + r < W) wv[r] = wm[xo + r];
                        }
#pragma unroll
                        for (int r = 0; r < 4; r++) sq[pb][r] = fmaf(wv[r], acc[r], sq[pb][r]);
                    }
                }
                const float gs = gscales[l];
#pragma unroll
                for (int pb = 0; pb < PB; pb++)
#pragma unroll
                    for (int r = 0; r < 4; r++)
                        mul[pb][r] = sc / (sqrtf(fmaxf(row16_sum(sq[pb][r]) * gs, 0.f)) + eps);
            }
            // the next dim block's fragments are loaded while this one computes
            const uint4* fp = fl + lane * 2;
            uint4 n0h = fp[0], n0l = fp[1], n1h = fp[128], n1l = fp[129];
#pragma unroll 1
            for (int db = 0; db < NDB; db++) {
                const h8 c0h = __builtin_bit_cast(h8, n0h), c0l = __builtin_bit_cast(h8, n0l);
                const h8 c1h = __builtin_bit_cast(h8, n1h), c1l = __builtin_bit_cast(h8, n1l);
                if (db + 1 < NDB) {
                    const uint4* f = fp + (size_t)(db + 1) * 256;
                    n0h = f[0]; n0l = f[1]; n1h = f[128]; n1l = f[129];
                }
                float* od = out + (size_t)(l * Df + db * 16 + li) * HW + (size_t)y * W;
#pragma unroll
                for (int pb = 0; pb < PB; pb++) {
                    f32x4q acc = {0.f, 0.f, 0.f, 0.f};
                    LSR_DEC_MFMA6(acc, pb);
                    const int xo = bx + 16 * pb + 4 * lg;
                    float* o = od + xo;
                    if (VEC && xo + 3 < W) {
                        *reinterpret_cast<float4*>(o) = make_float4(acc[0] * mul[pb][0], acc[1] * mul[pb][1],
                                                                    acc[2] * mul[pb][2], acc[3] * mul[pb][3]);
                    } else {
#pragma unroll
                        for (int r = 0; r < 4; r++)
                            if (xo + r < W) o[r] = acc[r] * mul[pb][r];
                    }
                }
            }
        }
    }
}

// ---------------------------------------------------------------------------
// Level-resident decode (default for Df <= 512).  k_quick_decode_h reloads each
// 16-dim block's codebook fragments from global memory inside its store loop,
// and a load issued while stores are pending waits for those stores too (one
// vmcnt counter for both): every dim block paid the write latency of the one
// before (2.38 ms at 1 Mpix = 2.6 TB/s, while the MFMA work alone takes 0.73 ms
// and the same store pattern alone sustains 5 TB/s, profiles/r02_decode_store_pattern.txt).
// Here a persistent workgroup of 8 waves owns one level: its codebook fragments
// (Df/16 x 4 KB) and the norm factor's fragments (4 x 4 KB) live in LDS for the
// whole kernel, so the dim loop reads only LDS and the only global loads are a
// tile's weights, prefetched one tile ahead.
//
// The L2 norm needs |F_p|^2 = w_p^T G w_p (G = CB CB^T) before any dim of pixel
// p is written.  With the Cholesky factor G = L L^T (f64, k_codebook_chol) it
// is |L^T w_p|^2: a 64-column product on the same A fragments (1/8 of the
// decode's matrix work), squared and summed along the output rows, with no
// second read of the weights.
// G[l][i][j] = sum_d CB[l][i][d] CB[l][j][d]: one 256-thread workgroup per
// (16 x 16 output tile, level), one output per thread, the two 16-row slices
// staged through LDS 128 dims at a time.
__global__ void __launch_bounds__(256) k_codebook_gram_t(const float* __restrict__ cb, int K, int Df,
                                                         float* __restrict__ G)
{
    __shared__ float sa[16][129], sb[16][129];
    const int nt = K / 16;
    const int ti = (int)blockIdx.x / nt, tj = (int)blockIdx.x % nt, l = blockIdx.y;
    const int r = threadIdx.x >> 4, c = threadIdx.x & 15;
    const float* base = cb + (size_t)l * K * Df;
    float v = 0.f;
    for (int d0 = 0; d0 < Df; d0 += 128) {
        __syncthreads();
        for (int e = threadIdx.x; e < 16 * 128; e += 256) {
            const int rr = e >> 7, dd = e & 127;
            const bool ok = d0 + dd < Df;
            sa[rr][dd] = ok ? base[(size_t)(16 * ti + rr) * Df + d0 + dd] : 0.f;
            sb[rr][dd] = ok ? base[(size_t)(16 * tj + rr) * Df + d0 + dd] : 0.f;
        }
        __syncthreads();
#pragma unroll 8
        for (int dd = 0; dd < 128; dd++) v = fmaf(sa[r][dd], sb[c][dd], v);
    }
    G[((size_t)l * K + 16 * ti + r) * K + 16 * tj + c] = v;
}

// Lower-triangular L with L L^T = G (per level, K <= 64, f64 in LDS), right-
// looking: per column j the pivot, the column scale, then the trailing lower
// triangle updated by all 256 threads.  A pivot at or below 1e-12 of the
// largest diagonal entry (rank-deficient codebook) leaves its column zero.
// Output row-major (K x K) f32, zeros above the diagonal.
__global__ void __launch_bounds__(256) k_codebook_chol(const float* __restrict__ G, int K, float* __restrict__ Lout)
{
    __shared__ double A[64][65];
    __shared__ double s_tol;
    const int l = blockIdx.x, t = threadIdx.x;
    const float* g = G + (size_t)l * K * K;
    for (int e = t; e < K * K; e += 256) A[e / K][e % K] = (double)g[e];
    __syncthreads();
    if (t == 0) {
        double mx = 0.0;
        for (int j = 0; j < K; j++) mx = fmax(mx, A[j][j]);
        s_tol = 1e-12 * mx;
    }
    __syncthreads();
    const double tol = s_tol;
    for (int j = 0; j < K; j++) {
        const double d = A[j][j];
        const double piv = d > tol ? sqrt(d) : 0.0;
        __syncthreads();   // every thread has read the pivot
        if (t == j) A[j][j] = piv;
        if (t > j && t < K) A[t][j] = piv > 0.0 ? A[t][j] / piv : 0.0;
        __syncthreads();
        // trailing lower triangle: rows i > j, columns j < k <= i
        const int m = K - 1 - j;
        for (int e = t; e < m * m; e += 256) {
            const int i = j + 1 + e / m, k = j + 1 + e % m;
            if (k <= i) A[i][k] -= A[i][j] * A[k][j];
        }
        __syncthreads();
    }
    float* o = Lout + (size_t)l * K * K;
    for (int e = t; e < K * K; e += 256) {
        const int r = e / K, c = e % K;
        o[e] = c <= r ? (float)A[r][c] : 0.f;
    }
}

#ifndef LSR_DEC2_WAVES
#define LSR_DEC2_WAVES 8     // waves per level-resident workgroup (one workgroup per CU: LDS)
#endif
#ifndef LSR_DEC2_PF
#define LSR_DEC2_PF 1        // next tile's weights loaded one tile ahead (64 VGPRs)
#endif
#ifndef LSR_DEC2_NT
#define LSR_DEC2_NT 0        // non-temporal output stores
#endif
#define LSR_DEC2_MAXDB 32    // Df <= 512: fragments + norm factor fit in 144 KB of LDS
#ifndef LSR_DEC2_STORE
#define LSR_DEC2_STORE 1     // 1: 4 planes x 256 B per store (register transpose); 0: 16 planes x 64 B
#endif

// Exchange a register bit with lane bit log2(D) (D = 4 or 8) between X (bit 0)
// and Y (bit 1): X's lanes with the lane bit set take Y's lanes D below, Y's
// lanes with it clear take X's lanes D above (DPP row shifts within 16-lane
// rows; bank masks select the 4-lane banks written).
template <int D>
__device__ __forceinline__ void dec_swap_lanebit(f32x4q& X, f32x4q& Y)
{
    static_assert(D == 4 || D == 8, "lane bit 2 or 3");
    constexpr int SHR = 0x110 + D, SHL = 0x100 + D;
    constexpr int HI = D == 4 ? 0xA : 0xC, LO = D == 4 ? 0x5 : 0x3;
#pragma unroll
    for (int r = 0; r < 4; r++) {
        const int x = __float_as_int(X[r]), y = __float_as_int(Y[r]);
        X[r] = __int_as_float(__builtin_amdgcn_update_dpp(x, y, SHR, 0xF, HI, false));
        Y[r] = __int_as_float(__builtin_amdgcn_update_dpp(y, x, SHL, 0xF, LO, false));
    }
}

// HWC: the weight map is pixel-major (H, W, lk) (LSR_LAYOUT_HWC): a lane's 8 codes
// of one pixel are 32 contiguous bytes, two 16-B loads instead of eight 4-B ones
// from eight channel planes.
template <bool NORM, bool VEC, bool HWC = false>
__global__ void __launch_bounds__(64 * LSR_DEC2_WAVES, 1)
    k_quick_decode_l(const float* __restrict__ wmap, int Df, int W, int H, const uint4* __restrict__ frag,
                     const float* __restrict__ scales, const uint4* __restrict__ nfrag,
                     const float* __restrict__ nscales, float* __restrict__ out, float eps, int nwg, int lk)
{
    extern __shared__ uint4 sfr[];   // [db][s][lane][hi, lo] codebook, then 4 blocks of the norm factor
    const int l = (int)blockIdx.x / nwg, wi = (int)blockIdx.x % nwg;
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, lg = lane >> 4, li = lane & 15;
    const int NDB = Df / 16;
    {
        const uint4* src = frag + (size_t)l * NDB * 256;
        for (int i = threadIdx.x; i < NDB * 256; i += 64 * LSR_DEC2_WAVES) sfr[i] = src[i];
        if constexpr (NORM) {
            const uint4* ns = nfrag + (size_t)l * 4 * 256;
            for (int i = threadIdx.x; i < 4 * 256; i += 64 * LSR_DEC2_WAVES) sfr[NDB * 256 + i] = ns[i];
        }
    }
    __syncthreads();
    const float sc = scales[l];
    const float ns2 = NORM ? nscales[l] * nscales[l] : 0.f;
    const size_t HW = (size_t)W * H;
    const int nbx = (W + 63) / 64;
    const int ntile = nbx * H;
    const int stride = nwg * LSR_DEC2_WAVES;
    // raw weights of a 64-pixel tile: lane (li, lg) holds W[64 l + 32 s + 8 lg + j][x = bx + 16 pb + li]
    float raw[4][2][8];
    auto load = [&](int tt) {
        const bool ok = tt < ntile;
        const int tq = ok ? tt : 0;
        const int bx = (tq % nbx) * 64, y = tq / nbx;
#pragma unroll
        for (int pb = 0; pb < 4; pb++) {
            const int xa = bx + 16 * pb + li;
            const size_t pa = (size_t)y * W + min(xa, W - 1);
            const bool in = ok && xa < W;
            if constexpr (HWC) {
                const float4* wp = reinterpret_cast<const float4*>(wmap + pa * lk + l * 64 + 8 * lg);
#pragma unroll
                for (int s2 = 0; s2 < 2; s2++) {
                    const float4 v0 = wp[8 * s2], v1 = wp[8 * s2 + 1];
                    raw[pb][s2][0] = in ? v0.x : 0.f;
                    raw[pb][s2][1] = in ? v0.y : 0.f;
                    raw[pb][s2][2] = in ? v0.z : 0.f;
                    raw[pb][s2][3] = in ? v0.w : 0.f;
                    raw[pb][s2][4] = in ? v1.x : 0.f;
                    raw[pb][s2][5] = in ? v1.y : 0.f;
                    raw[pb][s2][6] = in ? v1.z : 0.f;
                    raw[pb][s2][7] = in ? v1.w : 0.f;
                }
            } else {
#pragma unroll
                for (int s2 = 0; s2 < 2; s2++)
#pragma unroll
                    for (int j = 0; j < 8; j++) {
                        const float v = wmap[(size_t)(l * 64 + 32 * s2 + 8 * lg + j) * HW + pa];
                        raw[pb][s2][j] = in ? v : 0.f;
                    }
            }
        }
    };
    int t = wi * LSR_DEC2_WAVES + w;
#if LSR_DEC2_PF
    load(t);
#endif
    for (; t < ntile; t += stride) {
#if !LSR_DEC2_PF
        load(t);
#endif
        const int bx = (t % nbx) * 64, y = t / nbx;
        // per-pixel power-of-two scaling of the weights before the f16 split:
        // the pixel's largest |w| goes to [0.5, 1), so a nearly transparent
        // pixel's small weights keep all 22 bits of hi + lo instead of falling
        // into f16's subnormal range (exact: the scale is undone in `mul`, and
        // the L2 norm is scale-invariant).  Lane (li, lg) holds pixel (pb, li).
        float psc[4];   // 2^e of pixel (pb, li): w = psc * w_scaled
#pragma unroll
        for (int pb = 0; pb < 4; pb++) {
            float m = 0.f;
#pragma unroll
            for (int s2 = 0; s2 < 2; s2++)
#pragma unroll
                for (int j = 0; j < 8; j++) m = fmaxf(m, fabsf(raw[pb][s2][j]));
            m = fmaxf(m, __shfl_xor(m, 16, 64));
            m = fmaxf(m, __shfl_xor(m, 32, 64));
            int e = 0;
            if (m > 0.f && m < 3.0e38f) (void)frexpf(m, &e);
            // both factors stay finite normals: a subnormal m (e down to -148)
            // or m >= 2^127 would otherwise make inv or psc infinite
            e = min(max(e, -126), 126);
            psc[pb] = ldexpf(1.f, e);
            const float inv = ldexpf(1.f, -e);
#pragma unroll
            for (int s2 = 0; s2 < 2; s2++)
#pragma unroll
                for (int j = 0; j < 8; j++) raw[pb][s2][j] *= inv;
        }
        h8 Wh[4][2], Wl[4][2];
#pragma unroll
        for (int pb = 0; pb < 4; pb++)
#pragma unroll
            for (int s2 = 0; s2 < 2; s2++)
#pragma unroll
                for (int j = 0; j < 8; j++) {
                    const float v = raw[pb][s2][j];
                    const _Float16 h = (_Float16)v;
                    Wh[pb][s2][j] = h;
                    Wl[pb][s2][j] = (_Float16)(v - (float)h);
                }
#if LSR_DEC2_PF
        load(t + stride);   // next tile's weights in flight during this tile's products and stores
#endif
        // the scale of output pixel (pb, 4 lg + r) (the MFMA result layout)
        float osc[4][4];
#pragma unroll
        for (int pb = 0; pb < 4; pb++)
#pragma unroll
            for (int r = 0; r < 4; r++) osc[pb][r] = __shfl(psc[pb], 4 * lg + r, 64);
        float mul[4][4];
#pragma unroll
        for (int pb = 0; pb < 4; pb++)
#pragma unroll
            for (int r = 0; r < 4; r++) mul[pb][r] = sc * osc[pb][r];
        if constexpr (NORM) {
            // Y^T = W^T L: lane (k = 16 mb + li, lg) gets Y[k] of pixels 4 lg + r; |F_p|^2 = sum_k Y[k]^2
            float sq[4][4];
#pragma unroll
            for (int pb = 0; pb < 4; pb++)
#pragma unroll
                for (int r = 0; r < 4; r++) sq[pb][r] = 0.f;
#pragma unroll 1
            for (int mb = 0; mb < 4; mb++) {
                const uint4* f = sfr + (size_t)(NDB + mb) * 256 + lane * 2;
                const h8 c0h = __builtin_bit_cast(h8, f[0]), c0l = __builtin_bit_cast(h8, f[1]);
                const h8 c1h = __builtin_bit_cast(h8, f[128]), c1l = __builtin_bit_cast(h8, f[129]);
#pragma unroll
                for (int pb = 0; pb < 4; pb++) {
                    f32x4q acc = {0.f, 0.f, 0.f, 0.f};
                    LSR_DEC_MFMA6(acc, pb);
#pragma unroll
                    for (int r = 0; r < 4; r++) sq[pb][r] = fmaf(acc[r], acc[r], sq[pb][r]);
                }
            }
#pragma unroll
            for (int pb = 0; pb < 4; pb++)
#pragma unroll
                for (int r = 0; r < 4; r++)
                    mul[pb][r] = sc / (sqrtf(fmaxf(row16_sum(sq[pb][r]) * ns2, 0.f)) + eps / osc[pb][r]);
        }
#if LSR_DEC2_STORE == 1
        if (VEC) {
            // 4 planes x 256 B per store instruction (instead of 16 planes x 64 B):
            // the four 16-pixel tiles' results are transposed in registers by two
            // (register bit <-> lane bit) swaps — pb bit 0 <-> lane bit 2, pb bit 1
            // <-> lane bit 3 (DPP row shifts by 4 and 8 under bank masks) — so
            // register q holds dims 4 q + (li & 3) of pixel groups
            // g = lg + 4 ((li >> 2) & 3), each dim's 64 pixels in one 256-B piece.
            const int xo = bx + 4 * (lg + 4 * ((li >> 2) & 3));
            float* const orow = out + (size_t)(l * Df + (li & 3)) * HW + (size_t)y * W + xo;
            const bool st_ok = xo < W;   // W % 4 == 0: a pixel group is all in or all out
#pragma unroll 1
            for (int db = 0; db < NDB; db++) {
                const uint4* f = sfr + (size_t)db * 256 + lane * 2;
                const h8 c0h = __builtin_bit_cast(h8, f[0]), c0l = __builtin_bit_cast(h8, f[1]);
                const h8 c1h = __builtin_bit_cast(h8, f[128]), c1l = __builtin_bit_cast(h8, f[129]);
                f32x4q v[4];
#pragma unroll
                for (int pb = 0; pb < 4; pb++) {
                    f32x4q acc = {0.f, 0.f, 0.f, 0.f};
                    LSR_DEC_MFMA6(acc, pb);
#pragma unroll
                    for (int r = 0; r < 4; r++) v[pb][r] = acc[r] * mul[pb][r];
                }
                dec_swap_lanebit<4>(v[0], v[1]);   // pb bit 0 <-> lane bit 2
                dec_swap_lanebit<4>(v[2], v[3]);
                dec_swap_lanebit<8>(v[0], v[2]);   // pb bit 1 <-> lane bit 3
                dec_swap_lanebit<8>(v[1], v[3]);
                float* const od = orow + (size_t)db * 16 * HW;
                if (st_ok) {
#pragma unroll
                    for (int q = 0; q < 4; q++) *reinterpret_cast<f32x4q*>(od + (size_t)(4 * q) * HW) = v[q];
                }
            }
            continue;
        }
#endif
        float* const orow = out + (size_t)(l * Df + li) * HW + (size_t)y * W;
#pragma unroll 1
        for (int db = 0; db < NDB; db++) {
            const uint4* f = sfr + (size_t)db * 256 + lane * 2;
            const h8 c0h = __builtin_bit_cast(h8, f[0]), c0l = __builtin_bit_cast(h8, f[1]);
            const h8 c1h = __builtin_bit_cast(h8, f[128]), c1l = __builtin_bit_cast(h8, f[129]);
            float* const od = orow + (size_t)db * 16 * HW;
#pragma unroll
            for (int pb = 0; pb < 4; pb++) {
                f32x4q acc = {0.f, 0.f, 0.f, 0.f};
                LSR_DEC_MFMA6(acc, pb);
                const int xo = bx + 16 * pb + 4 * lg;
                float* o = od + xo;
                if (VEC && xo + 3 < W) {
#if LSR_DEC2_NT
                    f32x4q v = {acc[0] * mul[pb][0], acc[1] * mul[pb][1], acc[2] * mul[pb][2], acc[3] * mul[pb][3]};
                    __builtin_nontemporal_store(v, reinterpret_cast<f32x4q*>(o));
#else
                    *reinterpret_cast<float4*>(o) = make_float4(acc[0] * mul[pb][0], acc[1] * mul[pb][1],
                                                                acc[2] * mul[pb][2], acc[3] * mul[pb][3]);
#endif
                } else {
#pragma unroll
                    for (int r = 0; r < 4; r++)
                        if (xo + r < W) o[r] = acc[r] * mul[pb][r];
                }
            }
        }
    }
}

size_t quick_decode_workspace_bytes(int L, int K, int Df, int normalize)
{
#ifdef LSR_DECODE_F32
    return normalize ? sizeof(float) * (size_t)L * K * K : 0;
#else
    // codebook fragments (L * Df/16 * 2 * 64 * 32 B) + per-level scales; with normalisation the
    // Gram matrices and their Cholesky factors (2 * L * 64 * 64 f32), the factor's (or, for
    // Df > 512, the Gram matrices') fragments (L * 4 * 2 * 64 * 32 B) and scales
    return (size_t)L * Df * 256 + 256 + (normalize ? 2 * (size_t)L * K * K * 4 + (size_t)L * 64 * 256 + 256 : 0);
#endif
}

// The plan (= the workspace): codebook fragments + scales, and with
// normalisation the Gram matrices, their Cholesky factors and the factors'
// fragments + scales (for Df > 512 the Gram matrices' fragments instead).
// It depends on the codebooks only, so a caller decoding many frames with the
// same codebooks prepares it once (lsr_quick_decode_prepare).
hipError_t launch_quick_decode_prepare(const float* cb, int L, int K, int Df, int normalize, void* ws, hipStream_t st)
{
    if (L == 0) return hipSuccess;
#ifdef LSR_DECODE_F32
    if (normalize) {
        dim3 g((unsigned)((K * K + 255) / 256), (unsigned)L);
        k_codebook_gram<<<g, 256, 0, st>>>(cb, K, Df, (float*)ws);
    }
#else
    uint8_t* p = (uint8_t*)ws;
    uint4* frag = (uint4*)p;
    float* scales = (float*)(p + (size_t)L * Df * 256);
    k_codebook_frag<<<L, 256, 0, st>>>(cb, K, Df, frag, scales);
    if (normalize) {
        float* G = (float*)(p + (size_t)L * Df * 256 + 256);
        float* Lf = G + (size_t)L * K * K;
        uint4* nfrag = (uint4*)(Lf + (size_t)L * K * K);
        float* nscales = (float*)((uint8_t*)nfrag + (size_t)L * 64 * 256);
        k_codebook_gram_t<<<dim3((unsigned)((K / 16) * (K / 16)), (unsigned)L), 256, 0, st>>>(cb, K, Df, G);
#ifndef LSR_DECODE_H
        if (Df / 16 <= LSR_DEC2_MAXDB) {
            k_codebook_chol<<<L, 256, 0, st>>>(G, K, Lf);
            k_codebook_frag<<<L, 256, 0, st>>>(Lf, K, K, nfrag, nscales);
        } else
#endif
            k_codebook_frag<<<L, 256, 0, st>>>(G, K, K, nfrag, nscales);
    }
#endif
    return hipGetLastError();
}

hipError_t launch_quick_decode_run(const float* wmap, const float* cb, int L, int K, int Df, int H, int W,
                                   int normalize, float eps, const void* ws, float* out, hipStream_t st, bool hwc)
{
    if (L == 0 || H == 0 || W == 0) return hipSuccess;
#ifdef LSR_DECODE_F32
    if (hwc) return hipErrorInvalidValue;   // this A/B variant reads the channel-major map only
    const unsigned nb = (unsigned)(((W + 15) / 16) * ((H + 3) / 4));
    k_quick_decode<64><<<nb, 64, 0, st>>>(wmap, L, Df, W, H, cb, (const float*)ws, out, eps, normalize);
#else
    const uint8_t* p = (const uint8_t*)ws;
    const uint4* frag = (const uint4*)p;
    const float* scales = (const float*)(p + (size_t)L * Df * 256);
    const float* G = (const float*)(p + (size_t)L * Df * 256 + 256);
    const float* Lf = G + (size_t)L * K * K;
    const uint4* nfrag = (const uint4*)(Lf + (size_t)L * K * K);
    const float* nscales = (const float*)((const uint8_t*)nfrag + (size_t)L * 64 * 256);
    const bool vec = (W % 4) == 0;
    const int NDB = Df / 16;
#ifndef LSR_DECODE_H
    if (NDB <= LSR_DEC2_MAXDB) {
        // level-resident: one workgroup per CU, the CUs split evenly over the levels
        static int ncu = [] {
            int dev = 0, n = 256;
            if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
            return n > 0 ? n : 256;
        }();
        const int nwg = ncu / L > 0 ? ncu / L : 1;
        const size_t lds = (size_t)(NDB + (normalize ? 4 : 0)) * 256 * sizeof(uint4);
        auto run = [&](auto kern) {
            (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            kern<<<(unsigned)(nwg * L), 64 * LSR_DEC2_WAVES, lds, st>>>(wmap, Df, W, H, frag, scales, nfrag, nscales,
                                                                      out, eps, nwg, L * K);
        };
        if (hwc) {
            if (normalize) {
                if (vec) run(k_quick_decode_l<true, true, true>);
                else run(k_quick_decode_l<true, false, true>);
            } else {
                if (vec) run(k_quick_decode_l<false, true, true>);
                else run(k_quick_decode_l<false, false, true>);
            }
        } else if (normalize) {
            if (vec) run(k_quick_decode_l<true, true>);
            else run(k_quick_decode_l<true, false>);
        } else {
            if (vec) run(k_quick_decode_l<false, true>);
            else run(k_quick_decode_l<false, false>);
        }
        return hipGetLastError();
    }
#endif
    if (hwc) return hipErrorInvalidValue;   // the pixel-major map: level-resident kernel only
    const unsigned nb = (unsigned)(((W + 63) / 64) * H);
    if (normalize) {
        if (vec)
            k_quick_decode_h<true, true><<<nb, 64, 0, st>>>(wmap, L, Df, W, H, frag, scales, nfrag, nscales, out, eps);
        else
            k_quick_decode_h<true, false><<<nb, 64, 0, st>>>(wmap, L, Df, W, H, frag, scales, nfrag, nscales, out, eps);
    } else {
        if (vec)
            k_quick_decode_h<false, true><<<nb, 64, 0, st>>>(wmap, L, Df, W, H, frag, scales, nullptr, nullptr, out, eps);
        else
            k_quick_decode_h<false, false><<<nb, 64, 0, st>>>(wmap, L, Df, W, H, frag, scales, nullptr, nullptr, out,
                                                               eps);
    }
#endif
    return hipGetLastError();
}

hipError_t launch_quick_decode(const float* wmap, const float* cb, int L, int K, int Df, int H, int W, int normalize,
                               float eps, void* ws, float* out, hipStream_t st)
{
    if (L == 0 || H == 0 || W == 0) return hipSuccess;
    const hipError_t e = launch_quick_decode_prepare(cb, L, K, Df, normalize, ws, st);
    if (e != hipSuccess) return e;
    return launch_quick_decode_run(wmap, cb, L, K, Df, H, W, normalize, eps, ws, out, st);
}

}  // namespace lsr
