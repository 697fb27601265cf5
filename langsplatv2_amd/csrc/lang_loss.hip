// lang_loss.hip — the language-feature cosine loss of the feature-mode
// training step, fused behind lsr_lang_loss_forward /
// lsr_lang_loss_backward.  Replaces, per iteration (train.py:151-164):
//   gt, mask = viewpoint_cam.get_language_feature(...)        scene/cameras.py:59-96
//       gt[:, p] = feature_map[seg[p]], mask[p] = seg[p] != -1
//   f = compute_layer_feature_map(weight_map, 0)              scene/gaussian_model.py:533-543
//       f[:, p] = codebooks[0].T @ w_p                        (Df = 512 channels)
//   loss = cos_loss(f * mask, gt * mask)                      utils/loss_utils.py:24-25
//        = 1 - mean_p  f_p.gt_p / (max(|f_p|, eps) max(|gt_p|, eps))   (eps = 1e-8)
//
// The reference materialises f, gt and their products as (512, H, W) fp32
// tensors (4.2 GB each at 1080p).  Here nothing of size Df x pixels exists:
// every per-pixel quantity factors through the K = 64 code space,
//   |f_p|^2    = w_p^T G w_p,        G = CB CB^T          (K x K)
//   f_p.gt_p   = E[s_p] . w_p,       E = FEAT CB^T        (S x K, per segment)
//   |gt_p|     = |FEAT[s_p]|                              (per segment)
// and so do the gradients (cos_p = e/(N B), alpha = -m/(P N B),
// beta = m e/(P n^3 B) [n > eps]):
//   dL/dw_p    = alpha_p E[s_p] + beta_p (G w_p)
//   dL/dCB     = U^T FEAT + Q CB,  U[s] = sum_{p in s} alpha_p w_p,
//                                  Q    = sum_p beta_p w_p w_p^T.
// The two K x K x pixels products (G W and the beta-weighted Gram Q) run on
// exact-f32 MFMA (v_mfma_f32_16x16x4_f32) with the weight tile held in
// registers in the MFMA output layout (the quick.hip K-order trick), the
// segment sums U are run-length accumulated per wave and flushed with
// atomics when the segment changes.  Traffic: the weight map once
// (forward), the weight map + the gradient map once (backward).
#include "lsr_internal.h"

#include <algorithm>

namespace lsr {

typedef float f32x4l __attribute__((ext_vector_type(4)));

#define LL_K 64
#define LL_KB 4            // K / 16
#define LL_SP 65           // LDS row stride of the transposed weight tile
#define LL_COS_EPS 1e-8f   // torch.nn.functional.cosine_similarity default

// G[k][j] = CB[k].CB[j] (rows < K);  E[s][k] = FEAT[s].CB[k] (rows >= K);
// Bn[s] = max(|FEAT[s]|, eps).  One 256-thread block per row: thread
// (k, part) sums a quarter of the Df products with float4 loads, the four
// partial sums meet in LDS.
__global__ void __launch_bounds__(256) k_lang_prep(const float* __restrict__ cb, const float* __restrict__ feat,
                                                   int S, int Df, float* __restrict__ G, float* __restrict__ E,
                                                   float* __restrict__ Bn)
{
    __shared__ float red[4][LL_K + 1];
    const int row = blockIdx.x;
    const int k = threadIdx.x & 63, part = threadIdx.x >> 6;
    const float* a = row < LL_K ? cb + (size_t)row * Df : feat + (size_t)(row - LL_K) * Df;
    const float* b = cb + (size_t)k * Df;
    const int q = Df / 4;   // Df % 16 == 0 (checked by the caller)
    const int c0 = part * (q / 4) * 4;
    float s = 0.f, nn = 0.f;
#pragma unroll 4
    for (int c = c0; c < c0 + q; c += 4) {
        const float4 x = *reinterpret_cast<const float4*>(a + c);
        const float4 y = *reinterpret_cast<const float4*>(b + c);
        s = fmaf(x.x, y.x, fmaf(x.y, y.y, fmaf(x.z, y.z, fmaf(x.w, y.w, s))));
        if (k == 0) nn = fmaf(x.x, x.x, fmaf(x.y, x.y, fmaf(x.z, x.z, fmaf(x.w, x.w, nn))));
    }
    red[part][k] = s;
    if (k == 0) red[part][LL_K] = nn;
    __syncthreads();
    if (part != 0) return;
    s = red[0][k] + red[1][k] + red[2][k] + red[3][k];
    if (row < LL_K) {
        G[row * LL_K + k] = s;
    } else {
        E[(size_t)(row - LL_K) * LL_K + k] = s;
        if (k == 0)
            Bn[row - LL_K] = fmaxf(sqrtf(red[0][LL_K] + red[1][LL_K] + red[2][LL_K] + red[3][LL_K]), LL_COS_EPS);
    }
}

// Pixel-block geometry shared by both passes: one wave per 16x4 block, lane
// (lg, li) covers pixels (pb, li), pb = 0..3, and code rows kb*16 + 4lg + r.
struct LLBlock {
    bool inp[4];
    size_t pix[4];
    uint32_t lo[4];   // 32-bit element offset of (row 4lg, pixel pb); rows add (kb*16+r)*HW (wave-uniform)
    int sp[4];        // segment id, -1 = masked / outside
    __device__ __forceinline__ LLBlock(int blk, int nbx, int W, int H, size_t HW, const int32_t* seg, int S, int lg,
                                       int li)
    {
        const int bx = (blk % nbx) * 16, by = (blk / nbx) * 4;
#pragma unroll
        for (int pb = 0; pb < 4; pb++) {
            const int x = bx + li, y = by + pb;
            inp[pb] = x < W && y < H;
            pix[pb] = inp[pb] ? (size_t)y * W + x : 0;
            lo[pb] = (uint32_t)(4 * lg * HW + pix[pb]);
            const int s = inp[pb] ? seg[pix[pb]] : -1;
            sp[pb] = (s >= 0 && s < S) ? s : -1;
        }
    }
};

// Weight tile in the MFMA output layout: Wt[kb][r][pb] = w[kb*16 + 4lg + r][pixel (pb, li)].
__device__ __forceinline__ void ll_load_tile(const float* __restrict__ wmap, size_t HW, const LLBlock& bk,
                                             float (&Wt)[LL_KB][4][4])
{
#pragma unroll
    for (int kb = 0; kb < LL_KB; kb++)
#pragma unroll
        for (int r = 0; r < 4; r++)
#pragma unroll
            for (int pb = 0; pb < 4; pb++)
                Wt[kb][r][pb] = bk.inp[pb] ? wmap[(size_t)(kb * 16 + r) * HW + bk.lo[pb]] : 0.f;
}

// Y_kb = rows kb*16.. of G W for the four pixel columns (the tile registers
// are the B operand with K-order kb2*16 + 4lg + r2).
__device__ __forceinline__ void ll_gw_rows(const float* __restrict__ G, int kb, int lg, int li,
                                           const float (&Wt)[LL_KB][4][4], f32x4l (&Y)[4])
{
    float4 ga[LL_KB];
#pragma unroll
    for (int kb2 = 0; kb2 < LL_KB; kb2++)
        ga[kb2] = *reinterpret_cast<const float4*>(G + (kb * 16 + li) * LL_K + kb2 * 16 + 4 * lg);
#pragma unroll
    for (int pb = 0; pb < 4; pb++) Y[pb] = f32x4l{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kb2 = 0; kb2 < LL_KB; kb2++) {
        const float a4[4] = {ga[kb2].x, ga[kb2].y, ga[kb2].z, ga[kb2].w};
#pragma unroll
        for (int r2 = 0; r2 < 4; r2++)
#pragma unroll
            for (int pb = 0; pb < 4; pb++)
                Y[pb] = __builtin_amdgcn_mfma_f32_16x16x4f32(a4[r2], Wt[kb2][r2][pb], Y[pb], 0, 0, 0);
    }
}

// Rows kb*16.. of (G_kb,kb + 2 sum_{kb2 > kb} G_kb,kb2) applied to the tile:
// w_kb . this, summed over kb, is w.Gw (G symmetric).
__device__ __forceinline__ void ll_gw_rows_upper(const float* __restrict__ G, int kb, int lg, int li,
                                                 const float (&Wt)[LL_KB][4][4], f32x4l (&Y)[4])
{
#pragma unroll
    for (int pb = 0; pb < 4; pb++) Y[pb] = f32x4l{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kb2 = 0; kb2 < LL_KB; kb2++) {
        if (kb2 < kb) continue;
        const float4 g4 = *reinterpret_cast<const float4*>(G + (kb * 16 + li) * LL_K + kb2 * 16 + 4 * lg);
        const float f = kb2 == kb ? 1.f : 2.f;
        const float a4[4] = {f * g4.x, f * g4.y, f * g4.z, f * g4.w};
#pragma unroll
        for (int r2 = 0; r2 < 4; r2++)
#pragma unroll
            for (int pb = 0; pb < 4; pb++)
                Y[pb] = __builtin_amdgcn_mfma_f32_16x16x4f32(a4[r2], Wt[kb2][r2][pb], Y[pb], 0, 0, 0);
    }
}

__device__ __forceinline__ float4 ll_erow(const float* __restrict__ E, int s, int kb, int lg)
{
    return s >= 0 ? *reinterpret_cast<const float4*>(E + (size_t)s * LL_K + kb * 16 + 4 * lg)
                  : make_float4(0.f, 0.f, 0.f, 0.f);
}

// Forward: per pixel n = |f| = sqrt(w.Gw) and e = f.gt = E[s].w, written to
// the two stats planes (the backward's alpha/beta come from them), and the
// per-wave sum of cos_p.  Waves own contiguous block ranges.
__global__ void __launch_bounds__(64, 2) k_lang_loss_fwd(const float* __restrict__ wmap, int W, int H,
                                                         const int32_t* __restrict__ seg, int S,
                                                         const float* __restrict__ G, const float* __restrict__ E,
                                                         const float* __restrict__ Bn, float* __restrict__ stats,
                                                         float* __restrict__ part)
{
    const int lane = threadIdx.x, lg = lane >> 4, li = lane & 15;
    const int nbx = (W + 15) / 16, NB = nbx * ((H + 3) / 4);
    const size_t HW = (size_t)W * H;
    const int b0 = (int)(((int64_t)NB * blockIdx.x) / gridDim.x);
    const int b1 = (int)(((int64_t)NB * (blockIdx.x + 1)) / gridDim.x);
    float cos_sum = 0.f;
    for (int blk = b0; blk < b1; blk++) {
        const LLBlock bk(blk, nbx, W, H, HW, seg, S, lg, li);
        float Wt[LL_KB][4][4];
        ll_load_tile(wmap, HW, bk, Wt);
        float pn[4] = {0.f, 0.f, 0.f, 0.f}, pe[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int pb = 0; pb < 4; pb++) {
#pragma unroll
            for (int kb = 0; kb < LL_KB; kb++) {
                const float4 e4 = ll_erow(E, bk.sp[pb], kb, lg);
                pe[pb] = fmaf(Wt[kb][0][pb], e4.x, fmaf(Wt[kb][1][pb], e4.y,
                              fmaf(Wt[kb][2][pb], e4.z, fmaf(Wt[kb][3][pb], e4.w, pe[pb]))));
            }
        }
        __builtin_amdgcn_sched_barrier(0);
        // n^2 = w.Gw over the upper 16x16 blocks of the symmetric G only:
        // sum_kb w_kb.(G_kb,kb w_kb + 2 sum_{kb2 > kb} G_kb,kb2 w_kb2)  (160 MFMAs, not 256)
#pragma unroll
        for (int kb = 0; kb < LL_KB; kb++) {
            f32x4l Y[4];
            ll_gw_rows_upper(G, kb, lg, li, Wt, Y);
#pragma unroll
            for (int pb = 0; pb < 4; pb++)
#pragma unroll
                for (int r = 0; r < 4; r++) pn[pb] = fmaf(Wt[kb][r][pb], Y[pb][r], pn[pb]);
            asm volatile("" ::: "memory");
        }
#pragma unroll
        for (int pb = 0; pb < 4; pb++) {
            float vn = pn[pb], ve = pe[pb];
            vn += __shfl_xor(vn, 16, 64);
            vn += __shfl_xor(vn, 32, 64);
            ve += __shfl_xor(ve, 16, 64);
            ve += __shfl_xor(ve, 32, 64);
            const float n = sqrtf(fmaxf(vn, 0.f));
            if (lg == 0 && bk.inp[pb]) {
                stats[bk.pix[pb]] = n;
                stats[HW + bk.pix[pb]] = ve;
                if (bk.sp[pb] >= 0) cos_sum += ve / (fmaxf(n, LL_COS_EPS) * Bn[bk.sp[pb]]);
            }
        }
    }
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) cos_sum += __shfl_xor(cos_sum, m, 64);
    if (lane == 0) part[blockIdx.x] = cos_sum;
}

// Backward (scaled by the device scalar *gscale): alpha/beta per pixel from
// the forward's stats; dL/dw = alpha E[s] + beta G w written 16 rows at a
// time right after their MFMA block (no full G W kept); Q += beta-weighted
// Gram of the tile (LDS transpose, upper 16x16 tiles); U run-length sums.
__global__ void __launch_bounds__(64, 2) k_lang_loss_bwd(const float* __restrict__ wmap, int W, int H,
                                                         const int32_t* __restrict__ seg, int S,
                                                         const float* __restrict__ G, const float* __restrict__ E,
                                                         const float* __restrict__ Bn,
                                                         const float* __restrict__ stats,
                                                         const float* __restrict__ gscale, float* __restrict__ qpart,
                                                         float* __restrict__ gw, float* __restrict__ U)
{
    __shared__ float sW[LL_K * LL_SP];
    __shared__ float sA[64], sB[64];
    __shared__ int sS[64];
    const int lane = threadIdx.x, lg = lane >> 4, li = lane & 15;
    const int nbx = (W + 15) / 16, NB = nbx * ((H + 3) / 4);
    const size_t HW = (size_t)W * H;
    const float gP = gscale[0] / (float)HW;
    const int b0 = (int)(((int64_t)NB * blockIdx.x) / gridDim.x);
    const int b1 = (int)(((int64_t)NB * (blockIdx.x + 1)) / gridDim.x);

    f32x4l Q[10];
#pragma unroll
    for (int t = 0; t < 10; t++) Q[t] = f32x4l{0.f, 0.f, 0.f, 0.f};
    int ucur = -1;   // segment of the run being accumulated (wave-uniform)
    float uacc = 0.f;

    // software pipeline: the next block's tile is loaded into the same
    // registers once the current one is in LDS and its dL/dw is written, so
    // the loads overlap the Q MFMAs and the U sums
    LLBlock bk(b0 < b1 ? b0 : 0, nbx, W, H, HW, seg, S, lg, li);
    float Wt[LL_KB][4][4];
    if (b0 < b1) ll_load_tile(wmap, HW, bk, Wt);
    for (int blk = b0; blk < b1; blk++) {
        float al[4], be[4];
#pragma unroll
        for (int pb = 0; pb < 4; pb++) {
            const bool m = bk.sp[pb] >= 0;
            const float n = m ? stats[bk.pix[pb]] : 0.f;
            const float e = m ? stats[HW + bk.pix[pb]] : 0.f;
            const float B = m ? Bn[bk.sp[pb]] : 1.f;
            const float N = fmaxf(n, LL_COS_EPS);
            al[pb] = m ? -gP / (N * B) : 0.f;
            be[pb] = (m && n > LL_COS_EPS) ? gP * e / (n * n * n * B) : 0.f;
        }
#pragma unroll
        for (int kb = 0; kb < LL_KB; kb++)
#pragma unroll
            for (int r = 0; r < 4; r++)
#pragma unroll
                for (int pb = 0; pb < 4; pb++) sW[(kb * 16 + 4 * lg + r) * LL_SP + pb * 16 + li] = Wt[kb][r][pb];
        if (lg == 0) {
#pragma unroll
            for (int pb = 0; pb < 4; pb++) {
                sA[pb * 16 + li] = al[pb];
                sB[pb * 16 + li] = be[pb];
                sS[pb * 16 + li] = bk.sp[pb];
            }
        }
#pragma unroll
        for (int kb = 0; kb < LL_KB; kb++) {
            f32x4l Y[4];
            ll_gw_rows(G, kb, lg, li, Wt, Y);
#pragma unroll
            for (int pb = 0; pb < 4; pb++) {
                if (!bk.inp[pb]) continue;
                const float4 e4 = ll_erow(E, bk.sp[pb], kb, lg);
                const float ee[4] = {e4.x, e4.y, e4.z, e4.w};
#pragma unroll
                for (int r = 0; r < 4; r++)
                    gw[(size_t)(kb * 16 + r) * HW + bk.lo[pb]] = fmaf(al[pb], ee[r], be[pb] * Y[pb][r]);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        if (blk + 1 < b1) {
            bk = LLBlock(blk + 1, nbx, W, H, HW, seg, S, lg, li);
            ll_load_tile(wmap, HW, bk, Wt);
        }
        wave_lds_fence();
        // Q += sum_p beta_p w_p w_p^T: K-steps of 4 pixels (pixel 4s + lg per
        // lane group), upper-triangular 16x16 tiles only (Q is symmetric)
#pragma unroll 4
        for (int s = 0; s < 16; s++) {
            const int p = 4 * s + lg;
            const float bp = sB[p];
            float v[LL_KB];
#pragma unroll
            for (int mt = 0; mt < LL_KB; mt++) v[mt] = sW[(mt * 16 + li) * LL_SP + p];
            int t = 0;
#pragma unroll
            for (int mt = 0; mt < LL_KB; mt++)
#pragma unroll
                for (int nt = mt; nt < LL_KB; nt++, t++)
                    Q[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(bp * v[mt], v[nt], Q[t], 0, 0, 0);
        }
        // U[s] += alpha_p w_p over runs of equal segment (lane = code index).
        // Lane p reads pixel p's segment; a ballot marks where runs start, so
        // the per-pixel loop has no data-dependent branch.
        {
            const int sp_l = sS[lane];
            const int sp_prev = __shfl_up(sp_l, 1, 64);
            uint64_t starts = wave_ballot(lane == 0 || sp_l != sp_prev);
            while (starts) {
                const int p0 = __builtin_ctzll(starts);
                starts &= starts - 1;
                const int p1 = starts ? __builtin_ctzll(starts) : 64;
                const int s = __builtin_amdgcn_readlane(sp_l, p0);
                if (s < 0) continue;   // masked pixels: alpha = 0
                if (s != ucur) {
                    if (ucur >= 0) atomicAdd(&U[(size_t)ucur * LL_K + lane], uacc);
                    ucur = s;
                    uacc = 0.f;
                }
#pragma unroll 4
                for (int p = p0; p < p1; p++) uacc = fmaf(sA[p], sW[lane * LL_SP + p], uacc);
            }
        }
        wave_lds_fence();
    }
    if (ucur >= 0) atomicAdd(&U[(size_t)ucur * LL_K + lane], uacc);
    float* q = qpart + (size_t)blockIdx.x * LL_K * LL_K;
    int t = 0;
#pragma unroll
    for (int mt = 0; mt < LL_KB; mt++)
#pragma unroll
        for (int nt = mt; nt < LL_KB; nt++, t++)
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const int i = mt * 16 + 4 * lg + r, j = nt * 16 + li;
                q[i * LL_K + j] = Q[t][r];
                if (mt != nt) q[j * LL_K + i] = Q[t][r];
            }
}

// loss = 1 - (sum of the per-wave cos sums) / P, in double
__global__ void __launch_bounds__(256) k_lang_loss_total(const float* __restrict__ part, int n, size_t P,
                                                         float* __restrict__ loss)
{
    __shared__ double sh[256];
    double s = 0.0;
    for (int i = threadIdx.x; i < n; i += 256) s += (double)part[i];
    sh[threadIdx.x] = s;
    __syncthreads();
    for (int m = 128; m >= 1; m >>= 1) {
        if ((int)threadIdx.x < m) sh[threadIdx.x] += sh[threadIdx.x + m];
        __syncthreads();
    }
    if (threadIdx.x == 0) loss[0] = (float)(1.0 - sh[0] / (double)P);
}

// Q = sum of the per-wave partials: block (entry group x, wave slice y) sums
// LL_QSLICE partials of 256 entries and adds them into Q (zeroed).
#define LL_QSLICE 32
__global__ void __launch_bounds__(256) k_lang_q_reduce(const float* __restrict__ qpart, int n, float* __restrict__ Q)
{
    const int i = blockIdx.x * 256 + threadIdx.x;
    const int w0 = blockIdx.y * LL_QSLICE, w1 = min(n, w0 + LL_QSLICE);
    float s = 0.f;
#pragma unroll 8
    for (int w = w0; w < w1; w++) s += qpart[(size_t)w * LL_K * LL_K + i];
    atomicAdd(&Q[i], s);
}

// dL/dCB[k][c] = sum_s U[s][k] FEAT[s][c] + sum_j Q[k][j] CB[j][c]
__global__ void __launch_bounds__(256) k_lang_dcb(const float* __restrict__ U, const float* __restrict__ feat, int S,
                                                  const float* __restrict__ Q, const float* __restrict__ cb, int Df,
                                                  float* __restrict__ dcb)
{
    const int idx = blockIdx.x * 256 + threadIdx.x;
    if (idx >= LL_K * Df) return;
    const int k = idx / Df, c = idx % Df;
    float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
    int t = 0;
    for (; t + 4 <= S; t += 4) {
        s0 = fmaf(U[(size_t)t * LL_K + k], feat[(size_t)t * Df + c], s0);
        s1 = fmaf(U[(size_t)(t + 1) * LL_K + k], feat[(size_t)(t + 1) * Df + c], s1);
        s2 = fmaf(U[(size_t)(t + 2) * LL_K + k], feat[(size_t)(t + 2) * Df + c], s2);
        s3 = fmaf(U[(size_t)(t + 3) * LL_K + k], feat[(size_t)(t + 3) * Df + c], s3);
    }
    for (; t < S; t++) s0 = fmaf(U[(size_t)t * LL_K + k], feat[(size_t)t * Df + c], s0);
#pragma unroll
    for (int j = 0; j < LL_K; j += 4) {
        s0 = fmaf(Q[k * LL_K + j], cb[(size_t)j * Df + c], s0);
        s1 = fmaf(Q[k * LL_K + j + 1], cb[(size_t)(j + 1) * Df + c], s1);
        s2 = fmaf(Q[k * LL_K + j + 2], cb[(size_t)(j + 2) * Df + c], s2);
        s3 = fmaf(Q[k * LL_K + j + 3], cb[(size_t)(j + 3) * Df + c], s3);
    }
    dcb[idx] = (s0 + s1) + (s2 + s3);
}

size_t lang_loss_workspace_bytes(int S, int W, int H, int* waves)
{
    const int NB = ((W + 15) / 16) * ((H + 3) / 4);
    const int nw = std::max(1, std::min(NB, 2048));
    if (waves) *waves = nw;
    // G, E, Bn, U, Q, per-wave partials (K*K floats each), pixel stats (2 planes)
    return sizeof(float) * ((size_t)LL_K * LL_K * 2 + (size_t)S * LL_K * 2 + (size_t)S + (size_t)nw * LL_K * LL_K +
                            2 * (size_t)W * H + 256);
}

hipError_t launch_lang_loss(const float* wmap, const float* cb, int Df, int H, int W, const int32_t* seg,
                            const float* feat, int S, const float* gscale, float* loss, float* gw, float* dcb,
                            float* stats, float* ws, hipStream_t st)
{
    int nw = 0;
    lang_loss_workspace_bytes(S, W, H, &nw);
    float* G = ws;
    float* Q = G + LL_K * LL_K;
    float* E = Q + LL_K * LL_K;
    float* U = E + (size_t)S * LL_K;
    float* Bn = U + (size_t)S * LL_K;
    float* part = Bn + S + 64;                       // nw * K*K floats
    float* own_stats = part + (size_t)nw * LL_K * LL_K;
    k_lang_prep<<<LL_K + S, 256, 0, st>>>(cb, feat, S, Df, G, E, Bn);
    if (!gw) {   // forward: loss + per-pixel stats (into the caller's buffer)
        k_lang_loss_fwd<<<nw, 64, 0, st>>>(wmap, W, H, seg, S, G, E, Bn, stats ? stats : own_stats, part);
        if (loss) k_lang_loss_total<<<1, 256, 0, st>>>(part, nw, (size_t)W * H, loss);
        return hipGetLastError();
    }
    if (!stats) {   // backward without the forward's stats: recompute them
        stats = own_stats;
        k_lang_loss_fwd<<<nw, 64, 0, st>>>(wmap, W, H, seg, S, G, E, Bn, stats, part);
    }
    if (S > 0) (void)hipMemsetAsync(U, 0, sizeof(float) * (size_t)S * LL_K, st);
    (void)hipMemsetAsync(Q, 0, sizeof(float) * LL_K * LL_K, st);
    k_lang_loss_bwd<<<nw, 64, 0, st>>>(wmap, W, H, seg, S, G, E, Bn, stats, gscale, part, gw, U);
    k_lang_q_reduce<<<dim3(LL_K * LL_K / 256, (nw + LL_QSLICE - 1) / LL_QSLICE), 256, 0, st>>>(part, nw, Q);
    k_lang_dcb<<<(LL_K * Df + 255) / 256, 256, 0, st>>>(U, feat, S, Q, cb, Df, dcb);
    return hipGetLastError();
}

}  // namespace lsr
