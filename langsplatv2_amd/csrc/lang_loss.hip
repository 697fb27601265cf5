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
// Bn[s] = max(|FEAT[s]|, eps) (column 0 of the E rows).
__global__ void __launch_bounds__(256) k_lang_prep(const float* __restrict__ cb, const float* __restrict__ feat,
                                                   int S, int Df, float* __restrict__ G, float* __restrict__ E,
                                                   float* __restrict__ Bn)
{
    const int idx = blockIdx.x * 256 + threadIdx.x;
    const int row = idx / LL_K, k = idx % LL_K;
    if (row >= LL_K + S) return;
    const float* a = row < LL_K ? cb + (size_t)row * Df : feat + (size_t)(row - LL_K) * Df;
    const float* b = cb + (size_t)k * Df;
    float s = 0.f;
    for (int c = 0; c < Df; c++) s = fmaf(a[c], b[c], s);
    if (row < LL_K) {
        G[row * LL_K + k] = s;
    } else {
        E[(size_t)(row - LL_K) * LL_K + k] = s;
        if (k == 0) {
            float q = 0.f;
            for (int c = 0; c < Df; c++) q = fmaf(a[c], a[c], q);
            Bn[row - LL_K] = fmaxf(sqrtf(q), LL_COS_EPS);
        }
    }
}

// One wave per 16x4 pixel block (grid-stride over contiguous block ranges, so
// a wave's consecutive blocks are neighbours and segment runs stay long).
// BWD = false: per-wave sum of cos_p.  BWD = true: dL/dw, U, per-wave Q.
template <bool BWD>
__global__ void __launch_bounds__(64, BWD ? 1 : 2) k_lang_loss(const float* __restrict__ wmap, int W, int H,
                                                     const int32_t* __restrict__ seg, int S,
                                                     const float* __restrict__ G, const float* __restrict__ E,
                                                     const float* __restrict__ Bn, const float* __restrict__ gscale,
                                                     float* __restrict__ part, float* __restrict__ gw,
                                                     float* __restrict__ U)
{
    __shared__ float sW[LL_K * LL_SP];
    __shared__ float sA[64], sB[64];
    __shared__ int sS[64];
    const int lane = threadIdx.x, lg = lane >> 4, li = lane & 15;
    const int nbx = (W + 15) / 16, nby = (H + 3) / 4;
    const int NB = nbx * nby;
    const size_t HW = (size_t)W * H;
    const float invP = 1.0f / (float)HW;
    const float g = BWD ? gscale[0] : 1.0f;
    const int b0 = (int)(((int64_t)NB * blockIdx.x) / gridDim.x);
    const int b1 = (int)(((int64_t)NB * (blockIdx.x + 1)) / gridDim.x);

    float cos_sum = 0.f;
    f32x4l Q[10];
#pragma unroll
    for (int t = 0; t < 10; t++) Q[t] = f32x4l{0.f, 0.f, 0.f, 0.f};
    int ucur = -1;   // segment of the run being accumulated (wave-uniform)
    float uacc = 0.f;

    for (int blk = b0; blk < b1; blk++) {
        const int bx = (blk % nbx) * 16, by = (blk / nbx) * 4;
        bool inp[4];
        size_t pixo[4];
        int sp[4];
#pragma unroll
        for (int pb = 0; pb < 4; pb++) {
            const int x = bx + li, y = by + pb;
            inp[pb] = x < W && y < H;
            pixo[pb] = inp[pb] ? (size_t)y * W + x : 0;
            const int s = inp[pb] ? seg[pixo[pb]] : -1;
            sp[pb] = (s >= 0 && s < S) ? s : -1;
        }
        // lane offsets (32-bit: rows 4lg.. of the lane's pixels); the row
        // term (kb*16 + r)*HW is wave-uniform and stays in SGPRs
        uint32_t lo[4];
#pragma unroll
        for (int pb = 0; pb < 4; pb++) lo[pb] = (uint32_t)(4 * lg * HW + pixo[pb]);
        // weight tile in the MFMA output layout: Wt[kb][r][pb] = w[kb*16 + 4lg + r][pixel (pb, li)]
        float Wt[LL_KB][4][4];
#pragma unroll
        for (int kb = 0; kb < LL_KB; kb++)
#pragma unroll
            for (int r = 0; r < 4; r++)
#pragma unroll
                for (int pb = 0; pb < 4; pb++)
                    Wt[kb][r][pb] = inp[pb] ? wmap[(size_t)(kb * 16 + r) * HW + lo[pb]] : 0.f;
        if (BWD) {
            // the tile transposed through LDS for the Q and U phases:
            // sW[code][pixel], pixel = pb*16 + li
#pragma unroll
            for (int kb = 0; kb < LL_KB; kb++)
#pragma unroll
                for (int r = 0; r < 4; r++)
#pragma unroll
                    for (int pb = 0; pb < 4; pb++) sW[(kb * 16 + 4 * lg + r) * LL_SP + pb * 16 + li] = Wt[kb][r][pb];
        }
        // Y = G W (same registers serve as the B operand: K-order kb2*16 + 4lg + r2);
        // the A fragments of one 16-row block of G at a time (4 float4 loads)
        f32x4l Y[LL_KB][4];
#pragma unroll
        for (int kb = 0; kb < LL_KB; kb++) {
            float4 ga[LL_KB];
#pragma unroll
            for (int kb2 = 0; kb2 < LL_KB; kb2++)
                ga[kb2] = *reinterpret_cast<const float4*>(G + (kb * 16 + li) * LL_K + kb2 * 16 + 4 * lg);
#pragma unroll
            for (int pb = 0; pb < 4; pb++) Y[kb][pb] = f32x4l{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int kb2 = 0; kb2 < LL_KB; kb2++) {
                const float a4[4] = {ga[kb2].x, ga[kb2].y, ga[kb2].z, ga[kb2].w};
#pragma unroll
                for (int r2 = 0; r2 < 4; r2++)
#pragma unroll
                    for (int pb = 0; pb < 4; pb++)
                        Y[kb][pb] = __builtin_amdgcn_mfma_f32_16x16x4f32(a4[r2], Wt[kb2][r2][pb], Y[kb][pb], 0, 0, 0);
            }
            __builtin_amdgcn_sched_barrier(0);   // keep the next block's G loads from being hoisted here
        }
        // n^2 = w.Gw and e = E[s].w: lane-group partials, then across groups
        float n2[4], ev[4];
#pragma unroll
        for (int pb = 0; pb < 4; pb++) {
            float pn = 0.f, pe = 0.f;
            const float* Es = E + (size_t)max(sp[pb], 0) * LL_K;
#pragma unroll
            for (int kb = 0; kb < LL_KB; kb++) {
                const float4 e4 = sp[pb] >= 0 ? *reinterpret_cast<const float4*>(Es + kb * 16 + 4 * lg)
                                              : make_float4(0.f, 0.f, 0.f, 0.f);
                const float ee[4] = {e4.x, e4.y, e4.z, e4.w};
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    pn = fmaf(Wt[kb][r][pb], Y[kb][pb][r], pn);
                    pe = fmaf(Wt[kb][r][pb], ee[r], pe);
                }
            }
            __builtin_amdgcn_sched_barrier(0);   // bound the E loads in flight (register pressure)
            pn += __shfl_xor(pn, 16, 64);
            pn += __shfl_xor(pn, 32, 64);
            pe += __shfl_xor(pe, 16, 64);
            pe += __shfl_xor(pe, 32, 64);
            n2[pb] = pn;
            ev[pb] = pe;
        }
        float al[4], be[4];
#pragma unroll
        for (int pb = 0; pb < 4; pb++) {
            const bool m = sp[pb] >= 0;
            const float n = sqrtf(fmaxf(n2[pb], 0.f));
            const float N = fmaxf(n, LL_COS_EPS);
            const float B = m ? Bn[sp[pb]] : 1.f;
            const float cs = m ? ev[pb] / (N * B) : 0.f;
            if (lg == 0) cos_sum += cs;
            al[pb] = m ? -g * invP / (N * B) : 0.f;
            be[pb] = (m && n > LL_COS_EPS) ? g * invP * ev[pb] / (n * n * n * B) : 0.f;
        }
        if (!BWD) continue;

        // dL/dw = alpha E[s] + beta (G w), written once in the tile layout
#pragma unroll
        for (int pb = 0; pb < 4; pb++) {
            if (!inp[pb]) continue;
            const float* Es = E + (size_t)max(sp[pb], 0) * LL_K;
#pragma unroll
            for (int kb = 0; kb < LL_KB; kb++) {
                const float4 e4 = sp[pb] >= 0 ? *reinterpret_cast<const float4*>(Es + kb * 16 + 4 * lg)
                                              : make_float4(0.f, 0.f, 0.f, 0.f);
                const float ee[4] = {e4.x, e4.y, e4.z, e4.w};
#pragma unroll
                for (int r = 0; r < 4; r++)
                    gw[(size_t)(kb * 16 + r) * HW + lo[pb]] = fmaf(al[pb], ee[r], be[pb] * Y[kb][pb][r]);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        if (lg == 0) {
#pragma unroll
            for (int pb = 0; pb < 4; pb++) {
                sA[pb * 16 + li] = al[pb];
                sB[pb * 16 + li] = be[pb];
                sS[pb * 16 + li] = sp[pb];
            }
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
        // U[s] += alpha_p w_p over runs of equal segment (lane = code index)
        for (int p = 0; p < 64; p++) {
            const int s = sS[p];
            if (s < 0) continue;
            if (s != ucur) {
                if (ucur >= 0) atomicAdd(&U[(size_t)ucur * LL_K + lane], uacc);
                ucur = s;
                uacc = 0.f;
            }
            uacc = fmaf(sA[p], sW[lane * LL_SP + p], uacc);
        }
        wave_lds_fence();
    }

    // per-wave results: cos sum (forward) or Q (backward) into part[wave]
    if (!BWD) {
        float v = cos_sum;
#pragma unroll
        for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
        if (lane == 0) part[blockIdx.x] = v;
        return;
    }
    if (ucur >= 0) atomicAdd(&U[(size_t)ucur * LL_K + lane], uacc);
    float* q = part + (size_t)blockIdx.x * LL_K * LL_K;
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

// Q[i] = sum over the per-wave partials (in place into partial 0)
__global__ void __launch_bounds__(256) k_lang_q_reduce(float* __restrict__ part, int n)
{
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= LL_K * LL_K) return;
    float s = 0.f;
    for (int w = 0; w < n; w++) s += part[(size_t)w * LL_K * LL_K + i];
    part[i] = s;
}

// dL/dCB[k][c] = sum_s U[s][k] FEAT[s][c] + sum_j Q[k][j] CB[j][c]
__global__ void __launch_bounds__(256) k_lang_dcb(const float* __restrict__ U, const float* __restrict__ feat, int S,
                                                  const float* __restrict__ Q, const float* __restrict__ cb, int Df,
                                                  float* __restrict__ dcb)
{
    const int idx = blockIdx.x * 256 + threadIdx.x;
    if (idx >= LL_K * Df) return;
    const int k = idx / Df, c = idx % Df;
    float s = 0.f;
    for (int t = 0; t < S; t++) s = fmaf(U[(size_t)t * LL_K + k], feat[(size_t)t * Df + c], s);
    for (int j = 0; j < LL_K; j++) s = fmaf(Q[k * LL_K + j], cb[(size_t)j * Df + c], s);
    dcb[idx] = s;
}

size_t lang_loss_workspace_bytes(int S, int W, int H, int* waves)
{
    const int NB = ((W + 15) / 16) * ((H + 3) / 4);
    const int nw = std::max(1, std::min(NB, 2048));
    if (waves) *waves = nw;
    // G, E, Bn, U, per-wave partials (Q: K*K floats each)
    return sizeof(float) * ((size_t)LL_K * LL_K + (size_t)S * LL_K + (size_t)S + (size_t)S * LL_K +
                            (size_t)nw * LL_K * LL_K + 64);
}

hipError_t launch_lang_loss(const float* wmap, const float* cb, int Df, int H, int W, const int32_t* seg,
                            const float* feat, int S, const float* gscale, float* loss, float* gw, float* dcb,
                            float* ws, hipStream_t st)
{
    int nw = 0;
    lang_loss_workspace_bytes(S, W, H, &nw);
    float* G = ws;
    float* E = G + LL_K * LL_K;
    float* Bn = E + (size_t)S * LL_K;
    float* U = Bn + S;
    float* part = U + (size_t)S * LL_K;
    const int rows = LL_K + S;
    k_lang_prep<<<(rows * LL_K + 255) / 256, 256, 0, st>>>(cb, feat, S, Df, G, E, Bn);
    if (!gw) {
        k_lang_loss<false><<<nw, 64, 0, st>>>(wmap, W, H, seg, S, G, E, Bn, nullptr, part, nullptr, nullptr);
        k_lang_loss_total<<<1, 256, 0, st>>>(part, nw, (size_t)W * H, loss);
        return hipGetLastError();
    }
    if (S > 0) (void)hipMemsetAsync(U, 0, sizeof(float) * (size_t)S * LL_K, st);
    k_lang_loss<true><<<nw, 64, 0, st>>>(wmap, W, H, seg, S, G, E, Bn, gscale, part, gw, U);
    k_lang_q_reduce<<<(LL_K * LL_K + 255) / 256, 256, 0, st>>>(part, nw);
    k_lang_dcb<<<(LL_K * Df + 255) / 256, 256, 0, st>>>(U, feat, S, part, cb, Df, dcb);
    return hipGetLastError();
}

}  // namespace lsr
