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

hipError_t launch_quick_decode(const float* wmap, const float* cb, int L, int K, int Df, int H, int W, int normalize,
                               float eps, float* G, float* out, hipStream_t st)
{
    if (L == 0 || H == 0 || W == 0) return hipSuccess;
    if (normalize) {
        dim3 g((unsigned)((K * K + 255) / 256), (unsigned)L);
        k_codebook_gram<<<g, 256, 0, st>>>(cb, K, Df, G);
    }
    const unsigned nb = (unsigned)(((W + 15) / 16) * ((H + 3) / 4));
    k_quick_decode<64><<<nb, 64, 0, st>>>(wmap, L, Df, W, H, cb, G, out, eps, normalize);
    return hipGetLastError();
}

}  // namespace lsr
