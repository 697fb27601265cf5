// adam.hip — fused Adam step, behind lsr_adam_step.
// Replaces the update torch.optim.Adam(l, lr=0.0, eps=1e-15) performs for
// the reference's parameter groups (scene/gaussian_model.py:234-255; in
// feature mode the (N, 64) logits and the (1, 64, 512) codebooks,
// train.py:261-263): the default foreach implementation runs ~7 elementwise
// passes over each tensor (lerp, mul, addcmul, sqrt, div, add, addcdiv), 1.2 ms
// per step for 64M logits on MI355X.  One pass here: read p, g, m, v, write
// p, m, v (28 B per element), float4-vectorised, grid-stride.
//   m <- m + (1 - b1) (g - m)            (torch: exp_avg.lerp_(grad, 1 - b1))
//   v <- b2 v + (1 - b2) g^2             (exp_avg_sq.mul_(b2).addcmul_(g, g, 1 - b2))
//   p <- p - step_size * m / (sqrt(v) / bc2_sqrt + eps)
// with step_size = lr / (1 - b1^t) and bc2_sqrt = sqrt(1 - b2^t) computed on
// the host in double, as torch does.  weight_decay (L2, added to g first) is
// supported; amsgrad / maximize are not (the reference uses neither).
#include "lsr_internal.h"

namespace lsr {

__device__ __forceinline__ void adam_one(float& p, float g, float& m, float& v, const AdamArgs& a)
{
    if (a.weight_decay != 0.f) g = fmaf(a.weight_decay, p, g);
    m = fmaf(a.one_minus_b1, g - m, m);
    v = fmaf(a.one_minus_b2, g * g, a.b2 * v);
    const float denom = sqrtf(v) / a.bc2_sqrt + a.eps;
    p = fmaf(-a.step_size, m / denom, p);
}

template <bool VEC>
__global__ void __launch_bounds__(256) k_adam(float* __restrict__ p, const float* __restrict__ g,
                                              float* __restrict__ m, float* __restrict__ v, int64_t n, AdamArgs a)
{
    const int64_t n4 = VEC ? n / 4 : 0;
    const int64_t stride = (int64_t)gridDim.x * 256;
    float4* p4 = reinterpret_cast<float4*>(p);
    const float4* g4 = reinterpret_cast<const float4*>(g);
    float4* m4 = reinterpret_cast<float4*>(m);
    float4* v4 = reinterpret_cast<float4*>(v);
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += stride) {
        float4 P = p4[i], M = m4[i], V = v4[i];
        const float4 G = g4[i];
        adam_one(P.x, G.x, M.x, V.x, a);
        adam_one(P.y, G.y, M.y, V.y, a);
        adam_one(P.z, G.z, M.z, V.z, a);
        adam_one(P.w, G.w, M.w, V.w, a);
        p4[i] = P;
        m4[i] = M;
        v4[i] = V;
    }
    for (int64_t i = n4 * 4 + (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
        float P = p[i], M = m[i], V = v[i];
        adam_one(P, g[i], M, V, a);
        p[i] = P;
        m[i] = M;
        v[i] = V;
    }
}

hipError_t launch_adam(float* p, const float* g, float* m, float* v, int64_t n, const AdamArgs& a, hipStream_t st)
{
    if (n <= 0) return hipSuccess;
    const int64_t want = (n / 4 + 255) / 256;
    const int blocks = (int)(want < 4096 ? (want > 0 ? want : 1) : 4096);   // 16 per CU, grid-stride beyond
    const bool vec = (((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) & 15) == 0;
    if (vec)
        k_adam<true><<<blocks, 256, 0, st>>>(p, g, m, v, n, a);
    else
        k_adam<false><<<blocks, 256, 0, st>>>(p, g, m, v, n, a);
    return hipGetLastError();
}

}  // namespace lsr
