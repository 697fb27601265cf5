// lang_codes.hip — fused top-k soft-code producer for the rasterizer's
// language input.  Replaces the reference's chain of
// PyTorch ops
//   y = softmax(logits); top-k mask; y*mask / (sum(y*mask) + 1e-10)
// (softmax_to_topk_soft_code, utils/vq_utils.py:9-24), its packed sparse
// form (get_weights_and_indices, :26-40, ascending channel order, fp32
// indices), the per-level concatenation of GaussianModel.get_render_weights
// (scene/gaussian_model.py:510-518) and the level-offset concatenation the
// quick-path callers build (eval_lerf.py:340-348, backend_renderer.py:121-128)
// with ONE pass over the logits, and the autograd chain back to the logits
// with one more.
//
// Layout: a "row" is one (Gaussian, level) slice of K logits.  Sixteen lanes
// own a row (4 rows per wave); lane j holds channels 64q + 4j .. 64q + 4j + 3
// for q < K/64, so every global access is a coalesced float4 and the row
// reductions (max, sum, top-k arg-max) are 4 cross-lane steps inside a
// 16-lane group.  HBM-bound: 4K bytes read (+4K written dense / 8k sparse)
// per row.
#include "lsr_internal.h"

namespace lsr {

namespace {

constexpr int CODE_ROWS_PER_BLOCK = 16;   // 256 threads

// 16-lane group exchanges on DPP (no LDS round trip): quad_perm [1,0,3,2],
// quad_perm [2,3,0,1], row_half_mirror, row_mirror.  After the four steps
// of a commutative, associative combine every lane holds the group result.
constexpr int GRP_DPP[4] = {0xB1, 0x4E, 0x141, 0x140};

template <int CTRL>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t v)
{
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xF, 0xF, false);
}

template <int CTRL>
__device__ __forceinline__ float dpp_f32(float v)
{
    return __uint_as_float(dpp_u32<CTRL>(__float_as_uint(v)));
}

template <int S = 0>
__device__ __forceinline__ float grp_max(float v)
{
    if constexpr (S == 4) return v;
    else return grp_max<S + 1>(fmaxf(v, dpp_f32<GRP_DPP[S]>(v)));
}

template <int S = 0>
__device__ __forceinline__ float grp_sum(float v)
{
    if constexpr (S == 4) return v;
    else return grp_sum<S + 1>(v + dpp_f32<GRP_DPP[S]>(v));
}

template <int S = 0>
__device__ __forceinline__ uint64_t grp_or64(uint64_t v)
{
    if constexpr (S == 4) return v;
    else {
        const uint64_t o = ((uint64_t)dpp_u32<GRP_DPP[S]>((uint32_t)(v >> 32)) << 32) | dpp_u32<GRP_DPP[S]>((uint32_t)v);
        return grp_or64<S + 1>(v | o);
    }
}

// (value, channel) arg-max: larger value, then lower channel
template <int S = 0>
__device__ __forceinline__ void grp_argmax(float& bv, int& bc)
{
    if constexpr (S < 4) {
        const float ov = dpp_f32<GRP_DPP[S]>(bv);
        const int oc = (int)dpp_u32<GRP_DPP[S]>((uint32_t)bc);
        const bool take = ov > bv || (ov == bv && oc < bc);
        bv = take ? ov : bv;
        bc = take ? oc : bc;
        grp_argmax<S + 1>(bv, bc);
    }
}

// One row's softmax and top-k mask, shared by forward and backward so that
// both select the same channels.  Q = K / 64 float4 chunks per lane.
template <int Q>
struct CodeRow {
    float y[Q][4];      // softmax probabilities
    uint32_t sel[Q];    // bit r: channel 64q + 4j + r selected
    float s;            // sum of the selected probabilities

    __device__ void build(const float* __restrict__ row, int j, int k, bool live)
    {
        float x[Q][4];
#pragma unroll
        for (int q = 0; q < Q; q++) {
            float4 v = live ? reinterpret_cast<const float4*>(row + 64 * q)[j] : make_float4(0.f, 0.f, 0.f, 0.f);
            x[q][0] = v.x; x[q][1] = v.y; x[q][2] = v.z; x[q][3] = v.w;
        }
        // softmax over the row (utils/vq_utils.py:14)
        float m = -INFINITY;
#pragma unroll
        for (int q = 0; q < Q; q++)
#pragma unroll
            for (int r = 0; r < 4; r++) m = fmaxf(m, x[q][r]);
        m = grp_max(m);
        float e = 0.f;
#pragma unroll
        for (int q = 0; q < Q; q++)
#pragma unroll
            for (int r = 0; r < 4; r++) {
                y[q][r] = expf(x[q][r] - m);
                e += y[q][r];
            }
        const float inv = 1.0f / grp_sum(e);
#pragma unroll
        for (int q = 0; q < Q; q++) {
            sel[q] = 0u;
#pragma unroll
            for (int r = 0; r < 4; r++) y[q][r] *= inv;
        }
        // top-k (utils/vq_utils.py:16-18): k rounds of a (value, -channel)
        // arg-max over the unselected entries; ties go to the lower channel
        for (int it = 0; it < k; it++) {
            float bv = -1.0f;
            int bc = 0x7fffffff;
#pragma unroll
            for (int q = 0; q < Q; q++)
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    const int c = 64 * q + 4 * j + r;
                    const bool free_ = !((sel[q] >> r) & 1u);
                    if (free_ && (y[q][r] > bv || (y[q][r] == bv && c < bc))) { bv = y[q][r]; bc = c; }
                }
            grp_argmax(bv, bc);
            // the owner lane marks it (bc is group-uniform)
            const int q = bc >> 6, w = bc & 63;
            if ((w >> 2) == j) {
#pragma unroll
                for (int qq = 0; qq < Q; qq++)
                    if (qq == q) sel[qq] |= 1u << (w & 3);
            }
        }
        float t = 0.f;
#pragma unroll
        for (int q = 0; q < Q; q++)
#pragma unroll
            for (int r = 0; r < 4; r++) t += ((sel[q] >> r) & 1u) ? y[q][r] : 0.f;
        s = grp_sum(t);
    }
};

template <int Q>
__global__ void __launch_bounds__(256) k_topk_code_fwd(const float* __restrict__ logits, int64_t rows, int L, int k,
                                                        float* __restrict__ dense, float* __restrict__ sw, void* sidx,
                                                        int idx_dtype, int level_offset)
{
    constexpr int K = 64 * Q;
    const int j = threadIdx.x & 15;
    const int64_t row = (int64_t)blockIdx.x * CODE_ROWS_PER_BLOCK + (threadIdx.x >> 4);
    const bool live = row < rows;
    CodeRow<Q> cr;
    cr.build(logits + (live ? row : 0) * K, j, k, live);
    if (!live) return;
    const float d = cr.s + 1e-10f;   // utils/vq_utils.py:21
    if (dense) {
#pragma unroll
        for (int q = 0; q < Q; q++) {
            float o[4];
#pragma unroll
            for (int r = 0; r < 4; r++) o[r] = ((cr.sel[q] >> r) & 1u) ? cr.y[q][r] / d : 0.f;
            reinterpret_cast<float4*>(dense + row * K + 64 * q)[j] = make_float4(o[0], o[1], o[2], o[3]);
        }
    }
    if (sw || sidx) {
        // ascending channel order (the non-zero mask order of :37-38)
        const int64_t n = row / L;
        const int l = (int)(row - n * L);
        const int64_t obase = (n * L + l) * k;
        int before = 0;
#pragma unroll
        for (int q = 0; q < Q; q++) {
            const uint64_t bits = grp_or64((uint64_t)cr.sel[q] << (4 * j));
#pragma unroll
            for (int r = 0; r < 4; r++) {
                if (!((cr.sel[q] >> r) & 1u)) continue;
                const int w = 4 * j + r;
                const int rank = before + __popcll(bits & ((1ull << w) - 1ull));
                const int64_t o = obase + rank;
                const int c = 64 * q + w + (level_offset ? l * K : 0);
                if (sw) sw[o] = cr.y[q][r] / d;
                if (sidx) {
                    if (idx_dtype == LSR_INDEX_F32) ((float*)sidx)[o] = (float)c;
                    else if (idx_dtype == LSR_INDEX_I32) ((int32_t*)sidx)[o] = c;
                    else ((int64_t*)sidx)[o] = c;
                }
            }
            before += __popcll(bits);
        }
    }
}

// dL/dlogits from dL/dcode (dense): exact chain rule of :14-21.
//   d = s + 1e-10, code_j = mask_j y_j / d
//   dL/dy_j = mask_j (g_j / d - sum_i g_i code_i / d)      (division + sum)
//   dL/dx   = y (dL/dy - sum_i dL/dy_i y_i)                  (softmax)
// SPARSE: g is dL/dweights of the packed form (rows, k), the selected
// channels in ascending channel order (the forward's sparse output order);
// the dense (rows, K) code gradient is never formed.
template <int Q, bool SPARSE>
__global__ void __launch_bounds__(256) k_topk_code_bwd(const float* __restrict__ logits, const float* __restrict__ g,
                                                        int64_t rows, int k, float* __restrict__ dlogits)
{
    constexpr int K = 64 * Q;
    const int j = threadIdx.x & 15;
    const int64_t row = (int64_t)blockIdx.x * CODE_ROWS_PER_BLOCK + (threadIdx.x >> 4);
    const bool live = row < rows;
    CodeRow<Q> cr;
    cr.build(logits + (live ? row : 0) * K, j, k, live);
    float gv[Q][4];
    if constexpr (SPARSE) {
        int before = 0;
#pragma unroll
        for (int q = 0; q < Q; q++) {
            const uint64_t bits = grp_or64((uint64_t)cr.sel[q] << (4 * j));
#pragma unroll
            for (int r = 0; r < 4; r++) {
                gv[q][r] = 0.f;
                if (live && ((cr.sel[q] >> r) & 1u)) {
                    const int w = 4 * j + r;
                    const int rank = before + __popcll(bits & ((1ull << w) - 1ull));
                    gv[q][r] = g[row * k + rank];
                }
            }
            before += __popcll(bits);
        }
    } else {
#pragma unroll
        for (int q = 0; q < Q; q++) {
            const float4 v = live ? reinterpret_cast<const float4*>(g + row * K + 64 * q)[j] : make_float4(0.f, 0.f, 0.f, 0.f);
            gv[q][0] = v.x; gv[q][1] = v.y; gv[q][2] = v.z; gv[q][3] = v.w;
        }
    }
    const float d = cr.s + 1e-10f;
    float gc = 0.f;
#pragma unroll
    for (int q = 0; q < Q; q++)
#pragma unroll
        for (int r = 0; r < 4; r++)
            if ((cr.sel[q] >> r) & 1u) gc = fmaf(gv[q][r], cr.y[q][r] / d, gc);
    gc = grp_sum(gc);
    float dy[Q][4];
    float sdy = 0.f;
#pragma unroll
    for (int q = 0; q < Q; q++)
#pragma unroll
        for (int r = 0; r < 4; r++) {
            dy[q][r] = ((cr.sel[q] >> r) & 1u) ? (gv[q][r] - gc) / d : 0.f;
            sdy = fmaf(dy[q][r], cr.y[q][r], sdy);
        }
    sdy = grp_sum(sdy);
    if (!live) return;
#pragma unroll
    for (int q = 0; q < Q; q++) {
        float o[4];
#pragma unroll
        for (int r = 0; r < 4; r++) o[r] = cr.y[q][r] * (dy[q][r] - sdy);
        reinterpret_cast<float4*>(dlogits + row * K + 64 * q)[j] = make_float4(o[0], o[1], o[2], o[3]);
    }
}

}  // namespace

hipError_t launch_topk_code_fwd(const float* logits, int64_t N, int L, int K, int k, float* dense, float* sw,
                                void* sidx, int idx_dtype, int level_offset, hipStream_t st)
{
    const int64_t rows = N * L;
    if (rows == 0) return hipSuccess;
    const unsigned nb = (unsigned)((rows + CODE_ROWS_PER_BLOCK - 1) / CODE_ROWS_PER_BLOCK);
    switch (K / 64) {
        case 1: k_topk_code_fwd<1><<<nb, 256, 0, st>>>(logits, rows, L, k, dense, sw, sidx, idx_dtype, level_offset); break;
        case 2: k_topk_code_fwd<2><<<nb, 256, 0, st>>>(logits, rows, L, k, dense, sw, sidx, idx_dtype, level_offset); break;
        case 3: k_topk_code_fwd<3><<<nb, 256, 0, st>>>(logits, rows, L, k, dense, sw, sidx, idx_dtype, level_offset); break;
        case 4: k_topk_code_fwd<4><<<nb, 256, 0, st>>>(logits, rows, L, k, dense, sw, sidx, idx_dtype, level_offset); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_topk_code_bwd(const float* logits, const float* g, int64_t N, int L, int K, int k, float* dlogits,
                                hipStream_t st, bool sparse)
{
    const int64_t rows = N * L;
    if (rows == 0) return hipSuccess;
    const unsigned nb = (unsigned)((rows + CODE_ROWS_PER_BLOCK - 1) / CODE_ROWS_PER_BLOCK);
#define LSR_TOPK_BWD(Q)                                                                          \
    (sparse ? (k_topk_code_bwd<Q, true><<<nb, 256, 0, st>>>(logits, g, rows, k, dlogits), 0)      \
            : (k_topk_code_bwd<Q, false><<<nb, 256, 0, st>>>(logits, g, rows, k, dlogits), 0))
    switch (K / 64) {
        case 1: LSR_TOPK_BWD(1); break;
        case 2: LSR_TOPK_BWD(2); break;
        case 3: LSR_TOPK_BWD(3); break;
        case 4: LSR_TOPK_BWD(4); break;
        default: return hipErrorInvalidValue;
    }
#undef LSR_TOPK_BWD
    return hipGetLastError();
}

}  // namespace lsr
