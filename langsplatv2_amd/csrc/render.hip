// render.hip — per-pixel alpha blending over the per-tile depth-ordered
// Gaussian lists (A.3) and its reverse replay (A.4).
//
// Forward: one 256-thread workgroup (4 wave64) per 16x16 tile; batches of
// 256 instances staged into LDS (splat record 32 B + feature row); each lane
// owns one pixel and walks the batch front to back; __syncthreads_count
// retires the tile when all 256 pixels saturated (T < 1e-4).  A per-Gaussian
// conservative exponent cut (splat record .z) skips pairs whose alpha is
// certainly < 1/255 without evaluating exp.  No MFMA: the blend is a serial
// per-pixel recurrence.
//
// Backward: same tiling, batches staged back to front from the tile's
// largest n_contrib.  Per instance, each lane computes its pixel's
// contribution to the 9 + D per-Gaussian gradient values; the wave then
// reduces all values at once by recursive halving (gfx950 v_permlane32_swap,
// v_permlane16_swap, then row DPP), leaving value v's wave sum in lanes 2v and
// 2v+1, and 32 lanes issue ONE 128-byte global_atomic_add_f32 into the
// Gaussian's gradient row.  That is 70 VALU ops + 1 atomic instruction per
// (wave, instance) instead of (9 + D) atomics per contributing pixel.
#include "lsr_internal.h"

namespace lsr {

// ----------------------------------------------------------- reductions --
template <int CTRL>
__device__ __forceinline__ float dpp(float v)
{
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}

// Reduce 32 per-lane values across the wave.  On return, lane l holds the
// wave-wide sum of value (l >> 1) in v[0].
__device__ __forceinline__ float wave_reduce32(float (&v)[32])
{
    const int lane = threadIdx.x & 63;
    // bit 5: lanes l <-> l+32 (permlane32_swap)
#pragma unroll
    for (int k = 0; k < 16; k++) {
        auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v[k]), __float_as_uint(v[k + 16]), false, false);
        v[k] = __uint_as_float(r[0]) + __uint_as_float(r[1]);
    }
    // bit 4: rows 0<->1, 2<->3 (permlane16_swap)
#pragma unroll
    for (int k = 0; k < 8; k++) {
        auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v[k]), __float_as_uint(v[k + 8]), false, false);
        v[k] = __uint_as_float(r[0]) + __uint_as_float(r[1]);
    }
    // bit 3: row_ror:8 (== xor 8 inside a row)
    {
        const bool hi = lane & 8;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            float keep = hi ? v[k + 4] : v[k];
            float send = hi ? v[k] : v[k + 4];
            v[k] = keep + dpp<0x128>(send);
        }
    }
    // bit 2: row_half_mirror (pairs lanes across bit 2 inside each 8-lane half row)
    {
        const bool hi = lane & 4;
#pragma unroll
        for (int k = 0; k < 2; k++) {
            float keep = hi ? v[k + 2] : v[k];
            float send = hi ? v[k] : v[k + 2];
            v[k] = keep + dpp<0x141>(send);
        }
    }
    // bit 1: quad_perm [2,3,0,1]
    {
        const bool hi = lane & 2;
        float keep = hi ? v[1] : v[0];
        float send = hi ? v[0] : v[1];
        v[0] = keep + dpp<0x4E>(send);
    }
    // bit 0: quad_perm [1,0,3,2]
    v[0] = v[0] + dpp<0xB1>(v[0]);
    return v[0];
}

__device__ __forceinline__ int wave_max_i(int v)
{
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v = max(v, __shfl_xor(v, d, 64));
    return v;
}

// ---------------------------------------------------------- forward -------
template <int NL>
__global__ void __launch_bounds__(256) k_render_fwd(RenderArgs a)
{
    constexpr int C = 3 + NL;
    constexpr int F4 = (C + 3) / 4;  // float4 per feature row
    __shared__ float4 sA[256];
    __shared__ float4 sB[256];
    __shared__ float4 sF[256 * F4];

    const Cam& c = a.cam;
    const int tile = xcd_remap(blockIdx.x, gridDim.x);
    const int tx = tile % c.gx, ty = tile / c.gx;
    const int t = threadIdx.x;
    const int px = tx * LSR_TILE + (t & 15), py = ty * LSR_TILE + (t >> 4);
    const bool inside = px < c.W && py < c.H;
    const float pfx = (float)px, pfy = (float)py;
    const uint32_t rs = a.tile_start[tile], re = a.tile_start[tile + 1];
    const int D = a.D;

    float T = 1.0f;
    float acc[F4 * 4];
#pragma unroll
    for (int k = 0; k < F4 * 4; k++) acc[k] = 0.f;
    uint32_t contributor = 0, last = 0;
    bool done = !inside;

    for (uint32_t base = rs; base < re; base += 256) {
        if (__syncthreads_count(done) == 256) break;
        const uint32_t idx = base + t;
        if (idx < re) {
            const uint32_t gid = a.point_list[idx];
            sA[t] = a.splatA[gid];
            sB[t] = a.splatB[gid];
            float row[F4 * 4];
            row[0] = a.rgb[3 * gid];
            row[1] = a.rgb[3 * gid + 1];
            row[2] = a.rgb[3 * gid + 2];
#pragma unroll
            for (int k = 0; k < NL; k++) row[3 + k] = (k < D) ? a.lang[(size_t)gid * D + k] : 0.f;
#pragma unroll
            for (int k = 3 + NL; k < F4 * 4; k++) row[k] = 0.f;
#pragma unroll
            for (int q = 0; q < F4; q++) sF[t * F4 + q] = make_float4(row[4 * q], row[4 * q + 1], row[4 * q + 2], row[4 * q + 3]);
        }
        __syncthreads();
        const int n = (int)min(256u, re - base);
        for (int j = 0; !done && j < n; j++) {
            contributor++;
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
#pragma unroll
            for (int q = 0; q < F4; q++) {
                const float4 f = sF[j * F4 + q];
                acc[4 * q + 0] = fmaf(f.x, aT, acc[4 * q + 0]);
                acc[4 * q + 1] = fmaf(f.y, aT, acc[4 * q + 1]);
                acc[4 * q + 2] = fmaf(f.z, aT, acc[4 * q + 2]);
                acc[4 * q + 3] = fmaf(f.w, aT, acc[4 * q + 3]);
            }
            T = test_T;
            last = contributor;
        }
    }
    if (inside) {
        const size_t HW = (size_t)c.H * c.W;
        const size_t pix = (size_t)py * c.W + px;
        a.final_T[pix] = T;
        a.n_contrib[pix] = last;
#pragma unroll
        for (int ch = 0; ch < 3; ch++) a.out_color[ch * HW + pix] = fmaf(T, c.bg[ch], acc[ch]);
#pragma unroll
        for (int k = 0; k < NL; k++)
            if (k < D) a.out_lang[k * HW + pix] = acc[3 + k];
    }
}

// Sparse "quick" language path: Dq output channels, K (weight, index) pairs
// per Gaussian.  One wave per 16x4 pixel strip; per-pixel accumulators in LDS
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
    const int tile = xcd_remap(blockIdx.x >> 2, gridDim.x >> 2);
    const int strip = blockIdx.x & 3;
    const int tx = tile % c.gx, ty = tile / c.gx;
    const int t = threadIdx.x;
    const int px = tx * LSR_TILE + (t & 15), py = ty * LSR_TILE + strip * 4 + (t >> 4);
    const bool inside = px < c.W && py < c.H;
    const float pfx = (float)px, pfy = (float)py;
    const uint32_t rs = a.tile_start[tile], re = a.tile_start[tile + 1];
    for (int q = 0; q < Dq; q++) acc[q * 64 + t] = 0.f;

    float T = 1.0f, cr = 0.f, cg = 0.f, cb = 0.f;
    uint32_t contributor = 0, last = 0;
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
                int q;
                if (a.qidx_dtype == LSR_INDEX_F32)
                    q = f2i(((const float*)a.qi)[(size_t)gid * K + k] + 0.5f);
                else if (a.qidx_dtype == LSR_INDEX_I32)
                    q = ((const int32_t*)a.qi)[(size_t)gid * K + k];
                else
                    q = (int)((const int64_t*)a.qi)[(size_t)gid * K + k];
                sI[t * K + k] = (q >= 0 && q < Dq) ? q : -1;
            }
        }
        __syncthreads();
        const int n = (int)min(64u, re - base);
        for (int j = 0; !done && j < n; j++) {
            contributor++;
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
            last = contributor;
        }
    }
    if (inside) {
        const size_t HW = (size_t)c.H * c.W;
        const size_t pix = (size_t)py * c.W + px;
        a.final_T[pix] = T;
        a.n_contrib[pix] = last;
        a.out_color[pix] = fmaf(T, c.bg[0], cr);
        a.out_color[HW + pix] = fmaf(T, c.bg[1], cg);
        a.out_color[2 * HW + pix] = fmaf(T, c.bg[2], cb);
        for (int q = 0; q < Dq; q++) a.out_lang[q * HW + pix] = acc[q * 64 + t];
    }
}

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
        const size_t sm = (size_t)a.Dq * 64 * 4 + 64 * 32 + 64 * 12 + (size_t)64 * a.K * 8;
        k_render_fwd_quick<<<T * 4, 64, sm, st>>>(a);
        return hipGetLastError();
    }
    switch (lang_set_for(a.D)) {
        case 0: k_render_fwd<0><<<T, 256, 0, st>>>(a); break;
        case 4: k_render_fwd<4><<<T, 256, 0, st>>>(a); break;
        case 8: k_render_fwd<8><<<T, 256, 0, st>>>(a); break;
        case 16: k_render_fwd<16><<<T, 256, 0, st>>>(a); break;
        case 32: k_render_fwd<32><<<T, 256, 0, st>>>(a); break;
        case 64: k_render_fwd<64><<<T, 256, 0, st>>>(a); break;
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
    const int nv = 9 + (nl > 0 ? nl : 0);
    return (nv + 31) / 32 * 32;
}

template <int NL>
__global__ void __launch_bounds__(256) k_render_bwd(RenderBwdArgs b)
{
    constexpr int C = 3 + NL;
    constexpr int F4 = (C + 3) / 4;
    constexpr int NV = 9 + NL;
    constexpr int NG = (NV + 31) / 32;
    __shared__ float4 sA[256];
    __shared__ float4 sB[256];
    __shared__ float4 sF[256 * F4];
    __shared__ uint32_t sId[256];
    __shared__ int sMax;

    const RenderArgs& a = b.f;
    const Cam& c = a.cam;
    const int tile = xcd_remap(blockIdx.x, gridDim.x);
    const int tx = tile % c.gx, ty = tile / c.gx;
    const int t = threadIdx.x;
    const int lane = t & 63;
    const int px = tx * LSR_TILE + (t & 15), py = ty * LSR_TILE + (t >> 4);
    const bool inside = px < c.W && py < c.H;
    const float pfx = (float)px, pfy = (float)py;
    const uint32_t rs = a.tile_start[tile];
    const size_t HW = (size_t)c.H * c.W;
    const size_t pix = (size_t)py * c.W + px;
    const int D = a.D;
    const int VP = b.VP;
    const float ddelx_dx = 0.5f * (float)c.W, ddely_dy = 0.5f * (float)c.H;

    const float T_final = inside ? a.final_T[pix] : 0.f;
    const int last = inside ? (int)a.n_contrib[pix] : 0;
    float Gd[F4 * 4];
#pragma unroll
    for (int k = 0; k < F4 * 4; k++) Gd[k] = 0.f;
    if (inside) {
        Gd[0] = b.dout_color[pix];
        Gd[1] = b.dout_color[HW + pix];
        Gd[2] = b.dout_color[2 * HW + pix];
#pragma unroll
        for (int k = 0; k < NL; k++)
            if (k < D) Gd[3 + k] = b.dout_lang[k * HW + pix];
    }
    const float bg_dot = c.bg[0] * Gd[0] + c.bg[1] * Gd[1] + c.bg[2] * Gd[2];

    if (t == 0) sMax = 0;
    __syncthreads();
    const int wmax = wave_max_i(last);
    if (lane == 0) atomicMax(&sMax, wmax);
    __syncthreads();
    const int hi = sMax;

    float T = T_final;
    float last_alpha = 0.f, last_dot = 0.f, rec = 0.f;

    for (int bs = 0; bs < hi; bs += 256) {
        __syncthreads();
        {
            const int p = hi - 1 - (bs + t);
            if (p >= 0) {
                const uint32_t gid = a.point_list[rs + p];
                sId[t] = gid;
                sA[t] = a.splatA[gid];
                sB[t] = a.splatB[gid];
                float row[F4 * 4];
                row[0] = a.rgb[3 * gid];
                row[1] = a.rgb[3 * gid + 1];
                row[2] = a.rgb[3 * gid + 2];
#pragma unroll
                for (int k = 0; k < NL; k++) row[3 + k] = (k < D) ? a.lang[(size_t)gid * D + k] : 0.f;
#pragma unroll
                for (int k = 3 + NL; k < F4 * 4; k++) row[k] = 0.f;
#pragma unroll
                for (int q = 0; q < F4; q++) sF[t * F4 + q] = make_float4(row[4 * q], row[4 * q + 1], row[4 * q + 2], row[4 * q + 3]);
            }
        }
        __syncthreads();
        const int n = min(256, hi - bs);
        for (int j = 0; j < n; j++) {
            const int p = hi - 1 - (bs + j);   // wave-uniform position
            if (p >= wmax) continue;
            const float4 A = sA[j];
            const float4 B = sB[j];
            const float dx = A.x - pfx, dy = A.y - pfy;
            const float power = splat_power(A.z, A.w, B.x, dx, dy);
            bool contrib = (p < last) && !(power > 0.0f || power < B.z);
            float G = 0.f, alpha = 0.f;
            if (contrib) {
                G = expf_det(power);
                alpha = fminf(0.99f, B.y * G);
                contrib = alpha >= 1.0f / 255.0f;
            }
            if (!__any(contrib)) continue;
            float vals[NG * 32];
#pragma unroll
            for (int k = 0; k < NG * 32; k++) vals[k] = 0.f;
            if (contrib) {
                T = T / (1.f - alpha);
                const float aT = alpha * T;
                float f[F4 * 4];
#pragma unroll
                for (int q = 0; q < F4; q++) {
                    const float4 v = sF[j * F4 + q];
                    f[4 * q] = v.x; f[4 * q + 1] = v.y; f[4 * q + 2] = v.z; f[4 * q + 3] = v.w;
                }
                float dot = f[0] * Gd[0];
#pragma unroll
                for (int k = 1; k < C; k++) dot = fmaf(f[k], Gd[k], dot);
                rec = fmaf(last_alpha, last_dot, (1.f - last_alpha) * rec);
                float dL_dalpha = (dot - rec) * T;
                dL_dalpha = fmaf(-T_final / (1.f - alpha), bg_dot, dL_dalpha);
                last_alpha = alpha;
                last_dot = dot;
                const float dL_dG = B.y * dL_dalpha;
                const float gdx = G * dx, gdy = G * dy;
                const float dG_ddelx = -gdx * A.z - gdy * A.w;
                const float dG_ddely = -gdy * B.x - gdx * A.w;
                vals[0] = dL_dG * dG_ddelx * ddelx_dx;
                vals[1] = dL_dG * dG_ddely * ddely_dy;
                vals[2] = -0.5f * gdx * dx * dL_dG;
                vals[3] = -gdx * dy * dL_dG;
                vals[4] = -0.5f * gdy * dy * dL_dG;
                vals[5] = G * dL_dalpha;
#pragma unroll
                for (int k = 0; k < C; k++) vals[6 + k] = aT * Gd[k];
            }
            float* row = b.grad_acc + (size_t)sId[j] * VP;
#pragma unroll
            for (int g = 0; g < NG; g++) {
                float v32[32];
#pragma unroll
                for (int k = 0; k < 32; k++) v32[k] = vals[g * 32 + k];
                const float s = wave_reduce32(v32);
                const int vi = g * 32 + (lane >> 1);
                if (!(lane & 1) && vi < 9 + D && s != 0.f) atomicAdd(row + vi, s);
            }
        }
    }
}

hipError_t launch_render_bwd(const RenderBwdArgs& b, hipStream_t st)
{
    const int T = b.f.cam.gx * b.f.cam.gy;
    if (T == 0) return hipSuccess;
    switch (lang_set_for(b.f.D)) {
        case 0: k_render_bwd<0><<<T, 256, 0, st>>>(b); break;
        case 4: k_render_bwd<4><<<T, 256, 0, st>>>(b); break;
        case 8: k_render_bwd<8><<<T, 256, 0, st>>>(b); break;
        case 16: k_render_bwd<16><<<T, 256, 0, st>>>(b); break;
        case 32: k_render_bwd<32><<<T, 256, 0, st>>>(b); break;
        case 64: k_render_bwd<64><<<T, 256, 0, st>>>(b); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace lsr
