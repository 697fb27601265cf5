// preprocess.hip — per-Gaussian projection (A.1) and its chain rule (A.4).
//
// One thread per Gaussian, 256-thread blocks.  HBM-bound stream over N:
// reads means/scales/rotations/opacity/SH (44 + 4*S B), writes the splat
// records consumed by binning and render (2 x float4), rgb, depth, tile
// counts.  Operation sequence == oracle/lsr_oracle.c lso_preprocess.
#include "lsr_internal.h"

// Scale gradient convention (a named switch, SURVEY §8a style):
//  0 (default, upstream 3DGS): dL/dscales is the gradient w.r.t. the MODIFIED
//    scale s = scale_modifier * scale, i.e. the modifier factor is omitted;
//  1: the exact derivative dL/dscale = scale_modifier * dL/ds.
// Only scale_modifier != 1 tells them apart (training always renders at 1).
#ifndef LSR_SCALE_GRAD_EXACT
#define LSR_SCALE_GRAD_EXACT 0
#endif
#define LSR_SCALE_GRAD_MOD(mod) (LSR_SCALE_GRAD_EXACT ? (mod) : 1.0f)
#ifndef LSR_PRE_SH_EARLY
#define LSR_PRE_SH_EARLY 1   // SH row loads before the visibility tests: cfg3 preprocess 77.9 -> 71.7 us, cfg5 311 -> 289 us
#endif

namespace lsr {

// Backward SH16 path: one wave per 64 Gaussians.  The wave stages its 64 SH
// rows (64 x 192 B, contiguous) through a padded LDS tile with fully coalesced
// float4 loads, and writes the SH gradients back the same way, instead of 12
// lane-strided float4 accesses per thread (each touching 64 separate 192-B
// rows): 0.190 -> 0.159 ms at cfg3.  Row stride 49 floats: conflict-free
// per-lane row access.
#define LSR_SH_ROW 49

__device__ __forceinline__ void stage_sh_rows(float* shl, const float* shs, int b0, int cnt, int lane)
{
    const float4* src = reinterpret_cast<const float4*>(shs) + (size_t)b0 * 12;
    auto put = [&](int f, const float4 v) {
        const int row = f / 12, c4 = f - row * 12;
        float* d = shl + row * LSR_SH_ROW + c4 * 4;
        d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
    };
    if (cnt == 64) {
        // full wave: all 12 loads in flight before the first LDS write (a
        // rolled loop waits for each load in turn: 12 serial round trips)
        float4 v[12];
#pragma unroll
        for (int k = 0; k < 12; k++) v[k] = src[lane + 64 * k];
#pragma unroll
        for (int k = 0; k < 12; k++) put(lane + 64 * k, v[k]);
        return;
    }
    for (int f = lane; f < cnt * 12; f += 64) put(f, src[f]);
}

// dRGB/dsh_k of the forward's SH evaluation (sh_channel) at direction
// (x, y, z): the basis value multiplying coefficient k, same expressions as
// preprocess_bwd_one's.
__device__ __forceinline__ void sh_basis(int deg, float x, float y, float z, float (&bk)[16])
{
#pragma unroll
    for (int k = 0; k < 16; k++) bk[k] = 0.f;
    bk[0] = 0.28209479177387814f;
    if (deg > 0) {
        const float c1 = 0.4886025119029199f;
        bk[1] = -c1 * y;
        bk[2] = c1 * z;
        bk[3] = -c1 * x;
        if (deg > 1) {
            const float xx = x * x, yy = y * y, zz = z * z;
            const float xy = x * y, yz = y * z, xz = x * z;
            bk[4] = LSR_C2_0 * xy;
            bk[5] = LSR_C2_1 * yz;
            bk[6] = LSR_C2_2 * (2.f * zz - xx - yy);
            bk[7] = LSR_C2_3 * xz;
            bk[8] = LSR_C2_4 * (xx - yy);
            if (deg > 2) {
                bk[9] = LSR_C3_0 * y * (3.f * xx - yy);
                bk[10] = LSR_C3_1 * xy * z;
                bk[11] = LSR_C3_2 * y * (4.f * zz - xx - yy);
                bk[12] = LSR_C3_3 * z * (2.f * zz - 3.f * xx - 3.f * yy);
                bk[13] = LSR_C3_4 * x * (4.f * zz - xx - yy);
                bk[14] = LSR_C3_5 * z * (xx - yy);
                bk[15] = LSR_C3_6 * x * (xx - 3.f * yy);
            }
        }
    }
}

// The view-factored SH gradient: one thread per Gaussian sums R views'
// basis (x) dRGB products in view order and writes the (M,3) row once.
// d(RGB_ch)/d(dir) of the SH colour (sh_channel) at the unit direction (x, y, z):
// ddx/ddy/ddz[ch], the term order of upstream's backward.  Evaluated by the
// forward when a geometry gradient is pending (stored in GeomLayout::shjac) or,
// without that, by the preprocess backward from the SH row.
template <typename SHV>
__device__ __forceinline__ void sh_dir_jacobian(int deg, const SHV& sh, float x, float y, float z, float (&ddx)[3],
                                                float (&ddy)[3], float (&ddz)[3])
{
#pragma unroll
    for (int ch = 0; ch < 3; ch++) ddx[ch] = ddy[ch] = ddz[ch] = 0.f;
#define S(k) sh[(k)*3 + ch]
    if (deg > 0) {
        const float c1 = 0.4886025119029199f;
#pragma unroll
        for (int ch = 0; ch < 3; ch++) {
            ddx[ch] = -c1 * S(3);
            ddy[ch] = -c1 * S(1);
            ddz[ch] = c1 * S(2);
        }
        if (deg > 1) {
            const float xx = x * x, yy = y * y, zz = z * z;
            const float xy = x * y, yz = y * z, xz = x * z;
#pragma unroll
            for (int ch = 0; ch < 3; ch++) {
                ddx[ch] += LSR_C2_0 * y * S(4) + LSR_C2_2 * 2.f * -x * S(6) + LSR_C2_3 * z * S(7) + LSR_C2_4 * 2.f * x * S(8);
                ddy[ch] += LSR_C2_0 * x * S(4) + LSR_C2_1 * z * S(5) + LSR_C2_2 * 2.f * -y * S(6) + LSR_C2_4 * 2.f * -y * S(8);
                ddz[ch] += LSR_C2_1 * y * S(5) + LSR_C2_2 * 2.f * 2.f * z * S(6) + LSR_C2_3 * x * S(7);
            }
            if (deg > 2) {
#pragma unroll
                for (int ch = 0; ch < 3; ch++) {
                    ddx[ch] += LSR_C3_0 * S(9) * 3.f * 2.f * xy + LSR_C3_1 * S(10) * yz + LSR_C3_2 * S(11) * -2.f * xy +
                               LSR_C3_3 * S(12) * -3.f * 2.f * xz + LSR_C3_4 * S(13) * (-3.f * xx + 4.f * zz - yy) +
                               LSR_C3_5 * S(14) * 2.f * xz + LSR_C3_6 * S(15) * 3.f * (xx - yy);
                    ddy[ch] += LSR_C3_0 * S(9) * 3.f * (xx - yy) + LSR_C3_1 * S(10) * xz +
                               LSR_C3_2 * S(11) * (-3.f * yy + 4.f * zz - xx) + LSR_C3_3 * S(12) * -3.f * 2.f * yz +
                               LSR_C3_4 * S(13) * -2.f * xy + LSR_C3_5 * S(14) * -2.f * yz +
                               LSR_C3_6 * S(15) * -3.f * 2.f * xy;
                    ddz[ch] += LSR_C3_1 * S(10) * xy + LSR_C3_2 * S(11) * 4.f * 2.f * yz +
                               LSR_C3_3 * S(12) * 3.f * (2.f * zz - xx - yy) + LSR_C3_4 * S(13) * 4.f * 2.f * xz +
                               LSR_C3_5 * S(14) * (xx - yy);
                }
            }
        }
    }
#undef S
}

// The SH colour of a visible Gaussian (A.1: SH -> RGB, +0.5, clamp >= 0, and the
// clamp mask), and with `jac` the colour Jacobian d(RGB)/d(dir) the preprocess
// backward reads instead of the SH row.  sh: the 48 SH values when SH16.
template <bool SH16>
__device__ __forceinline__ void sh_colour_one(const Cam& c, const lsr_inputs& in, const GeomLayout& L,
                                              uint8_t* __restrict__ geom, int i, float mx, float my, float mz,
                                              const float* sh, bool jac)
{
    float* rgbo = (float*)(geom + L.rgb);
    uint32_t* clampm = (uint32_t*)(geom + L.clamped);
    float dir[3], dor[3];
    sh_dir(mx, my, mz, c.campos, dir, dor);
    float out[3];
    if constexpr (SH16) {
#pragma unroll
        for (int ch = 0; ch < 3; ch++) out[ch] = sh_channel(c.sh_degree, sh, ch, dir[0], dir[1], dir[2]);
    } else {
        const float* shg = in.shs + (size_t)i * in.max_coeffs * 3;
        for (int ch = 0; ch < 3; ch++) out[ch] = sh_channel(c.sh_degree, shg, ch, dir[0], dir[1], dir[2]);
    }
    if (jac) {
        // the backward's dRGB/d(dir), from the SH row already in registers: the
        // preprocess backward then reads 36 B instead of the 192-B SH row
        float ddx[3], ddy[3], ddz[3];
        if constexpr (SH16) sh_dir_jacobian(c.sh_degree, sh, dir[0], dir[1], dir[2], ddx, ddy, ddz);
        else sh_dir_jacobian(c.sh_degree, in.shs + (size_t)i * in.max_coeffs * 3, dir[0], dir[1], dir[2], ddx, ddy,
                             ddz);
        float3* J = (float3*)(geom + L.shjac) + (size_t)3 * i;
        J[0] = make_float3(ddx[0], ddx[1], ddx[2]);
        J[1] = make_float3(ddy[0], ddy[1], ddy[2]);
        J[2] = make_float3(ddz[0], ddz[1], ddz[2]);
    }
    uint32_t m = 0;
#pragma unroll
    for (int ch = 0; ch < 3; ch++) {
        m |= (out[ch] < 0.f ? 1u : 0u) << ch;
        rgbo[3 * i + ch] = fmaxf(out[ch], 0.f);
    }
    clampm[i] = m;
}

// PART 0: the whole of A.1 for Gaussian i; PART 1: the geometry only (no SH
// colour, rgb or clamp mask: k_preprocess_colour writes those, on a second
// stream, while the binning runs).
template <bool SH16, bool COV, int PART = 0>
__device__ __forceinline__ void preprocess_one(const Cam& c, const lsr_inputs& in, uint8_t* __restrict__ geom,
                                               int32_t* __restrict__ radii, int i, const float* shrow, bool jac)
{
    constexpr bool SHL = SH16 && PART == 0;   // this pass evaluates the SH colour from registers
    const int N = in.P;
    const GeomLayout L = geom_layout(N);
    float4* splatA = (float4*)(geom + L.splatA);
    float4* splatB = (float4*)(geom + L.splatB);
    float* rgbo = (float*)(geom + L.rgb);
    float* depth = (float*)(geom + L.depth);
    uint32_t* tiles = (uint32_t*)(geom + L.tiles);
    uint32_t* clampm = (uint32_t*)(geom + L.clamped);

    // every output is written exactly once: zeros on the invisible exits,
    // the values on the visible path
    auto invisible = [&]() {
        radii[i] = 0;
        tiles[i] = 0;
        if (PART == 0 || in.colors_precomp) clampm[i] = 0;
        depth[i] = 0.f;
        splatA[i] = make_float4(0.f, 0.f, 0.f, 0.f);
        splatB[i] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (PART == 0 && !in.colors_precomp) {
            rgbo[3 * i + 0] = 0.f;
            rgbo[3 * i + 1] = 0.f;
            rgbo[3 * i + 2] = 0.f;
        }
    };

    // Every input of the Gaussian is loaded up front (LSR_PRE_SH_EARLY), before
    // the visibility tests: one round trip instead of a chain means -> (tests)
    // -> covariance inputs -> SH row -> opacity; culled Gaussians read their
    // rows for nothing.  SH16 implies shs (and no colors_precomp).
    const float mx = in.means3D[3 * i], my = in.means3D[3 * i + 1], mz = in.means3D[3 * i + 2];
    float cov[6];
    float4 q = make_float4(1.f, 0.f, 0.f, 0.f);
    float s0 = 0.f, s1 = 0.f, s2 = 0.f;
    float o = 0.f;
    float sh[SHL ? 48 : 1];
    if (LSR_PRE_SH_EARLY) {
        if constexpr (COV) {
#pragma unroll
            for (int k = 0; k < 6; k++) cov[k] = in.cov3D_precomp[6 * i + k];
        } else {
            q = reinterpret_cast<const float4*>(in.rotations)[i];
            s0 = in.scales[3 * i]; s1 = in.scales[3 * i + 1]; s2 = in.scales[3 * i + 2];
        }
        o = in.opacities[i];
        if constexpr (SHL) {
            const float4* src = reinterpret_cast<const float4*>(in.shs) + (size_t)i * 12;
#pragma unroll
            for (int k = 0; k < 12; k++) {
                const float4 v = src[k];
                sh[4 * k] = v.x; sh[4 * k + 1] = v.y; sh[4 * k + 2] = v.z; sh[4 * k + 3] = v.w;
            }
        }
        // keep the loads here: the compiler otherwise sinks them past the
        // visibility tests into the blocks that use them (empty asm: no code)
        if constexpr (SHL) {
#pragma unroll
            for (int k = 0; k < 48; k++) asm volatile("" : "+v"(sh[k]));
        }
        asm volatile("" : "+v"(o));
        if constexpr (COV) {
#pragma unroll
            for (int k = 0; k < 6; k++) asm volatile("" : "+v"(cov[k]));
        } else {
            asm volatile("" : "+v"(q.x), "+v"(q.y), "+v"(q.z), "+v"(q.w), "+v"(s0), "+v"(s1), "+v"(s2));
        }
    }
    const float3 pv = xform43(c.view, mx, my, mz);
    if (pv.z <= 0.2f) {
        invisible();
        return;
    }
    const float4 ph = xform44(c.proj, mx, my, mz);
    const float pw = 1.0f / (ph.w + 0.0000001f);
    const float ppx = ph.x * pw, ppy = ph.y * pw;

    if (!LSR_PRE_SH_EARLY) {
        if constexpr (COV) {
#pragma unroll
            for (int k = 0; k < 6; k++) cov[k] = in.cov3D_precomp[6 * i + k];
        } else {
            q = reinterpret_cast<const float4*>(in.rotations)[i];
            s0 = in.scales[3 * i]; s1 = in.scales[3 * i + 1]; s2 = in.scales[3 * i + 2];
        }
    }
    if constexpr (!COV) compute_cov3D(s0, s1, s2, c.scale_modifier, q, cov);
    Ewa e;
    ewa_setup(c.view, pv, c.fx, c.fy, c.tanfovx, c.tanfovy, e);
    float a, b, cc;
    ewa_cov2D(e, cov, a, b, cc);
    const float det = a * cc - b * b;
    if (det == 0.0f) {
        invisible();
        return;
    }
    const float det_inv = 1.f / det;
    const float mid = 0.5f * (a + cc);
    const float l1 = mid + sqrtf(fmaxf(0.1f, mid * mid - det));
    const float radius = ceilf(3.f * sqrtf(l1));
    const int r = f2i(radius);
    const float px = ndc2pix(ppx, c.W), py = ndc2pix(ppy, c.H);
    int x0, y0, x1, y1;
    get_rect(px, py, r, c.gx, c.gy, x0, y0, x1, y1);
    const int area = (x1 - x0) * (y1 - y0);
    if (area == 0 || r <= 0) {
        invisible();
        return;
    }

    if (PART == 0 && !in.colors_precomp) {
        if constexpr (SHL) {
            // direct float4 loads (staging every row through LDS measured slower)
            if (!LSR_PRE_SH_EARLY) {
                const float4* src = reinterpret_cast<const float4*>(in.shs) + (size_t)i * 12;
#pragma unroll
                for (int k = 0; k < 12; k++) {
                    const float4 v = src[k];
                    sh[4 * k] = v.x; sh[4 * k + 1] = v.y; sh[4 * k + 2] = v.z; sh[4 * k + 3] = v.w;
                }
            }
        }
        sh_colour_one<SHL>(c, in, L, geom, i, mx, my, mz, sh, jac);
    } else if (in.colors_precomp) {
        clampm[i] = 0;
    }
    if (!LSR_PRE_SH_EARLY) o = in.opacities[i];
    depth[i] = pv.z;
    radii[i] = r;
    const float ca = cc * det_inv, cb = -b * det_inv, ccn = a * det_inv;   // the conic as stored
    splatA[i] = make_float4(px, py, ca, cb);
    const float cut = cut_widen(power_cut(o), ca, cb, ccn);
    splatB[i] = make_float4(ccn, o, cut, __uint_as_float(cut_extent(cut, a, cc, det)));
    tiles[i] = (uint32_t)area;
}

template <bool SH16, bool COV, int PART = 0>
__global__ void __launch_bounds__(256) k_preprocess(Cam c, lsr_inputs in, uint8_t* __restrict__ geom,
                                                    int32_t* __restrict__ radii, int jac, uint64_t* zero_word)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (PART == 0 && i == 0) ((uint32_t*)(geom + geom_layout(in.P).flags))[0] = jac ? 1u : 0u;
    if (zero_word && i == 0) *zero_word = 0;   // the tile count's total (k_bin_count, next on the stream)
    if (i >= in.P) return;
    preprocess_one<SH16, COV, PART>(c, in, geom, radii, i, nullptr, jac != 0);
}

// The SH colour pass of a split preprocess (PART 1 above did the geometry):
// every input loaded up front; invisible Gaussians get rgb 0 and mask 0 as in
// the fused pass.  Same expressions, so rgb / mask / Jacobian are bit-identical.
template <bool SH16>
__global__ void __launch_bounds__(256) k_preprocess_colour(Cam c, lsr_inputs in, uint8_t* __restrict__ geom,
                                                           const int32_t* __restrict__ radii, int jac)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const GeomLayout L = geom_layout(in.P);
    if (i == 0) ((uint32_t*)(geom + L.flags))[0] = jac ? 1u : 0u;
    if (i >= in.P) return;
    const int r = radii[i];
    const float mx = in.means3D[3 * i], my = in.means3D[3 * i + 1], mz = in.means3D[3 * i + 2];
    float sh[SH16 ? 48 : 1];
    if constexpr (SH16) {
        const float4* src = reinterpret_cast<const float4*>(in.shs) + (size_t)i * 12;
#pragma unroll
        for (int k = 0; k < 12; k++) {
            const float4 v = src[k];
            sh[4 * k] = v.x; sh[4 * k + 1] = v.y; sh[4 * k + 2] = v.z; sh[4 * k + 3] = v.w;
        }
    }
    if (r <= 0) {
        float* rgbo = (float*)(geom + L.rgb);
        rgbo[3 * i] = 0.f;
        rgbo[3 * i + 1] = 0.f;
        rgbo[3 * i + 2] = 0.f;
        ((uint32_t*)(geom + L.clamped))[i] = 0;
        return;
    }
    sh_colour_one<SH16>(c, in, L, geom, i, mx, my, mz, sh, jac != 0);
}

// jac: a geometry gradient is pending -- store the SH colour Jacobian for the
// preprocess backward (SH inputs only)
// The SH colour pass of a split preprocess on colour_st, behind everything
// enqueued on `st` so far (`ready` recorded there); records `done` on colour_st.
hipError_t launch_preprocess_colour(const Cam& c, const lsr_inputs& in, uint8_t* geom, const int32_t* radii, bool jac,
                                    hipStream_t st, hipStream_t colour_st, hipEvent_t ready, hipEvent_t done)
{
    if (in.P == 0) return hipSuccess;
    const bool sh16 = in.shs && in.max_coeffs == 16 && ((uintptr_t)in.shs % 16 == 0);
    const int j = (jac && in.shs && !in.colors_precomp) ? 1 : 0;
    const dim3 g((in.P + 255) / 256);
    hipError_t e;
    if ((e = hipEventRecord(ready, st)) != hipSuccess) return e;
    if ((e = hipStreamWaitEvent(colour_st, ready, 0)) != hipSuccess) return e;
    if (sh16) k_preprocess_colour<true><<<g, 256, 0, colour_st>>>(c, in, geom, radii, j);
    else k_preprocess_colour<false><<<g, 256, 0, colour_st>>>(c, in, geom, radii, j);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    return hipEventRecord(done, colour_st);
}

hipError_t launch_preprocess(const Cam& c, const lsr_inputs& in, uint8_t* geom, int32_t* radii, bool jac,
                             hipStream_t st, bool geom_only, uint64_t* zero_word)
{
    if (in.P == 0) return hipSuccess;
    const bool sh16 = in.shs && in.max_coeffs == 16 && ((uintptr_t)in.shs % 16 == 0);
    const bool cov = in.cov3D_precomp != nullptr;
    const int j = (jac && in.shs && !in.colors_precomp) ? 1 : 0;
    const dim3 g((in.P + 255) / 256);
    if (geom_only && in.shs && !in.colors_precomp) {
        // split: the geometry only (what the binning needs); the caller launches
        // the SH colour pass (launch_preprocess_colour) on its second stream
        if (cov) k_preprocess<false, true, 1><<<g, 256, 0, st>>>(c, in, geom, radii, j, zero_word);
        else k_preprocess<false, false, 1><<<g, 256, 0, st>>>(c, in, geom, radii, j, zero_word);
        return hipGetLastError();
    }
    if (sh16 && cov) k_preprocess<true, true><<<g, 256, 0, st>>>(c, in, geom, radii, j, zero_word);
    else if (sh16) k_preprocess<true, false><<<g, 256, 0, st>>>(c, in, geom, radii, j, zero_word);
    else if (cov) k_preprocess<false, true><<<g, 256, 0, st>>>(c, in, geom, radii, j, zero_word);
    else k_preprocess<false, false><<<g, 256, 0, st>>>(c, in, geom, radii, j, zero_word);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Backward: chain rule through A.1.  Gradient row layout: lsr_device.h
// (LSR_GROW_LANG).  Rows are read as float4; the SH gradient is written as
// 12 float4 per Gaussian (basis(k) * dRGB(ch)), the language gradient as
// float4 when D % 4 == 0.
// SH16: `shrow` holds this Gaussian's 48 SH values on entry and receives its
// 48 SH gradients (written back by the caller with coalesced stores).
// One Gaussian's backward inputs.  Every row is loaded up front, whether or
// not the Gaussian is visible (all are valid addresses): one round trip
// instead of a chain radius -> gradient row -> means / scales / rotation, and
// (SH16) issued before the SH rows are staged, so both are in flight at once.
struct BwdRow {
    int rad;
    float4 g0, g1, g2;
    float3 j0, j1, j2;   // the forward's SH colour Jacobian (jac: GeomLayout::shjac)
    float mx, my, mz;
    float4 q;
    float sc0, sc1, sc2;
    float cov[6];
    // COV: cov3D_precomp given (a kernel-wide choice, a template parameter so
    // no branch merges the two cases' loaded values: such merges cost a copy
    // each, and every copy waits for its load)
    template <bool COV>
    __device__ __forceinline__ void load(const lsr_inputs& in, const int32_t* __restrict__ radii,
                                         const float* __restrict__ gacc, int VP, int i, const float3* __restrict__ jac)
    {
        const float4* g4 = reinterpret_cast<const float4*>(gacc + (size_t)i * VP);
        rad = radii[i];
        g0 = g4[0];
        g1 = g4[1];
        g2 = g4[2];
        if (jac) {
            j0 = jac[3 * (size_t)i];
            j1 = jac[3 * (size_t)i + 1];
            j2 = jac[3 * (size_t)i + 2];
        }
        mx = in.means3D[3 * i]; my = in.means3D[3 * i + 1]; mz = in.means3D[3 * i + 2];
        q = make_float4(1.f, 0.f, 0.f, 0.f);
        sc0 = sc1 = sc2 = 0.f;
        if constexpr (COV) {
#pragma unroll
            for (int k = 0; k < 6; k++) cov[k] = in.cov3D_precomp[6 * i + k];
        } else {
            q = reinterpret_cast<const float4*>(in.rotations)[i];
            sc0 = in.scales[3 * i]; sc1 = in.scales[3 * i + 1]; sc2 = in.scales[3 * i + 2];
        }
    }
};

// jac: the forward stored the SH colour Jacobian (row.j0..j2); otherwise it is
// evaluated here from the SH row (SH16: shrow holds it on entry)
template <bool SH16>
__device__ __forceinline__ void preprocess_bwd_one(const Cam& c, const lsr_inputs& in, const uint8_t* __restrict__ geom,
                                                   const BwdRow& row, const float* __restrict__ gacc, int VP,
                                                   const lsr_bwd_out& out, int i, float* shrow, bool jac)
{
    const int N = in.P;
    const GeomLayout L = geom_layout(N);
    const int M = in.max_coeffs;
    const int D = in.lang_dim;
    const float4* g4 = reinterpret_cast<const float4*>(gacc + (size_t)i * VP);
    const float mx = row.mx, my = row.my, mz = row.mz;
    const float4 q = row.q;
    const float sc0 = row.sc0, sc1 = row.sc1, sc2 = row.sc2;
    float cov[6];
#pragma unroll
    for (int k = 0; k < 6; k++) cov[k] = row.cov[k];
    const bool vis = row.rad > 0;
    const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
    const float4 g0 = vis ? row.g0 : z4, g1 = vis ? row.g1 : z4, g2 = vis ? row.g2 : z4;
    const float gm2x = g0.x, gm2y = g0.y, dA = g0.z, dB = g0.w;
    const float dC = g1.x, gop = g1.y;
    const float gcol[3] = {g1.z, g1.w, g2.x};

    if (out.dL_dmeans2D) {
        out.dL_dmeans2D[3 * i + 0] = gm2x;
        out.dL_dmeans2D[3 * i + 1] = gm2y;
        out.dL_dmeans2D[3 * i + 2] = 0.f;
    }
    if (out.dL_dopacity) out.dL_dopacity[i] = gop;
    if (out.dL_dlang) {
        if ((D & 3) == 0) {
            float4* dl = reinterpret_cast<float4*>(out.dL_dlang + (size_t)i * D);
            for (int w = 0; w < D / 4; w++) dl[w] = vis ? g4[LSR_GROW_LANG / 4 + w] : make_float4(0.f, 0.f, 0.f, 0.f);
        } else {
            const float* g = gacc + (size_t)i * VP + LSR_GROW_LANG;
            for (int k = 0; k < D; k++) out.dL_dlang[(size_t)i * D + k] = vis ? g[k] : 0.f;
        }
    }
    if (out.dL_dcolors)
        for (int k = 0; k < 3; k++) out.dL_dcolors[3 * i + k] = gcol[k];

    const bool want_sh = out.dL_dsh && in.shs && !in.colors_precomp;
    if (!vis) {
        if (out.dL_dmeans3D) { out.dL_dmeans3D[3 * i] = 0.f; out.dL_dmeans3D[3 * i + 1] = 0.f; out.dL_dmeans3D[3 * i + 2] = 0.f; }
        if (want_sh) {
            if (SH16) {
#pragma unroll
                for (int k = 0; k < 48; k++) shrow[k] = 0.f;
            } else {
                for (int k = 0; k < M * 3; k++) out.dL_dsh[(size_t)i * M * 3 + k] = 0.f;
            }
        }
        if (out.dL_drgb_sh)
            for (int k = 0; k < 3; k++) out.dL_drgb_sh[3 * i + k] = 0.f;
        if (out.dL_dscales) for (int k = 0; k < 3; k++) out.dL_dscales[3 * i + k] = 0.f;
        if (out.dL_drotations) reinterpret_cast<float4*>(out.dL_drotations)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (out.dL_dcov3D) for (int k = 0; k < 6; k++) out.dL_dcov3D[6 * i + k] = 0.f;
        return;
    }
    (void)L;
    const float* V = c.view;
    const float* P = c.proj;
    if (!in.cov3D_precomp) compute_cov3D(sc0, sc1, sc2, c.scale_modifier, q, cov);
    const float3 pv = xform43(V, mx, my, mz);
    Ewa e;
    ewa_setup(V, pv, c.fx, c.fy, c.tanfovx, c.tanfovy, e);
    float a, b, cc;
    ewa_cov2D(e, cov, a, b, cc);
    const float det = a * cc - b * b;
    const float d2inv = 1.0f / ((det * det) + 0.0000001f);
    float dLa = 0.f, dLb = 0.f, dLc = 0.f;
    float dcov[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (d2inv != 0.f) {
        dLa = d2inv * (-cc * cc * dA + b * cc * dB - b * b * dC);
        dLb = d2inv * (2.f * b * cc * dA - (det + 2.f * b * b) * dB + 2.f * a * b * dC);
        dLc = d2inv * (-b * b * dA + a * b * dB - a * a * dC);
        const float* T0 = e.T0;
        const float* T1 = e.T1;
        dcov[0] = T0[0] * T0[0] * dLa + T0[0] * T1[0] * dLb + T1[0] * T1[0] * dLc;
        dcov[3] = T0[1] * T0[1] * dLa + T0[1] * T1[1] * dLb + T1[1] * T1[1] * dLc;
        dcov[5] = T0[2] * T0[2] * dLa + T0[2] * T1[2] * dLb + T1[2] * T1[2] * dLc;
        dcov[1] = 2.f * T0[0] * T0[1] * dLa + (T0[0] * T1[1] + T0[1] * T1[0]) * dLb + 2.f * T1[0] * T1[1] * dLc;
        dcov[2] = 2.f * T0[0] * T0[2] * dLa + (T0[0] * T1[2] + T0[2] * T1[0]) * dLb + 2.f * T1[0] * T1[2] * dLc;
        dcov[4] = 2.f * T0[1] * T0[2] * dLa + (T0[1] * T1[2] + T0[2] * T1[1]) * dLb + 2.f * T1[1] * T1[2] * dLc;
    }
    float u[3], v[3];
    ewa_uv(e, cov, u, v);
    float dT0[3], dT1[3];
#pragma unroll
    for (int k = 0; k < 3; k++) {
        dT0[k] = 2.f * dLa * u[k] + dLb * v[k];
        dT1[k] = 2.f * dLc * v[k] + dLb * u[k];
    }
    const float dJ00 = dT0[0] * V[0] + dT0[1] * V[4] + dT0[2] * V[8];
    const float dJ02 = dT0[0] * V[2] + dT0[1] * V[6] + dT0[2] * V[10];
    const float dJ11 = dT1[0] * V[1] + dT1[1] * V[5] + dT1[2] * V[9];
    const float dJ12 = dT1[0] * V[2] + dT1[1] * V[6] + dT1[2] * V[10];
    const float tz = 1.f / e.tz, tz2 = tz * tz, tz3 = tz2 * tz;
    const float dtx = e.xclamp ? 0.f : -c.fx * tz2 * dJ02;
    const float dty = e.yclamp ? 0.f : -c.fy * tz2 * dJ12;
    const float dtz = -c.fx * tz2 * dJ00 - c.fy * tz2 * dJ11 + (2.f * c.fx * e.tx) * tz3 * dJ02 +
                      (2.f * c.fy * e.ty) * tz3 * dJ12;
    float dm[3];
    dm[0] = V[0] * dtx + V[1] * dty + V[2] * dtz;
    dm[1] = V[4] * dtx + V[5] * dty + V[6] * dtz;
    dm[2] = V[8] * dtx + V[9] * dty + V[10] * dtz;

    const float4 ph = xform44(P, mx, my, mz);
    const float mw = 1.0f / (ph.w + 0.0000001f);
    const float mul1 = ph.x * mw * mw, mul2 = ph.y * mw * mw;
    dm[0] += (P[0] * mw - P[3] * mul1) * gm2x + (P[1] * mw - P[3] * mul2) * gm2y;
    dm[1] += (P[4] * mw - P[7] * mul1) * gm2x + (P[5] * mw - P[7] * mul2) * gm2y;
    dm[2] += (P[8] * mw - P[11] * mul1) * gm2x + (P[9] * mw - P[11] * mul2) * gm2y;

    if (in.shs && !in.colors_precomp) {
        const uint32_t clampm = ((const uint32_t*)(geom + L.clamped))[i];
        float dRGB[3];
#pragma unroll
        for (int k = 0; k < 3; k++) dRGB[k] = ((clampm >> k) & 1u) ? 0.f : gcol[k];
        if (out.dL_drgb_sh)
            for (int k = 0; k < 3; k++) out.dL_drgb_sh[3 * i + k] = dRGB[k];
        float dir[3], dor[3];
        sh_dir(mx, my, mz, c.campos, dir, dor);
        const float x = dir[0], y = dir[1], z = dir[2];
        const int deg = c.sh_degree;
        // basis functions (dRGB/dsh_k), term order of the forward
        float bk[16];
        sh_basis(deg, x, y, z, bk);
        float ddx[3], ddy[3], ddz[3];
        if (jac) {
            ddx[0] = row.j0.x; ddx[1] = row.j0.y; ddx[2] = row.j0.z;
            ddy[0] = row.j1.x; ddy[1] = row.j1.y; ddy[2] = row.j1.z;
            ddz[0] = row.j2.x; ddz[1] = row.j2.y; ddz[2] = row.j2.z;
        } else if (SH16) {
            float sh[48];
#pragma unroll
            for (int k = 0; k < 48; k++) sh[k] = shrow[k];
            sh_dir_jacobian(deg, sh, x, y, z, ddx, ddy, ddz);
        } else {
            float sh[48];
            const float* src = in.shs + (size_t)i * M * 3;
#pragma unroll
            for (int k = 0; k < 48; k++) sh[k] = (k < M * 3) ? src[k] : 0.f;
            sh_dir_jacobian(deg, sh, x, y, z, ddx, ddy, ddz);
        }
        if (want_sh) {
            if (SH16) {
#pragma unroll
                for (int el = 0; el < 48; el++) shrow[el] = bk[el / 3] * dRGB[el % 3];
            } else {
                float* ds = out.dL_dsh + (size_t)i * M * 3;
                for (int k = 0; k < M * 3; k++) ds[k] = (k < 48) ? bk[k / 3] * dRGB[k % 3] : 0.f;
            }
        }
        const float gd0 = ddx[0] * dRGB[0] + ddx[1] * dRGB[1] + ddx[2] * dRGB[2];
        const float gd1 = ddy[0] * dRGB[0] + ddy[1] * dRGB[1] + ddy[2] * dRGB[2];
        const float gd2 = ddz[0] * dRGB[0] + ddz[1] * dRGB[1] + ddz[2] * dRGB[2];
        const float sum2 = dor[0] * dor[0] + dor[1] * dor[1] + dor[2] * dor[2];
        const float inv32 = 1.0f / sqrtf(sum2 * sum2 * sum2);
        dm[0] += ((sum2 - dor[0] * dor[0]) * gd0 - dor[1] * dor[0] * gd1 - dor[2] * dor[0] * gd2) * inv32;
        dm[1] += (-dor[0] * dor[1] * gd0 + (sum2 - dor[1] * dor[1]) * gd1 - dor[2] * dor[1] * gd2) * inv32;
        dm[2] += (-dor[0] * dor[2] * gd0 - dor[1] * dor[2] * gd1 + (sum2 - dor[2] * dor[2]) * gd2) * inv32;
    }
    else if (out.dL_drgb_sh) {
        for (int k = 0; k < 3; k++) out.dL_drgb_sh[3 * i + k] = 0.f;
    }
    if (out.dL_dmeans3D) {
        out.dL_dmeans3D[3 * i] = dm[0];
        out.dL_dmeans3D[3 * i + 1] = dm[1];
        out.dL_dmeans3D[3 * i + 2] = dm[2];
    }
    if (in.cov3D_precomp) {
        if (out.dL_dcov3D)
            for (int k = 0; k < 6; k++) out.dL_dcov3D[6 * i + k] = dcov[k];
    } else {
        if (out.dL_dcov3D)
            for (int k = 0; k < 6; k++) out.dL_dcov3D[6 * i + k] = 0.f;
        const float mod = c.scale_modifier;
        float R[9];
        quat_to_R(q.x, q.y, q.z, q.w, R);
        const float sv[3] = {mod * sc0, mod * sc1, mod * sc2};
        const float Gm[9] = {dcov[0], 0.5f * dcov[1], 0.5f * dcov[2], 0.5f * dcov[1], dcov[3],
                             0.5f * dcov[4], 0.5f * dcov[2], 0.5f * dcov[4], dcov[5]};
        float Mm[9], dM[9], dR[9];
#pragma unroll
        for (int r = 0; r < 3; r++)
#pragma unroll
            for (int k = 0; k < 3; k++) Mm[r * 3 + k] = R[r * 3 + k] * sv[k];
#pragma unroll
        for (int r = 0; r < 3; r++)
#pragma unroll
            for (int k = 0; k < 3; k++)
                dM[r * 3 + k] = 2.f * (Gm[r * 3 + 0] * Mm[0 * 3 + k] + Gm[r * 3 + 1] * Mm[1 * 3 + k] + Gm[r * 3 + 2] * Mm[2 * 3 + k]);
        if (out.dL_dscales)
#pragma unroll
            for (int k = 0; k < 3; k++)
                out.dL_dscales[3 * i + k] = LSR_SCALE_GRAD_MOD(mod) * (dM[0 * 3 + k] * R[0 * 3 + k] + dM[1 * 3 + k] * R[1 * 3 + k] + dM[2 * 3 + k] * R[2 * 3 + k]);
#pragma unroll
        for (int r = 0; r < 3; r++)
#pragma unroll
            for (int k = 0; k < 3; k++) dR[r * 3 + k] = dM[r * 3 + k] * sv[k];
        const float qr = q.x, qx = q.y, qy = q.z, qz = q.w;
        if (out.dL_drotations) {
            float4 gq;
            gq.x = 2.f * (-qz * dR[1] + qy * dR[2] + qz * dR[3] - qx * dR[5] - qy * dR[6] + qx * dR[7]);
            gq.y = 2.f * (qy * dR[1] + qz * dR[2] + qy * dR[3] - qr * dR[5] + qz * dR[6] + qr * dR[7]) - 4.f * qx * (dR[4] + dR[8]);
            gq.z = 2.f * (qx * dR[1] + qr * dR[2] + qx * dR[3] + qz * dR[5] - qr * dR[6] + qz * dR[7]) - 4.f * qy * (dR[0] + dR[8]);
            gq.w = 2.f * (-qr * dR[1] + qx * dR[2] + qr * dR[3] + qy * dR[5] + qx * dR[6] + qy * dR[7]) - 4.f * qz * (dR[0] + dR[4]);
            reinterpret_cast<float4*>(out.dL_drotations)[i] = gq;
        }
    }
}

template <bool COV>
__global__ void __launch_bounds__(256) k_preprocess_bwd(Cam c, lsr_inputs in, const uint8_t* __restrict__ geom,
                                                        const int32_t* __restrict__ radii,
                                                        const float* __restrict__ gacc, int VP, lsr_bwd_out out)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= in.P) return;
    const bool jac = ((const uint32_t*)(geom + geom_layout(in.P).flags))[0] != 0u;
    const float3* J = jac ? (const float3*)(geom + geom_layout(in.P).shjac) : nullptr;
    BwdRow row;
    row.load<COV>(in, radii, gacc, VP, i, J);
    preprocess_bwd_one<false>(c, in, geom, row, gacc, VP, out, i, nullptr, jac);
}

template <bool COV>
__global__ void __launch_bounds__(64) k_preprocess_bwd_sh16(Cam c, lsr_inputs in, const uint8_t* __restrict__ geom,
                                                            const int32_t* __restrict__ radii,
                                                            const float* __restrict__ gacc, int VP, lsr_bwd_out out)
{
    __shared__ float shl[64 * LSR_SH_ROW];
    const int b0 = blockIdx.x * 64, lane = threadIdx.x;
    const int cnt = min(64, in.P - b0);
    const bool sh = !in.colors_precomp;
    // jac (uniform): the forward stored the SH colour Jacobian, so the SH rows
    // are not read at all (the LDS tile only stages the SH gradient's stores)
    const bool jac = ((const uint32_t*)(geom + geom_layout(in.P).flags))[0] != 0u;
    const float3* J = jac ? (const float3*)(geom + geom_layout(in.P).shjac) : nullptr;
    BwdRow row;
    row.load<COV>(in, radii, gacc, VP, b0 + min(lane, cnt - 1), J);
    if (sh && !jac) {
        stage_sh_rows(shl, in.shs, b0, cnt, lane);
        __syncthreads();
    }
    if (lane < cnt) preprocess_bwd_one<true>(c, in, geom, row, gacc, VP, out, b0 + lane, shl + lane * LSR_SH_ROW, jac);
    if (sh && out.dL_dsh) {
        __syncthreads();
        float4* dst = reinterpret_cast<float4*>(out.dL_dsh) + (size_t)b0 * 12;
        for (int f = lane; f < cnt * 12; f += 64) {
            const int row = f / 12, c4 = f - row * 12;
            const float* s4 = shl + row * LSR_SH_ROW + c4 * 4;
            dst[f] = make_float4(s4[0], s4[1], s4[2], s4[3]);
        }
    }
}

hipError_t launch_preprocess_bwd(const Cam& c, const lsr_inputs& in, const uint8_t* geom, const int32_t* radii,
                                 const float* grad_acc, int VP, const lsr_bwd_out& out, hipStream_t st)
{
    if (in.P == 0) return hipSuccess;
    const bool sh16 = in.shs && in.max_coeffs == 16 && ((uintptr_t)in.shs % 16 == 0) &&
                      (!out.dL_dsh || (uintptr_t)out.dL_dsh % 16 == 0);
    const bool cov = in.cov3D_precomp != nullptr;
    if (sh16 && cov)
        k_preprocess_bwd_sh16<true><<<(in.P + 63) / 64, 64, 0, st>>>(c, in, geom, radii, grad_acc, VP, out);
    else if (sh16)
        k_preprocess_bwd_sh16<false><<<(in.P + 63) / 64, 64, 0, st>>>(c, in, geom, radii, grad_acc, VP, out);
    else if (cov)
        k_preprocess_bwd<true><<<(in.P + 255) / 256, 256, 0, st>>>(c, in, geom, radii, grad_acc, VP, out);
    else
        k_preprocess_bwd<false><<<(in.P + 255) / 256, 256, 0, st>>>(c, in, geom, radii, grad_acc, VP, out);
    return hipGetLastError();
}

__global__ void __launch_bounds__(256) k_sh_grad_from_views(int64_t N, int M, int deg, const float* __restrict__ means3D,
                                                            int R, const float* __restrict__ campos,
                                                            const float* __restrict__ drgb, float* __restrict__ dL_dsh)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    const float mx = means3D[3 * i], my = means3D[3 * i + 1], mz = means3D[3 * i + 2];
    float acc[48];
#pragma unroll
    for (int k = 0; k < 48; k++) acc[k] = 0.f;
    for (int r = 0; r < R; r++) {
        const float* g = drgb + ((size_t)r * N + i) * 3;
        const float g0 = g[0], g1 = g[1], g2 = g[2];
        if (g0 == 0.f && g1 == 0.f && g2 == 0.f) continue;   // outside this view (or clamped): adds exact zeros
        float dir[3], dor[3];
        sh_dir(mx, my, mz, campos + 3 * r, dir, dor);
        float bk[16];
        sh_basis(deg, dir[0], dir[1], dir[2], bk);
#pragma unroll
        for (int k = 0; k < 16; k++) {
            acc[3 * k] += bk[k] * g0;
            acc[3 * k + 1] += bk[k] * g1;
            acc[3 * k + 2] += bk[k] * g2;
        }
    }
    float* o = dL_dsh + (size_t)i * M * 3;
    for (int k = 0; k < M * 3; k++) o[k] = k < 48 ? acc[k] : 0.f;
}

hipError_t launch_sh_grad_from_views(int64_t N, int M, int deg, const float* means3D, int R, const float* campos,
                                     const float* drgb, float* dL_dsh, hipStream_t st)
{
    if (N == 0) return hipSuccess;
    k_sh_grad_from_views<<<(unsigned)((N + 255) / 256), 256, 0, st>>>(N, M, deg, means3D, R, campos, drgb, dL_dsh);
    return hipGetLastError();
}

__global__ void k_mark_visible(int P, const float* __restrict__ means, const float* __restrict__ view,
                               uint8_t* __restrict__ present)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P) return;
    const float3 pv = xform43(view, means[3 * i], means[3 * i + 1], means[3 * i + 2]);
    present[i] = pv.z > 0.2f ? 1 : 0;
}

hipError_t launch_mark_visible(int P, const float* means, const float* view, uint8_t* present, hipStream_t st)
{
    if (P == 0) return hipSuccess;
    k_mark_visible<<<(P + 255) / 256, 256, 0, st>>>(P, means, view, present);
    return hipGetLastError();
}

}  // namespace lsr
