// lsr_device.h — device-side math and layouts of the gfx950 rasterizer.
//
// Floating-point contract: every .hip file is compiled with -ffp-contract=off
// and each fused multiply-add is an explicit fmaf().  The operation sequence
// of every function here is the one the CPU restatement (oracle/lsr_oracle.c)
// specifies, so forward results are bit-identical to it.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define LSR_TILE 16
#define LSR_TILE_PIX 256
#define LSR_WAVE 64
// Gradient row layout (floats): [0,1] dL/dmean2D  [2,3,4] dL/dconic
// [5] dL/dopacity  [6,7,8] dL/dcolor  [12, 12+D) dL/dlanguage (16-B aligned)
#define LSR_GROW_LANG 12

namespace lsr {

// ------------------------------------------------------------------ math --
// Deterministic exp for x <= 0, shared bit for bit with the oracle
// (lso_expf): n = round(x log2 e) by the 1.5*2^23 magic-number fma, Cody-Waite
// reduction, a degree-6 near-minimax polynomial on |r| <= ln2/2 (<= 0.96 ulp
// measured), and 2^n inserted by a shift of the magic sum's bits.  11 VALU
// instructions after the range guard.  Replaces the CUDA reference's expf so
// results are reproducible on the CPU.
__device__ __forceinline__ float expf_det(float x)
{
    if (x < -87.0f) return 0.0f;
    const float t = fmaf(x, 1.44269504088896341f, 12582912.0f);
    const float n = t - 12582912.0f;
    float r = fmaf(n, -0.693145751953125f, x);
    r = fmaf(n, -1.428606765330187e-06f, r);
    float p = 0x1.6aea1ap-10f;
    p = fmaf(p, r, 0x1.1267d2p-7f);
    p = fmaf(p, r, 0x1.555820p-5f);
    p = fmaf(p, r, 0x1.555418p-3f);
    p = fmaf(p, r, 0x1.fffffcp-2f);
    p = fmaf(p, r, 1.0f);
    p = fmaf(p, r, 1.0f);
    return p * __uint_as_float((__float_as_uint(t) << 23) + 0x3f800000u);
}

// Two expf_det at once on packed f32 (v_pk_fma/add/mul: each half rounds
// exactly as the scalar instruction), bitwise equal to expf_det for
// x >= -87.  Below, x is clamped to -87 (one v_med3_f32 per half): the result is then
// ~1e-38 where expf_det returns 0, and every caller rejects both (alpha <
// 1/255), so the decisions are expf_det's.  The clamp is needed: a staged
// 8x8 block of a needle splat (2D condition number 1e5+) holds pixels with
// power of -100 .. -1000, where n = round(x log2 e) < -127 wraps the exponent
// bits below to a huge positive scale (alpha 0.99 far off the needle).
typedef float lsr_f32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t lsr_u32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ lsr_f32x2 expf_det2(lsr_f32x2 x)
{
    x = lsr_f32x2{__builtin_amdgcn_fmed3f(x.x, -87.0f, 1.0e30f), __builtin_amdgcn_fmed3f(x.y, -87.0f, 1.0e30f)};
    const lsr_f32x2 t = __builtin_elementwise_fma(x, lsr_f32x2{1.44269504088896341f, 1.44269504088896341f},
                                                  lsr_f32x2{12582912.0f, 12582912.0f});
    const lsr_f32x2 n = t - lsr_f32x2{12582912.0f, 12582912.0f};
    lsr_f32x2 r = __builtin_elementwise_fma(n, lsr_f32x2{-0.693145751953125f, -0.693145751953125f}, x);
    r = __builtin_elementwise_fma(n, lsr_f32x2{-1.428606765330187e-06f, -1.428606765330187e-06f}, r);
    lsr_f32x2 p = lsr_f32x2{0x1.6aea1ap-10f, 0x1.6aea1ap-10f};
    p = __builtin_elementwise_fma(p, r, lsr_f32x2{0x1.1267d2p-7f, 0x1.1267d2p-7f});
    p = __builtin_elementwise_fma(p, r, lsr_f32x2{0x1.555820p-5f, 0x1.555820p-5f});
    p = __builtin_elementwise_fma(p, r, lsr_f32x2{0x1.555418p-3f, 0x1.555418p-3f});
    p = __builtin_elementwise_fma(p, r, lsr_f32x2{0x1.fffffcp-2f, 0x1.fffffcp-2f});
    p = __builtin_elementwise_fma(p, r, lsr_f32x2{1.0f, 1.0f});
    p = __builtin_elementwise_fma(p, r, lsr_f32x2{1.0f, 1.0f});
    const lsr_u32x2 tb = __builtin_bit_cast(lsr_u32x2, t);
    const lsr_u32x2 sb = (tb << 23) + lsr_u32x2{0x3f800000u, 0x3f800000u};
    return p * __builtin_bit_cast(lsr_f32x2, sb);
}

// Wave votes on a bool.  HIP's __ballot/__any take an int, which makes the
// compiler round-trip an SGPR lane mask through a VGPR (v_cndmask + v_cmp,
// 2 VALU per vote); the builtin on i1 stays on the scalar unit.
__device__ __forceinline__ uint64_t wave_ballot(bool b) { return __builtin_amdgcn_ballot_w64(b); }
__device__ __forceinline__ bool wave_any(bool b) { return __builtin_amdgcn_ballot_w64(b) != 0; }

// Wait for the wave's outstanding LDS operations; the memory clobber keeps
// the compiler from moving LDS accesses across it (wave-private LDS staging
// needs no workgroup barrier).
// (tools/variants/lds_nowait.patch: the compiler-only form, -0.8 % render_bwd, not taken)
__device__ __forceinline__ void wave_lds_fence() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// float -> int truncating + saturating; NaN -> 0 (matches oracle f2i).
// Branch-free: the clamp keeps the conversion in range (one v_cvt_i32_f32),
// the two selects give the saturated top and NaN.  (The branchy form made
// the quick render's staging wait on each code's LDS read separately.)
__device__ __forceinline__ int f2i(float v)
{
    const float c = fminf(fmaxf(v, -2147483648.0f), 2147483520.0f);   // NaN -> -2^31
    int r = (int)c;
    r = v >= 2147483520.0f ? 2147483647 : r;
    return v != v ? 0 : r;
}

// An fp32-encoded code index (u5): round half up, floor(v + 0.5); NaN and
// values outside [0, 2^31) -> -1 (dropped as every out-of-range code is).
__device__ __forceinline__ int quick_code_f32(float v)
{
    const float r = floorf(v + 0.5f);
    return (r >= 0.0f && r < 2147483648.0f) ? (int)r : -1;
}

// Quick-path code index m of a Gaussian's sparse language row: fp32-encoded
// integers as quick_code_f32, int32 as is, int64 outside [0, 2^31) -> -1;
// packed rows (LSR_INDEX_PACKED, K = 12): byte m of the row's 16 B, code + 1.
__device__ __forceinline__ int quick_index(const void* qi, int dtype, size_t off)
{
    if (dtype == 0) return quick_code_f32(((const float*)qi)[off]);
    if (dtype == 1) return ((const int32_t*)qi)[off];
    if (dtype == 3) {
        const size_t i = off / 12, m = off - i * 12;
        const uint32_t w = ((const uint32_t*)qi)[4 * i + (m >> 2)];
        return (int)((w >> (8 * (m & 3))) & 0xffu) - 1;
    }
    const int64_t v = ((const int64_t*)qi)[off];
    return (v < 0 || v > 0x7fffffff) ? -1 : (int)v;
}

__device__ __forceinline__ float ndc2pix(float v, int S)
{
    return (float)((((double)v + 1.0) * (double)S - 1.0) * 0.5);
}

__device__ __forceinline__ void get_rect(float px, float py, int r, int gx, int gy, int& x0, int& y0, int& x1, int& y1)
{
    x0 = min(gx, max(0, f2i((px - (float)r) / 16.0f)));
    y0 = min(gy, max(0, f2i((py - (float)r) / 16.0f)));
    x1 = min(gx, max(0, f2i((px + (float)r + 16.0f - 1.0f) / 16.0f)));
    y1 = min(gy, max(0, f2i((py + (float)r + 16.0f - 1.0f) / 16.0f)));
}

// Column-major 4x4 (m[c*4+r]) point transforms.
__device__ __forceinline__ float3 xform43(const float* m, float x, float y, float z)
{
    return make_float3(m[0] * x + m[4] * y + m[8] * z + m[12],
                       m[1] * x + m[5] * y + m[9] * z + m[13],
                       m[2] * x + m[6] * y + m[10] * z + m[14]);
}
__device__ __forceinline__ float4 xform44(const float* m, float x, float y, float z)
{
    return make_float4(m[0] * x + m[4] * y + m[8] * z + m[12],
                       m[1] * x + m[5] * y + m[9] * z + m[13],
                       m[2] * x + m[6] * y + m[10] * z + m[14],
                       m[3] * x + m[7] * y + m[11] * z + m[15]);
}

// Quaternion (r,x,y,z) -> row-major R (utils/general_utils.py:90-98, no renormalisation).
__device__ __forceinline__ void quat_to_R(float r, float x, float y, float z, float* R)
{
    R[0] = 1.f - 2.f * (y * y + z * z);
    R[1] = 2.f * (x * y - r * z);
    R[2] = 2.f * (x * z + r * y);
    R[3] = 2.f * (x * y + r * z);
    R[4] = 1.f - 2.f * (x * x + z * z);
    R[5] = 2.f * (y * z - r * x);
    R[6] = 2.f * (x * z - r * y);
    R[7] = 2.f * (y * z + r * x);
    R[8] = 1.f - 2.f * (x * x + y * y);
}

__device__ __forceinline__ void compute_cov3D(float s0, float s1, float s2, float mod, float4 q, float* cov)
{
    float R[9], Mm[9];
    quat_to_R(q.x, q.y, q.z, q.w, R);
    float sx = mod * s0, sy = mod * s1, sz = mod * s2;
#pragma unroll
    for (int i = 0; i < 3; i++) {
        Mm[i * 3 + 0] = R[i * 3 + 0] * sx;
        Mm[i * 3 + 1] = R[i * 3 + 1] * sy;
        Mm[i * 3 + 2] = R[i * 3 + 2] * sz;
    }
#define LSR_SIG(i, j) (Mm[(i)*3 + 0] * Mm[(j)*3 + 0] + Mm[(i)*3 + 1] * Mm[(j)*3 + 1] + Mm[(i)*3 + 2] * Mm[(j)*3 + 2])
    cov[0] = LSR_SIG(0, 0);
    cov[1] = LSR_SIG(0, 1);
    cov[2] = LSR_SIG(0, 2);
    cov[3] = LSR_SIG(1, 1);
    cov[4] = LSR_SIG(1, 2);
    cov[5] = LSR_SIG(2, 2);
#undef LSR_SIG
}

struct Ewa {
    float tx, ty, tz;
    bool xclamp, yclamp;
    float J00, J02, J11, J12;
    float T0[3], T1[3];
};

__device__ __forceinline__ void ewa_setup(const float* view, float3 pv, float fx, float fy, float tanfx, float tanfy, Ewa& e)
{
    const float limx = 1.3f * tanfx, limy = 1.3f * tanfy;
    float txtz = pv.x / pv.z, tytz = pv.y / pv.z;
    e.xclamp = (txtz < -limx) || (txtz > limx);
    e.yclamp = (tytz < -limy) || (tytz > limy);
    e.tz = pv.z;
    e.tx = fminf(limx, fmaxf(-limx, txtz)) * pv.z;
    e.ty = fminf(limy, fmaxf(-limy, tytz)) * pv.z;
    float tz2 = e.tz * e.tz;
    e.J00 = fx / e.tz;
    e.J02 = -(fx * e.tx) / tz2;
    e.J11 = fy / e.tz;
    e.J12 = -(fy * e.ty) / tz2;
#pragma unroll
    for (int j = 0; j < 3; j++) {
        e.T0[j] = e.J00 * view[j * 4 + 0] + e.J02 * view[j * 4 + 2];
        e.T1[j] = e.J11 * view[j * 4 + 1] + e.J12 * view[j * 4 + 2];
    }
}

__device__ __forceinline__ void ewa_uv(const Ewa& e, const float* c, float* u, float* v)
{
    u[0] = c[0] * e.T0[0] + c[1] * e.T0[1] + c[2] * e.T0[2];
    u[1] = c[1] * e.T0[0] + c[3] * e.T0[1] + c[4] * e.T0[2];
    u[2] = c[2] * e.T0[0] + c[4] * e.T0[1] + c[5] * e.T0[2];
    v[0] = c[0] * e.T1[0] + c[1] * e.T1[1] + c[2] * e.T1[2];
    v[1] = c[1] * e.T1[0] + c[3] * e.T1[1] + c[4] * e.T1[2];
    v[2] = c[2] * e.T1[0] + c[4] * e.T1[1] + c[5] * e.T1[2];
}

__device__ __forceinline__ void ewa_cov2D(const Ewa& e, const float* c, float& a, float& b, float& cc)
{
    float u[3], v[3];
    ewa_uv(e, c, u, v);
    a = e.T0[0] * u[0] + e.T0[1] * u[1] + e.T0[2] * u[2] + 0.3f;
    b = e.T0[0] * v[0] + e.T0[1] * v[1] + e.T0[2] * v[2];
    cc = e.T1[0] * v[0] + e.T1[1] * v[1] + e.T1[2] * v[2] + 0.3f;
}

__constant__ static const float SH_C0 = 0.28209479177387814f;
__constant__ static const float SH_C1 = 0.4886025119029199f;
#define LSR_C2_0 1.0925484305920792f
#define LSR_C2_1 (-1.0925484305920792f)
#define LSR_C2_2 0.31539156525252005f
#define LSR_C2_3 (-1.0925484305920792f)
#define LSR_C2_4 0.5462742152960396f
#define LSR_C3_0 (-0.5900435899266435f)
#define LSR_C3_1 2.890611442640554f
#define LSR_C3_2 (-0.4570457994644658f)
#define LSR_C3_3 0.3731763325901154f
#define LSR_C3_4 (-0.4570457994644658f)
#define LSR_C3_5 1.445305721320277f
#define LSR_C3_6 (-0.5900435899266435f)

// SH -> RGB (+0.5, pre-clamp), term order of utils/sh_utils.py:57-112.
// sh points at the Gaussian's (M,3) block.
__device__ __forceinline__ float sh_channel(int deg, const float* sh, int ch, float x, float y, float z)
{
#define S(k) sh[(k)*3 + ch]
    float r = 0.28209479177387814f * S(0);
    if (deg > 0) {
        const float c1 = 0.4886025119029199f;
        r = r - c1 * y * S(1) + c1 * z * S(2) - c1 * x * S(3);
        if (deg > 1) {
            float xx = x * x, yy = y * y, zz = z * z;
            float xy = x * y, yz = y * z, xz = x * z;
            r = r + LSR_C2_0 * xy * S(4) + LSR_C2_1 * yz * S(5) + LSR_C2_2 * (2.0f * zz - xx - yy) * S(6) +
                LSR_C2_3 * xz * S(7) + LSR_C2_4 * (xx - yy) * S(8);
            if (deg > 2) {
                r = r + LSR_C3_0 * y * (3.0f * xx - yy) * S(9) + LSR_C3_1 * xy * z * S(10) +
                    LSR_C3_2 * y * (4.0f * zz - xx - yy) * S(11) +
                    LSR_C3_3 * z * (2.0f * zz - 3.0f * xx - 3.0f * yy) * S(12) +
                    LSR_C3_4 * x * (4.0f * zz - xx - yy) * S(13) + LSR_C3_5 * z * (xx - yy) * S(14) +
                    LSR_C3_6 * x * (xx - 3.0f * yy) * S(15);
            }
        }
    }
#undef S
    return r + 0.5f;
}

__device__ __forceinline__ void sh_dir(float mx, float my, float mz, const float* campos, float* dir, float* dor)
{
    dor[0] = mx - campos[0];
    dor[1] = my - campos[1];
    dor[2] = mz - campos[2];
    float len = sqrtf(dor[0] * dor[0] + dor[1] * dor[1] + dor[2] * dor[2]);
    dir[0] = dor[0] / len;
    dir[1] = dor[1] / len;
    dir[2] = dor[2] / len;
}

// The per-pair Gaussian exponent (A.3), shared by forward and backward.
__device__ __forceinline__ float splat_power(float ca, float cb, float cc, float dx, float dy)
{
    return fmaf(-0.5f, fmaf(ca * dx, dx, (cc * dy) * dy), -((cb * dx) * dy));
}

// Conservative exponent cut: for power < cut, opacity*exp(power) < 1/255 is
// certain, so the pair is skipped without evaluating exp.  Never changes a
// result (the margin 0.02 dwarfs exp/log rounding); only saves work.
// The logarithm is taken in double and rounded once, so the value is the
// oracle's (lso_power_cut) bit for bit: the binning's tile cull (tile_keep)
// decides with it, and both sides must emit the same instance lists.
__device__ __forceinline__ float power_cut(float o)
{
    if (!(o * 255.0f > 1.0f)) return (o == o) ? -0.02f : -INFINITY;
    return (float)(-log((double)(255.0f * o))) - 0.02f;
}

// The cut as stored in the splat record: power_cut widened by the fp32
// conic's conditioning K = ca cc / det (>= 1).  Every test that uses the cut
// (the binning's cull_box / row_span, the render's block_overlap_exact and
// cut_extent) evaluates an ellipse from ca, cb, cc in fp32, and the render
// evaluates splat_power in fp32; for a needle splat (K ~ 1e5 after the 0.3 px
// dilation) det = ca cc - cb^2 keeps only ~log2(1/K) of its bits and the
// quadratic form's rounding grows like eps K |q|.  Scaling the cut by
// (1 + 8e-6 K) -- 4x the worst-case fp32 error of both (2 eps K for det,
// ~12 eps K for q) -- keeps every test conservative however thin the splat;
// at the usual K < 100 it widens the cut by < 1e-3.  A widened cut only keeps
// more instances / candidates, never changes an output.  det <= 0 in fp32:
// -inf (no cull at all).  The oracle restates it operation for operation
// (lso_cut_widen).
__device__ __forceinline__ float cut_widen(float cut, float ca, float cb, float cc)
{
    const float p = ca * cc;
    const float det = p - cb * cb;
    if (!(det > 0.f)) return -INFINITY;
    const float K = p / det;
    return cut * fmaf(K, 8e-6f, 1.0f);
}

// Conservative half-extents (pixels) of the region where power >= cut, i.e.
// where a pair can contribute: the cut ellipse Q(d) <= 2|cut| has bounding
// half-widths sqrt(2|cut| * cov2D.xx) and sqrt(2|cut| * cov2D.yy) (the conic
// is the inverse 2D covariance).  +2 px margin; packed as two u16 into the
// splat record's last word.  Anything degenerate gets the no-skip maximum.
__device__ __forceinline__ uint32_t cut_extent(float cut, float a, float c, float det)
{
    uint32_t hx = 65535u, hy = 65535u;
    if (det > 0.f && cut > -3.0e38f && cut <= 0.f) {
        const float r2 = -2.f * cut;
        const float ex = sqrtf(r2 * a), ey = sqrtf(r2 * c);
        if (ex < 65000.f) hx = (uint32_t)ceilf(ex) + 2u;
        if (ey < 65000.f) hy = (uint32_t)ceilf(ey) + 2u;
    }
    return hx | (hy << 16);
}

// Does the Gaussian (center x,y; packed extents) possibly touch the 8x8 pixel
// block whose top-left pixel is (bx, by)?
// rect_overlap: the same for a (EX+1) x (EY+1) pixel rectangle.
__device__ __forceinline__ bool rect_overlap(float x, float y, uint32_t ext, int bx, int by, int EX, int EY)
{
    const float hx = (float)(ext & 0xffffu), hy = (float)(ext >> 16);
    return (x + hx >= (float)bx) && (x - hx <= (float)(bx + EX)) && (y + hy >= (float)by) && (y - hy <= (float)(by + EY));
}
__device__ __forceinline__ bool block_overlap(float x, float y, uint32_t ext, int bx, int by)
{
    return rect_overlap(x, y, ext, bx, by, 7, 7);
}

// Exact (conservative) test: does the cut ellipse {d : Q(d) <= -2 cut},
// Q(d) = ca dx^2 + 2 cb dx dy + cc dy^2 with d = (x, y) - pixel, meet the
// pixel rectangle [bx, bx+7] x [by, by+7]?  Q is convex, so its minimum over
// the rectangle is 0 when the centre is inside, else it lies on an edge; on
// each edge Q is a 1-D quadratic minimised at a clamped stationary point.  A
// relative + absolute margin keeps the test conservative under rounding, so
// every pair the blend would accept survives (results stay bit-identical);
// the bounding-box test (block_overlap) keeps far more false candidates for
// thin, rotated splats.
// rect_overlap_exact: the test for the (EX+1) x (EY+1) rectangle at (bx, by)
// (the reciprocals only past the early exits: the render's staging mostly
// exits early).
__device__ __forceinline__ bool rect_overlap_exact(float x, float y, float ca, float cb, float cc, float cut,
                                                   int bx, int by, float EX, float EY)
{
    if (!(ca > 0.f) || !(cc > 0.f) || !(cut > -3.0e38f)) return true;   // degenerate / no cut: keep
    const float thr = fmaf(-2.f * cut, 1.001f, 1e-3f);
    const float u1 = x - (float)bx, u0 = u1 - EX;
    const float v1 = y - (float)by, v0 = v1 - EY;
    if (u0 <= 0.f && u1 >= 0.f && v0 <= 0.f && v1 >= 0.f) return true;
    // hardware reciprocals (1 ulp) instead of IEEE divisions (~10 VALU each):
    // they only place the edge minimisers, and q at a slightly displaced point
    // exceeds the edge minimum by ca * (displacement)^2 ~ 1e-14 relative, far
    // inside the 1e-3 + 0.1 % margin of thr (render_fwd -2.2 %, r04)
    const float ica = __builtin_amdgcn_rcpf(ca), icc = __builtin_amdgcn_rcpf(cc);
    auto q = [&](float u, float v) { return fmaf(ca * u, u, fmaf(2.f * cb * u, v, cc * v * v)); };
    const float va = fminf(fmaxf(-cb * u0 * icc, v0), v1);
    const float vb = fminf(fmaxf(-cb * u1 * icc, v0), v1);
    const float ua = fminf(fmaxf(-cb * v0 * ica, u0), u1);
    const float ub = fminf(fmaxf(-cb * v1 * ica, u0), u1);
    const float qmin = fminf(fminf(q(u0, va), q(u1, vb)), fminf(q(ua, v0), q(ub, v1)));
    return !(qmin > thr);
}
__device__ __forceinline__ bool block_overlap_exact(float x, float y, float ca, float cb, float cc, float cut,
                                                    int bx, int by)
{
    return rect_overlap_exact(x, y, ca, cb, cc, cut, bx, by, 7.f, 7.f);
}

// Binning's tile cull: can Gaussian (splat records A, B) contribute to any
// pixel of tile (tx, ty)?  The exact cut-ellipse test on the whole 16x16 tile
// (no clipping at the image border).  A rejected instance has alpha < 1/255 at
// every pixel of its tile, so dropping it from the tile's list changes no
// output; the reference's 3-sigma rect (A.2) emits 43 % more instances at cfg3
// (tools/bin_cull_census.py).
#ifndef LSR_TILE_CULL
#define LSR_TILE_CULL 1     // 0: the reference's full rect lists (A/B timing only; the oracle's cull=False)
#endif
// The tile cull's box: the tiles whose 16x16 pixel rectangle meets the
// axis-aligned box of the cut ellipse {q <= thr}, q(d) = ca dx^2 + 2 cb dx dy
// + cc dy^2, thr = -2 cut (1.001) + 1e-3, widened by 1e-4 relative + 0.5 px.
// The cull keeps an instance (Gaussian, tile) iff the tile is inside this box
// AND inside its row's span (row_span below); the oracle restates the same
// rule (lso_cull_box, lso_row_span).  A tile outside both cannot meet the
// ellipse, so nothing that contributes is dropped
// (tests/test_oracle.py::test_tile_cull_changes_no_output,
// tests/test_cull_vs_full.py).  Shrinks [x0, x1) x [y0, y1) in place.
__device__ __forceinline__ void cull_box(float x, float y, float ca, float cb, float cc, float cut, int& x0, int& y0,
                                         int& x1, int& y1)
{
    if (!LSR_TILE_CULL) return;
    if (!(ca > 0.f) || !(cc > 0.f) || !(cut > -3.0e38f)) return;
    const float det = ca * cc - cb * cb;
    if (!(det > 0.f)) return;
    const float thr = fmaf(-2.f * cut, 1.001f, 1e-3f);
    const float ue = fmaf(sqrtf(thr * cc / det), 1.0001f, 0.5f);
    const float ve = fmaf(sqrtf(thr * ca / det), 1.0001f, 0.5f);
    if (!(ue < 1.0e7f) || !(ve < 1.0e7f)) return;
    // tile t meets [x - ue, x + ue] iff 16 t <= x + ue and 16 t + 15 >= x - ue
    const float tx0 = ceilf((x - ue - 15.f) / 16.f), tx1 = floorf((x + ue) / 16.f) + 1.f;
    const float ty0 = ceilf((y - ve - 15.f) / 16.f), ty1 = floorf((y + ve) / 16.f) + 1.f;
    x0 = max(x0, f2i(fmaxf(tx0, -1.f)));
    y0 = max(y0, f2i(fmaxf(ty0, -1.f)));
    x1 = min(x1, f2i(fmaxf(tx1, -1.f)));
    y1 = min(y1, f2i(fmaxf(ty1, -1.f)));
}

// Row-span tile cull.  Per Gaussian, the cut ellipse {q <= thr} (cull_box)
// is intersected with each tile row's pixel band [16 ty,
// 16 ty + 15]; the x-extent of that piece, widened by 1e-3 of the ellipse's
// half width + 0.05 px, is a contiguous tile range.  The cull keeps (Gaussian,
// tile) iff the tile is in cull_box and in its row's range, so the binning
// walks exactly the kept instances, with no per-tile test.  Over a row the
// right edge u(v) = (-cb v + sqrt(thr ca - det v^2)) / ca is concave in v, so
// its maximum is at the row's v nearest v_r = -cb sqrt(thr / (det cc)) (the
// ellipse's rightmost point), the left edge's minimum at -v_r.  Rows outside
// |v| <= the (widened) vertical half extent are empty.  Restated operation
// for operation by the oracle (lso_span_prep / lso_row_span).
struct SpanPrep {
    float x, y, vm, vr, cb, det, tca, ica, me;
};
__device__ __forceinline__ SpanPrep span_prep(float x, float y, float ca, float cb, float cc, float cut)
{
    SpanPrep s;
    s.x = x;
    s.y = y;
    const float det = ca * cc - cb * cb;
    const float thr = fmaf(-2.f * cut, 1.001f, 1e-3f);
    const float tcd = thr / det;
    const bool all = !LSR_TILE_CULL || !(ca > 0.f) || !(cc > 0.f) || !(cut > -3.0e38f) || !(det > 0.f) ||
                     !(tcd < 1.0e30f);
    if (all) {   // degenerate / no cut: every tile of the box row
        s.vm = INFINITY; s.vr = 0.f; s.cb = 0.f; s.det = 1.f; s.tca = 1.f; s.ica = 1.f; s.me = INFINITY;
        return s;
    }
    s.vm = fmaf(sqrtf(tcd * ca), 1.0001f, 0.01f);
    s.vr = -cb * sqrtf(tcd / cc);
    s.cb = cb;
    s.det = det;
    s.tca = thr * ca;
    s.ica = 1.f / ca;
    s.me = fmaf(sqrtf(tcd * cc), 1e-3f, 0.05f);
    return s;
}
// Kept tiles [sx0, sx1) of tile row ty inside the box columns [bx0, bx1).
__device__ __forceinline__ void row_span(const SpanPrep& s, int ty, int bx0, int bx1, int& sx0, int& sx1)
{
    const float v1 = s.y - (float)(ty * LSR_TILE), v0 = v1 - 15.f;
    const float w0 = fmaxf(v0, -s.vm), w1 = fminf(v1, s.vm);
    const float a = fminf(fmaxf(s.vr, w0), w1), b = fminf(fmaxf(-s.vr, w0), w1);
    const float ra = sqrtf(fmaxf(fmaf(-s.det * a, a, s.tca), 0.f));
    const float rb = sqrtf(fmaxf(fmaf(-s.det * b, b, s.tca), 0.f));
    const float umax = fmaf(ra - s.cb * a, s.ica, s.me);
    const float umin = fmaf(-rb - s.cb * b, s.ica, -s.me);
    // tile t meets [x - umax, x - umin] iff 16 t <= x - umin and 16 t + 15 >= x - umax
    const float fx0 = ceilf((s.x - umax - 15.f) / 16.f);
    const float fx1 = floorf((s.x - umin) / 16.f) + 1.f;
    sx0 = f2i(fminf(fmaxf(fx0, (float)bx0), (float)bx1));
    sx1 = f2i(fminf(fmaxf(fx1, (float)bx0), (float)bx1));
    if (!(w0 <= w1) || sx1 < sx0) sx1 = sx0;
}
__device__ __forceinline__ SpanPrep span_prep(const float4& A, const float4& B)
{
    return span_prep(A.x, A.y, A.z, A.w, B.x, B.z);
}

// Partner value across lanes l <-> l ^ M without the LDS crossbar: the ISA
// has a register path for every distance: v_permlane32_swap (M = 32),
// v_permlane16_swap (M = 16), DPP row_ror:8 (M = 8), two DPP row rotations
// and a select (M = 4), DPP quad_perm (M = 2, 1).
template <int M>
__device__ __forceinline__ uint32_t xor_lane_u32(uint32_t x)
{
    const int lane = threadIdx.x & 63;
    if constexpr (M == 32) {
        auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
        return (lane & 32) ? r[0] : r[1];
    } else if constexpr (M == 16) {
        auto r = __builtin_amdgcn_permlane16_swap(x, x, false, false);
        return (lane & 16) ? r[0] : r[1];
    } else if constexpr (M == 8) {
        return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x128, 0xF, 0xF, false);   // row_ror:8
    } else if constexpr (M == 4) {
        // l ^ 4 inside a row of 16.  row_ror:N makes lane l read lane (l - N) mod 16
        // (as row_shr:N reads l - N), so row_ror:4 gives x[l - 4] (the partner
        // where bit 2 of l is set) and row_ror:12 gives x[l + 4] (bit 2 clear).
        const uint32_t from_below = (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x124, 0xF, 0xF, false);
        const uint32_t from_above = (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x12C, 0xF, 0xF, false);
        return (lane & 4) ? from_below : from_above;
    } else if constexpr (M == 2) {
        return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x4E, 0xF, 0xF, false);    // quad_perm [2,3,0,1]
    } else if constexpr (M == 1) {
        return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xF, 0xF, false);    // quad_perm [1,0,3,2]
    } else {
        return (uint32_t)__shfl_xor((int)x, M, 64);
    }
}

// ------------------------------------------------------------- layouts --
// Geometry workspace (per Gaussian, SoA, every section 256-B aligned).
struct GeomLayout {
    size_t splatA, splatB, rgb, depth, tiles, offsets, clamped, scan_part, shjac, flags, total;
    // splatA = {x, y, conic.a, conic.b}; splatB = {conic.c, opacity, cut, extent bits}
};

__host__ __device__ inline size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

__host__ __device__ inline GeomLayout geom_layout(size_t N)
{
    GeomLayout L;
    size_t o = 0;
    L.splatA = o;   o += align256(N * 16);  // float4 {x, y, conic.a, conic.b}
    L.splatB = o;   o += align256(N * 16);  // float4 {conic.c, opacity, cut, u16x2 cut extents}
    L.rgb = o;      o += align256(N * 12);
    L.depth = o;    o += align256(N * 4);
    L.tiles = o;    o += align256(N * 4);
    L.offsets = o;  o += align256(N * 4);   // inclusive scan of tiles
    L.clamped = o;  o += align256(N * 4);   // 3-bit mask
    L.scan_part = o; o += align256(((N + 4095) / 4096 + 1) * 8);
    // SH colour Jacobian d(RGB)/d(dir) (3 x float3 per Gaussian: ddx[0..2], ddy[0..2],
    // ddz[0..2]), written by a forward with a geometry gradient pending and read by
    // the preprocess backward instead of the 192-B SH row (preprocess.hip)
    L.shjac = o;    o += align256(N * 36);
    L.flags = o;    o += 256;               // [0] = 1: this forward wrote shjac
    L.total = o;
    return L;
}

// Row stride of the privatised binning's B x T count table (16-B rows).
__host__ __device__ inline int table_stride(int T) { return (T + 3) & ~3; }

// Image workspace (per pixel + per tile).
struct ImageLayout {
    size_t final_T, n_contrib, tile_cnt, tile_start, tile_part, cls_cnt, cls_list, border, total;
};

__host__ __device__ inline ImageLayout image_layout(size_t P, size_t T)
{
    ImageLayout L;
    size_t o = 0;
    L.final_T = o;    o += align256(P * 4);
    L.n_contrib = o;  o += align256(P * 4);
    L.tile_cnt = o;   o += align256(T * 4);
    L.tile_start = o; o += align256((T + 1) * 4);   // exclusive scan, [T] = num_rendered
    L.tile_part = o;  o += align256(((T + 63) / 64 + 1) * 8);   // scan partials / 64-tile group bases
    L.cls_cnt = o;    o += 512;                        // per-class tile counts (tile-sort classes); word 32: ticket;
                                                       // words 64-65: the tile count's total + arrivals
    L.cls_list = o;   o += align256(T * 6 * 4);        // per-class tile lists, T slots each
    L.border = o;     o += align256(T * 4 * 16);       // the list-driven backward's block order (k_bwd_order)
    L.total = o;
    return L;
}

// Binning workspace (per instance).
struct BinLayout {
    size_t rank, keys, point_list, total;
};

__host__ __device__ inline BinLayout bin_layout(size_t M)
{
    BinLayout L;
    size_t o = 0;
    L.rank = o;       o += align256(M * 4);
    L.keys = o;       o += align256(M * 8);
    L.point_list = o; o += align256(M * 4);
    L.total = o;
    return L;
}

// XCD-aware bijective block remap: blocks b, b+8, b+16 ... (one XCD under
// round-robin dispatch) receive consecutive work items, so neighbouring tiles
// share an L2.  Speed only; correctness never depends on placement.
__device__ __forceinline__ int xcd_remap(int b, int nb)
{
    const int q = nb / 8, r = nb % 8;
    const int xcd = b % 8, k = b / 8;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + k;
}

}  // namespace lsr
