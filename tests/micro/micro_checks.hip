// micro_checks.hip — GPU self-checks of two hardware facts the product relies
// on, folded into `pytest -m gpu` (tests/test_micro_checks.py) from the
// round-3 tools/micro programs.  Test infrastructure: built by build() into
// tests/micro/libmicro_checks.so, never linked by the product.
//
//  * micro_dpp_xor: the wave sort's register-path lane exchange
//    (lsr::xor_lane_u32, lsr_device.h: permlane32/16 swaps, DPP row rotations,
//    quad_perm) equals __shfl_xor for every distance M = 1..32 on several value
//    patterns.  Round 3's first distance-4 exchange had its two rotations
//    swapped and faulted the render through invalid ids.
//  * micro_mfma_order: v_mfma_f32_16x16x4_f32 (the forward's ML form and the
//    backward's contractions) is bitwise a fmaf chain over k = 0..3 in order,
//    including zeros, signed zeros, subnormal operands and accumulators,
//    infinities and NaN (compared as NaN), which is what keeps the MFMA
//    forward bit-identical to the oracle's sequential fmaf blend.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "lsr_device.h"

typedef float mc_f32x4 __attribute__((ext_vector_type(4)));

template <int M>
__device__ uint32_t xor_check(uint32_t x)
{
    return lsr::xor_lane_u32<M>(x) ^ (uint32_t)__shfl_xor((int)x, M, 64);
}

__global__ void k_dpp_xor(const uint32_t* __restrict__ vals, int npat, uint32_t* __restrict__ out)
{
    const int l = threadIdx.x;
    uint32_t bad[6] = {0, 0, 0, 0, 0, 0};
    for (int p = 0; p < npat; p++) {
        const uint32_t x = vals[p * 64 + l];
        bad[0] |= xor_check<1>(x);
        bad[1] |= xor_check<2>(x);
        bad[2] |= xor_check<4>(x);
        bad[3] |= xor_check<8>(x);
        bad[4] |= xor_check<16>(x);
        bad[5] |= xor_check<32>(x);
    }
    for (int m = 0; m < 6; m++) out[m * 64 + l] = bad[m];
}

__global__ void k_mfma(const float* A, const float* B, const float* C, float* D, int reps)
{
    const int l = threadIdx.x;
    for (int r = blockIdx.x; r < reps; r += gridDim.x) {
        const float* a = A + r * 64;
        const float* b = B + r * 64;
        const float* c = C + r * 256;
        // A[i][k]: lane l supplies A[l & 15][l >> 4]; B[k][j]: lane l supplies B[l >> 4][l & 15]
        const float av = a[(l & 15) * 4 + (l >> 4)];
        const float bv = b[(l >> 4) * 16 + (l & 15)];
        mc_f32x4 acc;
        for (int q = 0; q < 4; q++) acc[q] = c[(4 * (l >> 4) + q) * 16 + (l & 15)];
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc, 0, 0, 0);
        for (int q = 0; q < 4; q++) D[r * 256 + (4 * (l >> 4) + q) * 16 + (l & 15)] = acc[q];
    }
}

namespace {
struct Rng {
    uint64_t s;
    uint32_t next() { s = s * 6364136223846793005ull + 1442695040888963407ull; return (uint32_t)(s >> 32); }
    float unit() { return (next() >> 8) * (1.0f / 16777216.0f); }
};
float f_from_bits(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
uint32_t bits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
// a random operand: mostly wide-exponent normals; with `specials`, also
// +-0, subnormals, +-inf, NaN and values near the overflow edge
float operand(Rng& g, int specials)
{
    const float n = (g.unit() - 0.5f) * ldexpf(1.f, (int)(g.next() % 41) - 20);
    if (!specials) return n;
    switch (g.next() % 16) {
        case 0: return 0.f;
        case 1: return -0.f;
        case 2: return f_from_bits((g.next() & 0x007fffffu) | 1u);                  // +subnormal
        case 3: return f_from_bits(((g.next() & 0x007fffffu) | 1u) | 0x80000000u);  // -subnormal
        case 4: return f_from_bits(0x00800000u + (g.next() & 0xffffu));             // near FLT_MIN
        case 5: return (g.next() & 1) ? INFINITY : -INFINITY;
        case 6: return (g.unit() + 0.5f) * ldexpf(1.f, 120 + (int)(g.next() % 8));   // near overflow
        case 7: if (g.next() % 4 == 0) return NAN; return n;
        default: return n;
    }
}
bool same(float x, float y) { return (std::isnan(x) && std::isnan(y)) || bits(x) == bits(y); }
}  // namespace

extern "C" int micro_dpp_xor(int seed, int* mismatches6)
{
    const int npat = 8;
    std::vector<uint32_t> h(npat * 64);
    Rng g{(uint64_t)seed * 7919u + 1u};
    for (int p = 0; p < npat; p++)
        for (int l = 0; l < 64; l++)
            h[p * 64 + l] = p == 0 ? 1000u + (uint32_t)l : p == 1 ? 0xffffffffu - (uint32_t)l : g.next();
    uint32_t *dv = nullptr, *dout = nullptr;
    if (hipMalloc(&dv, h.size() * 4) != hipSuccess || hipMalloc(&dout, 6 * 64 * 4) != hipSuccess) return 2;
    if (hipMemcpy(dv, h.data(), h.size() * 4, hipMemcpyHostToDevice) != hipSuccess) return 2;
    k_dpp_xor<<<1, 64>>>(dv, npat, dout);
    uint32_t o[6 * 64];
    if (hipMemcpy(o, dout, sizeof(o), hipMemcpyDeviceToHost) != hipSuccess) return 2;
    for (int m = 0; m < 6; m++) {
        int nb = 0;
        for (int l = 0; l < 64; l++) nb += o[m * 64 + l] != 0u;
        mismatches6[m] = nb;
    }
    (void)hipFree(dv);
    (void)hipFree(dout);
    return 0;
}

// counts[0] = elements, [1] = equal to the fmaf chain k = 0..3, [2] = equal to
// the chain k = 3..0, [3] = elements with a special operand or accumulator
extern "C" int micro_mfma_order(int R, int seed, int specials, long long* counts)
{
    std::vector<float> A(R * 64), B(R * 64), C(R * 256), D(R * 256);
    Rng g{(uint64_t)seed * 104729u + 3u};
    for (auto& v : A) v = operand(g, specials);
    for (auto& v : B) v = operand(g, specials);
    for (auto& v : C) v = operand(g, specials);
    float *dA, *dB, *dC, *dD;
    if (hipMalloc(&dA, A.size() * 4) != hipSuccess || hipMalloc(&dB, B.size() * 4) != hipSuccess ||
        hipMalloc(&dC, C.size() * 4) != hipSuccess || hipMalloc(&dD, D.size() * 4) != hipSuccess)
        return 2;
    (void)hipMemcpy(dA, A.data(), A.size() * 4, hipMemcpyHostToDevice);
    (void)hipMemcpy(dB, B.data(), B.size() * 4, hipMemcpyHostToDevice);
    (void)hipMemcpy(dC, C.data(), C.size() * 4, hipMemcpyHostToDevice);
    k_mfma<<<64, 64>>>(dA, dB, dC, dD, R);
    if (hipMemcpy(D.data(), dD, D.size() * 4, hipMemcpyDeviceToHost) != hipSuccess) return 2;
    long long tot = 0, fwd = 0, rev = 0, spec = 0;
    for (int r = 0; r < R; r++)
        for (int i = 0; i < 16; i++)
            for (int j = 0; j < 16; j++) {
                const float* a = &A[r * 64 + i * 4];
                const float* b = &B[r * 64];
                const float c = C[r * 256 + i * 16 + j], d = D[r * 256 + i * 16 + j];
                float f = c, h = c;
                bool sp = !std::isnormal(c);
                for (int k = 0; k < 4; k++) {
                    f = fmaf(a[k], b[k * 16 + j], f);
                    sp |= !std::isnormal(a[k]) || !std::isnormal(b[k * 16 + j]);
                }
                for (int k = 3; k >= 0; k--) h = fmaf(a[k], b[k * 16 + j], h);
                tot++;
                fwd += same(f, d);
                rev += same(h, d);
                spec += sp;
            }
    counts[0] = tot;
    counts[1] = fwd;
    counts[2] = rev;
    counts[3] = spec;
    (void)hipFree(dA);
    (void)hipFree(dB);
    (void)hipFree(dC);
    (void)hipFree(dD);
    return 0;
}

// The render backward's fast exponential (v_exp_f32 of power * log2 e, render.hip
// k_render_bwd_mf phase 1) against the deterministic expf_det the forward and
// the oracle use, EXHAUSTIVELY over every float power in [lo, 0]: the largest
// relative difference |e_hw - e_det| / e_det.  The backward's alpha band
// (2e-8 around 1/255) must exceed it.
__global__ void k_exp_band(uint32_t b0, uint32_t b1, unsigned int* maxrel_bits, unsigned long long* count)
{
    const uint32_t stride = gridDim.x * blockDim.x;
    float mx = 0.f;
    unsigned long long n = 0;
    for (uint32_t b = b0 + blockIdx.x * blockDim.x + threadIdx.x; b <= b1 && b >= b0; b += stride) {
        const float x = __uint_as_float(b);
        const float eh = __builtin_amdgcn_exp2f(x * 1.4426950408889634f);
        const float ed = lsr::expf_det(x);
        if (ed > 0.f) {
            const float r = fabsf(eh - ed) / ed;
            mx = fmaxf(mx, r);
            n++;
        }
        if (b > 0xffffffffu - stride) break;
    }
    for (int d = 32; d >= 1; d >>= 1) {
        mx = fmaxf(mx, __shfl_xor(mx, d, 64));
        n += __shfl_xor(n, d, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        atomicMax(maxrel_bits, __float_as_uint(mx));
        atomicAdd(count, n);
    }
}

// out[0] = max relative difference over powers in [lo, -0.0], out[1] = values tested
extern "C" int micro_exp_band(float lo, double* out)
{
    unsigned int* dm = nullptr;
    unsigned long long* dn = nullptr;
    if (hipMalloc(&dm, 4) != hipSuccess || hipMalloc(&dn, 8) != hipSuccess) return 2;
    (void)hipMemset(dm, 0, 4);
    (void)hipMemset(dn, 0, 8);
    uint32_t b1;
    std::memcpy(&b1, &lo, 4);
    k_exp_band<<<2048, 256>>>(0x80000000u, b1, dm, dn);
    unsigned int m = 0;
    unsigned long long n = 0;
    if (hipMemcpy(&m, dm, 4, hipMemcpyDeviceToHost) != hipSuccess) return 2;
    if (hipMemcpy(&n, dn, 8, hipMemcpyDeviceToHost) != hipSuccess) return 2;
    float mf;
    std::memcpy(&mf, &m, 4);
    out[0] = mf;
    out[1] = (double)n;
    (void)hipFree(dm);
    (void)hipFree(dn);
    return 0;
}
