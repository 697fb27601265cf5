// bin_common.h — pieces shared by the binning kernels (binning.hip).
#pragma once
#include "lsr_internal.h"

namespace lsr {

// Screen bands: each block owns a band of `rows` tile rows, so a block's LDS
// histogram covers rows * gx tiles (<= LSR_BAND_LDS bytes) and several blocks
// stay resident per CU at any resolution; a Gaussian's rect is clipped to the
// band (each band re-reads the chunk's 20-B records, cheap next to the
// instance work).
#ifndef LSR_BAND_LDS
#define LSR_BAND_LDS 32768
#endif
#ifndef LSR_COUNT_XCD
#define LSR_COUNT_XCD 1   // chunk-major count grid: cfg5 bin_count 0.627 -> 0.604 ms (cfg3 ±0)
#endif
struct Band {
    int ty0, ty1, t0, nt;
    __device__ Band(const Cam& c, int rows, int band)
    {
        ty0 = band * rows;
        ty1 = min(c.gy, ty0 + rows);
        t0 = ty0 * c.gx;
        nt = (ty1 - ty0) * c.gx;
    }
};

// largest o in [0, 64) with pre[o] <= k (pre non-decreasing, pre[64] > k)
__device__ __forceinline__ int wave_search(const int* pre, int k)
{
    int o = 0;
#pragma unroll
    for (int step = 32; step >= 1; step >>= 1)
        if (pre[o + step] <= k) o += step;
    return o;
}

// One Gaussian's binning inputs (radius, the two splat records, depth),
// loaded one wave iteration ahead of their use (LSR_BIN_PF): the walk of
// iteration k runs while iteration k + 1's records are in flight, instead of
// every iteration waiting for a dependent radius -> record gather.  Lanes
// past the chunk read Gaussian g1 - 1 (a valid address) and get radius 0.
struct BinRec {
    int r;
    float4 A, B;
    float depth;
    uint32_t id;   // the Gaussian
    __device__ __forceinline__ void load(const uint8_t* geom, int P, int g1, const int32_t* __restrict__ radii, int i,
                                         bool with_depth)
    {
        const GeomLayout L = geom_layout(P);
        const int q = min(i, g1 - 1);
        id = (uint32_t)q;
        const int rr = radii[q];
        A = ((const float4*)(geom + L.splatA))[q];
        B = ((const float4*)(geom + L.splatB))[q];
        depth = with_depth ? ((const float*)(geom + L.depth))[q] : 0.f;
        r = i < g1 ? rr : 0;
    }
};

// Lane's Gaussian -> its cull box clipped to the band: columns [x0, x1),
// first row y0 (band-relative); returns the row count (0 if none).
__device__ __forceinline__ int band_box(const Cam& c, const Band& bd, const BinRec& g, int& x0, int& x1, int& y0)
{
    x0 = x1 = y0 = 0;
    if (g.r <= 0) return 0;
    int y1;
    get_rect(g.A.x, g.A.y, g.r, c.gx, c.gy, x0, y0, x1, y1);
    cull_box(g.A.x, g.A.y, g.A.z, g.A.w, g.B.x, g.B.z, x0, y0, x1, y1);
    y0 = max(y0, bd.ty0);
    y1 = min(y1, bd.ty1);
    const int h = (y1 > y0 && x1 > x0) ? y1 - y0 : 0;
    y0 -= bd.ty0;
    return h;
}

}  // namespace lsr
