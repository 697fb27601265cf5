// knn.hip — mean squared distance to the 3 nearest neighbours of every point
// (SURVEY.md §8f rank 3): the simple_knn._C.distCUDA2 call of
// GaussianModel.create_from_pcd (scene/gaussian_model.py:20,194), which turns
// it into initial scales (log sqrt of the clamp_min(1e-7) of this value).
//
// Semantics (the published simple-knn algorithm; the submodule source is
// absent from the reference checkout): for each point i, the three smallest
// squared distances d(i, j) = dx*dx + dy*dy + dz*dz over j != i, kept in
// ascending order by insertion, and out[i] = (b0 + b1 + b2) / 3.  Missing
// neighbours (N < 4) stay FLT_MAX.  The search is exact, so the result does
// not depend on traversal order: with -ffp-contract=off it is bit-identical
// to the brute-force oracle (oracle/lsr_oracle.c lso_knn_dist2).
//
// MI355X design:
//   1. bounding box (two-stage reduction), 63-bit Morton code per point
//      (21 bits per axis), rocPRIM radix sort of (code, index);
//   2. points gathered in Morton order as float4; boxes of 32 consecutive
//      points and superboxes of 32 boxes (1024 points), each with an AABB;
//   3. one wave = 64 consecutive sorted queries (spatially coherent): seed
//      the 3-best from the wave's own 64 points (LDS broadcast), then walk
//      the superboxes; a superbox / box is entered only if some lane's AABB
//      distance is below its current third-best (ballot), and an entered
//      box's 32 points are broadcast from LDS.  AABB distances are lower
//      bounds of the rounded point distances (rounding is monotonic), so
//      pruning never changes a result.
#include <float.h>

#include <rocprim/device/device_radix_sort.hpp>

#include "lsr_internal.h"

namespace lsr {

namespace {

constexpr int KNN_BOX = 32;      // points per box
constexpr int KNN_SUPER = 32;    // boxes per superbox
constexpr int KNN_RED_BLOCKS = 256;

__device__ __forceinline__ uint32_t ord_f32(float f)
{
    const uint32_t u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

__device__ __forceinline__ float unord_f32(uint32_t u)
{
    return __uint_as_float((u & 0x80000000u) ? (u & 0x7fffffffu) : ~u);
}

// partial min/max of each axis per block -> part[block][6] (order-preserving uint)
__global__ void __launch_bounds__(256) k_knn_bbox_partial(const float* __restrict__ p, int64_t N,
                                                           uint32_t* __restrict__ part)
{
    uint32_t mn[3] = {0xffffffffu, 0xffffffffu, 0xffffffffu}, mx[3] = {0u, 0u, 0u};
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < N; i += (int64_t)gridDim.x * 256)
        for (int a = 0; a < 3; a++) {
            const uint32_t v = ord_f32(p[3 * i + a]);
            mn[a] = min(mn[a], v);
            mx[a] = max(mx[a], v);
        }
    __shared__ uint32_t s[6][256];
    for (int a = 0; a < 3; a++) { s[a][threadIdx.x] = mn[a]; s[3 + a][threadIdx.x] = mx[a]; }
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w)
            for (int a = 0; a < 3; a++) {
                s[a][threadIdx.x] = min(s[a][threadIdx.x], s[a][threadIdx.x + w]);
                s[3 + a][threadIdx.x] = max(s[3 + a][threadIdx.x], s[3 + a][threadIdx.x + w]);
            }
        __syncthreads();
    }
    if (threadIdx.x < 6) part[blockIdx.x * 6 + threadIdx.x] = s[threadIdx.x][0];
}

__device__ __forceinline__ uint64_t spread3_21(uint32_t v)
{
    uint64_t x = v & 0x1fffffu;
    x = (x | x << 32) & 0x1f00000000ffffull;
    x = (x | x << 16) & 0x1f0000ff0000ffull;
    x = (x | x << 8) & 0x100f00f00f00f00full;
    x = (x | x << 4) & 0x10c30c30c30c30c3ull;
    x = (x | x << 2) & 0x1249249249249249ull;
    return x;
}

// bbox from the partials, then the Morton code of every point
__global__ void __launch_bounds__(256) k_knn_morton(const float* __restrict__ p, int64_t N,
                                                     const uint32_t* __restrict__ part, int nparts,
                                                     uint64_t* __restrict__ keys, uint32_t* __restrict__ vals)
{
    __shared__ float lo[3], sc[3];
    if (threadIdx.x < 3) {
        uint32_t mn = 0xffffffffu, mx = 0u;
        for (int b = 0; b < nparts; b++) {
            mn = min(mn, part[b * 6 + threadIdx.x]);
            mx = max(mx, part[b * 6 + 3 + threadIdx.x]);
        }
        const float a = unord_f32(mn), b = unord_f32(mx);
        lo[threadIdx.x] = a;
        sc[threadIdx.x] = (b > a) ? 2097151.0f / (b - a) : 0.f;
    }
    __syncthreads();
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= N) return;
    uint64_t code = 0;
    for (int a = 0; a < 3; a++) {
        float t = (p[3 * i + a] - lo[a]) * sc[a];
        t = fminf(fmaxf(t, 0.f), 2097151.0f);
        code |= spread3_21((uint32_t)t) << a;
    }
    keys[i] = code;
    vals[i] = (uint32_t)i;
}

__global__ void __launch_bounds__(256) k_knn_gather(const float* __restrict__ p, int64_t N,
                                                     const uint32_t* __restrict__ order, float4* __restrict__ sp)
{
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= N) return;
    const uint32_t j = order[i];
    sp[i] = make_float4(p[3 * (size_t)j], p[3 * (size_t)j + 1], p[3 * (size_t)j + 2], 0.f);
}

// AABB of each box (one lane per box; 32 sorted points, contiguous)
__global__ void __launch_bounds__(256) k_knn_boxes(const float4* __restrict__ sp, int64_t N, int nb,
                                                    float4* __restrict__ bmin, float4* __restrict__ bmax)
{
    const int b = blockIdx.x * 256 + threadIdx.x;
    if (b >= nb) return;
    float4 lo = make_float4(INFINITY, INFINITY, INFINITY, 0.f), hi = make_float4(-INFINITY, -INFINITY, -INFINITY, 0.f);
    const int64_t e = min((int64_t)(b + 1) * KNN_BOX, N);
    for (int64_t i = (int64_t)b * KNN_BOX; i < e; i++) {
        const float4 q = sp[i];
        lo.x = fminf(lo.x, q.x); lo.y = fminf(lo.y, q.y); lo.z = fminf(lo.z, q.z);
        hi.x = fmaxf(hi.x, q.x); hi.y = fmaxf(hi.y, q.y); hi.z = fmaxf(hi.z, q.z);
    }
    bmin[b] = lo;
    bmax[b] = hi;
}

__global__ void __launch_bounds__(256) k_knn_supers(const float4* __restrict__ bmin, const float4* __restrict__ bmax,
                                                     int nb, int ns, float4* __restrict__ smin, float4* __restrict__ smax)
{
    const int s = blockIdx.x * 256 + threadIdx.x;
    if (s >= ns) return;
    float4 lo = make_float4(INFINITY, INFINITY, INFINITY, 0.f), hi = make_float4(-INFINITY, -INFINITY, -INFINITY, 0.f);
    const int e = min((s + 1) * KNN_SUPER, nb);
    for (int b = s * KNN_SUPER; b < e; b++) {
        const float4 a = bmin[b], c = bmax[b];
        lo.x = fminf(lo.x, a.x); lo.y = fminf(lo.y, a.y); lo.z = fminf(lo.z, a.z);
        hi.x = fmaxf(hi.x, c.x); hi.y = fmaxf(hi.y, c.y); hi.z = fmaxf(hi.z, c.z);
    }
    smin[s] = lo;
    smax[s] = hi;
}

__device__ __forceinline__ float sq_dist(float4 a, float4 b)
{
    const float dx = b.x - a.x, dy = b.y - a.y, dz = b.z - a.z;
    return dx * dx + dy * dy + dz * dz;
}

// squared distance from q to an AABB (a lower bound of every rounded point
// distance inside it)
__device__ __forceinline__ float box_dist(float4 q, float4 lo, float4 hi)
{
    const float dx = fmaxf(fmaxf(lo.x - q.x, 0.f), q.x - hi.x);
    const float dy = fmaxf(fmaxf(lo.y - q.y, 0.f), q.y - hi.y);
    const float dz = fmaxf(fmaxf(lo.z - q.z, 0.f), q.z - hi.z);
    return dx * dx + dy * dy + dz * dz;
}

// insertion into the ascending 3-best (strict >: an equal distance is not inserted twice)
__device__ __forceinline__ void update3(float (&b)[3], float d)
{
#pragma unroll
    for (int j = 0; j < 3; j++) {
        const bool sw = b[j] > d;
        const float t = b[j];
        b[j] = sw ? d : t;
        d = sw ? t : d;
    }
}

__global__ void __launch_bounds__(64) k_knn_query(const float4* __restrict__ sp, const uint32_t* __restrict__ order,
                                                   int64_t N, const float4* __restrict__ bmin,
                                                   const float4* __restrict__ bmax, int nb,
                                                   const float4* __restrict__ smin, const float4* __restrict__ smax,
                                                   int ns, float* __restrict__ out)
{
    __shared__ float4 pts[64];
    const int lane = threadIdx.x;
    const int64_t base = (int64_t)blockIdx.x * 64;
    const int64_t i = base + lane;
    const bool live = i < N;
    const float4 q = live ? sp[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    float best[3] = {FLT_MAX, FLT_MAX, FLT_MAX};
    // seed: the wave's own 64 points (boxes b0, b0 + 1)
    const int nown = (int)min((int64_t)64, N - base);
    pts[lane] = q;
    __syncthreads();
    for (int t = 0; t < nown; t++)
        if (t != lane) update3(best, sq_dist(q, pts[t]));
    const int b0 = (int)(base / KNN_BOX);
    for (int s = 0; s < ns; s++) {
        const bool need_s = live && box_dist(q, smin[s], smax[s]) < best[2];
        if (!__any(need_s)) continue;
        const int be = min((s + 1) * KNN_SUPER, nb);
        for (int b = s * KNN_SUPER; b < be; b++) {
            if (b == b0 || b == b0 + 1) continue;
            const bool need_b = need_s && box_dist(q, bmin[b], bmax[b]) < best[2];
            if (!__any(need_b)) continue;
            const int64_t pb = (int64_t)b * KNN_BOX;
            const int cnt = (int)min((int64_t)KNN_BOX, N - pb);
            __syncthreads();
            if (lane < cnt) pts[lane] = sp[pb + lane];
            __syncthreads();
            if (need_b)
                for (int t = 0; t < cnt; t++) update3(best, sq_dist(q, pts[t]));
        }
    }
    if (live) out[order[i]] = (best[0] + best[1] + best[2]) / 3.0f;
}

}  // namespace

size_t knn_workspace_bytes(int64_t N, size_t sort_temp)
{
    const size_t nb = (size_t)((N + KNN_BOX - 1) / KNN_BOX), ns = (nb + KNN_SUPER - 1) / KNN_SUPER;
    return align256((size_t)KNN_RED_BLOCKS * 6 * 4) + 2 * align256((size_t)N * 8) + 2 * align256((size_t)N * 4) +
           align256((size_t)N * 16) + 2 * align256(nb * 16) + 2 * align256(ns * 16) + align256(sort_temp);
}

hipError_t knn_sort_temp_bytes(int64_t N, size_t* bytes)
{
    *bytes = 0;
    return rocprim::radix_sort_pairs(nullptr, *bytes, (const uint64_t*)nullptr, (uint64_t*)nullptr,
                                                         (const uint32_t*)nullptr, (uint32_t*)nullptr, (size_t)N, 0, 63);
}

hipError_t launch_knn_dist2(const float* points, int64_t N, float* out, uint8_t* ws, size_t sort_temp, hipStream_t st)
{
    if (N == 0) return hipSuccess;
    const int nb = (int)((N + KNN_BOX - 1) / KNN_BOX), ns = (nb + KNN_SUPER - 1) / KNN_SUPER;
    uint8_t* p = ws;
    auto take = [&](size_t bytes) { uint8_t* r = p; p += align256(bytes); return r; };
    uint32_t* part = (uint32_t*)take((size_t)KNN_RED_BLOCKS * 6 * 4);
    uint64_t* keys = (uint64_t*)take((size_t)N * 8);
    uint64_t* keys2 = (uint64_t*)take((size_t)N * 8);
    uint32_t* vals = (uint32_t*)take((size_t)N * 4);
    uint32_t* order = (uint32_t*)take((size_t)N * 4);
    float4* sp = (float4*)take((size_t)N * 16);
    float4* bmin = (float4*)take((size_t)nb * 16);
    float4* bmax = (float4*)take((size_t)nb * 16);
    float4* smin = (float4*)take((size_t)ns * 16);
    float4* smax = (float4*)take((size_t)ns * 16);
    void* temp = take(sort_temp);
    const int nparts = (int)min((int64_t)KNN_RED_BLOCKS, (N + 255) / 256);
    const unsigned g = (unsigned)((N + 255) / 256);
    k_knn_bbox_partial<<<nparts, 256, 0, st>>>(points, N, part);
    k_knn_morton<<<g, 256, 0, st>>>(points, N, part, nparts, keys, vals);
    size_t tb = sort_temp;
    hipError_t e = rocprim::radix_sort_pairs(temp, tb, keys, keys2, vals, order, (size_t)N, 0, 63, st);
    if (e != hipSuccess) return e;
    k_knn_gather<<<g, 256, 0, st>>>(points, N, order, sp);
    k_knn_boxes<<<(unsigned)((nb + 255) / 256), 256, 0, st>>>(sp, N, nb, bmin, bmax);
    k_knn_supers<<<(unsigned)((ns + 255) / 256), 256, 0, st>>>(bmin, bmax, nb, ns, smin, smax);
    k_knn_query<<<(unsigned)((N + 63) / 64), 64, 0, st>>>(sp, order, N, bmin, bmax, nb, smin, smax, ns, out);
    return hipGetLastError();
}

}  // namespace lsr
