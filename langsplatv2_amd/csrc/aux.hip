// aux.hip — small streaming kernels around the render path:
//
//  * k_nonfinite: the debug-mode NaN/Inf guard (SURVEY.md §5 "Failure
//    detection": C-ABI status codes + a NaN/Inf guard option).  With
//    settings.debug the driver scans every input and output array once per
//    call and returns LSR_ENONFINITE naming the first offending array; the
//    reference's nearest hooks are pipe.debug (gaussian_renderer/__init__.py:49)
//    and --detect_anomaly (train.py:362).
//  * k_check_lists: the debug-mode check of the binning lists (ids in range,
//    tile ranges monotone) before a render gathers through them.
//  * k_sparse_expand / k_sparse_gather: the quick (sparse) language input
//    (weights (N,K), indices (N,K), utils/vq_utils.py:26-40) expanded to dense
//    (N,Dq) rows, and the dense language gradient gathered back to dL/dweights.
//    Used only by the geometry-and-language backward in quick mode; the
//    language-only quick backward (the training path) never forms dense rows.
// All HBM-streaming, grid-stride, one pass.
#include "lsr_internal.h"

namespace lsr {

__global__ void __launch_bounds__(256) k_nonfinite(const float* __restrict__ p, size_t n, uint32_t* __restrict__ flag)
{
    const size_t stride = (size_t)gridDim.x * 256;
    bool bad = false;
    const size_t n4 = ((uintptr_t)p & 15) == 0 ? n / 4 : 0;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += stride) {
        const float4 v = reinterpret_cast<const float4*>(p)[i];
        bad |= !(isfinite(v.x) && isfinite(v.y) && isfinite(v.z) && isfinite(v.w));
    }
    for (size_t i = 4 * n4 + (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) bad |= !isfinite(p[i]);
    if (wave_any(bad) && (threadIdx.x & 63) == 0) atomicOr(flag, 1u);
}

hipError_t launch_nonfinite(const float* p, size_t n, uint32_t* flag, hipStream_t st)
{
    if (n == 0) return hipSuccess;
    const size_t blocks = (n / 4 + 255) / 256;
    k_nonfinite<<<(unsigned)(blocks < 2048 ? (blocks > 0 ? blocks : 1) : 2048), 256, 0, st>>>(p, n, flag);
    return hipGetLastError();
}

// Debug check of the binning lists before a render reads them (settings.debug):
// every point_list id < P, tile_start[0] == 0, tile_start non-decreasing and
// tile_start[T] == M.  A corrupt list (a sort or scatter bug) then returns
// LSR_ELISTS instead of faulting inside the render's gathers.
__global__ void __launch_bounds__(256) k_check_lists(const uint32_t* __restrict__ point_list, size_t M, uint32_t P,
                                                     const uint32_t* __restrict__ tile_start, size_t T,
                                                     uint32_t* __restrict__ flag)
{
    const size_t stride = (size_t)gridDim.x * 256;
    bool bad = false;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < M; i += stride) bad |= point_list[i] >= P;
    for (size_t t = (size_t)blockIdx.x * 256 + threadIdx.x; t < T; t += stride) bad |= tile_start[t + 1] < tile_start[t];
    if (blockIdx.x == 0 && threadIdx.x == 0) bad |= tile_start[0] != 0u || (size_t)tile_start[T] != M;
    if (wave_any(bad) && (threadIdx.x & 63) == 0) atomicOr(flag, 1u);
}

hipError_t launch_check_lists(const uint32_t* point_list, size_t M, uint32_t P, const uint32_t* tile_start, size_t T,
                              uint32_t* flag, hipStream_t st)
{
    const size_t n = M > T ? M : T;
    const size_t blocks = (n + 255) / 256;
    k_check_lists<<<(unsigned)(blocks < 2048 ? (blocks > 0 ? blocks : 1) : 2048), 256, 0, st>>>(point_list, M, P,
                                                                                                  tile_start, T, flag);
    return hipGetLastError();
}

// dense[j][q] = sum over m with idx[j][m] == q of w[j][m] (out-of-range codes
// dropped, as the quick forward drops them); one thread per row.
__global__ void __launch_bounds__(256) k_sparse_expand(const float* __restrict__ qw, const void* __restrict__ qi,
                                                       int dtype, int N, int K, int Dq, float* __restrict__ dense)
{
    const int j = blockIdx.x * 256 + threadIdx.x;
    if (j >= N) return;
    float* row = dense + (size_t)j * Dq;
    for (int q = 0; q < Dq; q++) row[q] = 0.f;
    for (int m = 0; m < K; m++) {
        const size_t off = (size_t)j * K + m;
        const int q = quick_index(qi, dtype, off);
        if (q >= 0 && q < Dq) row[q] += qw[off];
    }
}

// dw[j][m] = dense_grad[j][idx[j][m]] (0 for out-of-range codes)
__global__ void __launch_bounds__(256) k_sparse_gather(const float* __restrict__ g, const void* __restrict__ qi,
                                                       int dtype, int64_t NK, int K, int Dq, float* __restrict__ dw)
{
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= NK) return;
    const int64_t j = e / K;
    const int q = quick_index(qi, dtype, (size_t)e);
    dw[e] = (q >= 0 && q < Dq) ? g[(size_t)j * Dq + q] : 0.f;
}

hipError_t launch_sparse_expand(const float* qw, const void* qi, int dtype, int N, int K, int Dq, float* dense,
                                hipStream_t st)
{
    if (N == 0) return hipSuccess;
    k_sparse_expand<<<(N + 255) / 256, 256, 0, st>>>(qw, qi, dtype, N, K, Dq, dense);
    return hipGetLastError();
}

hipError_t launch_sparse_gather(const float* g, const void* qi, int dtype, int N, int K, int Dq, float* dw,
                                hipStream_t st)
{
    const int64_t NK = (int64_t)N * K;
    if (NK == 0) return hipSuccess;
    k_sparse_gather<<<(unsigned)((NK + 255) / 256), 256, 0, st>>>(g, qi, dtype, NK, K, Dq, dw);
    return hipGetLastError();
}

// Packed code rows (LSR_INDEX_PACKED): the 12 codes of Gaussian i as bytes
// code + 1 (0 = out of range), one 16-B row each; the quick render stages
// them as they are instead of converting 12 indices per candidate and frame.
__global__ void __launch_bounds__(256) k_quick_pack_codes(const void* __restrict__ qi, int dtype, int64_t N, int Dq,
                                                          uint4* __restrict__ out)
{
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= N) return;
    uint32_t w[3] = {0u, 0u, 0u};
#pragma unroll
    for (int m = 0; m < 12; m++) {
        const int q = quick_index(qi, dtype, (size_t)i * 12 + m);
        const uint32_t b = (q >= 0 && q < Dq) ? (uint32_t)(q + 1) : 0u;
        w[m >> 2] |= b << (8 * (m & 3));
    }
    out[i] = make_uint4(w[0], w[1], w[2], 0u);
}

hipError_t launch_quick_pack_codes(const void* qi, int dtype, int64_t N, int Dq, void* packed, hipStream_t st)
{
    if (N == 0) return hipSuccess;
    k_quick_pack_codes<<<(unsigned)((N + 255) / 256), 256, 0, st>>>(qi, dtype, N, Dq, (uint4*)packed);
    return hipGetLastError();
}

}  // namespace lsr
