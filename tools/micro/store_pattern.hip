// Store-pattern microbenchmark for the quick decode's output (3 x 512 planes of
// W x H fp32): which per-instruction store shape reaches HBM write bandwidth.
//   A: lane (d = l & 15, g = l >> 4) writes 16 B (4 px) of plane d: 16 planes x 64 B per instruction
//      (the split-f16 decode's MFMA output layout), a wave covering 64 px x all planes
//   B: 64 lanes x 16 B = 1 KB contiguous of ONE plane per instruction, a wave covering 256 px x all planes
//   C: as B but a wave covers 1024 px (4 instructions per plane)
//   D: 8 planes x 128 B per instruction (lanes of a 16-B piece pair across two
//      16-px MFMA tiles, DPP row_ror:8 merge), a wave covering 64 px x all planes
//   P<n>/PD<n>: A / D from a persistent grid of one n-wave workgroup per CU
//      looping over the 64-px tiles (the level-resident decode's occupancy)
// Build: hipcc --offload-arch=gfx950 -O3 store_pattern.hip -o store_pattern
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ void kA(float* out, int W, int H, int planes)
{
    const int lane = threadIdx.x, li = lane & 15, lg = lane >> 4;
    const int nbx = W / 64;
    const int bx = (blockIdx.x % nbx) * 64, y = blockIdx.x / nbx;
    const size_t HW = (size_t)W * H;
    for (int p0 = 0; p0 < planes; p0 += 16)
        for (int pb = 0; pb < 4; pb++) {
            float* o = out + (size_t)(p0 + li) * HW + (size_t)y * W + bx + 16 * pb + 4 * lg;
            *reinterpret_cast<float4*>(o) = make_float4((float)p0, (float)pb, 1.f, 2.f);
        }
}

template <int PXW>
__global__ void kB(float* out, int W, int H, int planes)
{
    const int lane = threadIdx.x;
    const int nbx = W / PXW;
    const int bx = (blockIdx.x % nbx) * PXW, y = blockIdx.x / nbx;
    const size_t HW = (size_t)W * H;
    for (int p = 0; p < planes; p++)
        for (int c = 0; c < PXW / 256; c++) {
            float* o = out + (size_t)p * HW + (size_t)y * W + bx + 256 * c + 4 * lane;
            *reinterpret_cast<float4*>(o) = make_float4((float)p, (float)c, 1.f, 2.f);
        }
}

__global__ void kD(float* out, int W, int H, int planes)
{
    const int lane = threadIdx.x, li = lane & 15, lg = lane >> 4;
    const int nbx = W / 64;
    const int bx = (blockIdx.x % nbx) * 64, y = blockIdx.x / nbx;
    const size_t HW = (size_t)W * H;
    // lane (li, lg): plane (li & 7) + 8 h, pixels 4 k, k = 4 (li >> 3) + lg of the 32-px pair
    for (int p0 = 0; p0 < planes; p0 += 16)
        for (int pp = 0; pp < 2; pp++)
            for (int h = 0; h < 2; h++) {
                const int k = 4 * (li >> 3) + lg;
                float* o = out + (size_t)(p0 + 8 * h + (li & 7)) * HW + (size_t)y * W + bx + 32 * pp + 4 * k;
                *reinterpret_cast<float4*>(o) = make_float4((float)p0, (float)pp, 1.f, 2.f);
            }
}

template <bool D128>
__global__ void kP(float* out, int W, int H, int planes, int nw)
{
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, li = lane & 15, lg = lane >> 4;
    const int nbx = W / 64, ntile = nbx * H;
    const size_t HW = (size_t)W * H;
    for (int t = blockIdx.x * nw + w; t < ntile; t += gridDim.x * nw) {
        const int bx = (t % nbx) * 64, y = t / nbx;
        for (int p0 = 0; p0 < planes; p0 += 16) {
            if (D128) {
                for (int pp = 0; pp < 2; pp++)
                    for (int h = 0; h < 2; h++) {
                        const int k = 4 * (li >> 3) + lg;
                        float* o = out + (size_t)(p0 + 8 * h + (li & 7)) * HW + (size_t)y * W + bx + 32 * pp + 4 * k;
                        *reinterpret_cast<float4*>(o) = make_float4((float)p0, (float)pp, 1.f, 2.f);
                    }
            } else {
                for (int pb = 0; pb < 4; pb++) {
                    float* o = out + (size_t)(p0 + li) * HW + (size_t)y * W + bx + 16 * pb + 4 * lg;
                    *reinterpret_cast<float4*>(o) = make_float4((float)p0, (float)pb, 1.f, 2.f);
                }
            }
        }
    }
}

int main()
{
    const int W = 1280, H = 800, planes = 1536;
    const size_t bytes = (size_t)W * H * planes * 4;
    float* out;
    if (hipMalloc(&out, bytes) != hipSuccess) return 1;
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    auto run = [&](const char* name, auto launch) {
        for (int i = 0; i < 3; i++) launch();
        hipDeviceSynchronize();
        hipEventRecord(a);
        for (int i = 0; i < 10; i++) launch();
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms = 0.f;
        hipEventElapsedTime(&ms, a, b);
        ms /= 10;
        printf("%s: %.3f ms  %.0f GB/s\n", name, ms, bytes / (ms * 1e-3) / 1e9);
    };
    run("A 16 planes x 64 B / instr, 64 px per wave", [&] { kA<<<(W / 64) * H, 64>>>(out, W, H, planes); });
    run("B 1 KB / instr, 256 px per wave", [&] { kB<256><<<(W / 256) * H, 64>>>(out, W, H, planes); });
    run("C 1 KB / instr, 1280 px per wave", [&] { kB<1280><<<(W / 1280) * H, 64>>>(out, W, H, planes); });
    run("D 8 planes x 128 B / instr, 64 px per wave", [&] { kD<<<(W / 64) * H, 64>>>(out, W, H, planes); });
    for (int nw : {8, 12, 16}) {
        char n1[64], n2[64];
        snprintf(n1, 64, "P%d  A persistent, %d waves per CU", nw, nw);
        snprintf(n2, 64, "PD%d D persistent, %d waves per CU", nw, nw);
        run(n1, [&] { kP<false><<<256, 64 * nw>>>(out, W, H, planes, nw); });
        run(n2, [&] { kP<true><<<256, 64 * nw>>>(out, W, H, planes, nw); });
    }
    hipFree(out);
    return 0;
}
