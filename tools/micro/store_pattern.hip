// Store-pattern microbenchmark for the quick decode's output (3 x 512 planes of
// W x H fp32): which per-instruction store shape reaches HBM write bandwidth.
//   A: lane (d = l & 15, g = l >> 4) writes 16 B (4 px) of plane d: 16 planes x 64 B per instruction
//      (the split-f16 decode's MFMA output layout), a wave covering 64 px x all planes
//   B: 64 lanes x 16 B = 1 KB contiguous of ONE plane per instruction, a wave covering 256 px x all planes
//   C: as B but a wave covers 1024 px (4 instructions per plane)
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
    hipFree(out);
    return 0;
}
