// Store-pattern microbenchmark for the quick decode's output (3 x 512 planes of
// W x H fp32): which per-instruction store shape reaches HBM write bandwidth.
//   A: lane (d = l & 15, g = l >> 4) writes 16 B (4 px) of plane d: 16 planes x 64 B per instruction
//      (the split-f16 decode's MFMA output layout), a wave covering 64 px x all planes
//   B: 64 lanes x 16 B = 1 KB contiguous of ONE plane per instruction, a wave covering 256 px x all planes
//   C: as B but a wave covers 1024 px (4 instructions per plane)
//   D: 8 planes x 128 B per instruction (lanes of a 16-B piece pair across two
//      16-px MFMA tiles, DPP row_ror:8 merge), a wave covering 64 px x all planes
//   E: 4 planes x 256 B per instruction (two register-bit <-> lane-bit swaps of
//      four 16-px MFMA tiles), a wave covering 64 px x all planes
//   P<n>/PD<n>/PE<n>/PC<n>: A / D / E / 1 KB-contiguous from a persistent grid of
//      one n-wave workgroup per CU looping over the 64-px tiles (the
//      level-resident decode's occupancy); ...R: each tile also reads its 16 KB
//      weight tile (64 planes x 256 B) first, as the decode does
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

__global__ void kE(float* out, int W, int H, int planes)
{
    const int lane = threadIdx.x, a = lane >> 4, b = lane & 15;
    const int nbx = W / 64;
    const int bx = (blockIdx.x % nbx) * 64, y = blockIdx.x / nbx;
    const size_t HW = (size_t)W * H;
    for (int p0 = 0; p0 < planes; p0 += 16)
        for (int q = 0; q < 4; q++) {
            float* o = out + (size_t)(p0 + 4 * q + a) * HW + (size_t)y * W + bx + 4 * b;
            *reinterpret_cast<float4*>(o) = make_float4((float)p0, (float)q, 1.f, 2.f);
        }
}

// MODE 0 = A, 1 = D, 2 = E, 3 = 1 KB contiguous (256 px of one plane) per instruction, 256-px tiles
template <int MODE, bool RD>
__global__ void kP(float* out, const float* in, int W, int H, int planes, int nw)
{
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, li = lane & 15, lg = lane >> 4;
    const int TW = MODE == 3 ? 256 : 64;
    const int nbx = W / TW, ntile = nbx * H;
    const size_t HW = (size_t)W * H;
    float acc = 0.f;
    for (int t = blockIdx.x * nw + w; t < ntile; t += gridDim.x * nw) {
        const int bx = (t % nbx) * TW, y = t / nbx;
        if (RD) {
            // 64 planes x 64 px of weights (16 KB per 64 px), as the decode's tile load
            for (int r = 0; r < TW / 64; r++)
#pragma unroll
                for (int j = 0; j < 16; j++) {
                    const float4 v = *reinterpret_cast<const float4*>(in + (size_t)(4 * j + lg) * HW + (size_t)y * W + bx + 64 * r + 4 * li);
                    acc += v.x + v.y + v.z + v.w;
                }
        }
        for (int p0 = 0; p0 < planes; p0 += 16) {
            if (MODE == 3) {
                for (int p = 0; p < 16; p++) {
                    float* o = out + (size_t)(p0 + p) * HW + (size_t)y * W + bx + 4 * lane;
                    *reinterpret_cast<float4*>(o) = make_float4((float)p0, acc, 1.f, 2.f);
                }
            } else if (MODE == 2) {
                for (int q = 0; q < 4; q++) {
                    float* o = out + (size_t)(p0 + 4 * q + lg) * HW + (size_t)y * W + bx + 4 * li;
                    *reinterpret_cast<float4*>(o) = make_float4((float)p0, acc, 1.f, 2.f);
                }
            } else if (MODE == 7 || MODE == 8) {
                // channel-last output ((H, W, planes): a pixel's planes contiguous), the 16
                // planes p0.. of the tile's 64 pixels: 7 = 4 px x 64 B per instruction
                // (lane: px 4 q + lg... 16 planes = 64 B per pixel), 8 = per instruction
                // 1 KB = 16 pixels x 64 B
                for (int q = 0; q < 4; q++) {
                    const int px = MODE == 7 ? (16 * q + li) : (16 * q + li);
                    float* o = out + ((size_t)y * W + bx + px) * planes + p0 + 4 * lg;
                    *reinterpret_cast<float4*>(o) = make_float4((float)p0, acc, 1.f, 2.f);
                }
            } else if (MODE >= 4) {   // E with a cache-policy modifier: 4 sc1, 5 nt, 6 sc0 sc1
                for (int q = 0; q < 4; q++) {
                    float* o = out + (size_t)(p0 + 4 * q + lg) * HW + (size_t)y * W + bx + 4 * li;
                    typedef float f4v __attribute__((ext_vector_type(4)));
                    const f4v v = {(float)p0, acc, 1.f, 2.f};
                    if (MODE == 4) asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(o), "v"(v) : "memory");
                    if (MODE == 5) asm volatile("global_store_dwordx4 %0, %1, off nt" ::"v"(o), "v"(v) : "memory");
                    if (MODE == 6) asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(o), "v"(v) : "memory");
                }
            } else if (MODE == 1) {
                for (int pp = 0; pp < 2; pp++)
                    for (int h = 0; h < 2; h++) {
                        const int k = 4 * (li >> 3) + lg;
                        float* o = out + (size_t)(p0 + 8 * h + (li & 7)) * HW + (size_t)y * W + bx + 32 * pp + 4 * k;
                        *reinterpret_cast<float4*>(o) = make_float4((float)p0, (float)pp, 1.f, 2.f);
                    }
            } else {
                for (int pb = 0; pb < 4; pb++) {
                    float* o = out + (size_t)(p0 + li) * HW + (size_t)y * W + bx + 16 * pb + 4 * lg;
                    *reinterpret_cast<float4*>(o) = make_float4((float)p0, acc, 1.f, 2.f);
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
    float* in;
    if (hipMalloc(&out, bytes) != hipSuccess) return 1;
    if (hipMalloc(&in, (size_t)W * H * 192 * 4) != hipSuccess) return 1;
    hipMemset(in, 0, (size_t)W * H * 192 * 4);
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
    run("E 4 planes x 256 B / instr, 64 px per wave", [&] { kE<<<(W / 64) * H, 64>>>(out, W, H, planes); });
    {
        // channel-last: each wave's 64 pixels x 1536 planes is one 384-KB contiguous block
        char n[96];
        snprintf(n, 96, "PL8 channel-last, 16 px x 64 B per instruction, 8 waves per CU");
        run(n, [&] { kP<7, false><<<256, 64 * 8>>>(out, in, W, H, planes, 8); });
        snprintf(n, 96, "PL8R channel-last + weight reads, 8 waves per CU");
        run(n, [&] { kP<7, true><<<256, 64 * 8>>>(out, in, W, H, planes, 8); });
    }
    {
        const char* nm[3] = {"E sc1", "E nt", "E sc0 sc1"};
        for (int m = 0; m < 3; m++) {
            char n[96];
            snprintf(n, 96, "P%s 8 waves per CU", nm[m]);
            auto L = [&](auto k) { run(n, [&] { k<<<256, 64 * 8>>>(out, in, W, H, planes, 8); }); };
            if (m == 0) L(kP<4, false>);
            if (m == 1) L(kP<5, false>);
            if (m == 2) L(kP<6, false>);
        }
    }
    for (int nw : {8, 16}) {
        char n[96];
        const char* nm[4] = {"A", "D", "E", "C"};
        for (int m = 0; m < 4; m++)
            for (int rd = 0; rd < 2; rd++) {
                snprintf(n, 96, "P%s%d%s %d waves per CU%s", nm[m], nw, rd ? "R" : "", nw, rd ? " + weight reads" : "");
                auto L = [&](auto k) { run(n, [&] { k<<<256, 64 * nw>>>(out, in, W, H, planes, nw); }); };
                if (m == 0) rd ? L(kP<0, true>) : L(kP<0, false>);
                if (m == 1) rd ? L(kP<1, true>) : L(kP<1, false>);
                if (m == 2) rd ? L(kP<2, true>) : L(kP<2, false>);
                if (m == 3) rd ? L(kP<3, true>) : L(kP<3, false>);
            }
    }
    hipFree(out);
    hipFree(in);
    return 0;
}
