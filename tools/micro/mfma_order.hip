// Is v_mfma_f32_16x16x4_f32 bitwise equal to a sequential fmaf chain over k?
// D[i][j] = C[i][j] + sum_k A[i][k] B[k][j].  Tests orders k=0..3 (fwd) and
// k=3..0 (rev), and the unfused sum, over random data with wide exponents.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <cstring>
typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ void k(const float* A, const float* B, const float* C, float* D, int reps)
{
    const int l = threadIdx.x;
    for (int r = 0; r < reps; r++) {
        const float* a = A + r * 64; const float* b = B + r * 64; const float* c = C + r * 256;
        // A[i][k]: lane l supplies A[l&15][l>>4]; B[k][j]: lane l supplies B[l>>4][l&15]
        float av = a[(l & 15) * 4 + (l >> 4)];
        float bv = b[(l >> 4) * 16 + (l & 15)];
        f32x4 acc;
        for (int q = 0; q < 4; q++) acc[q] = c[(4 * (l >> 4) + q) * 16 + (l & 15)];
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc, 0, 0, 0);
        for (int q = 0; q < 4; q++) D[r * 256 + (4 * (l >> 4) + q) * 16 + (l & 15)] = acc[q];
    }
}

static float rnd(unsigned& s) { s = s * 1664525u + 1013904223u; return ((s >> 8) & 0xffff) / 65536.0f - 0.5f; }

int main()
{
    const int R = 512;
    float *A = (float*)malloc(R * 64 * 4), *B = (float*)malloc(R * 64 * 4), *C = (float*)malloc(R * 256 * 4), *D = (float*)malloc(R * 256 * 4);
    unsigned s = 12345;
    for (int i = 0; i < R * 64; i++) { A[i] = rnd(s) * powf(2.f, (int)(rnd(s) * 20)); B[i] = rnd(s) * powf(2.f, (int)(rnd(s) * 20)); }
    for (int i = 0; i < R * 256; i++) C[i] = rnd(s) * powf(2.f, (int)(rnd(s) * 20));
    float *dA, *dB, *dC, *dD;
    hipMalloc(&dA, R * 64 * 4); hipMalloc(&dB, R * 64 * 4); hipMalloc(&dC, R * 256 * 4); hipMalloc(&dD, R * 256 * 4);
    hipMemcpy(dA, A, R * 64 * 4, hipMemcpyHostToDevice); hipMemcpy(dB, B, R * 64 * 4, hipMemcpyHostToDevice);
    hipMemcpy(dC, C, R * 256 * 4, hipMemcpyHostToDevice);
    k<<<1, 64>>>(dA, dB, dC, dD, R);
    hipMemcpy(D, dD, R * 256 * 4, hipMemcpyDeviceToHost);
    long fwd = 0, rev = 0, unf = 0, tot = 0;
    for (int r = 0; r < R; r++)
        for (int i = 0; i < 16; i++)
            for (int j = 0; j < 16; j++) {
                const float* a = A + r * 64 + i * 4; const float* b = B + r * 64;
                float c = C[r * 256 + i * 16 + j], d = D[r * 256 + i * 16 + j];
                float f = c; for (int k2 = 0; k2 < 4; k2++) f = fmaf(a[k2], b[k2 * 16 + j], f);
                float g = c; for (int k2 = 3; k2 >= 0; k2--) g = fmaf(a[k2], b[k2 * 16 + j], g);
                double e = c; for (int k2 = 0; k2 < 4; k2++) e += (double)a[k2] * b[k2 * 16 + j];
                fwd += memcmp(&f, &d, 4) == 0; rev += memcmp(&g, &d, 4) == 0; unf += (float)e == d; tot++;
            }
    printf("mfma_f32_16x16x4: bitwise equal to fmaf chain k=0..3: %ld/%ld, k=3..0: %ld/%ld, exact-sum-rounded-once: %ld/%ld\n", fwd, tot, rev, tot, unf, tot);
    return 0;
}
