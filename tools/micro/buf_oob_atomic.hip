// Does a raw-buffer float atomic whose offset is past num_records leave memory
// alone on gfx950?  (The render backward masks atomics by offset instead of
// exec.)  One allocation of 2048 floats; the descriptor covers the first 1024;
// lanes add 1.0 at offsets inside the range and at offsets in the second half
// second half untouched.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k(float* p)
{
    const int l = threadIdx.x;
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(p, 0, 1024 * 4, 0x00020000);
    const int in_off = l * 4;                          // floats 0..63
    const int oob_off = (1024 + l) * 4;                // floats 1024..1087: past num_records
    __builtin_amdgcn_raw_ptr_buffer_atomic_fadd_f32(1.0f, r, in_off, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_atomic_fadd_f32(1.0f, r, oob_off, 0, 0);
}

int main()
{
    float* d;
    if (hipMalloc(&d, 2048 * 4) != hipSuccess) return 2;
    (void)hipMemset(d, 0, 2048 * 4);
    k<<<1, 64>>>(d);
    if (hipDeviceSynchronize() != hipSuccess) { printf("kernel failed\n"); return 3; }
    float h[2048];
    (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    int in_ok = 0, oob_touched = 0;
    for (int i = 0; i < 64; i++) in_ok += h[i] == 1.0f;
    for (int i = 64; i < 2048; i++) oob_touched += h[i] != 0.0f;
    printf("in-range adds %d/64, out-of-range floats touched %d\n", in_ok, oob_touched);
    return (in_ok == 64 && oob_touched == 0) ? 0 : 1;
}
