"""Round-4 A/B variants of liblsr.so (tools/variant.py: patched copies of csrc).
Timing probes marked (probe) compute wrong results and exist only to price a
piece of work; the others are candidate changes.  Usage: python tools/r04_variants.py [NAME ...]"""
import subprocess
import sys

LOG2E = "1.4426950408889634f"
V = {
    # (probe) forward ML blend with the hardware exp instead of expf_det2
    "fastexp": [(
        "                    const f32x2 EX = expf_det2(P);\n                    const float a0 = fminf(0.99f, OP.x * EX.x), a1 = fminf(0.99f, OP.y * EX.y);",
        f"                    const f32x2 EX = f32x2{{__builtin_amdgcn_exp2f(P.x * {LOG2E}), __builtin_amdgcn_exp2f(P.y * {LOG2E})}};\n"
        "                    const float a0 = fminf(0.99f, OP.x * EX.x), a1 = fminf(0.99f, OP.y * EX.y);")],
    # (probe) backward without atomic memory traffic (every offset out of range)
    "noatom": [
        ("__builtin_amdgcn_raw_ptr_buffer_atomic_fadd_f32(v, rl, on ? off : LSR_BUF_OOB, 0, 0);",
         "__builtin_amdgcn_raw_ptr_buffer_atomic_fadd_f32(v, rl, LSR_BUF_OOB, 0, 0);"),
        ("__builtin_amdgcn_raw_ptr_buffer_atomic_fadd_f32(v, rg, on ? off : LSR_BUF_OOB, 0, 0);",
         "__builtin_amdgcn_raw_ptr_buffer_atomic_fadd_f32(v, rg, LSR_BUF_OOB, 0, 0);")],
    # (probe) backward prologue without the dL/dout fragment loads
    "nofrag": [(
        "        auto ld = [&](__amdgpu_buffer_rsrc_t r, uint32_t off) {\n"
        "            return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0));\n        };",
        "        auto ld = [&](__amdgpu_buffer_rsrc_t r, uint32_t off) {\n"
        "            return (float)(off & 1023) * 1e-3f;\n        };")],
    # (probe) backward without the 1/255 error-band lane collection
    "noband": [("                near_m |= lanes_abs_lt(d, 2e-8f);", "")],
    # candidate: the dot product's MFMA results transposed with permlane swaps instead of through LDS
    "dotperm": [
        ("            // dot[k][p] of the group's candidates on MFMA: (16 x C) . (C x 64)\n            if constexpr (!LO) {",
         "            // dot[k][p] of the group's candidates on MFMA: (16 x C) . (C x 64)\n            float dv[16];\n            (void)dv;\n            if constexpr (!LO) {"),
        ("#pragma unroll\n                for (int pb = 0; pb < 4; pb++)\n#pragma unroll\n"
         "                    for (int r = 0; r < 4; r++) sDU[(4 * lg + r) * GS + pb * 16 + li] = acc[pb][r];\n            }",
         "#pragma unroll\n                for (int r = 0; r < 4; r++) {\n"
         "                    uint32_t x0 = __float_as_uint(acc[0][r]), x1 = __float_as_uint(acc[1][r]);\n"
         "                    uint32_t x2 = __float_as_uint(acc[2][r]), x3 = __float_as_uint(acc[3][r]);\n"
         "                    auto s02 = __builtin_amdgcn_permlane32_swap(x0, x2, false, false);\n"
         "                    auto s13 = __builtin_amdgcn_permlane32_swap(x1, x3, false, false);\n"
         "                    auto s01 = __builtin_amdgcn_permlane16_swap(s02[0], s13[0], false, false);\n"
         "                    auto s23 = __builtin_amdgcn_permlane16_swap(s02[1], s13[1], false, false);\n"
         "                    dv[0 + r] = __uint_as_float(s01[0]);\n                    dv[4 + r] = __uint_as_float(s01[1]);\n"
         "                    dv[8 + r] = __uint_as_float(s23[0]);\n                    dv[12 + r] = __uint_as_float(s23[1]);\n"
         "                }\n            }"),
        ("                    const float dot = sDU[k * GS + lane];\n                    const float al = fminf(0.99f, BWD_OP(k) * G);\n"
         "                    const float om = 1.f - al;\n                    const float rcp",
         "                    const float dot = dv[k];\n                    const float al = fminf(0.99f, BWD_OP(k) * G);\n"
         "                    const float om = 1.f - al;\n                    const float rcp"),
        ("                    const float dot = sDU[k * GS + lane];\n                    const float al = fminf(0.99f, BWD_OP(k) * G);\n"
         "                    const float om = 1.f - al;\n                    T = T * __builtin_amdgcn_rcpf(om);",
         "                    const float dot = dv[k];\n                    const float al = fminf(0.99f, BWD_OP(k) * G);\n"
         "                    const float om = 1.f - al;\n                    T = T * __builtin_amdgcn_rcpf(om);")],
    # candidate: stage padded with INT_MAX positions -> no k < kn test per candidate in phase 1
    "fullgrp": [
        ("struct WaveStageG {\n    float4 A[80];\n    float4 B[80];\n    uint32_t gid[80];\n};",
         "struct WaveStageG {\n    float4 A[96];\n    float4 B[96];\n    uint32_t gid[96];\n};"),
        ("    for (int e = lane; e < 80; e += 64) {\n        st.A[e] = make_float4(0.f, 0.f, 0.f, 0.f);",
         "    for (int e = lane; e < 96; e += 64) {\n        st.A[e] = make_float4(0.f, 0.f, 0.f, 0.f);"),
        ("            n = carry + stage_candidates_geo_rec(st, carry, valid, gid, p, pm.bx, pm.by, Ac, Bc);",
         "            n = carry + stage_candidates_geo_rec(st, carry, valid, gid, p, pm.bx, pm.by, Ac, Bc);\n"
         "            if (lane < 16) reinterpret_cast<float*>(&st.B[n + lane])[3] = __int_as_float(0x7fffffff);\n"
         "            wave_lds_fence();"),
        ("                const bool cj = (k < kn_u) && (__float_as_int(B.w) < last) && !(power > 0.0f);",
         "                const bool cj = (__float_as_int(B.w) < last) && !(power > 0.0f);")],
}
# fullgrp + the conic pre-scaled by -log2e/2 (power in base 2: 7 VALU instead of 10) (timing)
V["p1lite"] = [
    (V["fullgrp"][0][0], "struct WaveStageG {\n    float4 A[96];\n    float4 B[96];\n    float4 Q[96];\n    uint32_t gid[96];\n};"),
    (V["fullgrp"][1][0], "    for (int e = lane; e < 96; e += 64) {\n        st.Q[e] = make_float4(0.f, 0.f, 0.f, 0.f);\n"
                         "        st.A[e] = make_float4(0.f, 0.f, 0.f, 0.f);"),
    V["fullgrp"][2],
    ("        st.B[r] = make_float4(B.x, B.y, B.z, __int_as_float(pos));\n        st.gid[r] = gid;\n    }\n    wave_lds_fence();\n"
     "    return __popcll(m);\n}\n\n// Feature c",
     "        st.B[r] = make_float4(B.x, B.y, B.z, __int_as_float(pos));\n"
     f"        st.Q[r] = make_float4(-0.5f * {LOG2E} * A.z, -{LOG2E} * A.w, -0.5f * {LOG2E} * B.x, 0.f);\n"
     "        st.gid[r] = gid;\n    }\n    wave_lds_fence();\n    return __popcll(m);\n}\n\n// Feature c"),
    ("                const float power = splat_power(A.z, A.w, B.x, A.x - pfx, A.y - pfy);\n"
     "                const bool cj = (k < kn_u) && (__float_as_int(B.w) < last) && !(power > 0.0f);\n"
     "                // G = 0 for a non-candidate pair: alpha - 1/255 is then far below the band\n"
     "                const float G = cj ? __builtin_amdgcn_exp2f(power * LSR_LOG2E) : 0.f;",
     "                const float4 Q = st.Q[g0 + k];\n                const float dx = A.x - pfx, dy = A.y - pfy;\n"
     "                const float p2 = fmaf(dx, fmaf(Q.x, dx, Q.y * dy), (Q.z * dy) * dy);\n"
     "                const bool cj = (__float_as_int(B.w) < last) && !(p2 > 0.0f);\n"
     "                const float G = cj ? __builtin_amdgcn_exp2f(p2) : 0.f;")]
# diagnostic: per-phase s_memtime census (tools/bwd_stamps.py)
V["stamps"] = [('#include "lsr_internal.h"\n\n#ifndef LSR_BWD_SPLAT_PF',
                '#define LSR_BWD_STAMPS 1\n#include "lsr_internal.h"\n\n#ifndef LSR_BWD_SPLAT_PF')]


def build(name):
    args = [sys.executable, "tools/variant.py", name]
    for i, (old, new, *fn) in enumerate(V[name]):
        if i:
            args.append("--")
        args += [old, new] + list(fn)
    r = subprocess.run(args, capture_output=True, text=True)
    if r.returncode:
        raise SystemExit(f"{name}: {r.stdout}{r.stderr}")
    print(r.stdout.strip())


if __name__ == "__main__":
    for n in sys.argv[1:] or list(V):
        build(n)
