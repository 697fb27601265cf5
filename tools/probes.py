"""A/B variants and timing probes of liblsr.so (tools/variant.py: patched copies of csrc).
Timing probes marked (probe) compute wrong results and exist only to price a
piece of work; the others are candidate changes.  Usage: python tools/probes.py [NAME ...]"""
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
}
# candidate: the ML forward's gathered language slices (A operand) loaded one 4-candidate step ahead
V["fwdpf"] = [(
    """            for (int q0 = 0; q0 < n; q0 += 4) {
                if (wave_ballot(!done) == 0) break;
                // A operand: language channel 16 nb + li of candidate q0 + lg
                // (0 past the chunk) -- from the staged rows, or (SF) gathered
                float av[MLB];
#pragma unroll
                for (int nb = 0; nb < MLB; nb++) {
                    // MLM: channels past D (a language set wider than D) read 0
                    const int ch = 16 * nb + li;
                    float fa;
                    if constexpr (SF)
                        fa = a.lang[(size_t)st.gid[min(q0 + lg, n - 1)] * D + (MLM ? min(ch, D - 1) : ch)];
                    else
                        fa = Fs[(q0 + lg) * (F4 * 4) + 3 + ch];
                    av[nb] = ((q0 + lg < n) & (!MLM || ch < D)) ? fa : 0.f;
                }""",
    """            auto a_op = [&](int q, float (&o)[MLB]) {
#pragma unroll
                for (int nb = 0; nb < MLB; nb++) {
                    const int ch = 16 * nb + li;
                    float fa;
                    if constexpr (SF)
                        fa = a.lang[(size_t)st.gid[min(q + lg, n - 1)] * D + (MLM ? min(ch, D - 1) : ch)];
                    else
                        fa = Fs[(q + lg) * (F4 * 4) + 3 + ch];
                    o[nb] = ((q + lg < n) & (!MLM || ch < D)) ? fa : 0.f;
                }
            };
            float avn[MLB];
            if (n > 0) a_op(0, avn);
            for (int q0 = 0; q0 < n; q0 += 4) {
                if (wave_ballot(!done) == 0) break;
                float av[MLB];
#pragma unroll
                for (int nb = 0; nb < MLB; nb++) av[nb] = avn[nb];
                if (q0 + 4 < n) a_op(q0 + 4, avn);""")]

# baseline: no per-block candidate lists (the backward re-stages from the tile lists)
V["nolst"] = [("    uint8_t* p = (uint8_t*)lb;\n    ra.listA = (float4*)p;",
               "    uint8_t* p = (uint8_t*)lb;\n    return;\n    ra.listA = (float4*)p;", "lsr_api.hip")]

# diagnostic: per-phase s_memtime census (tools/bwd_stamps.py)
V["stamps"] = [('#include "lsr_internal.h"\n\n#include <type_traits>',
                '#define LSR_BWD_STAMPS 1\n#include "lsr_internal.h"\n\n#include <type_traits>')]


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
