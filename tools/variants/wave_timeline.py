"""Recipe: python tools/variants/wave_timeline.py -> langsplatv2_amd/_build/var_wtl/liblsr.so (diagnostic only;
read by tools/wave_timeline.py)."""
# builds the wave-timeline variant: per-wave start/end s_memrealtime + HW ids for k_render_bwd_mf<16,.,LD,.,LST> (slot 1) and the training forward k_render_fwd<., true> (slot 0; work = tile instances | list count << 32)
import subprocess, sys
R = "render.hip"
decl = r'''
__device__ unsigned long long g_wtl[1 << 20];   // [kernel 0/1][wave] x {start, end, hwid|xcc<<32, work}
__device__ __forceinline__ void wtl_put(int k, unsigned long long t0, unsigned long long work)
{
    if (threadIdx.x == 0 && blockIdx.x < (1u << 17)) {
        const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
        const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);
        const unsigned xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);
        unsigned long long* p = g_wtl + ((size_t)k << 19) + 4 * (size_t)blockIdx.x;
        p[0] = t0; p[1] = t1; p[2] = hw | ((unsigned long long)xcc << 32); p[3] = work;
    }
}
'''
args = ["python", "tools/variant.py", "wtl",
        "struct WaveTile {", decl + "struct WaveTile {", R, "--",
        "    if constexpr (ZERO) zero_backward_accumulators(a);\n    constexpr int C = 3 + NL;",
        "    const unsigned long long wtl_t0 = __builtin_amdgcn_s_memrealtime();\n    if constexpr (ZERO) zero_backward_accumulators(a);\n    constexpr int C = 3 + NL;", R, "--",
        "            if (lane == 0) a.lcount[4 * wt.tile + wt.sub] = cnt;\n",
        "            if (lane == 0) a.lcount[4 * wt.tile + wt.sub] = cnt;\n            wtl_put(0, wtl_t0, (re - rs) | ((unsigned long long)cnt << 32));\n", R, "--",
        "    const RenderArgs& a = b.f;\n    const Cam& c = a.cam;\n    const WaveTile wt(a, LST ? a.border : nullptr);\n    const int lane = threadIdx.x;\n    const int lg = lane >> 4, li = lane & 15;",
        "    const unsigned long long wtl_t0 = __builtin_amdgcn_s_memrealtime();\n    const RenderArgs& a = b.f;\n    const Cam& c = a.cam;\n    const WaveTile wt(a, LST ? a.border : nullptr);\n    const int lane = threadIdx.x;\n    const int lg = lane >> 4, li = lane & 15;", R, "--",
        "    const int wmax = wave_max_i(last);\n    if (wmax == 0) return;\n    // Prologue order",
        "    const int wmax = wave_max_i(last);\n    if (wmax == 0) { if (LST && LD && !DET) wtl_put(1, wtl_t0, 0); return; }\n    // Prologue order", R, "--",
        "        wave_lds_fence();\n    }\n}\n\n\nhipError_t launch_render_bwd_lang",
        "        wave_lds_fence();\n    }\n    if (LST && LD && !DET) wtl_put(1, wtl_t0, LST ? lcnt : 0);\n}\n\n\nhipError_t launch_render_bwd_lang", R, "--",
        "}  // namespace lsr\n",
        "}  // namespace lsr\nextern \"C\" int lsr_dbg_wave_tl(unsigned long long* out)\n{\n    return hipMemcpyFromSymbol(out, HIP_SYMBOL(lsr::g_wtl), sizeof(unsigned long long) << 20) == hipSuccess ? 0 : 3;\n}\n", R]
subprocess.run(args, check=True)
