// lsr_api.hip — the C ABI (include/lsr.h): host-side driver that validates
// arguments, requests workspaces through the caller's allocator and enqueues
// the gfx950 kernels on the caller's stream.
//
// Forward pipeline (one host sync, for num_rendered):
//   preprocess -> scan(tiles_touched) -> [read M] -> duplicate (tile ranks)
//   -> scan(tile counts) -> scatter into tile buckets -> per-tile depth sort
//   -> render (dense or quick)
// Backward: zero gradient rows -> render bwd (wave-reduced atomics)
//   -> preprocess bwd (chain rule, writes every requested output).
#include <math.h>
#include <stdio.h>
#include <string.h>
#include <atomic>
#include <mutex>
#include <utility>
#include <vector>
#include "lsr_internal.h"

using namespace lsr;

namespace {

struct Status {
    int code = LSR_OK;
};

#define LSR_HIP(expr)                                                        \
    do {                                                                     \
        hipError_t _e = (expr);                                              \
        if (_e != hipSuccess) {                                              \
            fprintf(stderr, "[lsr] %s failed: %s (%s:%d)\n", #expr,          \
                    hipGetErrorString(_e), __FILE__, __LINE__);              \
            return LSR_EHIP;                                                 \
        }                                                                    \
    } while (0)

#define LSR_DEBUG_SYNC(s, st, stage)                                         \
    do {                                                                     \
        if ((s)->debug) {                                                    \
            hipError_t _e = hipStreamSynchronize(st);                        \
            if (_e == hipSuccess) _e = hipGetLastError();                    \
            if (_e != hipSuccess) {                                          \
                fprintf(stderr, "[lsr] stage %s failed: %s\n", stage,        \
                        hipGetErrorString(_e));                              \
                return LSR_EHIP;                                             \
            }                                                                \
        }                                                                    \
    } while (0)

// ---------------------------------------------------------------- profiling
// Optional per-stage HIP-event timing (diagnostics for bench.py's roofline):
// when enabled, each stage is bracketed by two events recorded on the
// caller's stream; lsr_profile_query sums their elapsed times.
enum Stage { ST_PRE, ST_SCAN, ST_DUP, ST_SCAN_T, ST_SCATTER, ST_SORT, ST_RENDER, ST_GZERO, ST_RENDER_BWD,
             ST_PRE_BWD, ST_DET_BOUNDS, ST_DET_FINISH, ST_N };
const char* kStageNames[ST_N] = {"preprocess", "scan_tiles", "bin_count", "scan_tile_counts", "bin_scatter",
                                 "tile_sort", "render_fwd", "grad_zero", "render_bwd", "preprocess_bwd",
                                 "det_bounds", "det_finish"};

// Process-wide (the autograd engine runs backward on its own thread, and the
// caller enables timing on its thread), thread-safe: the switch and mask are
// atomics read once per stage; the event pool is guarded by a mutex that is
// only taken while timing is on.  Off, the product path touches nothing.
struct Prof {
    std::atomic<bool> on{false};
    std::atomic<unsigned> mask{~0u};   // stages bracketed when on (lsr_profile_stages)
    std::mutex mu;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> ev[ST_N];
    size_t used[ST_N] = {};
};
Prof g_prof;

struct StageScope {
    Stage s;
    hipStream_t st;
    bool on;
    size_t slot = 0;
    StageScope(Stage s_, hipStream_t st_) : s(s_), st(st_), on(g_prof.on.load(std::memory_order_relaxed) &&
                                                                 ((g_prof.mask.load(std::memory_order_relaxed) >> s_) & 1u))
    {
        if (!on) return;
        std::lock_guard<std::mutex> lk(g_prof.mu);
        auto& v = g_prof.ev[s];
        if (g_prof.used[s] == v.size()) {
            hipEvent_t a, b;
            if (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess) { on = false; return; }
            v.push_back({a, b});
        }
        slot = g_prof.used[s]++;
        (void)hipEventRecord(v[slot].first, st);
    }
    ~StageScope()
    {
        if (!on) return;
        std::lock_guard<std::mutex> lk(g_prof.mu);
        (void)hipEventRecord(g_prof.ev[s][slot].second, st);
    }
};

// Debug-mode NaN/Inf guard: one streaming scan per array, a
// synchronous read of the flag, LSR_ENONFINITE naming the array.  Off unless
// settings.debug (which already synchronises after every stage).
struct Guard {
    const lsr_settings* s;
    lsr_alloc_fn alloc;
    void* ctx;
    hipStream_t st;
    uint32_t* flag = nullptr;
    Guard(const lsr_settings* s_, lsr_alloc_fn a_, void* c_, hipStream_t st_) : s(s_), alloc(a_), ctx(c_), st(st_) {}
    int check(const char* what, const float* p, size_t n)
    {
        if (!s->debug || !p || n == 0) return LSR_OK;
        if (!flag) {
            if (!alloc) return LSR_EINVAL;
            flag = (uint32_t*)alloc(ctx, 256, LSR_BUF_GUARD);
            if (!flag) return LSR_ENOMEM;
        }
        uint32_t h = 0;
        LSR_HIP(hipMemsetAsync(flag, 0, 4, st));
        LSR_HIP(launch_nonfinite(p, n, flag, st));
        LSR_HIP(hipMemcpyAsync(&h, flag, 4, hipMemcpyDeviceToHost, st));
        LSR_HIP(hipStreamSynchronize(st));
        if (h) {
            fprintf(stderr, "[lsr] non-finite values (NaN/Inf) in %s\n", what);
            return LSR_ENONFINITE;
        }
        return LSR_OK;
    }
    // the binning lists a render is about to gather through (debug only)
    int check_lists(const char* what, const uint32_t* point_list, size_t M, int P, const uint32_t* tile_start, size_t T)
    {
        if (!s->debug || !tile_start || T == 0) return LSR_OK;
        if (!flag) {
            if (!alloc) return LSR_EINVAL;
            flag = (uint32_t*)alloc(ctx, 256, LSR_BUF_GUARD);
            if (!flag) return LSR_ENOMEM;
        }
        uint32_t h = 0;
        LSR_HIP(hipMemsetAsync(flag, 0, 4, st));
        LSR_HIP(launch_check_lists(point_list, M, (uint32_t)P, tile_start, T, flag, st));
        LSR_HIP(hipMemcpyAsync(&h, flag, 4, hipMemcpyDeviceToHost, st));
        LSR_HIP(hipStreamSynchronize(st));
        if (h) {
            fprintf(stderr, "[lsr] corrupt binning lists before %s\n", what);
            return LSR_ELISTS;
        }
        return LSR_OK;
    }
};

#define LSR_GUARD(g, what, p, n)                          \
    do {                                                  \
        const int _rc = (g).check((what), (p), (n));      \
        if (_rc != LSR_OK) return _rc;                    \
    } while (0)

int guard_inputs(Guard& g, const lsr_settings* s, const lsr_inputs* in)
{
    const size_t P = (size_t)in->P;
    LSR_GUARD(g, "means3D", in->means3D, P * 3);
    LSR_GUARD(g, "opacities", in->opacities, P);
    LSR_GUARD(g, "shs", in->shs, P * (size_t)in->max_coeffs * 3);
    LSR_GUARD(g, "colors_precomp", in->colors_precomp, P * 3);
    LSR_GUARD(g, "scales", in->scales, P * 3);
    LSR_GUARD(g, "rotations", in->rotations, P * 4);
    LSR_GUARD(g, "cov3D_precomp", in->cov3D_precomp, P * 6);
    if (s->include_feature && !s->quick_render)
        LSR_GUARD(g, "language_feature_precomp", in->language_feature_precomp, P * (size_t)in->lang_dim);
    if (s->quick_render)
        LSR_GUARD(g, "language_feature_weights_quick", in->language_feature_weights_quick, P * (size_t)in->quick_k);
    return LSR_OK;
}

int dense_dim(const lsr_settings* s, const lsr_inputs* in)
{
    if (s->quick_render) return 0;
    if (!s->include_feature) return 0;
    return in->language_feature_precomp ? in->lang_dim : 0;
}

int quick_dim(const lsr_settings* s)
{
    return s->quick_dim > 0 ? s->quick_dim : 192;
}

int validate(const lsr_settings* s, const lsr_inputs* in)
{
    if (!s || !in) return LSR_EINVAL;
    if (s->image_height <= 0 || s->image_width <= 0 || in->P < 0) return LSR_EINVAL;
    if (!s->bg || !s->viewmatrix || !s->projmatrix || !s->campos) return LSR_EINVAL;
    if (s->quick_layout != LSR_LAYOUT_CHW && s->quick_layout != LSR_LAYOUT_HWC) return LSR_EINVAL;
    if (s->quick_layout == LSR_LAYOUT_HWC && !s->quick_render) return LSR_EINVAL;
    if (in->P > 0) {
        if (!in->means3D || !in->opacities) return LSR_EINVAL;
        if ((in->shs == nullptr) == (in->colors_precomp == nullptr)) return LSR_EINVAL;
        const bool sr = in->scales && in->rotations;
        if (sr == (in->cov3D_precomp != nullptr)) return LSR_EINVAL;
        if (in->shs && (in->max_coeffs <= 0 || s->sh_degree < 0 || s->sh_degree > 3 ||
                        (s->sh_degree + 1) * (s->sh_degree + 1) > in->max_coeffs))
            return LSR_EINVAL;
        if (in->shs && in->max_coeffs > 16) return LSR_EUNSUPPORTED;
    }
    if (s->quick_render) {
        if (in->P > 0 && (!in->language_feature_weights_quick || !in->language_feature_indices || in->quick_k <= 0))
            return LSR_EINVAL;
        if (in->quick_index_dtype < LSR_INDEX_F32 || in->quick_index_dtype > LSR_INDEX_PACKED) return LSR_EINVAL;
        if (in->quick_index_dtype == LSR_INDEX_PACKED) {
            // packed rows: the 12-code LDS-DMA kernel's staging format
            if (in->quick_k != 12 || quick_dim(s) > 192) return LSR_EUNSUPPORTED;
            if (in->P > 0 && (((uintptr_t)in->language_feature_weights_quick % 16) != 0 ||
                              ((uintptr_t)in->language_feature_indices % 16) != 0))
                return LSR_EUNSUPPORTED;
        }
        if ((size_t)quick_dim(s) * 256 + 64 * (32 + 12 + 8 * (size_t)in->quick_k) > 65536) return LSR_EUNSUPPORTED;
        if (s->quick_layout == LSR_LAYOUT_HWC) {
            // the pixel-major map is written by the 12-code, 192-channel LDS-DMA kernel only
            if (in->quick_k != 12 || quick_dim(s) != 192) return LSR_EUNSUPPORTED;
            if (in->P > 0 && (((uintptr_t)in->language_feature_weights_quick % 16) != 0 ||
                              ((uintptr_t)in->language_feature_indices % 16) != 0))
                return LSR_EUNSUPPORTED;
        }
    } else if (s->include_feature) {
        if (in->P > 0 && (!in->language_feature_precomp || in->lang_dim <= 0)) return LSR_EINVAL;
        if (lang_set_for(in->lang_dim) < 0) return LSR_EUNSUPPORTED;
    }
    return LSR_OK;
}

Cam make_cam(const lsr_settings* s)
{
    Cam c;
    c.W = s->image_width;
    c.H = s->image_height;
    c.gx = (c.W + LSR_TILE - 1) / LSR_TILE;
    c.gy = (c.H + LSR_TILE - 1) / LSR_TILE;
    c.tanfovx = s->tanfovx;
    c.tanfovy = s->tanfovy;
    c.fx = (float)c.W / (2.0f * s->tanfovx);
    c.fy = (float)c.H / (2.0f * s->tanfovy);
    c.scale_modifier = s->scale_modifier;
    c.view = s->viewmatrix;
    c.proj = s->projmatrix;
    c.campos = s->campos;
    c.bg = s->bg;
    c.sh_degree = s->sh_degree;
    return c;
}

RenderArgs make_render_args(const lsr_settings* s, const lsr_inputs* in, const Cam& c, const uint8_t* geom,
                            const uint8_t* bin, const uint8_t* img, int64_t M)
{
    RenderArgs a;
    const GeomLayout GL = geom_layout((size_t)in->P);
    const int T = c.gx * c.gy;
    const ImageLayout IL = image_layout((size_t)c.W * c.H, (size_t)T);
    const BinLayout BL = bin_layout((size_t)M);
    a.cam = c;
    a.P = in->P;
    a.splatA = (const float4*)(geom + GL.splatA);
    a.splatB = (const float4*)(geom + GL.splatB);
    a.rgb = in->colors_precomp ? in->colors_precomp : (const float*)(geom + GL.rgb);
    a.D = dense_dim(s, in);
    a.lang = a.D ? in->language_feature_precomp : nullptr;
    a.qw = s->quick_render ? in->language_feature_weights_quick : nullptr;
    a.qi = s->quick_render ? in->language_feature_indices : nullptr;
    a.qidx_dtype = in->quick_index_dtype;
    a.K = s->quick_render ? in->quick_k : 0;
    a.Dq = s->quick_render ? quick_dim(s) : 0;
    a.quick_hwc = s->quick_render && s->quick_layout == LSR_LAYOUT_HWC;
    a.point_list = (const uint32_t*)(bin + BL.point_list);
    a.tile_start = (const uint32_t*)(img + IL.tile_start);
    a.final_T = (float*)(img + IL.final_T);
    a.n_contrib = (uint32_t*)(img + IL.n_contrib);
    a.out_color = nullptr;
    a.out_lang = nullptr;
    return a;
}

}  // namespace

extern "C" {

const char* lsr_strerror(int code)
{
    switch (code) {
        case LSR_OK: return "success";
        case LSR_EINVAL: return "invalid argument (shapes, missing or conflicting inputs)";
        case LSR_EUNSUPPORTED: return "unsupported configuration (language dim / SH coefficients beyond the compiled sets)";
        case LSR_EHIP: return "HIP runtime or kernel launch failure";
        case LSR_ENOMEM: return "workspace allocation failed";
        case LSR_EOVERFLOW: return "num_rendered exceeds 32-bit instance indexing";
        case LSR_ENONFINITE: return "non-finite (NaN/Inf) values in an input or output (debug guard)";
        case LSR_ELISTS: return "corrupt binning lists: a Gaussian id out of range or tile ranges not monotone (debug check)";
        default: return "unknown error";
    }
}

int lsr_quick_decode(const float* weight_map, const float* codebooks, int L, int K, int Df, int H, int W,
                     int normalize, float eps, float* out, lsr_alloc_fn alloc, void* alloc_ctx, void* stream)
{
    if (L < 0 || H < 0 || W < 0 || Df <= 0 || (Df % 16) != 0) return LSR_EINVAL;
    if (K != 64) return LSR_EUNSUPPORTED;
    if (L == 0 || H == 0 || W == 0) return LSR_OK;
    if (!weight_map || !codebooks || !out) return LSR_EINVAL;
    hipStream_t st = (hipStream_t)stream;
    void* ws = nullptr;
    const size_t wsb = lsr::quick_decode_workspace_bytes(L, K, Df, normalize);
    if (wsb) {
        if (!alloc) return LSR_EINVAL;
        ws = alloc(alloc_ctx, wsb, LSR_BUF_DECODE);
        if (!ws) return LSR_ENOMEM;
    }
    if (lsr::launch_quick_decode(weight_map, codebooks, L, K, Df, H, W, normalize, eps, ws, out, st) != hipSuccess)
        return LSR_EHIP;
    return LSR_OK;
}

int lsr_quick_pack_codes(const void* indices, int index_dtype, int64_t N, int K, int quick_dim, uint32_t* packed,
                         void* stream)
{
    if (N < 0 || quick_dim < 0 || index_dtype < LSR_INDEX_F32 || index_dtype > LSR_INDEX_I64) return LSR_EINVAL;
    if (K != 12 || quick_dim > 255) return LSR_EUNSUPPORTED;
    if (N == 0) return LSR_OK;
    if (!indices || !packed || ((uintptr_t)packed % 16) != 0) return LSR_EINVAL;
    if (lsr::launch_quick_pack_codes(indices, index_dtype, N, quick_dim > 0 ? quick_dim : 192, packed,
                                     (hipStream_t)stream) != hipSuccess)
        return LSR_EHIP;
    return LSR_OK;
}

size_t lsr_quick_decode_plan_bytes(int L, int K, int Df, int normalize)
{
    if (L < 0 || K != 64 || Df <= 0 || (Df % 16) != 0) return 0;
    return lsr::quick_decode_workspace_bytes(L, K, Df, normalize);
}

int lsr_quick_decode_prepare(const float* codebooks, int L, int K, int Df, int normalize, void* plan, void* stream)
{
    if (L < 0 || Df <= 0 || (Df % 16) != 0) return LSR_EINVAL;
    if (K != 64) return LSR_EUNSUPPORTED;
    if (L == 0) return LSR_OK;
    if (!codebooks || !plan) return LSR_EINVAL;
    if (lsr::launch_quick_decode_prepare(codebooks, L, K, Df, normalize, plan, (hipStream_t)stream) != hipSuccess)
        return LSR_EHIP;
    return LSR_OK;
}

int lsr_quick_decode_run(const float* weight_map, int weight_layout, const void* plan, int L, int K, int Df, int H,
                         int W, int normalize, float eps, float* out, void* stream)
{
    if (L < 0 || H < 0 || W < 0 || Df <= 0 || (Df % 16) != 0) return LSR_EINVAL;
    if (weight_layout != LSR_LAYOUT_CHW && weight_layout != LSR_LAYOUT_HWC) return LSR_EINVAL;
    if (K != 64) return LSR_EUNSUPPORTED;
    if (L == 0 || H == 0 || W == 0) return LSR_OK;
    if (!weight_map || !plan || !out) return LSR_EINVAL;
    // the pixel-major map is read in 32-B pieces by the level-resident kernel (Df <= 512)
    if (weight_layout == LSR_LAYOUT_HWC && (Df > 512 || ((uintptr_t)weight_map % 16) != 0)) return LSR_EUNSUPPORTED;
    if (lsr::launch_quick_decode_run(weight_map, nullptr, L, K, Df, H, W, normalize, eps, plan, out,
                                     (hipStream_t)stream, weight_layout == LSR_LAYOUT_HWC) != hipSuccess)
        return LSR_EHIP;
    return LSR_OK;
}

static int lang_loss_args(const float* wm, const float* cb, int K, int Df, int H, int W, const int32_t* seg,
                          const float* feat, int S)
{
    if (K <= 0 || Df <= 0 || H <= 0 || W <= 0 || S < 0) return LSR_EINVAL;
    if (K != 64 || (Df % 16) != 0) return LSR_EUNSUPPORTED;
    if (!wm || !cb || !seg || (S > 0 && !feat)) return LSR_EINVAL;
    return LSR_OK;
}

int lsr_lang_loss_forward(const float* weight_map, const float* codebooks, int K, int Df, int H, int W,
                          const int32_t* seg, const float* features, int S, float* loss, float* pixel_stats,
                          lsr_alloc_fn alloc, void* alloc_ctx, void* stream)
{
    const int rc = lang_loss_args(weight_map, codebooks, K, Df, H, W, seg, features, S);
    if (rc != LSR_OK) return rc;
    if ((!loss && !pixel_stats) || !alloc) return LSR_EINVAL;
    float* ws = (float*)alloc(alloc_ctx, lsr::lang_loss_workspace_bytes(S, W, H, nullptr), LSR_BUF_LOSS);
    if (!ws) return LSR_ENOMEM;
    if (lsr::launch_lang_loss(weight_map, codebooks, Df, H, W, seg, features, S, nullptr, loss, nullptr, nullptr,
                              pixel_stats, ws, (hipStream_t)stream) != hipSuccess)
        return LSR_EHIP;
    return LSR_OK;
}

int lsr_lang_loss_backward(const float* weight_map, const float* codebooks, int K, int Df, int H, int W,
                           const int32_t* seg, const float* features, int S, const float* pixel_stats,
                           const float* grad_loss, float* grad_weight_map, float* grad_codebooks, lsr_alloc_fn alloc,
                           void* alloc_ctx, void* stream)
{
    const int rc = lang_loss_args(weight_map, codebooks, K, Df, H, W, seg, features, S);
    if (rc != LSR_OK) return rc;
    if (!grad_loss || !grad_weight_map || !grad_codebooks || !alloc) return LSR_EINVAL;
    float* ws = (float*)alloc(alloc_ctx, lsr::lang_loss_workspace_bytes(S, W, H, nullptr), LSR_BUF_LOSS);
    if (!ws) return LSR_ENOMEM;
    if (lsr::launch_lang_loss(weight_map, codebooks, Df, H, W, seg, features, S, grad_loss, nullptr,
                              grad_weight_map, grad_codebooks, const_cast<float*>(pixel_stats), ws,
                              (hipStream_t)stream) != hipSuccess)
        return LSR_EHIP;
    return LSR_OK;
}

int lsr_adam_step(float* params, const float* grads, float* exp_avg, float* exp_avg_sq, int64_t n, double lr,
                  double beta1, double beta2, double eps, double weight_decay, int64_t step, void* stream)
{
    if (n < 0 || step < 1 || !(beta1 >= 0.0 && beta1 < 1.0) || !(beta2 >= 0.0 && beta2 < 1.0)) return LSR_EINVAL;
    if (n == 0) return LSR_OK;
    if (!params || !grads || !exp_avg || !exp_avg_sq) return LSR_EINVAL;
    // scalars as torch forms them: Python doubles, rounded once to fp32
    const double bc1 = 1.0 - pow(beta1, (double)step);
    const double bc2 = 1.0 - pow(beta2, (double)step);
    lsr::AdamArgs a;
    a.one_minus_b1 = (float)(1.0 - beta1);
    a.b2 = (float)beta2;
    a.one_minus_b2 = (float)(1.0 - beta2);
    a.eps = (float)eps;
    a.step_size = (float)(lr / bc1);
    a.bc2_sqrt = (float)sqrt(bc2);
    a.weight_decay = (float)weight_decay;
    if (lsr::launch_adam(params, grads, exp_avg, exp_avg_sq, n, a, (hipStream_t)stream) != hipSuccess)
        return LSR_EHIP;
    return LSR_OK;
}

static bool topk_code_args_ok(int64_t N, int L, int K, int k)
{
    return N >= 0 && L >= 1 && K >= 64 && K <= 256 && (K % 64) == 0 && k >= 1 && k <= K &&
           N <= (int64_t)0x7fffffff / ((int64_t)L * K);
}

int lsr_topk_code_forward(const float* logits, int64_t N, int L, int K, int k, float* dense, float* sparse_w,
                          void* sparse_idx, int idx_dtype, int level_offset, void* stream)
{
    if (!topk_code_args_ok(N, L, K, k)) return (K % 64 || K > 256) && K > 0 ? LSR_EUNSUPPORTED : LSR_EINVAL;
    if (idx_dtype < LSR_INDEX_F32 || idx_dtype > LSR_INDEX_I64) return LSR_EINVAL;
    if (N == 0) return LSR_OK;
    if (!logits || (!dense && !sparse_w && !sparse_idx)) return LSR_EINVAL;
    if (lsr::launch_topk_code_fwd(logits, N, L, K, k, dense, sparse_w, sparse_idx, idx_dtype, level_offset,
                                  (hipStream_t)stream) != hipSuccess)
        return LSR_EHIP;
    return LSR_OK;
}

int lsr_topk_code_backward(const float* logits, const float* grad_dense, int64_t N, int L, int K, int k,
                           float* grad_logits, void* stream)
{
    if (!topk_code_args_ok(N, L, K, k)) return (K % 64 || K > 256) && K > 0 ? LSR_EUNSUPPORTED : LSR_EINVAL;
    if (N == 0) return LSR_OK;
    if (!logits || !grad_dense || !grad_logits) return LSR_EINVAL;
    if (lsr::launch_topk_code_bwd(logits, grad_dense, N, L, K, k, grad_logits, (hipStream_t)stream) != hipSuccess)
        return LSR_EHIP;
    return LSR_OK;
}

int lsr_topk_code_backward_sparse(const float* logits, const float* grad_weights, int64_t N, int L, int K, int k,
                                  float* grad_logits, void* stream)
{
    if (!topk_code_args_ok(N, L, K, k)) return (K % 64 || K > 256) && K > 0 ? LSR_EUNSUPPORTED : LSR_EINVAL;
    if (N == 0) return LSR_OK;
    if (!logits || !grad_weights || !grad_logits) return LSR_EINVAL;
    if (lsr::launch_topk_code_bwd(logits, grad_weights, N, L, K, k, grad_logits, (hipStream_t)stream, true) !=
        hipSuccess)
        return LSR_EHIP;
    return LSR_OK;
}

int lsr_knn_dist2(const float* points, int64_t N, float* out, lsr_alloc_fn alloc, void* alloc_ctx, void* stream)
{
    if (N < 0 || N > 0x7fffffffLL) return LSR_EINVAL;
    if (N == 0) return LSR_OK;
    if (!points || !out || !alloc) return LSR_EINVAL;
    size_t sort_temp = 0;
    if (lsr::knn_sort_temp_bytes(N, &sort_temp) != hipSuccess) return LSR_EHIP;
    uint8_t* ws = (uint8_t*)alloc(alloc_ctx, lsr::knn_workspace_bytes(N, sort_temp), LSR_BUF_KNN);
    if (!ws) return LSR_ENOMEM;
    if (lsr::launch_knn_dist2(points, N, out, ws, sort_temp, (hipStream_t)stream) != hipSuccess) return LSR_EHIP;
    return LSR_OK;
}

int lsr_sh_grad_from_views(int64_t N, int M, int sh_degree, const float* means3D, int R, const float* campos,
                           const float* drgb, float* dL_dsh, void* stream)
{
    if (N < 0 || M < 1 || M > 16 || sh_degree < 0 || sh_degree > 3 || (sh_degree + 1) * (sh_degree + 1) > M || R < 0)
        return LSR_EINVAL;
    if (N == 0) return LSR_OK;
    if (!means3D || !dL_dsh || (R > 0 && (!campos || !drgb))) return LSR_EINVAL;
    if (lsr::launch_sh_grad_from_views(N, M, sh_degree, means3D, R, campos, drgb, dL_dsh, (hipStream_t)stream) !=
        hipSuccess)
        return LSR_EHIP;
    return LSR_OK;
}

int lsr_abi_version(void) { return LSR_ABI_VERSION; }

// Process-wide options (lsr_set_option).  LSR_OPT_BIN_MODE: the forward's tile
// binning; one mode is built (binning.hip: scatter into tile buckets + per-tile
// sort).  The depth-ordered mode of round 4 (order.hip) measured slower at every
// size (cfg5 scatter 4.55 vs 0.84 ms) and was removed in round 5.
static std::atomic<int64_t> g_bin_mode{LSR_BIN_AUTO};
// LSR_OPT_LISTS_MAX_MB: the backward's per-block candidate lists (128 B per
// instance of capacity) are written only while they fit this budget; above it
// the backward re-stages its candidates from the tile lists (same results,
// measured 2.8 % slower at cfg3).  cfg3: 0.6 GB; cfg5 (M = 60 M): 7.7 GB -> off.
static std::atomic<int64_t> g_lists_max_mb{2048};
// LSR_OPT_SPLIT_PREPROCESS: the SH colour pass on a second stream, concurrent
// with the binning (preprocess.hip k_preprocess_colour).
static std::atomic<int64_t> g_split_pre{1};
// LSR_OPT_DETERMINISTIC: the render backward's cross-block sums as 64-bit
// fixed-point atomics (render.hip det_shift), converted back by k_det_finish
static std::atomic<int64_t> g_det{0};
#ifndef LSR_SPLIT_MIN_P
#define LSR_SPLIT_MIN_P (1 << 19)
#endif
#ifndef LSR_COLOUR_EVENT_FLAGS
#define LSR_COLOUR_EVENT_FLAGS hipEventDisableTiming   // A/B: | hipEventReleaseToDevice
#endif
#ifndef LSR_SPLIT_AFTER_COUNT
#define LSR_SPLIT_AFTER_COUNT 0   // 1: the colour pass starts behind the tile count instead of the geometry
#endif
static constexpr int kSplitPreMinP = LSR_SPLIT_MIN_P;

int lsr_set_option(int option, int64_t value)
{
    switch (option) {
        case LSR_OPT_BIN_MODE:
            if (value != LSR_BIN_AUTO && value != LSR_BIN_SORTED_TILES) return LSR_EINVAL;
            g_bin_mode.store(value, std::memory_order_relaxed);
            return LSR_OK;
        case LSR_OPT_LISTS_MAX_MB:
            if (value < 0) return LSR_EINVAL;
            g_lists_max_mb.store(value, std::memory_order_relaxed);
            return LSR_OK;
        case LSR_OPT_SPLIT_PREPROCESS:
            if (value != 0 && value != 1) return LSR_EINVAL;
            g_split_pre.store(value, std::memory_order_relaxed);
            return LSR_OK;
        case LSR_OPT_DETERMINISTIC:
            if (value != 0 && value != 1) return LSR_EINVAL;
            g_det.store(value, std::memory_order_relaxed);
            return LSR_OK;
        default:
            return LSR_EINVAL;
    }
}

int lsr_get_option(int option, int64_t* value)
{
    if (!value) return LSR_EINVAL;
    switch (option) {
        case LSR_OPT_BIN_MODE: *value = g_bin_mode.load(std::memory_order_relaxed); return LSR_OK;
        case LSR_OPT_LISTS_MAX_MB: *value = g_lists_max_mb.load(std::memory_order_relaxed); return LSR_OK;
        case LSR_OPT_SPLIT_PREPROCESS: *value = g_split_pre.load(std::memory_order_relaxed); return LSR_OK;
        case LSR_OPT_DETERMINISTIC: *value = g_det.load(std::memory_order_relaxed); return LSR_OK;
        default: return LSR_EINVAL;
    }
}

int lsr_max_lang_dim(void) { return 64; }

int lsr_stream_create(void** stream)
{
    if (!stream) return LSR_EINVAL;
    hipStream_t s = nullptr;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return LSR_EHIP;
    *stream = (void*)s;
    return LSR_OK;
}

int lsr_stream_destroy(void* stream)
{
    if (!stream) return LSR_EINVAL;
    return hipStreamDestroy((hipStream_t)stream) == hipSuccess ? LSR_OK : LSR_EHIP;
}

void lsr_profile_enable(int on)
{
    g_prof.on.store(on != 0);
}

int lsr_profile_stages(const char* names)
{
    if (!names || !*names) { g_prof.mask.store(~0u); return LSR_OK; }
    unsigned m = 0;
    const char* p = names;
    while (*p) {
        const char* e = p;
        while (*e && *e != ',') e++;
        int hit = -1;
        for (int k = 0; k < ST_N; k++)
            if (strlen(kStageNames[k]) == (size_t)(e - p) && strncmp(kStageNames[k], p, (size_t)(e - p)) == 0) hit = k;
        if (hit < 0) return LSR_EINVAL;
        m |= 1u << hit;
        p = *e ? e + 1 : e;
    }
    g_prof.mask.store(m);
    return LSR_OK;
}

void lsr_profile_reset(void)
{
    std::lock_guard<std::mutex> lk(g_prof.mu);
    for (int k = 0; k < ST_N; k++) g_prof.used[k] = 0;
}

int lsr_profile_query(const char** names, double* ms, int64_t* calls, int max_stages)
{
    std::lock_guard<std::mutex> lk(g_prof.mu);
    int n = 0;
    for (int k = 0; k < ST_N && n < max_stages; k++, n++) {
        double tot = 0.0;
        for (size_t i = 0; i < g_prof.used[k]; i++) {
            float e = 0.f;
            if (hipEventSynchronize(g_prof.ev[k][i].second) != hipSuccess) return -LSR_EHIP;
            if (hipEventElapsedTime(&e, g_prof.ev[k][i].first, g_prof.ev[k][i].second) != hipSuccess) return -LSR_EHIP;
            tot += e;
        }
        if (names) names[n] = kStageNames[k];
        if (ms) ms[n] = tot;
        if (calls) calls[n] = (int64_t)g_prof.used[k];
    }
    return n;
}

// ------------------------------------------- split preprocess: colour stream
// One non-blocking stream and two events per host thread and device (created
// on first use, destroyed when the thread exits), on the device of the
// caller's stream (not the thread's current device: a caller may pass another
// device's stream).  The SH colour pass runs there behind the geometry pass
// while the caller's stream bins.  When no colour stream can be had (device
// index >= 16, creation failure) the forward runs the fused preprocess, which
// gives identical results.
struct ColourStream {
    hipStream_t stream = nullptr;
    hipEvent_t geom_done = nullptr, colour_done = nullptr;
    void release()
    {
        if (colour_done) (void)hipEventDestroy(colour_done);
        if (geom_done) (void)hipEventDestroy(geom_done);
        if (stream) (void)hipStreamDestroy(stream);
        stream = nullptr;
        geom_done = colour_done = nullptr;
    }
    ~ColourStream() { release(); }
};

static ColourStream* colour_stream(hipStream_t st)
{
    thread_local ColourStream tab[16];
    hipDevice_t sdev = 0;
    int cur = 0;
    if (hipStreamGetDevice(st, &sdev) != hipSuccess || hipGetDevice(&cur) != hipSuccess) return nullptr;
    const int dev = (int)sdev;
    if (dev < 0 || dev >= 16) return nullptr;
    ColourStream& cs = tab[dev];
    if (!cs.stream) {
        // streams and events belong to the device current at their creation
        if (dev != cur && hipSetDevice(dev) != hipSuccess) return nullptr;
        const bool ok = hipStreamCreateWithFlags(&cs.stream, hipStreamNonBlocking) == hipSuccess &&
                        hipEventCreateWithFlags(&cs.geom_done, LSR_COLOUR_EVENT_FLAGS) == hipSuccess &&
                        hipEventCreateWithFlags(&cs.colour_done, LSR_COLOUR_EVENT_FLAGS) == hipSuccess;
        if (dev != cur) (void)hipSetDevice(cur);
        if (!ok) {
            cs.release();
            return nullptr;
        }
    }
    return &cs;
}

// Makes the caller's stream wait for the colour pass exactly once: before the
// render, or on any early return (the pass writes into the caller's geometry
// buffer, which must not be released while it runs).
struct ColourJoin {
    ColourStream* cs;
    hipStream_t st;
    bool done = false;
    hipError_t wait()
    {
        if (!cs || done) return hipSuccess;
        done = true;
        return hipStreamWaitEvent(st, cs->colour_done, 0);
    }
    ~ColourJoin() { (void)wait(); }
};

// ------------------------------------------------- host-visible scan total
// One coherent pinned line per host thread: word 0 receives (seq << 32 | M)
// from k_bin_count (k_publish_total on the global-atomic path), words 1..3 the
// tile-sort class counts and word LSR_CLS_SLOT (seq << 32 | M) once those are
// out (k_bin_table); the host spins until a word's sequence matches.
struct HostSlot {
    uint64_t* word = nullptr;   // host view
    uint64_t* dev = nullptr;    // device view of the same word
    uint32_t seq = 0;
    uint64_t last_m = 0;        // previous forward's M (binning size guess)
    ~HostSlot() { if (word) (void)hipHostFree(word); }
};

static HostSlot& host_slot()
{
    thread_local HostSlot hs;
    if (!hs.word) {
        void* p = nullptr;
        if (hipHostMalloc(&p, 64, hipHostMallocCoherent | hipHostMallocPortable | hipHostMallocMapped) != hipSuccess)
            return hs;
        void* d = nullptr;
        if (hipHostGetDevicePointer(&d, p, 0) != hipSuccess) { (void)hipHostFree(p); return hs; }
        hs.word = (uint64_t*)p;
        hs.dev = (uint64_t*)d;
        *(volatile uint64_t*)hs.word = 0;
    }
    return hs;
}

// Spin on the published word; every 4096 polls ask the runtime whether the
// stream has drained (which also covers a stream the runtime has not
// submitted yet, and reports a faulted stream instead of spinning forever).
static int wait_published(HostSlot& hs, uint32_t seq, hipStream_t st, uint64_t* M, int slot = 0)
{
    volatile uint64_t* w = hs.word + slot;
    for (uint64_t it = 1;; it++) {
        uint64_t v = __atomic_load_n((uint64_t*)w, __ATOMIC_ACQUIRE);
        if ((uint32_t)(v >> 32) == seq) {
            *M = v & 0xffffffffull;
            return LSR_OK;
        }
        if ((it & 4095) == 0) {
            const hipError_t q = hipStreamQuery(st);
            if (q == hipSuccess) {
                v = __atomic_load_n((uint64_t*)w, __ATOMIC_ACQUIRE);
                if ((uint32_t)(v >> 32) != seq) {
                    fprintf(stderr, "[lsr] scan total was not published (stream drained)\n");
                    return LSR_EHIP;
                }
                *M = v & 0xffffffffull;
                return LSR_OK;
            }
            if (q != hipErrorNotReady) {
                fprintf(stderr, "[lsr] stream failed while waiting for the scan total: %s\n", hipGetErrorString(q));
                return LSR_EHIP;
            }
        }
        __builtin_ia32_pause();
    }
}

// The dense backward's accumulators (lsr_fwd_out.grad_ws / grad_ws_lang):
// gradient rows (P x VP, unless only dL/dlang is requested) and, where the
// render backward adds dL/dlang straight into an (P, D) array (language-only,
// or D = 16 / 32 with aligned rows), that array -- a separate allocation, so
// the gradient the caller keeps holds no gradient rows alive.  kind encodes
// the configuration, so a backward uses a forward's accumulators only when it
// needs exactly these.
struct GradWs {
    int kind = 0;          // 0: nothing to prepare
    int VP = 0;
    size_t rows_bytes = 0, lang_bytes = 0;
    bool lang_only = false, lang_direct = false;
};
static GradWs grad_ws_layout(int P, int Dd, bool geom, bool lang, bool lang_aligned)
{
    GradWs w;
    lang = lang && Dd > 0;
    if (P <= 0 || (!geom && !lang)) return w;
    w.lang_only = lang && !geom;
    w.lang_direct = lang && geom && bwd_lang_direct(Dd) && lang_aligned;
    if (w.lang_only || w.lang_direct) w.lang_bytes = (size_t)P * Dd * 4;
    if (!w.lang_only) {
        w.VP = w.lang_direct ? 16 : grad_row_width(Dd);
        w.rows_bytes = (size_t)P * w.VP * 4;
    }
    w.kind = (geom ? 1 : 0) | (lang ? 2 : 0) | (w.lang_direct ? 4 : 0) | (w.VP << 8);
    return w;
}

// The backward's per-block candidate lists (RenderArgs::listA/B/lcount): A and
// B arrays of 4 M entries (block b = 4 tile + sub owns [4 tile_start + sub n_tile,
// + n_tile)), then the 4 T per-block counts.  The forward that writes them also
// writes the backward's block order (RenderArgs::border, ImageLayout::border).
static size_t block_lists_bytes(size_t M, size_t T)
{
    if (M == 0 || T == 0) return 0;
    return 2 * align256(4 * M * 16) + align256(4 * T * 4);
}
static void set_block_lists(RenderArgs& ra, void* lb, size_t M)
{
    uint8_t* p = (uint8_t*)lb;
    ra.listA = (float4*)p;
    ra.listB = (float4*)(p + align256(4 * M * 16));
    ra.lcount = (uint32_t*)(p + 2 * align256(4 * M * 16));
}
// the backward's view of the lists, with the block order the same forward wrote
static void set_block_lists_bwd(RenderArgs& ra, const void* lb, const void* img, size_t M)
{
    set_block_lists(ra, (void*)lb, M);
    const size_t T = (size_t)ra.cam.gx * ra.cam.gy;
    if (bwd_order_on((int)T)) ra.border = (const uint4*)((const uint8_t*)img + image_layout((size_t)ra.cam.W * ra.cam.H, T).border);
}

int lsr_forward(const lsr_settings* s, const lsr_inputs* in, lsr_fwd_out* out, lsr_alloc_fn alloc, void* ctx,
                void* stream)
{
    int rc = validate(s, in);
    if (rc != LSR_OK) return rc;
    if (!out || !alloc || !out->out_color || (in->P > 0 && !out->radii)) return LSR_EINVAL;
    const int Dd = dense_dim(s, in);
    if ((Dd > 0 || s->quick_render) && !out->out_lang) return LSR_EINVAL;
    hipStream_t st = (hipStream_t)stream;
    const Cam c = make_cam(s);
    const int P = in->P;
    const int T = c.gx * c.gy;
    const size_t NPIX = (size_t)c.W * c.H;

    Guard guard(s, alloc, ctx, st);
    rc = guard_inputs(guard, s, in);
    if (rc != LSR_OK) return rc;

    const GeomLayout GL = geom_layout((size_t)P);
    const ImageLayout IL = image_layout(NPIX, (size_t)T);
    // privatised binning needs a B x T table (tail of the image workspace)
    const bool priv = P > 0 && bin_privatised_ok(c);
    int chunk = 0;
    const int B = priv ? bin_blocks(P, c, chunk) : 0;
    const size_t table_bytes = priv ? align256((size_t)B * table_stride(T) * 4) : 0;
    uint8_t* geom = (uint8_t*)alloc(ctx, GL.total, LSR_BUF_GEOM);
    uint8_t* img = (uint8_t*)alloc(ctx, IL.total + table_bytes, LSR_BUF_IMAGE);
    if (!geom || !img) return LSR_ENOMEM;
    out->geom = geom;
    out->geom_bytes = GL.total;
    out->image = img;
    out->image_bytes = IL.total + table_bytes;
    uint32_t* table = (uint32_t*)(img + IL.total);
    uint32_t* tile_cnt = (uint32_t*)(img + IL.tile_cnt);
    uint32_t* tile_start = (uint32_t*)(img + IL.tile_start);
    uint64_t* tpart = (uint64_t*)(img + IL.tile_part);
    const size_t tnb = scan_partials((size_t)T) - 1;
    uint32_t* cls_cnt = (uint32_t*)(img + IL.cls_cnt);
    uint32_t* cls_list = (uint32_t*)(img + IL.cls_list);

    // 1. preprocess (the SH colour pass on the second stream when split)
    ColourStream* colour = nullptr;
    // from 512K Gaussians up (cfg5 5M: whole forward 2.974 -> 2.812 and 2.995 -> 2.835 ms;
    // cfg3 1M fwd+bwd: 1.1188 -> 1.1176 and 1.1259 -> 1.1156 ms, the colour pass slowing
    // the short count; cfg2 100K: slower, its forward is bound by host launches; the
    // colour pass started behind the count instead: cfg5 2.946, cfg3 1.1159 ms;
    // profiles/r05s3_ab_split_cfg*.txt, r05s3_ab_split_start_cfg*.txt)
    if (g_split_pre.load(std::memory_order_relaxed) && !s->debug && P >= kSplitPreMinP && in->shs &&
        !in->colors_precomp) {
        colour = colour_stream(st);   // nullptr: the fused preprocess below (same results)
    }
    ColourJoin join{colour, st};   // every return after the launch leaves `st` behind the colour pass
    {
        // a pending geometry gradient: the preprocess also stores the SH colour
        // Jacobian the preprocess backward needs (48 B instead of the 192-B SH row)
        const bool jac = (out->grad_ws_request & LSR_GWS_GEOM) != 0 && !s->quick_render;
        StageScope sc(ST_PRE, st);
        LSR_HIP(launch_preprocess(c, *in, geom, out->radii, jac, st, colour != nullptr,
                                  priv ? (uint64_t*)(cls_cnt + LSR_COUNT_WORD) : nullptr));
        if (colour && !LSR_SPLIT_AFTER_COUNT)
            LSR_HIP(launch_preprocess_colour(c, *in, geom, out->radii, jac, st, colour->stream, colour->geom_done,
                                             colour->colour_done));
    }
    LSR_DEBUG_SYNC(s, st, "preprocess");
    HostSlot& hs = host_slot();
    if (!hs.word) return LSR_EHIP;
    const uint32_t seq = ++hs.seq;
    if (priv) {
        // 2. per-block tile histograms -> column scan -> tile starts; M = total
        {
            StageScope sc(ST_DUP, st);
            LSR_HIP(launch_bin_count(c, P, chunk, B, geom, out->radii, table, tile_cnt, tile_start, tpart, cls_cnt,
                                     cls_list, hs.dev, seq, st));
        }
        {
            StageScope sc(ST_SCAN_T, st);
            LSR_HIP(launch_tile_start_apply(T, B, tile_cnt, tpart, tile_start, st));
        }
    } else {
        uint64_t* gpart = (uint64_t*)(geom + GL.scan_part);
        const size_t gnb = scan_partials((size_t)P) - 1;
        StageScope sc(ST_SCAN, st);
        LSR_HIP(launch_scan_u32((const uint32_t*)(geom + GL.tiles), (uint32_t*)(geom + GL.offsets), gpart,
                                (size_t)P, false, st));
        LSR_HIP(launch_publish_total(gpart + gnb, nullptr, hs.dev, seq, nullptr, st));
    }
    if (colour && LSR_SPLIT_AFTER_COUNT) {
        const bool jac = (out->grad_ws_request & LSR_GWS_GEOM) != 0 && !s->quick_render;
        LSR_HIP(launch_preprocess_colour(c, *in, geom, out->radii, jac, st, colour->stream, colour->geom_done,
                                         colour->colour_done));
    }
    // speculative binning workspace sized from the previous call's M, taken
    // while the GPU is still counting, so the host usually has nothing but
    // launches to do once M is known
    uint8_t* bin = nullptr;
    size_t bin_cap = 0;
    if (hs.last_m > 0) {
        const size_t guess = (size_t)(hs.last_m + hs.last_m / 4 + 4096);
        bin_cap = bin_layout(guess).total;
        bin = (uint8_t*)alloc(ctx, bin_cap, LSR_BUF_BINNING);
        if (!bin) return LSR_ENOMEM;
    }
    uint64_t M = 0;
    rc = wait_published(hs, seq, st, &M);
    if (rc != LSR_OK) return rc;
    LSR_DEBUG_SYNC(s, st, "count");
    if (M >= 0xffffffffull) return LSR_EOVERFLOW;
    out->num_rendered = (int64_t)M;
    hs.last_m = M;

    // 3. binning workspace + scatter into tile buckets
    const BinLayout BL = bin_layout((size_t)M);
    if (!bin || BL.total > bin_cap) {
        bin_cap = BL.total > 0 ? BL.total : 256;
        bin = (uint8_t*)alloc(ctx, bin_cap, LSR_BUF_BINNING);
        if (!bin) return LSR_ENOMEM;
    }
    out->binning = bin;
    out->binning_bytes = bin_cap;
    if (priv) {
        StageScope sc(ST_SCATTER, st);
        LSR_HIP(launch_bin_scatter(c, P, chunk, B, geom, out->radii, table, tile_start, (uint64_t*)(bin + BL.keys),
                                   st));
    } else {
        {
            StageScope sc(ST_DUP, st);
            LSR_HIP(hipMemsetAsync(tile_cnt, 0, (size_t)T * 4, st));
            LSR_HIP(launch_duplicate(c, P, geom, out->radii, tile_cnt, (uint32_t*)(bin + BL.rank), st));
        }
        {
            StageScope sc(ST_SCAN_T, st);
            LSR_HIP(launch_scan_u32(tile_cnt, tile_start, tpart, (size_t)T, true, st));
            LSR_HIP(hipMemcpyAsync(tile_start + T, tpart + tnb, sizeof(uint32_t), hipMemcpyDeviceToDevice, st));
        }
        StageScope sc(ST_SCATTER, st);
        LSR_HIP(launch_scatter(c, P, geom, out->radii, tile_start, (const uint32_t*)(bin + BL.rank),
                               (uint64_t*)(bin + BL.keys), st));
    }
    LSR_DEBUG_SYNC(s, st, "scatter");
    // the privatised path's tile-sort class counts: published by the column
    // scan (k_bin_table) with its own M, after the count published M -- the
    // scatter above was launched in between
    uint32_t host_cls[SORT_NCLS];
    if (priv) {
        uint64_t M2 = 0;
        rc = wait_published(hs, seq, st, &M2, LSR_CLS_SLOT);
        if (rc != LSR_OK) return rc;
        if (M2 != M) {
            fprintf(stderr, "[lsr] tile count and column scan disagree on M (%llu vs %llu)\n",
                    (unsigned long long)M, (unsigned long long)M2);
            return LSR_EHIP;
        }
        for (int k = 0; k < SORT_NCLS; k++) host_cls[k] = ((volatile uint32_t*)(hs.word + 1))[k];
    }
    {
        StageScope sc(ST_SORT, st);
        LSR_HIP(launch_tile_sort(T, tile_start, (uint64_t*)(bin + BL.keys), (uint32_t*)(bin + BL.point_list), cls_cnt,
                                 cls_list, priv ? host_cls : nullptr, st));
    }
    LSR_DEBUG_SYNC(s, st, "tile_sort");

    // 4. render (and the backward's accumulators zeroed alongside it)
    RenderArgs ra = make_render_args(s, in, c, geom, bin, img, (int64_t)M);
    {
        const int lrc = guard.check_lists("render", ra.point_list, (size_t)M, P, ra.tile_start, (size_t)T);
        if (lrc != LSR_OK) return lrc;
    }
    ra.out_color = out->out_color;
    ra.out_lang = out->out_lang;
    out->grad_ws = nullptr;
    out->grad_ws_bytes = 0;
    out->grad_ws_kind = 0;
    out->grad_ws_lang = nullptr;
    out->lists = nullptr;
    out->lists_bytes = 0;
    if (out->grad_ws_request && !s->quick_render) {
        const GradWs w = grad_ws_layout(P, Dd, (out->grad_ws_request & LSR_GWS_GEOM) != 0,
                                        (out->grad_ws_request & LSR_GWS_LANG) != 0,
                                        (uintptr_t)in->language_feature_precomp % 16 == 0);
        if (w.kind) {
            if (w.rows_bytes) {
                const size_t bytes = (w.rows_bytes + 255) / 256 * 256;
                void* ws = alloc(ctx, bytes, LSR_BUF_GRAD);
                if (!ws) return LSR_ENOMEM;
                out->grad_ws = ws;
                out->grad_ws_bytes = w.rows_bytes;
                ra.zero = (float4*)ws;
                ra.zero_n16 = bytes / 16;
            }
            if (w.lang_bytes) {
                const size_t bytes = (w.lang_bytes + 255) / 256 * 256;
                void* wl = alloc(ctx, bytes, LSR_BUF_GRAD_LANG);
                if (!wl) return LSR_ENOMEM;
                out->grad_ws_lang = wl;
                ra.zero2 = (float4*)wl;
                ra.zero2_n16 = bytes / 16;
            }
            out->grad_ws_kind = w.kind;
            // the backward's per-block candidate lists (render.hip LST): the render
            // writes each 8x8 block's staged candidates; capacity 4 entries per instance
            const size_t L = block_lists_bytes((size_t)M, (size_t)T);
            if (L && L <= ((size_t)g_lists_max_mb.load(std::memory_order_relaxed) << 20)) {
                void* lb = alloc(ctx, L, LSR_BUF_LISTS);
                if (!lb) return LSR_ENOMEM;
                out->lists = lb;
                out->lists_bytes = L;
                set_block_lists(ra, lb, (size_t)M);
            }
        }
    }
    LSR_HIP(join.wait());   // the SH colours of a split preprocess
    { StageScope sc(ST_RENDER, st); LSR_HIP(launch_render_fwd(ra, st)); }
    // the backward's block order from the lists the render just counted
    if (bwd_order_on(T) && ra.lcount) LSR_HIP(launch_bwd_order(ra, (uint4*)(img + IL.border), st));
    LSR_DEBUG_SYNC(s, st, "render");
    LSR_GUARD(guard, "out_color", out->out_color, 3 * NPIX);
    LSR_GUARD(guard, "out_lang", out->out_lang, (size_t)(s->quick_render ? quick_dim(s) : Dd) * NPIX);
    return LSR_OK;
}

static int guard_bwd_outputs(Guard& g, const lsr_inputs* in, const lsr_bwd_out* o, int D)
{
    const size_t P = (size_t)in->P;
    LSR_GUARD(g, "dL_dmeans2D", o->dL_dmeans2D, P * 3);
    LSR_GUARD(g, "dL_dcolors", o->dL_dcolors, P * 3);
    LSR_GUARD(g, "dL_dlang", o->dL_dlang, P * (size_t)D);
    LSR_GUARD(g, "dL_dopacity", o->dL_dopacity, P);
    LSR_GUARD(g, "dL_dmeans3D", o->dL_dmeans3D, P * 3);
    LSR_GUARD(g, "dL_dcov3D", o->dL_dcov3D, P * 6);
    LSR_GUARD(g, "dL_dsh", o->dL_dsh, P * (size_t)in->max_coeffs * 3);
    LSR_GUARD(g, "dL_dscales", o->dL_dscales, P * 3);
    LSR_GUARD(g, "dL_drotations", o->dL_drotations, P * 4);
    LSR_GUARD(g, "dL_dlang_weights", o->dL_dlang_weights, P * (size_t)in->quick_k);
    LSR_GUARD(g, "dL_drgb_sh", o->dL_drgb_sh, P * 3);
    return LSR_OK;
}

static bool geometry_requested(const lsr_bwd_out* o)
{
    return o->dL_dmeans2D || o->dL_dcolors || o->dL_dopacity || o->dL_dmeans3D || o->dL_dcov3D || o->dL_dsh ||
           o->dL_dscales || o->dL_drotations || o->dL_drgb_sh;
}

static int record_lang_ready(const lsr_bwd_out* out, hipStream_t st)
{
    if (out->lang_ready_event) LSR_HIP(hipEventRecord((hipEvent_t)out->lang_ready_event, st));
    return LSR_OK;
}

static int backward_dense(const lsr_settings* s, const lsr_inputs* in, const lsr_bwd_in* b, lsr_bwd_out* out,
                          lsr_alloc_fn alloc, void* ctx, hipStream_t st, Guard& guard);

// Quick (sparse) language input: weights (P,K) + codes (P,K) rendered into
// Dq channels.  dL/dweights[j][m] = sum_p aT_j(p) dL/dout_lang[idx[j][m]][p].
//  - weights alone requested (feature-mode training, geometry frozen): the
//    language-only render backward gathers the channel gradients at the codes
//    (no dense (P,Dq) rows anywhere);
//  - geometry requested too: the quick channels take part in dL/dalpha when
//    their upstream gradient is given, so the sparse rows are expanded to
//    dense (P,Dq) rows and the dense backward runs (Dq <= 64), dL/dweights
//    gathered from its dL/dlang; without an upstream language gradient the
//    backward is the RGB-only one.
static int backward_quick(const lsr_settings* s, const lsr_inputs* in, const lsr_bwd_in* b, lsr_bwd_out* out,
                          lsr_alloc_fn alloc, void* ctx, hipStream_t st, Guard& guard)
{
    const int P = in->P;
    const int Dq = quick_dim(s);
    float* dw = out->dL_dlang_weights;
    const bool geom = geometry_requested(out);
    if (!dw && !geom) return record_lang_ready(out, st);
    if (dw && !geom && !b->dL_dout_lang) {
        // the weights requested but the language output received no gradient
        // (autograd passes none when the loss ignores it): dL/dweights = 0
        LSR_HIP(hipMemsetAsync(dw, 0, (size_t)P * in->quick_k * 4, st));
        return record_lang_ready(out, st);
    }
    // (deterministic mode: the expansion path below, whose dense language-only
    // backward sums in fixed point; the sparse gather adds floats in any order)
    if (dw && !geom && !g_det.load(std::memory_order_relaxed)) {
        if (lang_set_for(Dq) < 0) return LSR_EUNSUPPORTED;
        const Cam c = make_cam(s);
        RenderBwdArgs rb;
        rb.f = make_render_args(s, in, c, (const uint8_t*)b->geom, (const uint8_t*)b->binning,
                                (const uint8_t*)b->image, b->num_rendered);
        rb.f.D = Dq;
        rb.f.lang = nullptr;
        rb.dout_color = b->dL_dout_color;
        rb.dout_lang = b->dL_dout_lang;
        rb.grad_acc = nullptr;
        rb.VP = Dq;
        rb.qw_acc = dw;
        { StageScope sc(ST_GZERO, st); LSR_HIP(hipMemsetAsync(dw, 0, (size_t)P * in->quick_k * 4, st)); }
        { StageScope sc(ST_RENDER_BWD, st); LSR_HIP(launch_render_bwd_lang_sparse(rb, st)); }
        LSR_DEBUG_SYNC(s, st, "render_bwd_lang_sparse");
        int rc = record_lang_ready(out, st);
        if (rc != LSR_OK) return rc;
        return guard_bwd_outputs(guard, in, out, 0);
    }
    lsr_settings s2 = *s;
    s2.quick_render = 0;
    s2.quick_dim = 0;
    lsr_inputs in2 = *in;
    in2.quick_k = 0;
    in2.language_feature_weights_quick = nullptr;
    in2.language_feature_indices = nullptr;
    lsr_bwd_out o2 = *out;
    o2.dL_dlang_weights = nullptr;
    o2.lang_ready_event = nullptr;
    lsr_bwd_in b2 = *b;
    float* dense_grad = nullptr;
    if (b->dL_dout_lang) {
        if (lang_set_for(Dq) < 0) return LSR_EUNSUPPORTED;
        const size_t row = (size_t)P * Dq * 4;
        uint8_t* ws = (uint8_t*)alloc(ctx, align256(row) + (dw ? row : 0), LSR_BUF_SPARSE);
        if (!ws) return LSR_ENOMEM;
        float* dense = (float*)ws;
        dense_grad = dw ? (float*)(ws + align256(row)) : nullptr;
        LSR_HIP(launch_sparse_expand(in->language_feature_weights_quick, in->language_feature_indices,
                                     in->quick_index_dtype, P, in->quick_k, Dq, dense, st));
        s2.include_feature = 1;
        in2.lang_dim = Dq;
        in2.language_feature_precomp = dense;
        o2.dL_dlang = dense_grad;
    } else {
        s2.include_feature = 0;
        in2.lang_dim = 0;
        in2.language_feature_precomp = nullptr;
        o2.dL_dlang = nullptr;
        b2.dL_dout_lang = nullptr;
        if (dw) LSR_HIP(hipMemsetAsync(dw, 0, (size_t)P * in->quick_k * 4, st));
    }
    // the dense backward shares this call's guard (its flag word stays owned by one Guard)
    int rc = backward_dense(&s2, &in2, &b2, &o2, alloc, ctx, st, guard);
    if (rc != LSR_OK) return rc;
    if (dw && dense_grad)
        LSR_HIP(launch_sparse_gather(dense_grad, in->language_feature_indices, in->quick_index_dtype, P, in->quick_k,
                                     Dq, dw, st));
    rc = record_lang_ready(out, st);
    if (rc != LSR_OK) return rc;
    return guard_bwd_outputs(guard, in, out, 0);
}

int lsr_backward(const lsr_settings* s, const lsr_inputs* in, const lsr_bwd_in* b, lsr_bwd_out* out,
                 lsr_alloc_fn alloc, void* ctx, void* stream)
{
    int rc = validate(s, in);
    if (rc != LSR_OK) return rc;
    if (!b || !out || !alloc || !b->geom || !b->image || !b->binning || !b->dL_dout_color) return LSR_EINVAL;
    const int Dd = dense_dim(s, in);
    if (Dd > 0 && !b->dL_dout_lang) return LSR_EINVAL;
    if (out->dL_dlang_weights && !s->quick_render) return LSR_EINVAL;
    if (s->quick_render && out->dL_dlang) return LSR_EINVAL;   // the quick input has no dense rows
    if (in->P == 0) return LSR_OK;
    if (!b->radii) return LSR_EINVAL;
    hipStream_t st = (hipStream_t)stream;
    const Cam c = make_cam(s);
    const int P = in->P;
    const size_t NPIX = (size_t)c.W * c.H;
    Guard guard(s, alloc, ctx, st);
    LSR_GUARD(guard, "dL_dout_color", b->dL_dout_color, 3 * NPIX);
    LSR_GUARD(guard, "dL_dout_lang", b->dL_dout_lang, (size_t)(s->quick_render ? quick_dim(s) : Dd) * NPIX);
    if (s->debug) {   // the saved lists the render backward gathers through
        const RenderArgs la = make_render_args(s, in, c, (const uint8_t*)b->geom, (const uint8_t*)b->binning,
                                               (const uint8_t*)b->image, b->num_rendered);
        const int lrc = guard.check_lists("render_bwd", la.point_list, (size_t)b->num_rendered, P, la.tile_start,
                                          (size_t)c.gx * c.gy);
        if (lrc != LSR_OK) return lrc;
    }
    if (s->quick_render) return backward_quick(s, in, b, out, alloc, ctx, st, guard);
    return backward_dense(s, in, b, out, alloc, ctx, st, guard);
}

// LSR_OPT_DETERMINISTIC: the bounds word ({max |dL/dout|, max |feature|,
// flags}) and the zeroed 64-bit fixed-point twins of the accumulators the
// render backward adds into (rb.grad_acc's (P, VP) rows, and with lang_direct
// the (P, D) language rows); rb.radii = the forward's radii.
static int det_prepare(RenderBwdArgs& rb, const int32_t* radii, bool lang_direct, lsr_alloc_fn alloc, void* ctx,
                       hipStream_t st)
{
    rb.radii = radii;
    const size_t P = (size_t)rb.f.P;
    const size_t rows = align256(P * (size_t)rb.VP * 8);
    const size_t lang = lang_direct ? align256(P * (size_t)rb.f.D * 8) : 0;
    const size_t hdr = LSR_DET_HDR + align256(P * 4);   // + the shift table
    uint8_t* ws = (uint8_t*)alloc(ctx, hdr + rows + lang, LSR_BUF_DET);
    if (!ws) return LSR_ENOMEM;
    rb.det_bounds = (float*)ws;
    rb.det_sh = (uint32_t*)(ws + LSR_DET_HDR);
    rb.det_rows = (long long*)(ws + hdr);
    rb.det_lang = lang_direct ? (long long*)(ws + hdr + rows) : nullptr;
    {
        // the header and the shift table are written whole by launch_det_bounds
        StageScope sc(ST_DET_BOUNDS, st);
        LSR_HIP(launch_det_bounds(rb, rb.det_bounds, st));
    }
    // after the bounds pass: its reads would otherwise pay for writing the
    // cleared lines back from the last-level cache (bounds 0.094 -> 0.079 ms)
    StageScope sc(ST_GZERO, st);
    LSR_HIP(hipMemsetAsync(ws + hdr, 0, rows + lang, st));
    return LSR_OK;
}

// The dense-input backward (lsr_backward's body past validation; also the
// geometry path of the quick input, with that call's guard).
static int backward_dense(const lsr_settings* s, const lsr_inputs* in, const lsr_bwd_in* b, lsr_bwd_out* out,
                          lsr_alloc_fn alloc, void* ctx, hipStream_t st, Guard& guard)
{
    int rc = LSR_OK;
    const Cam c = make_cam(s);
    const int P = in->P;
    const int Dd = dense_dim(s, in);
    if (Dd > 0 && !b->dL_dout_lang) return LSR_EINVAL;
    // Only dL/dlanguage requested (feature-mode training with frozen geometry
    // and no means2D gradient): the language-only render backward writes the
    // output directly; no gradient rows, no preprocess backward.
    const bool lang_only = Dd > 0 && out->dL_dlang && !geometry_requested(out);
    // the forward's zeroed accumulators, when they are exactly what this call needs
    const GradWs W = grad_ws_layout(P, Dd, geometry_requested(out), out->dL_dlang != nullptr,
                                    (uintptr_t)in->language_feature_precomp % 16 == 0);
    const bool ws_kind = W.kind != 0 && b->grad_ws_kind == W.kind;
    const bool ws_ok = ws_kind && W.rows_bytes > 0 && b->grad_ws && b->grad_ws_bytes >= W.rows_bytes;
    const bool ws_lang = ws_kind && W.lang_bytes > 0 && b->grad_ws_lang && out->dL_dlang == (float*)b->grad_ws_lang;
    const bool det = g_det.load(std::memory_order_relaxed) != 0;
    if (lang_only) {
        RenderBwdArgs rb;
        rb.f = make_render_args(s, in, c, (const uint8_t*)b->geom, (const uint8_t*)b->binning,
                                (const uint8_t*)b->image, b->num_rendered);
        if (b->lists) set_block_lists_bwd(rb.f, b->lists, b->image, (size_t)b->num_rendered);
        rb.f.qw = nullptr;
        rb.f.D = Dd;
        rb.f.lang = in->language_feature_precomp;
        rb.dout_color = b->dL_dout_color;
        rb.dout_lang = b->dL_dout_lang;
        rb.grad_acc = out->dL_dlang;
        rb.VP = Dd;
        if (det) {
            rc = det_prepare(rb, b->radii, false, alloc, ctx, st);
            if (rc != LSR_OK) return rc;
        } else if (!ws_lang) {
            StageScope sc(ST_GZERO, st);
            LSR_HIP(hipMemsetAsync(out->dL_dlang, 0, (size_t)P * Dd * 4, st));
        }
        { StageScope sc(ST_RENDER_BWD, st); LSR_HIP(launch_render_bwd_lang(rb, st)); }
        if (det) { StageScope sc(ST_DET_FINISH, st); LSR_HIP(launch_det_finish(rb, true, nullptr, out->dL_dlang, st)); }
        LSR_DEBUG_SYNC(s, st, "render_bwd_lang");
        rc = record_lang_ready(out, st);
        if (rc != LSR_OK) return rc;
        return guard_bwd_outputs(guard, in, out, Dd);
    }
    // D = 16 / 32 with dL/dlang requested: the render backward adds the
    // language gradients straight into the output; the rows keep geometry +
    // colour (one 64-B line) and preprocess_bwd no longer copies language
    // (and 16-B aligned language rows: the kernel gathers them as float4 lines)
    const bool lang_direct = Dd > 0 && out->dL_dlang && bwd_lang_direct(Dd) &&
                             (uintptr_t)in->language_feature_precomp % 16 == 0;
    const int VP = lang_direct ? 16 : grad_row_width(Dd);
    float* gacc = ws_ok ? (float*)b->grad_ws : (float*)alloc(ctx, (size_t)P * VP * 4, LSR_BUF_GRAD);
    if (!gacc) return LSR_ENOMEM;
    // (deterministic: k_det_finish writes every element of gacc and dL/dlang)
    if (!det && (!ws_ok || (lang_direct && !ws_lang))) {
        StageScope sc(ST_GZERO, st);
        if (!ws_ok) LSR_HIP(hipMemsetAsync(gacc, 0, (size_t)P * VP * 4, st));
        if (lang_direct && !ws_lang) LSR_HIP(hipMemsetAsync(out->dL_dlang, 0, (size_t)P * Dd * 4, st));
    }

    RenderBwdArgs rb;
    rb.f = make_render_args(s, in, c, (const uint8_t*)b->geom, (const uint8_t*)b->binning, (const uint8_t*)b->image,
                            b->num_rendered);
    if (b->lists) set_block_lists_bwd(rb.f, b->lists, b->image, (size_t)b->num_rendered);
    rb.f.qw = nullptr;
    rb.f.D = Dd;
    rb.f.lang = Dd ? in->language_feature_precomp : nullptr;
    rb.dout_color = b->dL_dout_color;
    rb.dout_lang = Dd ? b->dL_dout_lang : nullptr;
    rb.grad_acc = gacc;
    rb.VP = VP;
    rb.lang_acc = lang_direct ? out->dL_dlang : nullptr;
    if (det) {
        rc = det_prepare(rb, b->radii, lang_direct, alloc, ctx, st);
        if (rc != LSR_OK) return rc;
    }
    { StageScope sc(ST_RENDER_BWD, st); LSR_HIP(launch_render_bwd(rb, st)); }
    if (det) {
        StageScope sc(ST_DET_FINISH, st);
        LSR_HIP(launch_det_finish(rb, false, gacc, lang_direct ? out->dL_dlang : nullptr, st));
    }
    LSR_DEBUG_SYNC(s, st, "render_bwd");
    // the language gradient is final here unless preprocess_bwd copies it out
    if (lang_direct || !out->dL_dlang) {
        rc = record_lang_ready(out, st);
        if (rc != LSR_OK) return rc;
    }

    lsr_inputs in2 = *in;
    in2.lang_dim = Dd;
    lsr_bwd_out o2 = *out;
    if (!Dd || lang_direct) o2.dL_dlang = nullptr;
    { StageScope sc(ST_PRE_BWD, st); LSR_HIP(launch_preprocess_bwd(c, in2, (const uint8_t*)b->geom, b->radii, gacc, VP, o2, st)); }
    LSR_DEBUG_SYNC(s, st, "preprocess_bwd");
    if (!(lang_direct || !out->dL_dlang)) {
        rc = record_lang_ready(out, st);
        if (rc != LSR_OK) return rc;
    }
    return guard_bwd_outputs(guard, in, out, Dd);
}

int lsr_mark_visible(int P, const float* means3D, const float* viewmatrix, const float* projmatrix, uint8_t* present,
                     void* stream)
{
    (void)projmatrix;
    if (P < 0 || (P > 0 && (!means3D || !viewmatrix || !present))) return LSR_EINVAL;
    LSR_HIP(launch_mark_visible(P, means3D, viewmatrix, present, (hipStream_t)stream));
    return LSR_OK;
}

}  // extern "C"
