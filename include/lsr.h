/*
 * lsr.h — C ABI of the MI355X-native language-Gaussian tile rasterizer
 * (liblsr.so, hand-written HIP for gfx950).
 *
 * This is the drop-in boundary under the reference's operator surface
 * `diff_gaussian_rasterization` (imported at gaussian_renderer/__init__.py:15,
 * constructed :37-54, called :108-119).  Each entry point replaces one
 * binding of the reference's (absent) torch extension `_C`
 * (submodules/efficient-langsplat-rasterization, .gitmodules:1-3):
 *
 *   lsr_forward      <- _C.rasterize_gaussians           (forward of
 *                       GaussianRasterizer.__call__, gaussian_renderer/__init__.py:108-119)
 *   lsr_backward     <- _C.rasterize_gaussians_backward  (autograd backward,
 *                       reached from loss.backward() at train.py:173)
 *   lsr_mark_visible <- _C.mark_visible                  (GaussianRasterizer.markVisible)
 *   lsr_strerror     <- the RuntimeError text the binding raises
 *
 * Conventions
 *  - All tensor pointers are DEVICE pointers to contiguous fp32 (int32 for
 *    radii) arrays with the shapes documented per field; optional inputs are
 *    NULL.  N = number of Gaussians, H×W image, D dense language channels,
 *    K quick entries per Gaussian, Dq quick output channels.
 *  - Matrices are the reference's `world_view_transform` /
 *    `full_proj_transform` tensors as stored (row-major transposed, i.e.
 *    column-major math matrices; scene/cameras.py:55-57).
 *  - The library never allocates device memory itself: workspaces are
 *    requested through `alloc(ctx, bytes, which)` (torch's caching allocator
 *    on the Python side) and returned in the out struct so the caller can
 *    keep them for backward (the upstream geomBuffer/binningBuffer/imgBuffer
 *    pattern).  Returned pointers must be 256-byte aligned.
 *  - All work is enqueued on `stream` (a hipStream_t).  lsr_forward performs
 *    exactly one host synchronisation (the num_rendered read-back that sizes
 *    the binning workspace).
 *  - Return value 0 = success; otherwise an LSR_E* code (lsr_strerror).
 */
#ifndef LSR_H
#define LSR_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LSR_ABI_VERSION 12  /* 12 (r06): LSR_OPT_DETERMINISTIC;
                               11 (r05): LSR_INDEX_PACKED, lsr_quick_pack_codes, LSR_OPT_SPLIT_PREPROCESS;
                               10 (r05): lsr_settings.quick_layout, lsr_quick_decode_run weight_layout;
                               9 (r05): LSR_OPT_LISTS_MAX_MB; LSR_BIN_ORDERED removed */

enum {
    LSR_OK = 0,
    LSR_EINVAL = 1,        /* invalid argument / shape / missing input */
    LSR_EUNSUPPORTED = 2,  /* e.g. language dim beyond the compiled channel sets */
    LSR_EHIP = 3,          /* HIP launch / runtime failure */
    LSR_ENOMEM = 4,        /* alloc callback returned NULL */
    LSR_EOVERFLOW = 5,     /* num_rendered does not fit 32-bit instance indices */
    LSR_ENONFINITE = 6,    /* debug guard: NaN/Inf in an input or output */
    LSR_ELISTS = 7         /* debug check: corrupt binning lists (id >= P, tile ranges not monotone) */
};

/* GaussianRasterizationSettings (gaussian_renderer/__init__.py:37-52),
 * field for field, plus the optional trailing quick_dim (u4). */
typedef struct lsr_settings {
    int image_height;
    int image_width;
    float tanfovx;
    float tanfovy;
    const float* bg;          /* (3,) device */
    float scale_modifier;
    const float* viewmatrix;  /* (4,4) device */
    const float* projmatrix;  /* (4,4) device */
    int sh_degree;            /* active SH degree (0..3) */
    const float* campos;      /* (3,) device */
    int prefiltered;
    int debug;                /* sync + check after every stage */
    int include_feature;      /* dense language channels on */
    int quick_render;         /* sparse (weights, indices) language channels on */
    int quick_dim;            /* Dq; 0 selects the reference default 192 */
    int quick_layout;         /* LSR_LAYOUT_CHW (0, the reference's (Dq,H,W)) or LSR_LAYOUT_HWC:
                                 out_lang is written pixel-major, (H,W,Dq) — every pixel's Dq
                                 weights in one 768-B row at Dq = 192 (the quick_render kernel
                                 with K = 12, Dq = 192 only; else LSR_EUNSUPPORTED) */
} lsr_settings;

enum { LSR_LAYOUT_CHW = 0, LSR_LAYOUT_HWC = 1 };

/* Code-index dtypes of language_feature_indices.  LSR_INDEX_PACKED: an (N, 4)
 * uint32 array written by lsr_quick_pack_codes (K = 12 codes per Gaussian as
 * bytes code + 1, 0 = no code, 16-B rows): what the quick render stages per
 * candidate, so a caller rendering many views of one model converts the
 * reference's fp32 indices once instead of every frame.  Forward and backward
 * of quick_render with K = 12, Dq <= 192 and 16-B aligned weights / indices
 * only (else LSR_EUNSUPPORTED); bytes above Dq are dropped as out-of-range
 * codes are. */
enum { LSR_INDEX_F32 = 0, LSR_INDEX_I32 = 1, LSR_INDEX_I64 = 2, LSR_INDEX_PACKED = 3 };

/* GaussianRasterizer.forward kwargs (gaussian_renderer/__init__.py:108-119). */
typedef struct lsr_inputs {
    int P;                          /* N */
    int max_coeffs;                 /* shs.shape[1] (16 at degree 3) */
    int lang_dim;                   /* D = language_feature_precomp.shape[1] */
    int quick_k;                    /* K = language_feature_weights_quick.shape[1] */
    int quick_index_dtype;          /* LSR_INDEX_* of language_feature_indices */
    const float* means3D;           /* (N,3) */
    const float* shs;               /* (N,M,3) or NULL */
    const float* colors_precomp;    /* (N,3) or NULL (exactly one of shs/colors) */
    const float* opacities;         /* (N,1) */
    const float* scales;            /* (N,3) or NULL */
    const float* rotations;         /* (N,4) wxyz or NULL (normalised by caller) */
    const float* cov3D_precomp;     /* (N,6) or NULL (exactly one of scale+rot/cov) */
    const float* language_feature_precomp;       /* (N,D) or NULL */
    const float* language_feature_weights_quick; /* (N,K) or NULL */
    const void* language_feature_indices;        /* (N,K) or NULL */
} lsr_inputs;

/* Workspace allocator.  lsr_forward may request LSR_BUF_BINNING twice in
 * one call: a speculative buffer sized from the previous call's M (taken
 * while the GPU is still counting) and, only if M outgrew it, a second one;
 * the last pointer returned for a kind is the one the call uses. */
typedef void* (*lsr_alloc_fn)(void* ctx, size_t bytes, int which);
enum { LSR_BUF_GEOM = 0, LSR_BUF_BINNING = 1, LSR_BUF_IMAGE = 2, LSR_BUF_GRAD = 3, LSR_BUF_DECODE = 4,
       LSR_BUF_KNN = 5, LSR_BUF_LOSS = 6, LSR_BUF_GUARD = 7, LSR_BUF_SPARSE = 8, LSR_BUF_GRAD_LANG = 9,
       LSR_BUF_LISTS = 10, LSR_BUF_DET = 11 /* LSR_OPT_DETERMINISTIC: bounds + fixed-point accumulators */ };

typedef struct lsr_fwd_out {
    float* out_color;     /* (3,H,W)  caller-allocated */
    float* out_lang;      /* (Dout,H,W) caller-allocated, Dout = D (dense), Dq (quick) or 0 */
    int32_t* radii;       /* (N,) caller-allocated */
    /* filled by lsr_forward: */
    void* geom;    size_t geom_bytes;
    void* binning; size_t binning_bytes;   /* capacity (>= layout for num_rendered) */
    void* image;   size_t image_bytes;
    int64_t num_rendered;
    /* Optional: the backward's accumulators, prepared by the forward.  In:
     * grad_ws_request = LSR_GWS_GEOM (the backward will request geometry /
     * colour gradients) | LSR_GWS_LANG (it will request dL_dlang).  The
     * forward then allocates them and zeroes them inside the render kernel
     * instead of the backward clearing them with memsets; out: grad_ws /
     * grad_ws_bytes (the gradient rows, LSR_BUF_GRAD; NULL when only dL/dlang
     * is requested), grad_ws_lang (an (N,D) dL/dlang accumulator in its OWN
     * allocation, LSR_BUF_GRAD_LANG, so the gradient returned from it keeps
     * nothing else alive; NULL: none) and grad_ws_kind.
     * Dense language path only (quick_render: nothing prepared). */
    int grad_ws_request;
    int grad_ws_kind;
    void* grad_ws; size_t grad_ws_bytes; void* grad_ws_lang;
    /* With grad_ws_request set (dense path), also: each 8x8 block's candidate
     * list for the backward (LSR_BUF_LISTS; NULL when not prepared), written by
     * the render: pass it in lsr_bwd_in.lists to let the backward read its
     * candidates instead of re-staging them from the tile lists. */
    void* lists; size_t lists_bytes;
} lsr_fwd_out;
enum { LSR_GWS_GEOM = 1, LSR_GWS_LANG = 2 };

/* _C.rasterize_gaussians: preprocess → binning (tile buckets + per-tile depth
 * sort) → per-pixel alpha blend of RGB + language channels.  With
 * settings.debug set, inputs and outputs are also scanned for NaN/Inf
 * (LSR_ENONFINITE). */
int lsr_forward(const lsr_settings* s, const lsr_inputs* in, lsr_fwd_out* out,
                lsr_alloc_fn alloc, void* alloc_ctx, void* stream);

typedef struct lsr_bwd_in {
    const void* geom;
    const void* binning;
    const void* image;
    int64_t num_rendered;
    const int32_t* radii;           /* (N,) from forward */
    const float* dL_dout_color;     /* (3,H,W) */
    const float* dL_dout_lang;      /* (D,H,W) or NULL */
    /* Optional: lsr_fwd_out.grad_ws / _bytes / _kind / _lang of the same
     * forward (zeroed accumulators; hand them to ONE backward).  Used when the
     * kind matches what this call's requested outputs need (otherwise the call
     * allocates and clears its own); dL_dlang == grad_ws_lang then needs no
     * clearing either. */
    void* grad_ws; size_t grad_ws_bytes; int grad_ws_kind;
    void* grad_ws_lang;
    /* Optional: lsr_fwd_out.lists of the same forward (read only; any number of
     * backwards over that forward may use it). */
    const void* lists;
} lsr_bwd_in;

/* Gradient outputs; NULL = not requested (needs_input_grad False).  Every
 * non-NULL array is fully written (no pre-zeroing needed). */
typedef struct lsr_bwd_out {
    float* dL_dmeans2D;     /* (N,3): [:, :2] = dL/d(NDC xy), [:, 2] = 0 */
    float* dL_dcolors;      /* (N,3): dL/dcolors_precomp */
    float* dL_dlang;        /* (N,D): dL/dlanguage_feature_precomp */
    float* dL_dopacity;     /* (N,1) */
    float* dL_dmeans3D;     /* (N,3) */
    float* dL_dcov3D;       /* (N,6) */
    float* dL_dsh;          /* (N,M,3) */
    float* dL_dscales;      /* (N,3) */
    float* dL_drotations;   /* (N,4) */
    /* Quick (sparse) language input with a gradient: with
     * quick_render set, dL/dlanguage_feature_weights_quick (N,K),
     *   dL/dw[j][m] = sum_p alpha_j(p) T_j(p) dL/dout_lang[idx[j][m]][p];
     * the indices are not differentiable. */
    float* dL_dlang_weights;
    /* Optional hipEvent_t, recorded on `stream` as soon as dL_dlang /
     * dL_dlang_weights are final (before the preprocess backward), so a
     * data-parallel caller can start their all-reduce early (§8e). */
    void* lang_ready_event;
    /* View-factored SH gradient (multi-GPU exchange): when set,
     * (N,3) receives the SH evaluation's colour gradient dL/dRGB of each
     * Gaussian (0 where the SH colour was clamped, 0 for Gaussians outside the
     * view).  dL/dsh of this view is basis(dir) (x) that vector, so a
     * data-parallel caller exchanges these 3 floats (plus the camera centre)
     * instead of the 3*M of dL_dsh and rebuilds the summed SH gradient with
     * lsr_sh_grad_from_views.  dL_dsh may then be NULL. */
    float* dL_drgb_sh;
} lsr_bwd_out;

/* _C.rasterize_gaussians_backward.  With settings.debug set, every stage is
 * synchronised and checked, and inputs / outputs are scanned for NaN/Inf
 * (LSR_ENONFINITE; the offending array is named on stderr). */
int lsr_backward(const lsr_settings* s, const lsr_inputs* in, const lsr_bwd_in* b,
                 lsr_bwd_out* out, lsr_alloc_fn alloc, void* alloc_ctx, void* stream);

/* Sum over R views of the SH coefficient gradient, from each view's
 * dL_drgb_sh (lsr_bwd_out): dL_dsh[i][k][c] = sum_r basis_k(dir_ri) *
 * drgb[r][i][c] with dir_ri = normalize(means3D[i] - campos[r]) and the basis
 * of the forward's SH evaluation at `sh_degree` (coefficients above it get 0).
 * Views are summed in order r = 0..R-1, so every rank computes identical
 * values.  means3D (N,3), campos (R,3), drgb (R,N,3), dL_dsh (N,M,3): device
 * pointers; M = max SH coefficients per Gaussian (<= 16). */
int lsr_sh_grad_from_views(int64_t N, int M, int sh_degree, const float* means3D, int R, const float* campos,
                           const float* drgb, float* dL_dsh, void* stream);

/* _C.mark_visible: present[i] = (view-space z of means3D[i]) > 0.2. */
int lsr_mark_visible(int P, const float* means3D, const float* viewmatrix,
                     const float* projmatrix, uint8_t* present, void* stream);

/* Codebook decode of a rendered language weight map;
 * replaces, after render(), the reference's
 *   F = einsum('ldk,lkn->ldn', codebooks.permute(0,2,1), W.view(L, K, H*W))
 *   F = F / (F.norm(dim=1, keepdim=True) + eps)
 * of render_language_feature_map_quick (eval_lerf.py:210-220,
 * backend_renderer.py:16-36); with L = 1 and normalize = 0 it is
 * compute_final_feature_map (scene/gaussian_model.py:545-550).
 * weight_map (L*K, H, W), codebooks (L, K, Df), out (L, Df, H, W), all fp32
 * device pointers.  K must be 64 and Df a multiple of 16. */
int lsr_quick_decode(const float* weight_map, const float* codebooks, int L, int K, int Df, int H, int W,
                     int normalize, float eps, float* out, lsr_alloc_fn alloc, void* alloc_ctx, void* stream);

/* The same decode in two steps for many frames with fixed codebooks (the
 * eval loops of eval_lerf.py decode every view with one model's codebooks):
 * lsr_quick_decode_prepare writes the codebook-only part (fragments, norm
 * factor) into a caller-owned device buffer of lsr_quick_decode_plan_bytes
 * bytes (0 = unsupported shape); lsr_quick_decode_run decodes a frame with it.
 * The plan is valid until the codebooks change.  weight_layout: LSR_LAYOUT_CHW
 * for an (L*K, H, W) weight map, LSR_LAYOUT_HWC for a pixel-major (H, W, L*K)
 * one (lsr_settings.quick_layout); the output is (L, Df, H, W) either way. */
/* The packed code rows (LSR_INDEX_PACKED) of K = 12 code indices per Gaussian:
 * indices (N, 12) of LSR_INDEX_F32 / I32 / I64 index_dtype (fp32 values round
 * half up, u5), packed (N, 4) uint32, 16-B aligned: byte m of row i holds
 * code m + 1 when 0 <= code < quick_dim (0 selects 192), else 0. */
int lsr_quick_pack_codes(const void* indices, int index_dtype, int64_t N, int K, int quick_dim, uint32_t* packed,
                         void* stream);

size_t lsr_quick_decode_plan_bytes(int L, int K, int Df, int normalize);
int lsr_quick_decode_prepare(const float* codebooks, int L, int K, int Df, int normalize, void* plan, void* stream);
int lsr_quick_decode_run(const float* weight_map, int weight_layout, const void* plan, int L, int K, int Df, int H,
                         int W, int normalize, float eps, float* out, void* stream);

/* Fused top-k soft codes (replaces softmax_to_topk_soft_code,
 * utils/vq_utils.py:9-24; get_weights_and_indices, :26-40; the per-level
 * loop of GaussianModel.get_render_weights, scene/gaussian_model.py:510-518;
 * and the level-offset concatenation of eval_lerf.py:340-348).
 * logits (N, L*K) fp32: L levels of K-way codes; K in {64,128,192,256},
 * 1 <= k <= K.  Outputs (any may be NULL, at least one not):
 *   dense      (N, L*K) fp32: y*mask / (sum(y*mask) + 1e-10) per level;
 *   sparse_w   (N, L*k) fp32: the k non-zeros of each level in ascending
 *              channel order;
 *   sparse_idx (N, L*k) of LSR_INDEX_* idx_dtype: their channel indices,
 *              + l*K for level l when level_offset != 0.
 * Top-k ties go to the lower channel (torch.topk's tie order is
 * implementation-defined). */
int lsr_topk_code_forward(const float* logits, int64_t N, int L, int K, int k, float* dense, float* sparse_w,
                          void* sparse_idx, int idx_dtype, int level_offset, void* stream);
/* dL/dlogits (N, L*K) from dL/ddense (N, L*K): the autograd chain of
 * softmax_to_topk_soft_code (mask recomputed from the logits). */
int lsr_topk_code_backward(const float* logits, const float* grad_dense, int64_t N, int L, int K, int k,
                           float* grad_logits, void* stream);
/* dL/dlogits (N, L*K) from dL/dsparse_w (N, L*k): the gradient of the packed
 * weights (ascending channel order, as lsr_topk_code_forward's sparse_w),
 * e.g. lsr_bwd_out.dL_dlang_weights of a quick-mode render; the dense code
 * gradient is never formed (the sparse training path). */
int lsr_topk_code_backward_sparse(const float* logits, const float* grad_weights, int64_t N, int L, int K, int k,
                                  float* grad_logits, void* stream);

/* Language-feature cosine loss of the feature-mode training step (SURVEY
 * §8f rank 4; train.py:151-164 with vq_layer_num = 1, layer_idx = 0):
 *   f[:, p]  = codebooks[0]^T w_p        compute_layer_feature_map,
 *                                        scene/gaussian_model.py:533-543
 *   gt[:, p] = features[seg[p]], mask[p] = seg[p] != -1
 *                                        get_language_feature, scene/cameras.py:59-96
 *   loss     = 1 - mean_p cos(f_p*mask_p, gt_p*mask_p)   cos_loss,
 *                                        utils/loss_utils.py:24-25 (eps 1e-8)
 * weight_map (K, H, W), codebooks (K, Df), features (S, Df) fp32; seg (H, W)
 * int32 segment ids, -1 (or any id outside [0, S)) = masked.  K must be 64,
 * Df a multiple of 16.  Nothing of size Df x pixels is materialised
 * (everything factors through the K-dim code space).  Forward writes loss[0]
 * and/or pixel_stats (2, H, W) (|f_p| and f_p.gt_p; either may be NULL).
 * Backward writes grad_weight_map (K, H, W) and grad_codebooks (K, Df), both
 * scaled by the device scalar *grad_loss, from the forward's pixel_stats
 * (NULL: recomputed).  Workspace via alloc (LSR_BUF_LOSS). */
int lsr_lang_loss_forward(const float* weight_map, const float* codebooks, int K, int Df, int H, int W,
                          const int32_t* seg, const float* features, int S, float* loss, float* pixel_stats,
                          lsr_alloc_fn alloc, void* alloc_ctx, void* stream);
int lsr_lang_loss_backward(const float* weight_map, const float* codebooks, int K, int Df, int H, int W,
                           const int32_t* seg, const float* features, int S, const float* pixel_stats,
                           const float* grad_loss, float* grad_weight_map, float* grad_codebooks, lsr_alloc_fn alloc,
                           void* alloc_ctx, void* stream);

/* Fused Adam step: the update of torch.optim.Adam as the
 * reference builds it (scene/gaussian_model.py:234-255, no amsgrad), one pass
 * over n fp32 elements of params / grads / exp_avg / exp_avg_sq (device
 * pointers, same layout).  step is the 1-based step count after increment;
 * the scalars are doubles (Python floats) and the bias corrections are
 * formed in double on the host, as torch does. */
int lsr_adam_step(float* params, const float* grads, float* exp_avg, float* exp_avg_sq, int64_t n, double lr,
                  double beta1, double beta2, double eps, double weight_decay, int64_t step, void* stream);

/* simple_knn._C.distCUDA2 (scene/gaussian_model.py:20,194): for points
 * (N, 3) fp32, out[i] = mean of the three smallest squared distances
 * dx*dx + dy*dy + dz*dz to points j != i (exact; FLT_MAX for missing
 * neighbours when N < 4).  Workspace (~40 B/point) via alloc. */
int lsr_knn_dist2(const float* points, int64_t N, float* out, lsr_alloc_fn alloc, void* alloc_ctx, void* stream);

const char* lsr_strerror(int code);
int lsr_abi_version(void);

/* Process-wide options.  LSR_OPT_BIN_MODE picks the forward's tile binning:
 * LSR_BIN_SORTED_TILES (= LSR_BIN_AUTO, the default) scatters (depth, id) keys
 * into the tile buckets and sorts each bucket.  (ABI <= 8's LSR_BIN_ORDERED, a
 * depth-ordered mode measured slower at every size, is no longer built: the
 * value is rejected with LSR_EINVAL.)  LSR_OPT_LISTS_MAX_MB (default 2048): a
 * forward with a backward pending writes the backward's per-block candidate
 * lists (128 B per tile instance) only while they fit this many MiB; above it
 * the backward re-stages from the tile lists (identical results).  LSR_EINVAL
 * for an unknown option/value. */
#define LSR_OPT_BIN_MODE 1
#define LSR_OPT_LISTS_MAX_MB 2
/* LSR_OPT_SPLIT_PREPROCESS (default 1): a forward with SH colours of at least
 * 2^19 Gaussians evaluates the SH colour on a library-owned second stream
 * of the current device, concurrent with the tile binning (the geometry the
 * binning needs stays on the caller's stream, and the render waits for both);
 * 0: one fused preprocess kernel on the caller's stream.  Results identical. */
#define LSR_OPT_SPLIT_PREPROCESS 3
/* LSR_OPT_DETERMINISTIC (default 0): 1 makes lsr_backward bit-reproducible.
 * The render backward's cross-block sums (every per-Gaussian gradient is a sum
 * of per-8x8-block partials, added by atomics in whatever order the blocks
 * finish) are accumulated as 64-bit fixed-point integers, whose addition is
 * associative: one binary exponent per (Gaussian, gradient column) chosen from
 * an a-priori bound (the launch's max |dL/dout| and max |feature|, the
 * Gaussian's radius, the image size), so the sum cannot overflow, and each
 * block partial is rounded once to 2^-s (s is 30-60 bits below the bound).
 * Two backwards of the same inputs give identical bits.  A non-finite input or
 * term turns every gradient of that call into NaN (never a silently wrong
 * value).  Costs one bound pass, a zeroed 8-B-per-value accumulator, 64-bit
 * atomics (twice the atomic bytes) and one conversion pass. */
#define LSR_OPT_DETERMINISTIC 4
#define LSR_BIN_AUTO 0
#define LSR_BIN_SORTED_TILES 1
#define LSR_BIN_ORDERED 2
int lsr_set_option(int option, int64_t value);
int lsr_get_option(int option, int64_t* value);

/* A non-blocking HIP stream on the current device (no implicit
 * synchronisation with the legacy default stream), created with the HIP
 * runtime this library uses; for callers that overlap renders across streams
 * (langsplatv2_amd.view_stream).  lsr_stream_destroy releases it. */
int lsr_stream_create(void** stream);
int lsr_stream_destroy(void* stream);

/* Dense language channel sets compiled into this build (ascending; D is
 * rounded up to the next set).  Returns the largest supported D. */
int lsr_max_lang_dim(void);

/* Diagnostics: per-stage HIP-event timing on the caller's stream (used by
 * bench.py for the live roofline).  One process-wide, thread-safe timer
 * (atomic switch, mutex-guarded event pool; autograd runs the backward on its
 * own thread): off by default, and while off the entry points above read one
 * atomic flag per stage and nothing else.
 * lsr_profile_query fills up to max_stages (name, total ms, call count)
 * triples since the last reset and returns the number filled. */
void lsr_profile_enable(int on);
/* Restrict the timed stages to a comma-separated list of stage names
 * ("render_bwd,render_fwd"); NULL or "" selects every stage.  Each timed
 * stage adds two event records (a few us of stream idle each), so bench.py
 * times only the roofline kernel inside its timed region.  Returns
 * LSR_EINVAL for an unknown name (mask unchanged). */
int lsr_profile_stages(const char* names);
void lsr_profile_reset(void);
int lsr_profile_query(const char** names, double* ms, int64_t* calls, int max_stages);

#ifdef __cplusplus
}
#endif
#endif
