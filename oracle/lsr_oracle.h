/*
 * lsr_oracle.h — CPU restatement of the language-Gaussian tile rasterizer.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product path (langsplatv2_amd/,
 * diff_gaussian_rasterization/) may include, link or call this code.  Only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use it, and
 * only as the checker / the CPU baseline being timed.
 *
 * Parity status: the rasterizer's CUDA source (git submodule
 * submodules/efficient-langsplat-rasterization, .gitmodules:1-3, pinned SHA
 * not recorded) is ABSENT from the reference checkout, and the reference has
 * no tests or golden vectors for it.  This oracle
 * restates the 3DGS-lineage algorithm and is pinned by
 * the reference's importable Python on the path's edges (utils/sh_utils.py,
 * utils/general_utils.py, utils/graphics_utils.py, utils/vq_utils.py — see
 * tests/golden/make_ref_golden.py) and by a float64 torch-autograd
 * restatement of the forward for the backward (tests/test_oracle.py).
 * Against the CUDA kernels themselves: PARITY UNPINNED.
 *
 * Floating-point contract: compiled with -ffp-contract=off; every fused
 * multiply-add is an explicit fmaf().  The HIP kernels use the identical
 * operation sequence, so forward outputs (radii, xy, conic, rgb, tile lists,
 * image, final_T, n_contrib) are bit-identical between oracle and GPU.
 * Backward per-pair math is identical; only the order of the per-Gaussian
 * sums differs (GPU: wave reduction + atomics; oracle: sequential, in
 * double), so gradients are compared with a tolerance.
 */
#ifndef LSR_ORACLE_H
#define LSR_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    int W, H;
    float tanfovx, tanfovy;
    const float* bg;          /* 3 */
    float scale_modifier;
    const float* viewmatrix;  /* 16, column-major (torch row-major of world_view_transform) */
    const float* projmatrix;  /* 16, column-major (full_proj_transform) */
    int sh_degree;            /* active degree */
    const float* campos;      /* 3 */
    int include_feature;      /* dense language channels */
    int quick_render;         /* sparse (weights, indices) language channels */
    int quick_dim;            /* D_q, output channels of the quick path */
} lso_settings;

typedef struct {
    int N;
    int M;                    /* max_coeffs = shs.shape[1] */
    int D;                    /* dense language channels (language_feature_precomp.shape[1]) */
    int K;                    /* quick: entries per Gaussian */
    const float* means3D;     /* N*3 */
    const float* shs;         /* N*M*3 or NULL */
    const float* colors_precomp; /* N*3 or NULL */
    const float* opacities;   /* N */
    const float* scales;      /* N*3 or NULL */
    const float* rotations;   /* N*4 or NULL */
    const float* cov3D_precomp; /* N*6 or NULL */
    const float* lang;        /* N*D or NULL */
    const float* qweights;    /* N*K or NULL */
    const float* qindices;    /* N*K (float-encoded ints) or NULL */
} lso_inputs;

/* Per-Gaussian geometry (oracle-owned host arrays, sized N). */
typedef struct {
    float* depth;       /* N */
    int32_t* radii;     /* N */
    float* xy;          /* N*2 */
    float* conic_opacity; /* N*4 */
    float* rgb;         /* N*3 */
    uint8_t* clamped;   /* N*3 */
    float* cov3D;       /* N*6 */
    uint32_t* tiles_touched; /* N */
} lso_geom;

/* A.1 preprocess. */
void lso_preprocess(const lso_settings* s, const lso_inputs* in, lso_geom* g);

/* A.2 binning: returns M = num_rendered; point_list (M) sorted by
 * (tile, depth bits, gaussian id); ranges (T*2). point_list must hold
 * sum(tiles_touched) entries. */
int64_t lso_num_rendered(int N, const uint32_t* tiles_touched);
void lso_binning(const lso_settings* s, int N, const lso_geom* g,
                 uint32_t* point_list, uint32_t* ranges);

/* The same with the product's tile cull (cull != 0): an instance (Gaussian,
 * tile) of the rect is kept only if the tile lies in the Gaussian's cull box
 * and in its row's span of the widened cut ellipse (lso_cull_box,
 * lso_row_span: the restatements of lsr_device.h cull_box / row_span).
 * Dropped instances have alpha < 1/255 at every pixel of their tile, so the
 * rendered outputs equal lso_binning's; the lists shrink.  cull = 0 is
 * lso_num_rendered / lso_binning. */
int64_t lso_num_rendered_ex(const lso_settings* s, int N, const lso_geom* g, int cull);
void lso_binning_ex(const lso_settings* s, int N, const lso_geom* g,
                    uint32_t* point_list, uint32_t* ranges, int cull);
float lso_power_cut(float opacity);
float lso_cut_widen(float cut, float ca, float cb, float cc);
/* the cull's box (lsr_device.h cull_box): shrinks the rect [r0, r1) to the
 * tiles meeting the cut ellipse's bounding box */
void lso_cull_box(float x, float y, float ca, float cb, float cc, float cut, int* r0, int* r1);
/* the per-Gaussian part of the row-span cull and one row's kept tile range
 * [sx0, sx1) inside the box columns [bx0, bx1) (lsr_device.h span_prep / row_span) */
typedef struct { float x, y, vm, vr, cb, det, tca, ica, me; } lso_span;
void lso_span_prep(float x, float y, float ca, float cb, float cc, float cut, lso_span* s);
void lso_row_span(const lso_span* s, int ty, int bx0, int bx1, int* sx0, int* sx1);

/* A.3 render forward.  out_color 3*H*W; out_lang Dout*H*W (Dout = D dense
 * or quick_dim); final_T, n_contrib H*W.  Tiles are processed in parallel
 * with OpenMP when nthreads > 1 (results do not depend on nthreads). */
void lso_render_fwd(const lso_settings* s, const lso_inputs* in, const lso_geom* g,
                    const uint32_t* point_list, const uint32_t* ranges,
                    float* out_color, float* out_lang, float* final_T,
                    uint32_t* n_contrib, int nthreads);
/* Same, restricted to a list of tiles (bounded CPU-baseline samples). */
void lso_render_fwd_tiles(const lso_settings* s, const lso_inputs* in, const lso_geom* g,
                          const uint32_t* point_list, const uint32_t* ranges,
                          const int32_t* tiles, int ntiles,
                          float* out_color, float* out_lang, float* final_T,
                          uint32_t* n_contrib, int nthreads);

/* A.4 render backward: per-Gaussian sums (double accumulators, then cast). */
typedef struct {
    float* dmean2D;   /* N*3 (z = 0): dL/d(NDC xy) */
    float* dconic;    /* N*3 : dL/d(conic a, b, c) (full derivative) */
    float* dopacity;  /* N */
    float* dcolor;    /* N*3 */
    float* dlang;     /* N*D or NULL */
} lso_render_grads;

void lso_render_bwd(const lso_settings* s, const lso_inputs* in, const lso_geom* g,
                    const uint32_t* point_list, const uint32_t* ranges,
                    const float* final_T, const uint32_t* n_contrib,
                    const float* dout_color, const float* dout_lang,
                    lso_render_grads* rg);
void lso_render_bwd_tiles(const lso_settings* s, const lso_inputs* in, const lso_geom* g,
                          const uint32_t* point_list, const uint32_t* ranges,
                          const int32_t* tiles, int ntiles,
                          const float* final_T, const uint32_t* n_contrib,
                          const float* dout_color, const float* dout_lang,
                          lso_render_grads* rg);
/* as lso_render_bwd_tiles on nthreads OpenMP threads (tiles in parallel, fp64
 * atomic accumulation): the multi-threaded CPU baseline of bench.py */
void lso_render_bwd_tiles_mt(const lso_settings* s, const lso_inputs* in, const lso_geom* g,
                             const uint32_t* point_list, const uint32_t* ranges,
                             const int32_t* tiles, int ntiles,
                             const float* final_T, const uint32_t* n_contrib,
                             const float* dout_color, const float* dout_lang,
                             lso_render_grads* rg, int nthreads);

/* A-priori bound of |product deterministic backward - this oracle| per
 * render-gradient element (the same fields as lso_render_grads); see the
 * derivation at its definition.  Excludes the fixed-point rounding and the
 * two final fp32 roundings, which the caller adds.  Optional (NULL: skipped):
 * mag = each element's sum of |term| (geometry terms in their factorised form),
 * nblocks = per Gaussian, the 8x8 blocks it has a contributing pixel in; the
 * default float-atomic cross-block sum adds at most nblocks u mag. */
void lso_render_bwd_bound_tiles_mt(const lso_settings* s, const lso_inputs* in, const lso_geom* g,
                                   const uint32_t* point_list, const uint32_t* ranges, const int32_t* tiles,
                                   int ntiles, const float* final_T, const uint32_t* n_contrib,
                                   const float* dout_color, const float* dout_lang, lso_render_grads* bound,
                                   lso_render_grads* mag, float* nblocks, int nthreads);

typedef struct {
    float* dmeans3D;  /* N*3 */
    float* dsh;       /* N*M*3 or NULL */
    float* dcolors;   /* N*3 (== dL/dcolors_precomp when precomp given) */
    float* dscales;   /* N*3 or NULL */
    float* drot;      /* N*4 or NULL */
    float* dcov3D;    /* N*6 or NULL (when cov3D_precomp given) */
} lso_param_grads;

/* Chain rule through A.1 (consumes the render grads). */
void lso_preprocess_bwd(const lso_settings* s, const lso_inputs* in, const lso_geom* g,
                        const lso_render_grads* rg, lso_param_grads* pg);

/* The deterministic exponential shared (as a specification) with the HIP
 * kernels: magic-number rounding, Cody-Waite reduction, degree-6 near-minimax
 * polynomial in fmaf (<= 0.96 ulp). */
float lso_expf(float x);

/* Primitives: SH evaluation (sh: N*M*3, no +0.5), quaternion -> row-major R,
 * packed covariance (R S)(R S)^T with S = diag(mod * s). */
void lso_sh_eval(int deg, int N, int M, const float* sh, const float* dirs, float* out);
void lso_quat_to_R(int N, const float* q, float* R);
void lso_cov3D(int N, const float* s, float mod, const float* q, float* cov);

/* simple_knn distCUDA2 (scene/gaussian_model.py:20,194), by brute force:
 * out[i] = (b0 + b1 + b2) / 3 of the three smallest squared distances
 * dx*dx + dy*dy + dz*dz (left to right, no contraction) to points j != i,
 * b ascending by insertion (strict >), FLT_MAX where fewer than 3 exist.
 * O(N^2); OpenMP over i. */
void lso_knn_dist2(int N, const float* pts, float* out);

#ifdef __cplusplus
}
#endif
#endif
