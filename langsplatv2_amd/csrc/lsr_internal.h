// lsr_internal.h — launcher declarations shared by the kernel translation
// units and the C-ABI driver (lsr_api.hip).  Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../include/lsr.h"
#include "lsr_device.h"

namespace lsr {

struct Cam {
    int W, H, gx, gy;
    float tanfovx, tanfovy, fx, fy, scale_modifier;
    const float* view;
    const float* proj;
    const float* campos;
    const float* bg;
    int sh_degree;
};

// preprocess.hip
// geom_only (SH inputs): the geometry pass only; the SH colour pass is
// launch_preprocess_colour, on a second stream (lsr_api.hip, split preprocess)
hipError_t launch_preprocess(const Cam& c, const lsr_inputs& in, uint8_t* geom, int32_t* radii, bool jac,
                             hipStream_t st, bool geom_only = false, uint64_t* zero_word = nullptr);
hipError_t launch_preprocess_colour(const Cam& c, const lsr_inputs& in, uint8_t* geom, const int32_t* radii, bool jac,
                                    hipStream_t st, hipStream_t colour_st, hipEvent_t ready, hipEvent_t done);
hipError_t launch_sh_grad_from_views(int64_t N, int M, int deg, const float* means3D, int R, const float* campos,
                                     const float* drgb, float* dL_dsh, hipStream_t st);
hipError_t launch_preprocess_bwd(const Cam& c, const lsr_inputs& in, const uint8_t* geom, const int32_t* radii,
                                 const float* grad_acc, int VP, const lsr_bwd_out& out, hipStream_t st);
hipError_t launch_mark_visible(int P, const float* means, const float* view, uint8_t* present, hipStream_t st);

// binning.hip
// Inclusive scan of n uint32 values (in-place allowed); writes the 64-bit total
// to part[0] (part must hold scan_partials(n) uint64 entries).
size_t scan_partials(size_t n);
hipError_t launch_scan_u32(const uint32_t* in, uint32_t* out, uint64_t* part, size_t n, bool exclusive, hipStream_t st);
// Tile-sort size classes (binning.hip tile_class); their per-class tile counts
// and lists live in the image workspace (cls_cnt, cls_list).
#define SORT_NCLS 6
#define LSR_TICKET_WORD 32   // cls_cnt word k_bin_table counts arrivals in (own 128-B line)
#define LSR_COUNT_WORD 64    // cls_cnt words (one u64) k_bin_count sums M and arrivals in (own line;
                             // zeroed by the preprocess)
#define LSR_CLS_SLOT 4       // pinned host word (u64 index) k_bin_table publishes the class counts under
hipError_t launch_publish_total(const uint64_t* total, uint32_t* tile_end, uint64_t* host_slot, uint32_t seq,
                                const uint32_t* cls_cnt, hipStream_t st);
hipError_t launch_duplicate(const Cam& c, int P, const uint8_t* geom, const int32_t* radii, uint32_t* tile_cnt,
                            uint32_t* rank, hipStream_t st);
hipError_t launch_scatter(const Cam& c, int P, const uint8_t* geom, const int32_t* radii, const uint32_t* tile_start,
                          const uint32_t* rank, uint64_t* keys, hipStream_t st);
int bin_blocks(int P, const Cam& c, int& chunk);
bool bin_privatised_ok(const Cam& c);
// count + column scan + group-level tile scan; publishes M (and the sort
// class counts) to host_slot like launch_publish_total
hipError_t launch_bin_count(const Cam& c, int P, int chunk, int B, const uint8_t* geom, const int32_t* radii,
                            uint32_t* table, uint32_t* tile_cnt, uint32_t* tile_start, uint64_t* tpart,
                            uint32_t* cls_cnt, uint32_t* cls_list, uint64_t* host_slot, uint32_t seq, hipStream_t st);
int bin_scatter_rows(const Cam& c);
int scatter_merge(int P);
int bin_block(int P);
// tile_start[0..T) from tile_cnt and the group bases launch_bin_count left in tpart
hipError_t launch_tile_start_apply(int T, int B, const uint32_t* tile_cnt, const uint64_t* tpart, uint32_t* tile_start,
                                   hipStream_t st);
hipError_t launch_bin_scatter(const Cam& c, int P, int chunk, int B, const uint8_t* geom, const int32_t* radii,
                              const uint32_t* table, const uint32_t* tile_start, uint64_t* keys, hipStream_t st);
hipError_t launch_tile_sort(int T, const uint32_t* tile_start, uint64_t* keys, uint32_t* point_list,
                            uint32_t* cls_cnt, uint32_t* cls_list, const uint32_t* host_cnt, hipStream_t st);


// render.hip
struct RenderArgs {
    Cam cam;
    int P;
    const float4* splatA;
    const float4* splatB;
    const float* rgb;            // (P,3): preprocess output or colors_precomp
    const float* lang;           // (P,D) dense or NULL
    int D;                       // dense language channels rendered (0 if off)
    const float* qw;             // quick weights (P,K) or NULL
    const void* qi;              // quick indices (P,K)
    int qidx_dtype, K, Dq;
    int quick_hwc;   // out_lang pixel-major (H, W, Dq) (lsr_settings.quick_layout)
    const uint32_t* point_list;
    const uint32_t* tile_start;  // T+1
    float* final_T;
    uint32_t* n_contrib;
    float* out_color;
    float* out_lang;
    // the backward's accumulators, zeroed by the dense forward render (NULL: none)
    float4* zero = nullptr;
    size_t zero_n16 = 0;
    float4* zero2 = nullptr;   // the (N, D) dL/dlang accumulator (its own allocation)
    size_t zero2_n16 = 0;
    // per-8x8-block candidate lists for the backward (lsr_fwd_out.lists; NULL: none).
    // Block b = 4 tile + sub owns entries [4 tile_start[tile] + sub n_tile, + n_tile)
    // of listA / listB (n_tile = the tile's instance count); lcount[b] = its entries
    // below the block's largest n_contrib (an over-count is harmless)
    float4* listA = nullptr;   // the candidate's splat record A {x, y, conic.a, conic.b}
    float4* listB = nullptr;   // {conic.c, opacity, id bits, 0-based tile-list position bits}
    uint32_t* lcount = nullptr;
    // backward only: the blocks in dispatch order, heaviest list first inside
    // each XCD's range (k_bwd_order; null = band order)
    const uint4* border = nullptr;   // {block 4 tile + sub, tile_start[tile], tile_start[tile + 1], lcount[block]}
};
hipError_t launch_render_fwd(const RenderArgs& a, hipStream_t st);
// the backward's block order (RenderArgs::border, 4 T entries) from the forward's lcount
#ifndef LSR_BWD_ORDER
#define LSR_BWD_ORDER 1   // list-driven backward: heaviest block lists dispatched first (0: band order)
#endif
// from this many 8x8 blocks (4 T) up: four or more generations of the
// backward's 4,096 resident waves, where its drain is worth the order
// kernel's ~7.5 us (cfg3: 32,640 blocks)
#define LSR_BWD_ORDER_MIN_BLOCKS 16384
inline bool bwd_order_on(int T) { return LSR_BWD_ORDER && 4 * (int64_t)T >= LSR_BWD_ORDER_MIN_BLOCKS; }
hipError_t launch_bwd_order(const RenderArgs& a, uint4* border, hipStream_t st);

struct RenderBwdArgs {
    RenderArgs f;
    const float* dout_color;
    const float* dout_lang;
    float* grad_acc;   // (P, VP) atomically accumulated
    int VP;
    // non-null: dL/dlanguage is accumulated straight into this (P, D) output
    // (zeroed by the caller) and the gradient rows hold geometry + colour only
    float* lang_acc = nullptr;
    // non-null (language-only backward in quick mode): dL/dweights (P, K) of
    // the sparse input f.qw / f.qi, accumulated with the channel gradient
    // gathered at each Gaussian's codes (zeroed by the caller)
    float* qw_acc = nullptr;
    // LSR_OPT_DETERMINISTIC: the atomics add 64-bit fixed-point twins of grad_acc
    // (det_rows, same (P, VP) indexing) and lang_acc (det_lang, (P, D)), each value
    // scaled by 2^det_shift(...) (render.hip); det_bounds = {max |dL/dout|,
    // max |feature|, flag bits} from launch_det_bounds, radii the forward's
    long long* det_rows = nullptr;
    long long* det_lang = nullptr;
    float* det_bounds = nullptr;
    const int32_t* radii = nullptr;
    // per Gaussian, the four column classes' shifts as signed bytes (class k in
    // byte k), written by launch_det_bounds and read by the adds and the
    // conversion alike
    uint32_t* det_sh = nullptr;
};
bool bwd_lang_direct(int D);  // D for which the full backward supports lang_acc
int grad_row_width(int D);   // VP for a dense language dim
hipError_t launch_render_bwd(const RenderBwdArgs& a, hipStream_t st);
// language-only backward: grad_acc is the (P, D) dL/dlanguage output itself
// (zeroed by the caller), VP = D
hipError_t launch_render_bwd_lang(const RenderBwdArgs& a, hipStream_t st);
// language-only backward of the quick (sparse) input: a.qw_acc (P, K) from
// the Dq-channel gradient (Dq must be a compiled channel set, <= 64)
hipError_t launch_render_bwd_lang_sparse(const RenderBwdArgs& a, hipStream_t st);
int lang_set_for(int D);     // compiled channel set >= D, or -1
// LSR_OPT_DETERMINISTIC: bounds = {max |dL/dout| over the 3 + D planes,
// max |feature| over the visible Gaussians' colours and the dense language input,
// flag} (flag bit 0: a non-finite value).  bounds points at LSR_DET_HDR bytes:
// the 3 words, then the per-block partials (every word written, no atomics)
constexpr int LSR_DET_BLOCKS = 32768;
constexpr size_t LSR_DET_HDR = 256 + 3 * 4 * LSR_DET_BLOCKS;
hipError_t launch_det_bounds(const RenderBwdArgs& b, float* bounds, hipStream_t st);
// the fixed-point sums back to fp32: rows (P, VP) -> grad_out (every element
// written; VP = 16 with lang_direct), lang (P, D) -> lang_out; lang_only: rows
// is the (P, D) language accumulator and lang_out its output.  A flagged
// bounds word writes NaN everywhere.
hipError_t launch_det_finish(const RenderBwdArgs& b, bool lang_only, float* grad_out, float* lang_out,
                             hipStream_t st);

// quick.hip
hipError_t launch_topk_code_fwd(const float* logits, int64_t N, int L, int K, int k, float* dense, float* sw,
                                void* sidx, int idx_dtype, int level_offset, hipStream_t st);
// sparse: g is dL/dweights of the packed (N, L*k) form (ascending channel order)
hipError_t launch_topk_code_bwd(const float* logits, const float* g, int64_t N, int L, int K, int k, float* dlogits,
                                hipStream_t st, bool sparse = false);
size_t knn_workspace_bytes(int64_t N, size_t sort_temp);
hipError_t knn_sort_temp_bytes(int64_t N, size_t* bytes);
hipError_t launch_knn_dist2(const float* points, int64_t N, float* out, uint8_t* ws, size_t sort_temp, hipStream_t st);
size_t quick_decode_workspace_bytes(int L, int K, int Df, int normalize);
hipError_t launch_quick_decode_prepare(const float* cb, int L, int K, int Df, int normalize, void* ws, hipStream_t st);
hipError_t launch_quick_decode_run(const float* wmap, const float* cb, int L, int K, int Df, int H, int W,
                                   int normalize, float eps, const void* ws, float* out, hipStream_t st,
                                   bool hwc = false);
hipError_t launch_quick_decode(const float* wmap, const float* cb, int L, int K, int Df, int H, int W, int normalize,
                               float eps, void* ws, float* out, hipStream_t st);

// lang_loss.hip
size_t lang_loss_workspace_bytes(int S, int W, int H, int* waves);
// gw == nullptr: forward (loss and/or the per-pixel stats (2, H, W));
// else dL/dweight_map and dL/dcodebooks scaled by *gscale, from the
// forward's stats (recomputed when stats == nullptr)
hipError_t launch_lang_loss(const float* wmap, const float* cb, int Df, int H, int W, const int32_t* seg,
                            const float* feat, int S, const float* gscale, float* loss, float* gw, float* dcb,
                            float* stats, float* ws, hipStream_t st);

// aux.hip: debug NaN/Inf guard (flag |= 1 if any element of p[0..n) is not
// finite) and the quick-input dense expansion / gradient gather
hipError_t launch_nonfinite(const float* p, size_t n, uint32_t* flag, hipStream_t st);
hipError_t launch_check_lists(const uint32_t* point_list, size_t M, uint32_t P, const uint32_t* tile_start, size_t T,
                              uint32_t* flag, hipStream_t st);
hipError_t launch_sparse_expand(const float* qw, const void* qi, int dtype, int N, int K, int Dq, float* dense,
                                hipStream_t st);
hipError_t launch_sparse_gather(const float* g, const void* qi, int dtype, int N, int K, int Dq, float* dw,
                                hipStream_t st);
hipError_t launch_quick_pack_codes(const void* qi, int dtype, int64_t N, int Dq, void* packed, hipStream_t st);

// adam.hip
struct AdamArgs {
    float one_minus_b1, b2, one_minus_b2, eps, step_size, bc2_sqrt, weight_decay;
};
hipError_t launch_adam(float* p, const float* g, float* m, float* v, int64_t n, const AdamArgs& a, hipStream_t st);

}  // namespace lsr
