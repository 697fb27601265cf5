/*
 * lsr_oracle.c — CPU restatement of the language-Gaussian tile rasterizer.
 * TEST INFRASTRUCTURE ONLY (see lsr_oracle.h for the contract and parity
 * status).  Build: oracle/Makefile (gcc -O2 -ffp-contract=off -fopenmp).
 *
 * Algorithm: SURVEY.md Appendix A (3DGS lineage).  Citations point at the
 * reference call sites / Python restatements that pin each step:
 *   SH → RGB            utils/sh_utils.py:57-112, gaussian_renderer/__init__.py:76-81
 *   cov3D = R S S^T R^T  utils/general_utils.py:78-110, scene/gaussian_model.py:28-32
 *   camera conventions   utils/graphics_utils.py:38-71, scene/cameras.py:55-58
 *   dense language input utils/vq_utils.py:9-24  (scene/gaussian_model.py:510-518)
 *   quick language input utils/vq_utils.py:26-40 (eval_lerf.py:333-348)
 *   outputs              gaussian_renderer/__init__.py:108-129
 */
#include "lsr_oracle.h"
#include <float.h>
/* Scale-gradient convention, mirroring csrc/preprocess.hip's LSR_SCALE_GRAD_EXACT:
 * 0 (default) = upstream 3DGS (dL/dscales w.r.t. scale_modifier * scale). */
#ifndef LSO_SCALE_GRAD_EXACT
#define LSO_SCALE_GRAD_EXACT 0
#endif
#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define TILE 16
#define TILE_PIX (TILE * TILE)

static const float SH_C0 = 0.28209479177387814f;
static const float SH_C1 = 0.4886025119029199f;
static const float SH_C2[5] = {1.0925484305920792f, -1.0925484305920792f, 0.31539156525252005f,
                               -1.0925484305920792f, 0.5462742152960396f};
static const float SH_C3[7] = {-0.5900435899266435f, 2.890611442640554f, -0.4570457994644658f,
                               0.3731763325901154f, -0.4570457994644658f, 1.445305721320277f,
                               -0.5900435899266435f};

/* ---------------------------------------------------------------- exp -- */
float lso_expf(float x)
{
    if (x < -87.0f) return 0.0f;
    const float t = fmaf(x, 1.44269504088896341f, 12582912.0f);
    const float n = t - 12582912.0f;
    float r = fmaf(n, -0.693145751953125f, x);
    r = fmaf(n, -1.428606765330187e-06f, r);
    float p = 0x1.6aea1ap-10f;
    p = fmaf(p, r, 0x1.1267d2p-7f);
    p = fmaf(p, r, 0x1.555820p-5f);
    p = fmaf(p, r, 0x1.555418p-3f);
    p = fmaf(p, r, 0x1.fffffcp-2f);
    p = fmaf(p, r, 1.0f);
    p = fmaf(p, r, 1.0f);
    uint32_t tb;
    memcpy(&tb, &t, 4);
    const uint32_t bits = (tb << 23) + 0x3f800000u;
    float sc;
    memcpy(&sc, &bits, 4);
    return p * sc;
}

/* ------------------------------------------------------- small helpers -- */
/* transformPoint4x3 / 4x4 over a column-major 4x4 (m[c*4+r]). */
static inline void xform43(const float* m, float x, float y, float z, float* o)
{
    o[0] = m[0] * x + m[4] * y + m[8] * z + m[12];
    o[1] = m[1] * x + m[5] * y + m[9] * z + m[13];
    o[2] = m[2] * x + m[6] * y + m[10] * z + m[14];
}
static inline void xform44(const float* m, float x, float y, float z, float* o)
{
    o[0] = m[0] * x + m[4] * y + m[8] * z + m[12];
    o[1] = m[1] * x + m[5] * y + m[9] * z + m[13];
    o[2] = m[2] * x + m[6] * y + m[10] * z + m[14];
    o[3] = m[3] * x + m[7] * y + m[11] * z + m[15];
}
/* ndc2Pix evaluated in double, rounded to float (A.1). */
static inline float ndc2pix(float v, int S) { return (float)((((double)v + 1.0) * (double)S - 1.0) * 0.5); }

static inline int imin(int a, int b) { return a < b ? a : b; }
static inline int imax(int a, int b) { return a > b ? a : b; }

/* float → int, truncating, saturating (defined for every input, as the GPU's
 * v_cvt_i32_f32; NaN → 0). */
static inline int f2i(float v)
{
    if (v != v) return 0;
    if (v >= 2147483520.0f) return 2147483647;
    if (v <= -2147483648.0f) return (int)(-2147483647 - 1);
    return (int)v;
}

static inline void get_rect(float px, float py, int r, int gx, int gy, int* r0, int* r1)
{
    r0[0] = imin(gx, imax(0, f2i((px - (float)r) / 16.0f)));
    r0[1] = imin(gy, imax(0, f2i((py - (float)r) / 16.0f)));
    r1[0] = imin(gx, imax(0, f2i((px + (float)r + 16.0f - 1.0f) / 16.0f)));
    r1[1] = imin(gy, imax(0, f2i((py + (float)r + 16.0f - 1.0f) / 16.0f)));
}

/* Quaternion (r,x,y,z) → row-major R exactly as utils/general_utils.py:90-98
 * (without the normalisation of :79-81; the caller normalises,
 * scene/gaussian_model.py:146-147). */
static inline void quat_to_R(const float* q, float* R)
{
    float r = q[0], x = q[1], y = q[2], z = q[3];
    R[0] = 1.f - 2.f * (y * y + z * z);
    R[1] = 2.f * (x * y - r * z);
    R[2] = 2.f * (x * z + r * y);
    R[3] = 2.f * (x * y + r * z);
    R[4] = 1.f - 2.f * (x * x + z * z);
    R[5] = 2.f * (y * z - r * x);
    R[6] = 2.f * (x * z - r * y);
    R[7] = 2.f * (y * z + r * x);
    R[8] = 1.f - 2.f * (x * x + y * y);
}

/* cov3D = (R S)(R S)^T packed (xx,xy,xz,yy,yz,zz) — general_utils.py:64-73,101-110. */
static void compute_cov3D(const float* s, float mod, const float* q, float* cov)
{
    float R[9], Mm[9];
    quat_to_R(q, R);
    float sx = mod * s[0], sy = mod * s[1], sz = mod * s[2];
    for (int i = 0; i < 3; i++) {
        Mm[i * 3 + 0] = R[i * 3 + 0] * sx;
        Mm[i * 3 + 1] = R[i * 3 + 1] * sy;
        Mm[i * 3 + 2] = R[i * 3 + 2] * sz;
    }
#define SIG(i, j) (Mm[(i) * 3 + 0] * Mm[(j) * 3 + 0] + Mm[(i) * 3 + 1] * Mm[(j) * 3 + 1] + Mm[(i) * 3 + 2] * Mm[(j) * 3 + 2])
    cov[0] = SIG(0, 0);
    cov[1] = SIG(0, 1);
    cov[2] = SIG(0, 2);
    cov[3] = SIG(1, 1);
    cov[4] = SIG(1, 2);
    cov[5] = SIG(2, 2);
#undef SIG
}

/* EWA projection of cov3D with J evaluated at the (clamped) view-space mean. */
typedef struct {
    float tx, ty, tz;        /* clamped t.x, t.y and t.z */
    int xclamp, yclamp;
    float J00, J02, J11, J12;
    float T0[3], T1[3];      /* rows of J*W */
} ewa_t;

static void ewa_setup(const float* view, const float* pv, float fx, float fy, float tanfx, float tanfy, ewa_t* e)
{
    const float limx = 1.3f * tanfx, limy = 1.3f * tanfy;
    float txtz = pv[0] / pv[2], tytz = pv[1] / pv[2];
    e->xclamp = (txtz < -limx) || (txtz > limx);
    e->yclamp = (tytz < -limy) || (tytz > limy);
    e->tz = pv[2];
    e->tx = fminf(limx, fmaxf(-limx, txtz)) * pv[2];
    e->ty = fminf(limy, fmaxf(-limy, tytz)) * pv[2];
    float tz2 = e->tz * e->tz;
    e->J00 = fx / e->tz;
    e->J02 = -(fx * e->tx) / tz2;
    e->J11 = fy / e->tz;
    e->J12 = -(fy * e->ty) / tz2;
    for (int j = 0; j < 3; j++) {
        /* W[r][j] = view[j*4 + r] */
        e->T0[j] = e->J00 * view[j * 4 + 0] + e->J02 * view[j * 4 + 2];
        e->T1[j] = e->J11 * view[j * 4 + 1] + e->J12 * view[j * 4 + 2];
    }
}

static void ewa_cov2D(const ewa_t* e, const float* c, float* a, float* b, float* cc)
{
    /* u = Σ T0^T, v = Σ T1^T with Σ from the packed 6-vector. */
    float u0 = c[0] * e->T0[0] + c[1] * e->T0[1] + c[2] * e->T0[2];
    float u1 = c[1] * e->T0[0] + c[3] * e->T0[1] + c[4] * e->T0[2];
    float u2 = c[2] * e->T0[0] + c[4] * e->T0[1] + c[5] * e->T0[2];
    float v0 = c[0] * e->T1[0] + c[1] * e->T1[1] + c[2] * e->T1[2];
    float v1 = c[1] * e->T1[0] + c[3] * e->T1[1] + c[4] * e->T1[2];
    float v2 = c[2] * e->T1[0] + c[4] * e->T1[1] + c[5] * e->T1[2];
    *a = e->T0[0] * u0 + e->T0[1] * u1 + e->T0[2] * u2 + 0.3f;
    *b = e->T0[0] * v0 + e->T0[1] * v1 + e->T0[2] * v2;
    *cc = e->T1[0] * v0 + e->T1[1] * v1 + e->T1[2] * v2 + 0.3f;
}

/* SH → RGB, term order of utils/sh_utils.py:57-112 (degrees 0..3). */
static void sh_eval(int deg, const float* sh /* M*3 */, const float* dir, float* out);
static void sh_to_rgb(int deg, const float* sh /* M*3 */, const float* dir, float* out)
{
    sh_eval(deg, sh, dir, out);
    for (int ch = 0; ch < 3; ch++) out[ch] = out[ch] + 0.5f;
}

static void sh_eval(int deg, const float* sh /* M*3 */, const float* dir, float* out)
{
    float x = dir[0], y = dir[1], z = dir[2];
    for (int ch = 0; ch < 3; ch++) {
#define S(k) sh[(k) * 3 + ch]
        float r = SH_C0 * S(0);
        if (deg > 0) {
            r = r - SH_C1 * y * S(1) + SH_C1 * z * S(2) - SH_C1 * x * S(3);
            if (deg > 1) {
                float xx = x * x, yy = y * y, zz = z * z;
                float xy = x * y, yz = y * z, xz = x * z;
                r = r + SH_C2[0] * xy * S(4) + SH_C2[1] * yz * S(5) + SH_C2[2] * (2.0f * zz - xx - yy) * S(6) +
                    SH_C2[3] * xz * S(7) + SH_C2[4] * (xx - yy) * S(8);
                if (deg > 2) {
                    r = r + SH_C3[0] * y * (3.0f * xx - yy) * S(9) + SH_C3[1] * xy * z * S(10) +
                        SH_C3[2] * y * (4.0f * zz - xx - yy) * S(11) +
                        SH_C3[3] * z * (2.0f * zz - 3.0f * xx - 3.0f * yy) * S(12) +
                        SH_C3[4] * x * (4.0f * zz - xx - yy) * S(13) + SH_C3[5] * z * (xx - yy) * S(14) +
                        SH_C3[6] * x * (xx - 3.0f * yy) * S(15);
                }
            }
        }
#undef S
        out[ch] = r;
    }
}

/* Primitive entry points (golden-vector tests against the reference's own
 * eval_sh / build_rotation / build_scaling_rotation). */
void lso_sh_eval(int deg, int N, int M, const float* sh, const float* dirs, float* out)
{
    for (int i = 0; i < N; i++) sh_eval(deg, sh + (size_t)i * M * 3, dirs + 3 * i, out + 3 * i);
}

void lso_quat_to_R(int N, const float* q, float* R)
{
    for (int i = 0; i < N; i++) quat_to_R(q + 4 * i, R + 9 * i);
}

void lso_cov3D(int N, const float* s, float mod, const float* q, float* cov)
{
    for (int i = 0; i < N; i++) compute_cov3D(s + 3 * i, mod, q + 4 * i, cov + 6 * i);
}

static inline void sh_dir(const float* mean, const float* campos, float* dir, float* dir_orig)
{
    dir_orig[0] = mean[0] - campos[0];
    dir_orig[1] = mean[1] - campos[1];
    dir_orig[2] = mean[2] - campos[2];
    float len = sqrtf(dir_orig[0] * dir_orig[0] + dir_orig[1] * dir_orig[1] + dir_orig[2] * dir_orig[2]);
    dir[0] = dir_orig[0] / len;
    dir[1] = dir_orig[1] / len;
    dir[2] = dir_orig[2] / len;
}

/* ---------------------------------------------------------- preprocess -- */
void lso_preprocess(const lso_settings* s, const lso_inputs* in, lso_geom* g)
{
    const int N = in->N;
    const int gx = (s->W + TILE - 1) / TILE, gy = (s->H + TILE - 1) / TILE;
    const float fx = (float)s->W / (2.0f * s->tanfovx);
    const float fy = (float)s->H / (2.0f * s->tanfovy);
    for (int i = 0; i < N; i++) {
        g->radii[i] = 0;
        g->tiles_touched[i] = 0;
        g->depth[i] = 0.f;
        g->xy[2 * i] = g->xy[2 * i + 1] = 0.f;
        for (int k = 0; k < 4; k++) g->conic_opacity[4 * i + k] = 0.f;
        for (int k = 0; k < 3; k++) { g->rgb[3 * i + k] = 0.f; g->clamped[3 * i + k] = 0; }
        for (int k = 0; k < 6; k++) g->cov3D[6 * i + k] = 0.f;

        const float* p = in->means3D + 3 * i;
        float pv[3], ph[4];
        xform43(s->viewmatrix, p[0], p[1], p[2], pv);
        if (pv[2] <= 0.2f) continue;
        xform44(s->projmatrix, p[0], p[1], p[2], ph);
        float pw = 1.0f / (ph[3] + 0.0000001f);
        float ppx = ph[0] * pw, ppy = ph[1] * pw;

        float cov[6];
        if (in->cov3D_precomp) {
            memcpy(cov, in->cov3D_precomp + 6 * i, sizeof(cov));
        } else {
            compute_cov3D(in->scales + 3 * i, s->scale_modifier, in->rotations + 4 * i, cov);
        }
        memcpy(g->cov3D + 6 * i, cov, sizeof(cov));

        ewa_t e;
        ewa_setup(s->viewmatrix, pv, fx, fy, s->tanfovx, s->tanfovy, &e);
        float a, b, c;
        ewa_cov2D(&e, cov, &a, &b, &c);
        float det = a * c - b * b;
        if (det == 0.0f) continue;
        float det_inv = 1.f / det;
        float mid = 0.5f * (a + c);
        float l1 = mid + sqrtf(fmaxf(0.1f, mid * mid - det));
        float radius = ceilf(3.f * sqrtf(l1));
        int r = f2i(radius);
        float px = ndc2pix(ppx, s->W), py = ndc2pix(ppy, s->H);
        int r0[2], r1[2];
        get_rect(px, py, r, gx, gy, r0, r1);
        int area = (r1[0] - r0[0]) * (r1[1] - r0[1]);
        if (area == 0 || r <= 0) continue;

        if (!in->colors_precomp) {
            float dir[3], dor[3], rgb[3];
            sh_dir(p, s->campos, dir, dor);
            sh_to_rgb(s->sh_degree, in->shs + (size_t)i * in->M * 3, dir, rgb);
            for (int k = 0; k < 3; k++) {
                g->clamped[3 * i + k] = rgb[k] < 0.f;
                g->rgb[3 * i + k] = fmaxf(rgb[k], 0.f);
            }
        } else {
            for (int k = 0; k < 3; k++) g->rgb[3 * i + k] = in->colors_precomp[3 * i + k];
        }
        g->depth[i] = pv[2];
        g->radii[i] = r;
        g->xy[2 * i] = px;
        g->xy[2 * i + 1] = py;
        g->conic_opacity[4 * i + 0] = c * det_inv;
        g->conic_opacity[4 * i + 1] = -b * det_inv;
        g->conic_opacity[4 * i + 2] = a * det_inv;
        g->conic_opacity[4 * i + 3] = in->opacities[i];
        g->tiles_touched[i] = (uint32_t)area;
    }
}

/* ------------------------------------------------------------- binning -- */
int64_t lso_num_rendered(int N, const uint32_t* t)
{
    int64_t m = 0;
    for (int i = 0; i < N; i++) m += t[i];
    return m;
}

/* Conservative cut of the pair exponent: opacity * exp(power) < 1/255 for
 * every power below it (lsr_device.h power_cut, the log taken in double and
 * rounded once on both sides). */
float lso_power_cut(float o)
{
    if (!(o * 255.0f > 1.0f)) return (o == o) ? -0.02f : -INFINITY;
    return (float)(-log((double)(255.0f * o))) - 0.02f;
}

/* The cut as the product stores it in the splat record (lsr_device.h
 * cut_widen): power_cut scaled by (1 + 8e-6 K), K = ca cc / det of the fp32
 * conic, so the cull stays conservative for needle splats; -inf when det <= 0
 * in fp32. */
float lso_cut_widen(float cut, float ca, float cb, float cc)
{
    const float p = ca * cc;
    const float det = p - cb * cb;
    if (!(det > 0.f)) return -INFINITY;
    const float K = p / det;
    return cut * fmaf(K, 8e-6f, 1.0f);
}

/* The product's cull box (csrc/lsr_device.h cull_box), restated operation for
 * operation: the tiles meeting the cut ellipse's axis-aligned box, widened by
 * 1e-4 relative + 0.5 px.  The cull keeps (Gaussian, tile) iff the tile is in
 * the box AND in its row's span (lso_row_span). */
void lso_cull_box(float x, float y, float ca, float cb, float cc, float cut, int* r0, int* r1)
{
    if (!(ca > 0.f) || !(cc > 0.f) || !(cut > -3.0e38f)) return;
    const float det = ca * cc - cb * cb;
    if (!(det > 0.f)) return;
    const float thr = fmaf(-2.f * cut, 1.001f, 1e-3f);
    const float ue = fmaf(sqrtf(thr * cc / det), 1.0001f, 0.5f);
    const float ve = fmaf(sqrtf(thr * ca / det), 1.0001f, 0.5f);
    if (!(ue < 1.0e7f) || !(ve < 1.0e7f)) return;
    const float tx0 = ceilf((x - ue - 15.f) / 16.f), tx1 = floorf((x + ue) / 16.f) + 1.f;
    const float ty0 = ceilf((y - ve - 15.f) / 16.f), ty1 = floorf((y + ve) / 16.f) + 1.f;
    r0[0] = imax(r0[0], f2i(fmaxf(tx0, -1.f)));
    r0[1] = imax(r0[1], f2i(fmaxf(ty0, -1.f)));
    r1[0] = imin(r1[0], f2i(fmaxf(tx1, -1.f)));
    r1[1] = imin(r1[1], f2i(fmaxf(ty1, -1.f)));
}

/* The product's row-span cull (csrc/lsr_device.h span_prep / row_span),
 * restated operation for operation: per tile row ty, the cut ellipse's
 * x-extent over the row's pixel band [16 ty, 16 ty + 15], widened by 1e-3 of
 * its half width + 0.05 px, as the tile range [sx0, sx1) inside the box
 * columns [bx0, bx1).  The right edge (-cb v + sqrt(thr ca - det v^2)) / ca
 * is concave in v: its maximum over the row is at the row's v nearest the
 * ellipse's rightmost point v_r = -cb sqrt(thr / (det cc)); the left edge's
 * minimum at -v_r; rows beyond the widened vertical half extent are empty. */
void lso_span_prep(float x, float y, float ca, float cb, float cc, float cut, lso_span* s)
{
    s->x = x;
    s->y = y;
    const float det = ca * cc - cb * cb;
    const float thr = fmaf(-2.f * cut, 1.001f, 1e-3f);
    const float tcd = thr / det;
    if (!(ca > 0.f) || !(cc > 0.f) || !(cut > -3.0e38f) || !(det > 0.f) || !(tcd < 1.0e30f)) {
        s->vm = INFINITY; s->vr = 0.f; s->cb = 0.f; s->det = 1.f; s->tca = 1.f; s->ica = 1.f; s->me = INFINITY;
        return;
    }
    s->vm = fmaf(sqrtf(tcd * ca), 1.0001f, 0.01f);
    s->vr = -cb * sqrtf(tcd / cc);
    s->cb = cb;
    s->det = det;
    s->tca = thr * ca;
    s->ica = 1.f / ca;
    s->me = fmaf(sqrtf(tcd * cc), 1e-3f, 0.05f);
}

void lso_row_span(const lso_span* s, int ty, int bx0, int bx1, int* sx0, int* sx1)
{
    const float v1 = s->y - (float)(ty * TILE), v0 = v1 - 15.f;
    const float w0 = fmaxf(v0, -s->vm), w1 = fminf(v1, s->vm);
    const float a = fminf(fmaxf(s->vr, w0), w1), b = fminf(fmaxf(-s->vr, w0), w1);
    const float ra = sqrtf(fmaxf(fmaf(-s->det * a, a, s->tca), 0.f));
    const float rb = sqrtf(fmaxf(fmaf(-s->det * b, b, s->tca), 0.f));
    const float umax = fmaf(ra - s->cb * a, s->ica, s->me);
    const float umin = fmaf(-rb - s->cb * b, s->ica, -s->me);
    const float fx0 = ceilf((s->x - umax - 15.f) / 16.f);
    const float fx1 = floorf((s->x - umin) / 16.f) + 1.f;
    *sx0 = f2i(fminf(fmaxf(fx0, (float)bx0), (float)bx1));
    *sx1 = f2i(fminf(fmaxf(fx1, (float)bx0), (float)bx1));
    if (!(w0 <= w1) || *sx1 < *sx0) *sx1 = *sx0;
}

/* The culled instances of Gaussian i: rows [r0[1], r1[1]) of the box, each
 * with its kept column range (cull) or the whole rect row (no cull). */
static inline void gaussian_prep(const lso_geom* g, int i, float cut, int cull, int* r0, int* r1, lso_span* sp)
{
    if (!cull) return;
    const float* co = g->conic_opacity + 4 * i;
    lso_cull_box(g->xy[2 * i], g->xy[2 * i + 1], co[0], co[1], co[2], cut, r0, r1);
    lso_span_prep(g->xy[2 * i], g->xy[2 * i + 1], co[0], co[1], co[2], cut, sp);
}
static inline void row_range(const lso_span* sp, int cull, int y, const int* r0, const int* r1, int* x0, int* x1)
{
    if (!cull) {
        *x0 = r0[0];
        *x1 = r1[0];
        return;
    }
    lso_row_span(sp, y, r0[0], r1[0], x0, x1);
}

int64_t lso_num_rendered_ex(const lso_settings* s, int N, const lso_geom* g, int cull)
{
    if (!cull) return lso_num_rendered(N, g->tiles_touched);
    const int gx = (s->W + TILE - 1) / TILE, gy = (s->H + TILE - 1) / TILE;
    int64_t m = 0;
    for (int i = 0; i < N; i++) {
        if (g->radii[i] <= 0) continue;
        int r0[2], r1[2];
        get_rect(g->xy[2 * i], g->xy[2 * i + 1], g->radii[i], gx, gy, r0, r1);
        const float* coi = g->conic_opacity + 4 * i;
        const float cut = lso_cut_widen(lso_power_cut(coi[3]), coi[0], coi[1], coi[2]);
        lso_span sp;
        gaussian_prep(g, i, cut, 1, r0, r1, &sp);
        if (r1[0] <= r0[0]) continue;
        for (int y = r0[1]; y < r1[1]; y++) {
            int x0, x1;
            row_range(&sp, 1, y, r0, r1, &x0, &x1);
            m += x1 - x0;
        }
    }
    return m;
}

static int cmp_u64(const void* a, const void* b)
{
    uint64_t x = *(const uint64_t*)a, y = *(const uint64_t*)b;
    return x < y ? -1 : (x > y ? 1 : 0);
}

void lso_binning(const lso_settings* s, int N, const lso_geom* g, uint32_t* point_list, uint32_t* ranges)
{
    lso_binning_ex(s, N, g, point_list, ranges, 0);
}

void lso_binning_ex(const lso_settings* s, int N, const lso_geom* g, uint32_t* point_list, uint32_t* ranges,
                    int cull)
{
    const int gx = (s->W + TILE - 1) / TILE, gy = (s->H + TILE - 1) / TILE;
    const int T = gx * gy;
    int64_t M = lso_num_rendered_ex(s, N, g, cull);
    /* Counting sort by tile, then per-tile sort by (depth bits, id): the
     * order of a stable sort on (tile<<32 | depth bits) with duplicates
     * emitted in Gaussian order (Appendix A.2). */
    uint32_t* cnt = (uint32_t*)calloc((size_t)T + 1, sizeof(uint32_t));
    for (int i = 0; i < N; i++) {
        if (g->radii[i] <= 0) continue;
        int r0[2], r1[2];
        get_rect(g->xy[2 * i], g->xy[2 * i + 1], g->radii[i], gx, gy, r0, r1);
        const float* coi = g->conic_opacity + 4 * i;
        const float cut = lso_cut_widen(lso_power_cut(coi[3]), coi[0], coi[1], coi[2]);
        lso_span sp;
        gaussian_prep(g, i, cut, cull, r0, r1, &sp);
        if (r1[0] <= r0[0]) continue;
        for (int y = r0[1]; y < r1[1]; y++) {
            int x0, x1;
            row_range(&sp, cull, y, r0, r1, &x0, &x1);
            for (int x = x0; x < x1; x++) cnt[y * gx + x + 1]++;
        }
    }
    for (int t = 0; t < T; t++) cnt[t + 1] += cnt[t];
    uint64_t* keys = (uint64_t*)malloc((size_t)(M > 0 ? M : 1) * sizeof(uint64_t));
    uint32_t* cur = (uint32_t*)malloc((size_t)T * sizeof(uint32_t));
    memcpy(cur, cnt, (size_t)T * sizeof(uint32_t));
    for (int i = 0; i < N; i++) {
        if (g->radii[i] <= 0) continue;
        int r0[2], r1[2];
        get_rect(g->xy[2 * i], g->xy[2 * i + 1], g->radii[i], gx, gy, r0, r1);
        uint32_t db;
        memcpy(&db, &g->depth[i], 4);
        const float* coi = g->conic_opacity + 4 * i;
        const float cut = lso_cut_widen(lso_power_cut(coi[3]), coi[0], coi[1], coi[2]);
        lso_span sp;
        gaussian_prep(g, i, cut, cull, r0, r1, &sp);
        if (r1[0] <= r0[0]) continue;
        for (int y = r0[1]; y < r1[1]; y++) {
            int x0, x1;
            row_range(&sp, cull, y, r0, r1, &x0, &x1);
            for (int x = x0; x < x1; x++) {
                int t = y * gx + x;
                keys[cur[t]++] = ((uint64_t)db << 32) | (uint32_t)i;
            }
        }
    }
    for (int t = 0; t < T; t++) {
        uint32_t a = cnt[t], b = cnt[t + 1];
        if (b > a + 1) qsort(keys + a, b - a, sizeof(uint64_t), cmp_u64);
        ranges[2 * t] = a;
        ranges[2 * t + 1] = b;
    }
    for (int64_t k = 0; k < M; k++) point_list[k] = (uint32_t)(keys[k] & 0xffffffffu);
    free(keys);
    free(cur);
    free(cnt);
}

/* ---------------------------------------------------------- render fwd -- */
/* u5: round half up, floor(v + 0.5); NaN and values outside [0, 2^31) -> -1 */
static inline int quick_index(float v)
{
    const float r = floorf(v + 0.5f);
    return (r >= 0.f && r < 2147483648.f) ? (int)r : -1;
}

static void render_tile_fwd(const lso_settings* s, const lso_inputs* in, const lso_geom* g,
                            const uint32_t* point_list, const uint32_t* ranges, int tile,
                            float* out_color, float* out_lang, float* final_T, uint32_t* n_contrib)
{
    const int W = s->W, H = s->H;
    const int gx = (W + TILE - 1) / TILE;
    const int tx = tile % gx, ty = tile / gx;
    const int D = s->include_feature ? in->D : 0;
    const int quick = s->quick_render && in->qweights;
    const int Dq = quick ? s->quick_dim : 0;
    const int Dout = quick ? Dq : D;
    const uint32_t start = ranges[2 * tile], end = ranges[2 * tile + 1];
    float* acc = (float*)malloc(sizeof(float) * (size_t)(Dout > 0 ? Dout : 1));
    for (int py = ty * TILE; py < ty * TILE + TILE && py < H; py++)
        for (int px = tx * TILE; px < tx * TILE + TILE && px < W; px++) {
            const float pfx = (float)px, pfy = (float)py;
            float T = 1.0f, C[3] = {0.f, 0.f, 0.f};
            for (int k = 0; k < Dout; k++) acc[k] = 0.f;
            uint32_t contributor = 0, last = 0;
            for (uint32_t idx = start; idx < end; idx++) {
                contributor++;
                const uint32_t j = point_list[idx];
                const float* co = g->conic_opacity + 4 * j;
                float dx = g->xy[2 * j] - pfx, dy = g->xy[2 * j + 1] - pfy;
                float power = fmaf(-0.5f, fmaf(co[0] * dx, dx, (co[2] * dy) * dy), -((co[1] * dx) * dy));
                if (power > 0.0f) continue;
                float G = lso_expf(power);
                float alpha = fminf(0.99f, co[3] * G);
                if (alpha < 1.0f / 255.0f) continue;
                float test_T = T * (1.0f - alpha);
                if (test_T < 0.0001f) break;
                float aT = alpha * T;
                for (int ch = 0; ch < 3; ch++) C[ch] = fmaf(g->rgb[3 * j + ch], aT, C[ch]);
                if (quick) {
                    const float* w = in->qweights + (size_t)j * in->K;
                    const float* ix = in->qindices + (size_t)j * in->K;
                    for (int k = 0; k < in->K; k++) {
                        int q = quick_index(ix[k]);
                        if (q >= 0 && q < Dq) acc[q] = fmaf(w[k], aT, acc[q]);
                    }
                } else {
                    const float* f = in->lang + (size_t)j * in->D;
                    for (int k = 0; k < D; k++) acc[k] = fmaf(f[k], aT, acc[k]);
                }
                T = test_T;
                last = contributor;
            }
            const size_t pix = (size_t)py * W + px;
            final_T[pix] = T;
            n_contrib[pix] = last;
            for (int ch = 0; ch < 3; ch++) out_color[(size_t)ch * H * W + pix] = fmaf(T, s->bg[ch], C[ch]);
            for (int k = 0; k < Dout; k++) out_lang[(size_t)k * H * W + pix] = acc[k];
        }
    free(acc);
}

void lso_render_fwd_tiles(const lso_settings* s, const lso_inputs* in, const lso_geom* g,
                          const uint32_t* point_list, const uint32_t* ranges, const int32_t* tiles, int ntiles,
                          float* out_color, float* out_lang, float* final_T, uint32_t* n_contrib, int nthreads)
{
#ifdef _OPENMP
    if (nthreads < 1) nthreads = 1;
#pragma omp parallel for schedule(dynamic, 4) num_threads(nthreads)
#endif
    for (int k = 0; k < ntiles; k++)
        render_tile_fwd(s, in, g, point_list, ranges, tiles[k], out_color, out_lang, final_T, n_contrib);
}

void lso_render_fwd(const lso_settings* s, const lso_inputs* in, const lso_geom* g, const uint32_t* point_list,
                    const uint32_t* ranges, float* out_color, float* out_lang, float* final_T,
                    uint32_t* n_contrib, int nthreads)
{
    const int gx = (s->W + TILE - 1) / TILE, gy = (s->H + TILE - 1) / TILE;
    const int T = gx * gy;
    int32_t* tiles = (int32_t*)malloc(sizeof(int32_t) * (size_t)T);
    for (int t = 0; t < T; t++) tiles[t] = t;
    lso_render_fwd_tiles(s, in, g, point_list, ranges, tiles, T, out_color, out_lang, final_T, n_contrib, nthreads);
    free(tiles);
}

/* ---------------------------------------------------------- render bwd -- */
typedef struct {
    double* dmean2D; double* dconic; double* dopacity; double* dcolor; double* dlang;
} dacc_t;

/* atomic: tiles rendered by several threads at once (the multi-threaded CPU
 * baseline); the sequential path (the parity checker) keeps plain adds */
static inline void acc_add(double* p, double v, int atomic)
{
    if (atomic) {
#pragma omp atomic update
        *p += v;
    } else {
        *p += v;
    }
}

static void render_tile_bwd(const lso_settings* s, const lso_inputs* in, const lso_geom* g,
                            const uint32_t* point_list, const uint32_t* ranges, int tile,
                            const float* final_Ts, const uint32_t* n_contrib,
                            const float* dout_color, const float* dout_lang, dacc_t* A, int atomic)
{
    const int W = s->W, H = s->H;
    const int gx = (W + TILE - 1) / TILE;
    const int tx = tile % gx, ty = tile / gx;
    const int D = s->include_feature ? in->D : 0;
    const uint32_t start = ranges[2 * tile];
    const float ddelx_dx = 0.5f * (float)W, ddely_dy = 0.5f * (float)H;
    float* Gl = (float*)malloc(sizeof(float) * (size_t)(D > 0 ? D : 1));
    for (int py = ty * TILE; py < ty * TILE + TILE && py < H; py++)
        for (int px = tx * TILE; px < tx * TILE + TILE && px < W; px++) {
            const size_t pix = (size_t)py * W + px;
            const float pfx = (float)px, pfy = (float)py;
            const float T_final = final_Ts[pix];
            const uint32_t last = n_contrib[pix];
            float Gc[3];
            for (int ch = 0; ch < 3; ch++) Gc[ch] = dout_color[(size_t)ch * H * W + pix];
            for (int k = 0; k < D; k++) Gl[k] = dout_lang[(size_t)k * H * W + pix];
            const float bg_dot = s->bg[0] * Gc[0] + s->bg[1] * Gc[1] + s->bg[2] * Gc[2];
            float T = T_final;
            float last_alpha = 0.f, last_dot = 0.f, rec = 0.f;
            /* back to front over positions [0, last) */
            for (int64_t p = (int64_t)last - 1; p >= 0; p--) {
                const uint32_t j = point_list[start + p];
                const float* co = g->conic_opacity + 4 * j;
                float dx = g->xy[2 * j] - pfx, dy = g->xy[2 * j + 1] - pfy;
                float power = fmaf(-0.5f, fmaf(co[0] * dx, dx, (co[2] * dy) * dy), -((co[1] * dx) * dy));
                if (power > 0.0f) continue;
                float G = lso_expf(power);
                float alpha = fminf(0.99f, co[3] * G);
                if (alpha < 1.0f / 255.0f) continue;
                T = T / (1.f - alpha);
                const float aT = alpha * T;
                /* dot = f_j · dL/dpixel over RGB + dense language channels (u2) */
                float dot = g->rgb[3 * j] * Gc[0];
                dot = fmaf(g->rgb[3 * j + 1], Gc[1], dot);
                dot = fmaf(g->rgb[3 * j + 2], Gc[2], dot);
                const float* f = D ? in->lang + (size_t)j * in->D : NULL;
                for (int k = 0; k < D; k++) dot = fmaf(f[k], Gl[k], dot);
                rec = fmaf(last_alpha, last_dot, (1.f - last_alpha) * rec);
                float dL_dalpha = (dot - rec) * T;
                dL_dalpha = fmaf(-T_final / (1.f - alpha), bg_dot, dL_dalpha);
                last_alpha = alpha;
                last_dot = dot;
                for (int ch = 0; ch < 3; ch++) acc_add(&A->dcolor[3 * (size_t)j + ch], (double)(aT * Gc[ch]), atomic);
                for (int k = 0; k < D; k++) acc_add(&A->dlang[(size_t)j * D + k], (double)(aT * Gl[k]), atomic);
                const float dL_dG = co[3] * dL_dalpha;
                const float gdx = G * dx, gdy = G * dy;
                const float dG_ddelx = -gdx * co[0] - gdy * co[1];
                const float dG_ddely = -gdy * co[2] - gdx * co[1];
                acc_add(&A->dmean2D[3 * (size_t)j + 0], (double)(dL_dG * dG_ddelx * ddelx_dx), atomic);
                acc_add(&A->dmean2D[3 * (size_t)j + 1], (double)(dL_dG * dG_ddely * ddely_dy), atomic);
                acc_add(&A->dconic[3 * (size_t)j + 0], (double)(-0.5f * gdx * dx * dL_dG), atomic);
                acc_add(&A->dconic[3 * (size_t)j + 1], (double)(-gdx * dy * dL_dG), atomic);
                acc_add(&A->dconic[3 * (size_t)j + 2], (double)(-0.5f * gdy * dy * dL_dG), atomic);
                acc_add(&A->dopacity[j], (double)(G * dL_dalpha), atomic);
            }
        }
    free(Gl);
}

void lso_render_bwd_tiles_mt(const lso_settings* s, const lso_inputs* in, const lso_geom* g,
                             const uint32_t* point_list, const uint32_t* ranges, const int32_t* tiles, int ntiles,
                             const float* final_T, const uint32_t* n_contrib, const float* dout_color,
                             const float* dout_lang, lso_render_grads* rg, int nthreads)
{
    const int N = in->N;
    const int D = s->include_feature ? in->D : 0;
    dacc_t A;
    A.dmean2D = (double*)calloc((size_t)N * 3 + 1, sizeof(double));
    A.dconic = (double*)calloc((size_t)N * 3 + 1, sizeof(double));
    A.dopacity = (double*)calloc((size_t)N + 1, sizeof(double));
    A.dcolor = (double*)calloc((size_t)N * 3 + 1, sizeof(double));
    A.dlang = (double*)calloc((size_t)N * (D > 0 ? D : 1) + 1, sizeof(double));
    if (nthreads <= 1) {
        for (int k = 0; k < ntiles; k++)
            render_tile_bwd(s, in, g, point_list, ranges, tiles[k], final_T, n_contrib, dout_color, dout_lang, &A, 0);
    } else {
#pragma omp parallel for schedule(dynamic, 4) num_threads(nthreads)
        for (int k = 0; k < ntiles; k++)
            render_tile_bwd(s, in, g, point_list, ranges, tiles[k], final_T, n_contrib, dout_color, dout_lang, &A, 1);
    }
    for (size_t i = 0; i < (size_t)N * 3; i++) {
        rg->dmean2D[i] = (i % 3 == 2) ? 0.f : (float)A.dmean2D[i];
        rg->dconic[i] = (float)A.dconic[i];
        rg->dcolor[i] = (float)A.dcolor[i];
    }
    for (int i = 0; i < N; i++) rg->dopacity[i] = (float)A.dopacity[i];
    if (rg->dlang && D)
        for (size_t i = 0; i < (size_t)N * D; i++) rg->dlang[i] = (float)A.dlang[i];
    free(A.dmean2D); free(A.dconic); free(A.dopacity); free(A.dcolor); free(A.dlang);
}

void lso_render_bwd_tiles(const lso_settings* s, const lso_inputs* in, const lso_geom* g,
                          const uint32_t* point_list, const uint32_t* ranges, const int32_t* tiles, int ntiles,
                          const float* final_T, const uint32_t* n_contrib, const float* dout_color,
                          const float* dout_lang, lso_render_grads* rg)
{
    lso_render_bwd_tiles_mt(s, in, g, point_list, ranges, tiles, ntiles, final_T, n_contrib, dout_color, dout_lang,
                            rg, 1);
}

void lso_render_bwd(const lso_settings* s, const lso_inputs* in, const lso_geom* g, const uint32_t* point_list,
                    const uint32_t* ranges, const float* final_T, const uint32_t* n_contrib,
                    const float* dout_color, const float* dout_lang, lso_render_grads* rg)
{
    const int gx = (s->W + TILE - 1) / TILE, gy = (s->H + TILE - 1) / TILE;
    const int T = gx * gy;
    int32_t* tiles = (int32_t*)malloc(sizeof(int32_t) * (size_t)T);
    for (int t = 0; t < T; t++) tiles[t] = t;
    lso_render_bwd_tiles(s, in, g, point_list, ranges, tiles, T, final_T, n_contrib, dout_color, dout_lang, rg);
    free(tiles);
}

/* ------------------------------------------- render bwd: error bounds -- */
/* A-priori bound of |GPU - oracle| for every render-gradient element, for the
 * product's deterministic backward (include/lsr.h LSR_OPT_DETERMINISTIC), by a
 * running forward-error analysis of both evaluations of Appendix A.4 along the
 * oracle's own traversal.  Units: u = 2^-24 (fp32 unit roundoff); the result is
 * u x (sum over the element's per-pixel terms of their error bounds).
 *
 * Per contributing pair, back to front at one pixel:
 *   G:      the power is the same fp32 bits on both sides (the forward is
 *           bit-exact); GPU 2^(power log2e) (product u|power|, v_exp_f32 2u),
 *           oracle lso_expf (2u), |power| <= ln 255 for a contributing pair
 *           => |dG|/G <= 10u; alpha = min(0.99, o G): |dalpha|/alpha <= 12u.
 *   T:      T <- T / (1 - alpha) from the bit-identical final T; d(1-alpha) =
 *           dalpha, so each step adds 12u alpha/(1-alpha) plus 4u (GPU rcp +
 *           mul, oracle divide): eT.
 *   aT:     eT + 14u; colour / language term aT dL/dout: + 2u.
 *   dot:    sum over C = 3 + D channels (GPU MFMA, oracle fmaf chain):
 *           2 C u sum_c |f_c dL/dout_c|.
 *   S:      S <- alpha dot + (1 - alpha) S with the errors above: eS
 *           (absolute) carried like S itself.
 *   dL/dalpha = (dot - S) T - T_final/(1-alpha) bg.dL/dout:
 *           T (2 C u |f.dout| + eS) + |dot - S| T (eT + 2u)
 *           + |bg term| (12u alpha/(1-alpha) + 4u) + 2u |dL/dalpha|.
 *   opacity G dL/dalpha; mean2D / conic o G dL/dalpha x (dx, dy polynomial):
 *           value error o |poly| (G e(dL/dalpha) + 12u G |dL/dalpha|).
 *   GPU pixel sums: each 8x8 block's 64 terms summed in fp32 (MFMA K chain
 *           or a 16-term VALU chain + 2 reduction levels, then the moment
 *           combination): <= 72u sum |term|, where a geometry term's magnitude
 *           is that of its factorised form, |u| (|X|+|lx|)^k (|Y|+|ly|)^m with
 *           X = mean - block centre, lx = pixel - block centre (the product
 *           sums u lx^k ly^m per block and combines with X, Y afterwards).
 * Not included (added by the caller): the fixed-point rounding of each block
 * partial (2^-(s+1), s from the product's det_shift) and the final fp32
 * roundings of the two results (u |value| each); the oracle's fp64 sums are
 * exact to 2^-53 relative. */
static void render_tile_bwd_bound(const lso_settings* s, const lso_inputs* in, const lso_geom* g,
                                  const uint32_t* point_list, const uint32_t* ranges, int tile,
                                  const float* final_Ts, const uint32_t* n_contrib,
                                  const float* dout_color, const float* dout_lang, dacc_t* A, dacc_t* M,
                                  int32_t* seen_tile, uint8_t* seen_mask, double* nblk, int atomic)
{
    const int W = s->W, H = s->H;
    const int gx = (W + TILE - 1) / TILE;
    const int tx = tile % gx, ty = tile / gx;
    const int D = s->include_feature ? in->D : 0;
    const double C2 = 2.0 * (3 + D);
    const uint32_t start = ranges[2 * tile];
    const double hW = 0.5 * (double)W, hH = 0.5 * (double)H;
    float* Gl = (float*)malloc(sizeof(float) * (size_t)(D > 0 ? D : 1));
    for (int py = ty * TILE; py < ty * TILE + TILE && py < H; py++)
        for (int px = tx * TILE; px < tx * TILE + TILE && px < W; px++) {
            const size_t pix = (size_t)py * W + px;
            const float pfx = (float)px, pfy = (float)py;
            const double cx = (double)(px & ~7) + 3.5, cy = (double)(py & ~7) + 3.5;
            const double alx = fabs((double)px - cx), aly = fabs((double)py - cy);
            const float T_final = final_Ts[pix];
            const uint32_t last = n_contrib[pix];
            float Gc[3];
            for (int ch = 0; ch < 3; ch++) Gc[ch] = dout_color[(size_t)ch * H * W + pix];
            for (int k = 0; k < D; k++) Gl[k] = dout_lang[(size_t)k * H * W + pix];
            const float bg_dot = s->bg[0] * Gc[0] + s->bg[1] * Gc[1] + s->bg[2] * Gc[2];
            float T = T_final;
            float last_alpha = 0.f, last_dot = 0.f, rec = 0.f;
            double eT = 0.0, eS = 0.0, last_dabs = 0.0;
            for (int64_t p = (int64_t)last - 1; p >= 0; p--) {
                const uint32_t j = point_list[start + p];
                const float* co = g->conic_opacity + 4 * j;
                float dx = g->xy[2 * j] - pfx, dy = g->xy[2 * j + 1] - pfy;
                float power = fmaf(-0.5f, fmaf(co[0] * dx, dx, (co[2] * dy) * dy), -((co[1] * dx) * dy));
                if (power > 0.0f) continue;
                float G = lso_expf(power);
                float alpha = fminf(0.99f, co[3] * G);
                if (alpha < 1.0f / 255.0f) continue;
                T = T / (1.f - alpha);
                const double ra = (double)alpha / (1.0 - (double)alpha);
                eT += 12.0 * ra + 4.0;
                const double aT = (double)alpha * (double)T;
                float dot = g->rgb[3 * j] * Gc[0];
                dot = fmaf(g->rgb[3 * j + 1], Gc[1], dot);
                dot = fmaf(g->rgb[3 * j + 2], Gc[2], dot);
                double dabs = fabs((double)g->rgb[3 * j] * Gc[0]) + fabs((double)g->rgb[3 * j + 1] * Gc[1]) +
                              fabs((double)g->rgb[3 * j + 2] * Gc[2]);
                const float* f = D ? in->lang + (size_t)j * in->D : NULL;
                for (int k = 0; k < D; k++) {
                    dot = fmaf(f[k], Gl[k], dot);
                    dabs += fabs((double)f[k] * Gl[k]);
                }
                /* S absorbs the previous (nearer-the-back) pair, as the oracle's rec */
                eS = 12.0 * last_alpha * (fabs((double)last_dot) + fabs((double)rec)) + last_alpha * C2 * last_dabs +
                     (1.0 - last_alpha) * eS +
                     3.0 * (last_alpha * fabs((double)last_dot) + (1.0 - last_alpha) * fabs((double)rec));
                rec = fmaf(last_alpha, last_dot, (1.f - last_alpha) * rec);
                float dL_dalpha = (dot - rec) * T;
                const float bgt = -T_final / (1.f - alpha) * bg_dot;
                dL_dalpha = fmaf(-T_final / (1.f - alpha), bg_dot, dL_dalpha);
                const double EdLa = (double)T * (C2 * dabs + eS) + fabs((double)dot - rec) * T * (eT + 2.0) +
                                    fabs((double)bgt) * (12.0 * ra + 4.0) + 2.0 * fabs((double)dL_dalpha);
                last_alpha = alpha;
                last_dot = dot;
                last_dabs = dabs;
                if (nblk) {
                    /* the 8x8 blocks j has a contributing pixel in (the cross-block sum's terms) */
                    const uint8_t bit = (uint8_t)(1u << (((py >> 3) & 1) * 2 + ((px >> 3) & 1)));
                    if (seen_tile[j] != tile) {
                        seen_tile[j] = tile;
                        seen_mask[j] = 0;
                    }
                    if (!(seen_mask[j] & bit)) {
                        seen_mask[j] |= bit;
                        acc_add(&nblk[j], 1.0, atomic);
                    }
                }
                const double eaT = eT + 16.0 + 72.0;   /* + the product and the block sum */
                for (int ch = 0; ch < 3; ch++) acc_add(&A->dcolor[3 * (size_t)j + ch], eaT * fabs(aT * Gc[ch]), atomic);
                for (int k = 0; k < D; k++) acc_add(&A->dlang[(size_t)j * D + k], eaT * fabs(aT * Gl[k]), atomic);
                const double o = co[3];
                const double Ub = (double)G * fabs((double)dL_dalpha);
                acc_add(&A->dopacity[j], (double)G * EdLa + (14.0 + 72.0) * Ub, atomic);
                const double VE = o * ((double)G * EdLa + 12.0 * Ub);     /* per unit of the pair's polynomial */
                const double adx = fabs((double)dx), ady = fabs((double)dy);
                const double AX = fabs((double)g->xy[2 * j] - cx) + alx, AY = fabs((double)g->xy[2 * j + 1] - cy) + aly;
                const double ca = fabs((double)co[0]), cb = fabs((double)co[1]), cc = fabs((double)co[2]);
                acc_add(&A->dmean2D[3 * (size_t)j + 0], hW * (VE * (ca * adx + cb * ady) + 72.0 * o * Ub * (ca * AX + cb * AY)),
                        atomic);
                acc_add(&A->dmean2D[3 * (size_t)j + 1], hH * (VE * (cb * adx + cc * ady) + 72.0 * o * Ub * (cb * AX + cc * AY)),
                        atomic);
                acc_add(&A->dconic[3 * (size_t)j + 0], 0.5 * (VE * adx * adx + 72.0 * o * Ub * AX * AX), atomic);
                acc_add(&A->dconic[3 * (size_t)j + 1], VE * adx * ady + 72.0 * o * Ub * AX * AY, atomic);
                acc_add(&A->dconic[3 * (size_t)j + 2], 0.5 * (VE * ady * ady + 72.0 * o * Ub * AY * AY), atomic);
                if (M) {
                    /* the terms' magnitudes (geometry: factorised forms), in units of 1 */
                    for (int ch = 0; ch < 3; ch++) acc_add(&M->dcolor[3 * (size_t)j + ch], fabs(aT * Gc[ch]), atomic);
                    for (int k = 0; k < D; k++) acc_add(&M->dlang[(size_t)j * D + k], fabs(aT * Gl[k]), atomic);
                    acc_add(&M->dopacity[j], Ub, atomic);
                    acc_add(&M->dmean2D[3 * (size_t)j + 0], hW * o * Ub * (ca * AX + cb * AY), atomic);
                    acc_add(&M->dmean2D[3 * (size_t)j + 1], hH * o * Ub * (cb * AX + cc * AY), atomic);
                    acc_add(&M->dconic[3 * (size_t)j + 0], 0.5 * o * Ub * AX * AX, atomic);
                    acc_add(&M->dconic[3 * (size_t)j + 1], o * Ub * AX * AY, atomic);
                    acc_add(&M->dconic[3 * (size_t)j + 2], 0.5 * o * Ub * AY * AY, atomic);
                }
            }
        }
    free(Gl);
}

static void dacc_alloc(dacc_t* A, int N, int D)
{
    A->dmean2D = (double*)calloc((size_t)N * 3 + 1, sizeof(double));
    A->dconic = (double*)calloc((size_t)N * 3 + 1, sizeof(double));
    A->dopacity = (double*)calloc((size_t)N + 1, sizeof(double));
    A->dcolor = (double*)calloc((size_t)N * 3 + 1, sizeof(double));
    A->dlang = (double*)calloc((size_t)N * (D > 0 ? D : 1) + 1, sizeof(double));
}

static void dacc_store(const dacc_t* A, int N, int D, double scale, lso_render_grads* out)
{
    for (size_t i = 0; i < (size_t)N * 3; i++) {
        out->dmean2D[i] = (i % 3 == 2) ? 0.f : (float)(scale * A->dmean2D[i]);
        out->dconic[i] = (float)(scale * A->dconic[i]);
        out->dcolor[i] = (float)(scale * A->dcolor[i]);
    }
    for (int i = 0; i < N; i++) out->dopacity[i] = (float)(scale * A->dopacity[i]);
    if (out->dlang && D)
        for (size_t i = 0; i < (size_t)N * D; i++) out->dlang[i] = (float)(scale * A->dlang[i]);
    free(A->dmean2D); free(A->dconic); free(A->dopacity); free(A->dcolor); free(A->dlang);
}

void lso_render_bwd_bound_tiles_mt(const lso_settings* s, const lso_inputs* in, const lso_geom* g,
                                   const uint32_t* point_list, const uint32_t* ranges, const int32_t* tiles,
                                   int ntiles, const float* final_T, const uint32_t* n_contrib,
                                   const float* dout_color, const float* dout_lang, lso_render_grads* bound,
                                   lso_render_grads* mag, float* nblocks, int nthreads)
{
    const int N = in->N;
    const int D = s->include_feature ? in->D : 0;
    const double u = 5.9604644775390625e-08; /* 2^-24 */
    dacc_t A, M;
    dacc_alloc(&A, N, D);
    if (mag) dacc_alloc(&M, N, D);
    double* nb = nblocks ? (double*)calloc((size_t)N + 1, sizeof(double)) : NULL;
    const int nt = nthreads <= 1 ? 1 : nthreads;
#pragma omp parallel num_threads(nt) if (nt > 1)
    {
        /* per thread: the tile and 4-block mask j was last counted in */
        int32_t* seen_tile = NULL;
        uint8_t* seen_mask = NULL;
        if (nb) {
            seen_tile = (int32_t*)malloc(sizeof(int32_t) * ((size_t)N + 1));
            seen_mask = (uint8_t*)calloc((size_t)N + 1, 1);
            for (int i = 0; i < N; i++) seen_tile[i] = -1;
        }
#pragma omp for schedule(dynamic, 4)
        for (int k = 0; k < ntiles; k++)
            render_tile_bwd_bound(s, in, g, point_list, ranges, tiles[k], final_T, n_contrib, dout_color, dout_lang,
                                  &A, mag ? &M : NULL, seen_tile, seen_mask, nb, nt > 1);
        free(seen_tile);
        free(seen_mask);
    }
    dacc_store(&A, N, D, u, bound);
    if (mag) dacc_store(&M, N, D, 1.0, mag);
    if (nb) {
        for (int i = 0; i < N; i++) nblocks[i] = (float)nb[i];
        free(nb);
    }
}

/* ------------------------------------------------------ preprocess bwd -- */
/* Chain rule through A.1; conventions as the upstream 3DGS backward:
 * straight-through 0.99 clamp (render), ±1.3 tanfov clamp zeroes the
 * clamped coordinate's gradient and J is differentiated at the clamped t
 * (t.x treated as constant when clamped), colour clamp zeroes clamped
 * channels, quaternion gradient w.r.t. the (caller-normalised) input. */
void lso_preprocess_bwd(const lso_settings* s, const lso_inputs* in, const lso_geom* g,
                        const lso_render_grads* rg, lso_param_grads* pg)
{
    const int N = in->N;
    const float fx = (float)s->W / (2.0f * s->tanfovx);
    const float fy = (float)s->H / (2.0f * s->tanfovy);
    const float* V = s->viewmatrix;
    const float* P = s->projmatrix;
    for (int i = 0; i < N; i++) {
        float* dm = pg->dmeans3D + 3 * i;
        dm[0] = dm[1] = dm[2] = 0.f;
        if (pg->dsh && in->shs) for (int k = 0; k < in->M * 3; k++) pg->dsh[(size_t)i * in->M * 3 + k] = 0.f;
        if (pg->dscales) for (int k = 0; k < 3; k++) pg->dscales[3 * i + k] = 0.f;
        if (pg->drot) for (int k = 0; k < 4; k++) pg->drot[4 * i + k] = 0.f;
        if (pg->dcov3D) for (int k = 0; k < 6; k++) pg->dcov3D[6 * i + k] = 0.f;
        for (int k = 0; k < 3; k++) pg->dcolors[3 * i + k] = rg->dcolor[3 * i + k];
        if (g->radii[i] <= 0) {
            for (int k = 0; k < 3; k++) pg->dcolors[3 * i + k] = 0.f;
            continue;
        }
        const float* p = in->means3D + 3 * i;
        const float* cov = g->cov3D + 6 * i;
        float pv[3];
        xform43(V, p[0], p[1], p[2], pv);
        ewa_t e;
        ewa_setup(V, pv, fx, fy, s->tanfovx, s->tanfovy, &e);
        float a, b, c;
        ewa_cov2D(&e, cov, &a, &b, &c);
        /* dL/d(a,b,c) from dL/dconic */
        const float dA = rg->dconic[3 * i], dB = rg->dconic[3 * i + 1], dC = rg->dconic[3 * i + 2];
        float det = a * c - b * b;
        float d2inv = 1.0f / ((det * det) + 0.0000001f);
        float dLa = 0.f, dLb = 0.f, dLc = 0.f;
        float dcov[6] = {0, 0, 0, 0, 0, 0};
        if (d2inv != 0.f) {
            dLa = d2inv * (-c * c * dA + b * c * dB - b * b * dC);
            dLb = d2inv * (2.f * b * c * dA - (det + 2.f * b * b) * dB + 2.f * a * b * dC);
            dLc = d2inv * (-b * b * dA + a * b * dB - a * a * dC);
            const float* T0 = e.T0; const float* T1 = e.T1;
            dcov[0] = T0[0] * T0[0] * dLa + T0[0] * T1[0] * dLb + T1[0] * T1[0] * dLc;
            dcov[3] = T0[1] * T0[1] * dLa + T0[1] * T1[1] * dLb + T1[1] * T1[1] * dLc;
            dcov[5] = T0[2] * T0[2] * dLa + T0[2] * T1[2] * dLb + T1[2] * T1[2] * dLc;
            dcov[1] = 2.f * T0[0] * T0[1] * dLa + (T0[0] * T1[1] + T0[1] * T1[0]) * dLb + 2.f * T1[0] * T1[1] * dLc;
            dcov[2] = 2.f * T0[0] * T0[2] * dLa + (T0[0] * T1[2] + T0[2] * T1[0]) * dLb + 2.f * T1[0] * T1[2] * dLc;
            dcov[4] = 2.f * T0[1] * T0[2] * dLa + (T0[1] * T1[2] + T0[2] * T1[1]) * dLb + 2.f * T1[1] * T1[2] * dLc;
        }
        /* dL/dT rows: a = T0ΣT0', b = T0ΣT1', c = T1ΣT1' */
        float u[3], v[3];
        u[0] = cov[0] * e.T0[0] + cov[1] * e.T0[1] + cov[2] * e.T0[2];
        u[1] = cov[1] * e.T0[0] + cov[3] * e.T0[1] + cov[4] * e.T0[2];
        u[2] = cov[2] * e.T0[0] + cov[4] * e.T0[1] + cov[5] * e.T0[2];
        v[0] = cov[0] * e.T1[0] + cov[1] * e.T1[1] + cov[2] * e.T1[2];
        v[1] = cov[1] * e.T1[0] + cov[3] * e.T1[1] + cov[4] * e.T1[2];
        v[2] = cov[2] * e.T1[0] + cov[4] * e.T1[1] + cov[5] * e.T1[2];
        float dT0[3], dT1[3];
        for (int k = 0; k < 3; k++) {
            dT0[k] = 2.f * dLa * u[k] + dLb * v[k];
            dT1[k] = 2.f * dLc * v[k] + dLb * u[k];
        }
        /* T0j = J00 W0j + J02 W2j ; T1j = J11 W1j + J12 W2j ; Wrj = V[j*4+r] */
        float dJ00 = dT0[0] * V[0] + dT0[1] * V[4] + dT0[2] * V[8];
        float dJ02 = dT0[0] * V[2] + dT0[1] * V[6] + dT0[2] * V[10];
        float dJ11 = dT1[0] * V[1] + dT1[1] * V[5] + dT1[2] * V[9];
        float dJ12 = dT1[0] * V[2] + dT1[1] * V[6] + dT1[2] * V[10];
        float tz = 1.f / e.tz, tz2 = tz * tz, tz3 = tz2 * tz;
        float dtx = e.xclamp ? 0.f : -fx * tz2 * dJ02;
        float dty = e.yclamp ? 0.f : -fy * tz2 * dJ12;
        float dtz = -fx * tz2 * dJ00 - fy * tz2 * dJ11 + (2.f * fx * e.tx) * tz3 * dJ02 + (2.f * fy * e.ty) * tz3 * dJ12;
        /* view-space → world: W^T (dtx, dty, dtz) */
        dm[0] = V[0] * dtx + V[1] * dty + V[2] * dtz;
        dm[1] = V[4] * dtx + V[5] * dty + V[6] * dtz;
        dm[2] = V[8] * dtx + V[9] * dty + V[10] * dtz;

        /* projection: means2D (NDC) → mean */
        float ph[4];
        xform44(P, p[0], p[1], p[2], ph);
        float mw = 1.0f / (ph[3] + 0.0000001f);
        float mul1 = ph[0] * mw * mw, mul2 = ph[1] * mw * mw;
        float g2x = rg->dmean2D[3 * i], g2y = rg->dmean2D[3 * i + 1];
        dm[0] += (P[0] * mw - P[3] * mul1) * g2x + (P[1] * mw - P[3] * mul2) * g2y;
        dm[1] += (P[4] * mw - P[7] * mul1) * g2x + (P[5] * mw - P[7] * mul2) * g2y;
        dm[2] += (P[8] * mw - P[11] * mul1) * g2x + (P[9] * mw - P[11] * mul2) * g2y;

        /* colour: SH chain (colour clamp zeroes clamped channels) */
        if (!in->colors_precomp && in->shs) {
            float dRGB[3];
            for (int k = 0; k < 3; k++) dRGB[k] = g->clamped[3 * i + k] ? 0.f : rg->dcolor[3 * i + k];
            float dir[3], dor[3];
            sh_dir(p, s->campos, dir, dor);
            const float x = dir[0], y = dir[1], z = dir[2];
            const float* sh = in->shs + (size_t)i * in->M * 3;
            float* dsh = pg->dsh + (size_t)i * in->M * 3;
            float ddx[3] = {0, 0, 0}, ddy[3] = {0, 0, 0}, ddz[3] = {0, 0, 0};
            const int deg = s->sh_degree;
            for (int ch = 0; ch < 3; ch++) {
#define S(k) sh[(k) * 3 + ch]
#define DS(k) dsh[(k) * 3 + ch]
                const float gch = dRGB[ch];
                DS(0) = SH_C0 * gch;
                if (deg > 0) {
                    DS(1) = -SH_C1 * y * gch;
                    DS(2) = SH_C1 * z * gch;
                    DS(3) = -SH_C1 * x * gch;
                    ddx[ch] = -SH_C1 * S(3);
                    ddy[ch] = -SH_C1 * S(1);
                    ddz[ch] = SH_C1 * S(2);
                    if (deg > 1) {
                        float xx = x * x, yy = y * y, zz = z * z;
                        float xy = x * y, yz = y * z, xz = x * z;
                        DS(4) = SH_C2[0] * xy * gch;
                        DS(5) = SH_C2[1] * yz * gch;
                        DS(6) = SH_C2[2] * (2.f * zz - xx - yy) * gch;
                        DS(7) = SH_C2[3] * xz * gch;
                        DS(8) = SH_C2[4] * (xx - yy) * gch;
                        ddx[ch] += SH_C2[0] * y * S(4) + SH_C2[2] * 2.f * -x * S(6) + SH_C2[3] * z * S(7) + SH_C2[4] * 2.f * x * S(8);
                        ddy[ch] += SH_C2[0] * x * S(4) + SH_C2[1] * z * S(5) + SH_C2[2] * 2.f * -y * S(6) + SH_C2[4] * 2.f * -y * S(8);
                        ddz[ch] += SH_C2[1] * y * S(5) + SH_C2[2] * 2.f * 2.f * z * S(6) + SH_C2[3] * x * S(7);
                        if (deg > 2) {
                            DS(9) = SH_C3[0] * y * (3.f * xx - yy) * gch;
                            DS(10) = SH_C3[1] * xy * z * gch;
                            DS(11) = SH_C3[2] * y * (4.f * zz - xx - yy) * gch;
                            DS(12) = SH_C3[3] * z * (2.f * zz - 3.f * xx - 3.f * yy) * gch;
                            DS(13) = SH_C3[4] * x * (4.f * zz - xx - yy) * gch;
                            DS(14) = SH_C3[5] * z * (xx - yy) * gch;
                            DS(15) = SH_C3[6] * x * (xx - 3.f * yy) * gch;
                            ddx[ch] += SH_C3[0] * S(9) * 3.f * 2.f * xy + SH_C3[1] * S(10) * yz +
                                       SH_C3[2] * S(11) * -2.f * xy + SH_C3[3] * S(12) * -3.f * 2.f * xz +
                                       SH_C3[4] * S(13) * (-3.f * xx + 4.f * zz - yy) + SH_C3[5] * S(14) * 2.f * xz +
                                       SH_C3[6] * S(15) * 3.f * (xx - yy);
                            ddy[ch] += SH_C3[0] * S(9) * 3.f * (xx - yy) + SH_C3[1] * S(10) * xz +
                                       SH_C3[2] * S(11) * (-3.f * yy + 4.f * zz - xx) + SH_C3[3] * S(12) * -3.f * 2.f * yz +
                                       SH_C3[4] * S(13) * -2.f * xy + SH_C3[5] * S(14) * -2.f * yz +
                                       SH_C3[6] * S(15) * -3.f * 2.f * xy;
                            ddz[ch] += SH_C3[1] * S(10) * xy + SH_C3[2] * S(11) * 4.f * 2.f * yz +
                                       SH_C3[3] * S(12) * 3.f * (2.f * zz - xx - yy) + SH_C3[4] * S(13) * 4.f * 2.f * xz +
                                       SH_C3[5] * S(14) * (xx - yy);
                        }
                    }
                }
#undef S
#undef DS
            }
            float gdir[3];
            gdir[0] = ddx[0] * dRGB[0] + ddx[1] * dRGB[1] + ddx[2] * dRGB[2];
            gdir[1] = ddy[0] * dRGB[0] + ddy[1] * dRGB[1] + ddy[2] * dRGB[2];
            gdir[2] = ddz[0] * dRGB[0] + ddz[1] * dRGB[1] + ddz[2] * dRGB[2];
            /* d normalize(v) / dv */
            float sum2 = dor[0] * dor[0] + dor[1] * dor[1] + dor[2] * dor[2];
            float inv32 = 1.0f / sqrtf(sum2 * sum2 * sum2);
            dm[0] += ((sum2 - dor[0] * dor[0]) * gdir[0] - dor[1] * dor[0] * gdir[1] - dor[2] * dor[0] * gdir[2]) * inv32;
            dm[1] += (-dor[0] * dor[1] * gdir[0] + (sum2 - dor[1] * dor[1]) * gdir[1] - dor[2] * dor[1] * gdir[2]) * inv32;
            dm[2] += (-dor[0] * dor[2] * gdir[0] - dor[1] * dor[2] * gdir[1] + (sum2 - dor[2] * dor[2]) * gdir[2]) * inv32;
        }

        /* cov3D: to scales / rotations, or straight out */
        if (in->cov3D_precomp) {
            if (pg->dcov3D) for (int k = 0; k < 6; k++) pg->dcov3D[6 * i + k] = dcov[k];
        } else if (in->scales && in->rotations) {
            const float* q = in->rotations + 4 * i;
            const float* sc = in->scales + 3 * i;
            const float mod = s->scale_modifier;
            float R[9];
            quat_to_R(q, R);
            float sv[3] = {mod * sc[0], mod * sc[1], mod * sc[2]};
            /* Σ = M M^T, M = R S ; dL/dM = 2 G M, G symmetric from packed grads */
            float Gm[9] = {dcov[0], 0.5f * dcov[1], 0.5f * dcov[2],
                           0.5f * dcov[1], dcov[3], 0.5f * dcov[4],
                           0.5f * dcov[2], 0.5f * dcov[4], dcov[5]};
            float Mm[9];
            for (int r = 0; r < 3; r++)
                for (int cc = 0; cc < 3; cc++) Mm[r * 3 + cc] = R[r * 3 + cc] * sv[cc];
            float dM[9];
            for (int r = 0; r < 3; r++)
                for (int cc = 0; cc < 3; cc++)
                    dM[r * 3 + cc] = 2.f * (Gm[r * 3 + 0] * Mm[0 * 3 + cc] + Gm[r * 3 + 1] * Mm[1 * 3 + cc] + Gm[r * 3 + 2] * Mm[2 * 3 + cc]);
            /* dL/ds_c = Σ_r dM[r][c] R[r][c] (upstream: w.r.t. the modified scale;
             * LSO_SCALE_GRAD_EXACT 1: times mod, the exact derivative);
             * dL/dR[r][c] = dM[r][c] sv[c] */
            for (int cc = 0; cc < 3; cc++)
                pg->dscales[3 * i + cc] = (LSO_SCALE_GRAD_EXACT ? mod : 1.0f) * (dM[0 * 3 + cc] * R[0 * 3 + cc] + dM[1 * 3 + cc] * R[1 * 3 + cc] + dM[2 * 3 + cc] * R[2 * 3 + cc]);
            float dR[9];
            for (int r = 0; r < 3; r++)
                for (int cc = 0; cc < 3; cc++) dR[r * 3 + cc] = dM[r * 3 + cc] * sv[cc];
            const float qr = q[0], qx = q[1], qy = q[2], qz = q[3];
            /* R polynomial derivatives (see quat_to_R) */
            float gr = 2.f * (-qz * dR[1] + qy * dR[2] + qz * dR[3] - qx * dR[5] - qy * dR[6] + qx * dR[7]);
            float gx = 2.f * (qy * dR[1] + qz * dR[2] + qy * dR[3] - qr * dR[5] + qz * dR[6] + qr * dR[7]) - 4.f * qx * (dR[4] + dR[8]);
            float gy = 2.f * (qx * dR[1] + qr * dR[2] + qx * dR[3] + qz * dR[5] - qr * dR[6] + qz * dR[7]) - 4.f * qy * (dR[0] + dR[8]);
            float gz = 2.f * (-qr * dR[1] + qx * dR[2] + qr * dR[3] + qy * dR[5] + qx * dR[6] + qy * dR[7]) - 4.f * qz * (dR[0] + dR[4]);
            pg->drot[4 * i + 0] = gr;
            pg->drot[4 * i + 1] = gx;
            pg->drot[4 * i + 2] = gy;
            pg->drot[4 * i + 3] = gz;
        }
    }
}

void lso_knn_dist2(int N, const float* pts, float* out)
{
#pragma omp parallel for schedule(dynamic, 64)
    for (int i = 0; i < N; i++) {
        float b[3] = {FLT_MAX, FLT_MAX, FLT_MAX};
        const float qx = pts[3 * i], qy = pts[3 * i + 1], qz = pts[3 * i + 2];
        for (int j = 0; j < N; j++) {
            if (j == i) continue;
            const float dx = pts[3 * j] - qx, dy = pts[3 * j + 1] - qy, dz = pts[3 * j + 2] - qz;
            float d = dx * dx + dy * dy + dz * dz;
            for (int k = 0; k < 3; k++)
                if (b[k] > d) {
                    const float t = b[k];
                    b[k] = d;
                    d = t;
                }
        }
        out[i] = (b[0] + b[1] + b[2]) / 3.0f;
    }
}
