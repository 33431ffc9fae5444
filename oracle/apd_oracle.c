/*
 * apd_oracle.c — CPU restatement of APDe-MVS's per-view PatchMatch (RunPatchMatch, APD.cu:2663-2737).
 *
 * TEST INFRASTRUCTURE ONLY. This file is the parity oracle and the host-CPU baseline. Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it; the product library
 * (libapd_hip.so) never links, loads or calls it.
 *
 * Parity status: "parity unpinned" against the reference itself. The reference CUDA path cannot be
 * built in this pipeline (nvcc, OpenCV and Boost are absent), the reference ships no
 * tests, fixtures or golden vectors, and it seeds cuRAND with clock64() (APD.cu:916),
 * so no run of it is reproducible anyway. The oracle is pinned by analytic known-answer tests
 * (tests/test_oracle_kat.py) and follows APD.cu function by function; every function below cites the
 * reference lines it restates.
 *
 * Semantic contract shared bit-for-bit with the HIP kernels (written twice, independently):
 *  - fp32 everywhere the reference uses fp32; double exactly where the reference promotes to double
 *    (0.8 x expf, 0.25 x and 0.75 x, cost - 0.1). Both sides compile with -ffp-contract=off; fused
 *    multiply-adds appear only as explicit fmaf() at a FIXED set of sites: the NCC moments and
 *    variances, the weighted view sums, the CDF, the homography projection. nvcc --fmad=true (the
 *    reference's default) may contract every other a*b+c as well -- e.g. the anchor position
 *    point.x + direction.x * radius (APD.cu:1925), restated here as a separate multiply and add --
 *    and which sites it contracts is the compiler's choice, not the source's. This contract is
 *    therefore one fixed, documented rounding of the reference's arithmetic: the HIP kernels equal
 *    it bit for bit, and agreement with a real CUDA build of the reference can only be statistical
 *    (within rounding), never bitwise.
 *  - Division and sqrt are IEEE correctly rounded. rsqrtf(x) is restated as 1.0f/sqrtf(x).
 *    exp/sin/cos are the deterministic polynomials o_expf/o_sinf/o_cosf below.
 *  - Homography: H = A - b*(n^T Kr^-1)/w with A = Ks*R_rel*Kr^-1, b = Ks*t_rel precomputed per source
 *    view in double; algebraically identical to ComputeHomography (APD.cu:334-394).
 *  - Projection: X = fma(H1,y,fma(H0,x,H2)) (same for Y,Z), then x' = X*(1/Z) (the reference's
 *    --use_fast_math X/Z is __fdividef, i.e. X*rcp(Z)).
 *  - tex2D with cudaFilterModeLinear, unnormalised coordinates (APD.cpp:691-706): bilinear with the
 *    coordinate rounded to 1/256 (CUDA's 8-bit fractional weights), clamp-to-edge addressing
 *    (Wrap is not honoured with unnormalised coordinates). NaN/huge coordinates are clamped to
 *    [-1, W] first. Integer+0.5 fetches (reference image, depth maps) are plain texel reads.
 *  - RNG: Philox4x32-10 counter stream keyed by (seed, pixel index, launch ordinal) replaces the
 *    per-pixel cuRAND XORWOW state seeded by clock64() (APD.cu:904-917); draws happen in the
 *    program order listed in SURVEY.md Appendix B. uniform() = ((u>>8)+1)*2^-24 in (0,1].
 *  - Buffers the reference leaves uninitialised (view_weight_cuda, APD.cpp:750) start at zero.
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <float.h>
#ifdef _OPENMP
#include <omp.h>
#endif
#include <time.h>

#include "../include/apd_hip.h"

typedef struct { float x, y, z, w; } f4;

/* Float division and square roots of the restated arithmetic. In the parity build these are the IEEE
   operations of the contract above. ORACLE_FASTMATH (liboracle_fm.so, the numerics-sensitivity study
   tools/numerics_sensitivity.py; NOT the parity contract) restates the reference's own build flags,
   nvcc --use_fast_math (CMakeLists.txt:26), in spirit: the file is compiled with -ffp-contract=fast
   (every a*b+c the source writes may become a fused multiply-add, as nvcc --fmad=true does), a/b is
   a * rcp(b) and 1/sqrt(x) is rsqrt(x) with ~1-2 ulp approximations (the SSE 12-bit estimate plus one
   Newton step, as -prec-div=false / -prec-sqrt=false allow), sqrt(x) = x * rsqrt(x), exp is __expf's
   exp2 of a rounded x * log2(e), sin/cos come from libm instead of the contract's polynomials, and
   denormals are flushed to zero (FTZ/DAZ, -ftz=true). */
#ifdef ORACLE_FASTMATH
#include <immintrin.h>
static inline float fm_rcp(float x) {
    const float ax = fabsf(x);
    if (!(ax > 1e-36f && ax < 1e36f)) return 1.0f / x; /* zero, denormal, huge, inf, NaN */
    float r = _mm_cvtss_f32(_mm_rcp_ss(_mm_set_ss(x)));
    return r * (2.0f - x * r);
}
static inline float fm_rsqrt(float x) {
    if (!(x > 1e-36f && x < 1e36f)) return 1.0f / sqrtf(x);
    float r = _mm_cvtss_f32(_mm_rsqrt_ss(_mm_set_ss(x)));
    return r * (1.5f - 0.5f * x * r * r);
}
static inline float fm_sqrt(float x) { return (x > 1e-36f && x < 1e36f) ? x * fm_rsqrt(x) : sqrtf(x); }
#define FDIV(a, b) ((a) * fm_rcp(b))
#define FRSQRT(x) fm_rsqrt(x)
#define FSQRT(x) fm_sqrt(x)
#else
#define FDIV(a, b) ((a) / (b))
#define FRSQRT(x) (1.0f / sqrtf(x))
#define FSQRT(x) sqrtf(x)
#endif

#define WEAK APD_WEAK
#define STRONG APD_STRONG
#define UNKNOWN APD_UNKNOWN
#define ANCHOR_NUM APD_ANCHOR_NUM
#define COST_MAX 2.0f
#define M_PI_D 3.14159265358979323846

/* OpenCV's MIN/MAX macros as used by the reference (cvdef.h). */
#define CV_MIN(a, b) ((a) > (b) ? (b) : (a))
#define CV_MAX(a, b) ((a) < (b) ? (b) : (a))

/* launch ordinals of the RNG contract */
#define ORD_ANCHORS 1u
#define ORD_INIT 2u
#define ORD_STRONG(i) (16u + 3u * (uint32_t)(i))
#define ORD_FIT(i) (17u + 3u * (uint32_t)(i))
#define ORD_WEAK(i) (18u + 3u * (uint32_t)(i))
#define RNG_TAG 0x41504421u

/* ------------------------------------------------------------------------------------------------
 * deterministic math
 * ----------------------------------------------------------------------------------------------*/
static inline float bits_f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }

/* exp(x): Cody-Waite reduction + degree-7 Taylor/Horner (|r| <= ln2/2), 2^k by two exact scalings.
   Restates expf at APD.cu:440 (Softmax), 1340/1347/1358 (view selection). */
float o_expf(float x) {
#ifdef ORACLE_FASTMATH
    return (float)exp2((double)(x * 1.44269504f)); /* __expf: ex2.approx(x * log2e) */
#endif
    if (x != x) return x;
    if (x > 88.7228394f) return INFINITY;
    if (x < -103.972084f) return 0.0f;
    float kf = floorf(fmaf(x, 1.44269502f, 0.5f));
    int k = (int)kf;
    float r = fmaf(kf, -0.693145752f, x);
    r = fmaf(kf, -1.42860677e-06f, r);
    float p = 1.98412698e-04f;          /* 1/5040 */
    p = fmaf(p, r, 1.38888889e-03f);    /* 1/720  */
    p = fmaf(p, r, 8.33333333e-03f);    /* 1/120  */
    p = fmaf(p, r, 4.16666667e-02f);    /* 1/24   */
    p = fmaf(p, r, 1.66666667e-01f);    /* 1/6    */
    p = fmaf(p, r, 0.5f);
    p = fmaf(p, r, 1.0f);
    p = fmaf(p, r, 1.0f);
    int k1 = k / 2, k2 = k - k1;
    p *= bits_f((uint32_t)(k1 + 127) << 23);
    p *= bits_f((uint32_t)(k2 + 127) << 23);
    return p;
}

/* sin/cos for |x| <= 0.8 (arguments are the +-0.01*pi perturbation angles, APD.cu:274-283). */
float o_sinf(float x) {
#ifdef ORACLE_FASTMATH
    return (float)sin((double)x);
#endif
    float s2 = x * x;
    float p = -2.50521084e-08f;
    p = fmaf(p, s2, 2.75573192e-06f);
    p = fmaf(p, s2, -1.98412698e-04f);
    p = fmaf(p, s2, 8.33333333e-03f);
    p = fmaf(p, s2, -1.66666667e-01f);
    return fmaf(x * s2, p, x);
}
float o_cosf(float x) {
#ifdef ORACLE_FASTMATH
    return (float)cos((double)x);
#endif
    float s2 = x * x;
    float p = 2.08767570e-09f;
    p = fmaf(p, s2, -2.75573192e-07f);
    p = fmaf(p, s2, 2.48015873e-05f);
    p = fmaf(p, s2, -1.38888889e-03f);
    p = fmaf(p, s2, 4.16666667e-02f);
    p = fmaf(p, s2, -0.5f);
    return fmaf(s2, p, 1.0f);
}

/* ------------------------------------------------------------------------------------------------
 * RNG contract: Philox4x32-10 (Salmon et al. 2011), counter = (pixel, ordinal, block, TAG)
 * ----------------------------------------------------------------------------------------------*/
typedef struct { uint32_t k0, k1, c0, c1, n; uint32_t b[4]; } orng;

void o_philox(uint32_t c[4], uint32_t k0, uint32_t k1) {
    for (int r = 0; r < 10; ++r) {
        uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
        uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
        uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        uint32_t n0 = hi1 ^ c[1] ^ k0, n2 = hi0 ^ c[3] ^ k1;
        c[0] = n0; c[1] = lo1; c[2] = n2; c[3] = lo0;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
}
static inline void orng_init(orng *g, uint64_t seed, uint32_t pixel, uint32_t ordinal) {
    g->k0 = (uint32_t)seed; g->k1 = (uint32_t)(seed >> 32);
    g->c0 = pixel; g->c1 = ordinal; g->n = 0;
}
/* curand(): APD.cu:1921-1922, 1994-1996, 2536-2538 */
static inline uint32_t orng_u32(orng *g) {
    uint32_t j = g->n & 3u;
    if (j == 0) {
        uint32_t c[4] = {g->c0, g->c1, g->n >> 2, RNG_TAG};
        o_philox(c, g->k0, g->k1);
        g->b[0] = c[0]; g->b[1] = c[1]; g->b[2] = c[2]; g->b[3] = c[3];
    }
    g->n++;
    return g->b[j];
}
/* curand_uniform(): (0,1] */
static inline float orng_uniform(orng *g) {
    return (float)((orng_u32(g) >> 8) + 1u) * 5.96046448e-08f;
}

/* ------------------------------------------------------------------------------------------------
 * problem context
 * ----------------------------------------------------------------------------------------------*/
typedef struct {
    int W, H, HW, N, NI;
    int row_limit;
    const float *img[APD_MAX_IMAGES];
    const float *dep[APD_MAX_IMAGES];
    apd_camera cam[APD_MAX_IMAGES];
    apd_params P;
    uint64_t seed;
    /* per-source homography precompute */
    float A[APD_MAX_IMAGES][9], b[APD_MAX_IMAGES][3];
    float ikx, iky, cxk, cyk;
    /* state */
    f4 *plane;
    float *cost;
    uint32_t *sel;
    uint32_t *sel_next; /* RandomInitialization output (launch-start snapshot semantics) */
    uint8_t *vw;      /* view-major: vw[v*HW + pix] */
    uint8_t *weak;
    uint8_t *conf;
    const uint8_t *sa;
    uint8_t *sa_zero;
    int32_t *amap;
    int16_t *anchors; /* weak_count*9 (x,y) */
    int32_t weak_count;
    uint8_t *reliable;
    int16_t *nearest; /* HW (x,y) */
    f4 *fit;
    float *curve;
} octx;

/* ------------------------------------------------------------------------------------------------
 * Access-set checking ("a CPU oracle with a per-colour write-set ∩ read-set = ∅
 * assertion mode"). Every access to the per-pixel state goes through RD / WR. In the normal build
 * they are the plain subscript. Built with -DORACLE_RACECHECK (liboracle_rc.so, single-threaded),
 * each FOR_ALL / FOR_COLOUR phase records, per state element, the pixel task that wrote it and the
 * task(s) that read it, and counts a conflict whenever one task's write meets another task's read or
 * write in the same phase: exactly the accesses whose outcome would depend on the order in which
 * the GPU's threads run (the reference's kernels and ours run a phase's pixels concurrently; the
 * in-place DepthToWeak / LocalRefine / filter tiles and the checkerboard colours rely on this).
 * ----------------------------------------------------------------------------------------------*/
#ifdef ORACLE_RACECHECK
enum { RC_plane, RC_cost, RC_sel, RC_sel_next, RC_vw, RC_weak, RC_conf, RC_fit, RC_reliable, RC_nearest,
       RC_anchors, RC_curve, RC_amap, RC_COUNT };
static const char *const rc_names[RC_COUNT] = {"plane", "cost", "sel", "sel_next", "vw", "weak", "conf", "fit",
                                               "reliable", "nearest", "anchors", "curve", "amap"};
typedef struct { int32_t *wr, *rd; size_t n, cap; } rc_shadow;
static rc_shadow rc_sh[RC_COUNT];
static int32_t rc_task = -1;        /* the pixel task running, -1 outside a phase */
static char rc_phase_name[96];
static int64_t rc_conflicts, rc_phases, rc_accesses;
static char rc_first[320];
static int rc_merge_colours;        /* negative control: both colours of a checkerboard in one phase */

static void rc_conflict(int a, size_t i, int32_t t1, int32_t t2, const char *what) {
    if (!rc_conflicts)
        snprintf(rc_first, sizeof rc_first, "%s: %s[%zu] %s (tasks %d, %d)", rc_phase_name, rc_names[a], i, what,
                 (int)t1, (int)t2);
    rc_conflicts++;
}
static inline void rc_touch(int a, size_t i, int write) {
    if (rc_task < 0) return;
    rc_shadow *s = &rc_sh[a];
    if (i >= s->n) { rc_conflict(a, i, rc_task, -1, "out of range"); return; }
    rc_accesses++;
    const int32_t t = rc_task;
    if (write) {
        if (s->wr[i] >= 0 && s->wr[i] != t) rc_conflict(a, i, s->wr[i], t, "written by two tasks");
        if (s->rd[i] == -2 || (s->rd[i] >= 0 && s->rd[i] != t)) rc_conflict(a, i, s->rd[i], t, "read by one task, written by another");
        s->wr[i] = t;
    } else {
        if (s->wr[i] >= 0 && s->wr[i] != t) rc_conflict(a, i, s->wr[i], t, "written by one task, read by another");
        s->rd[i] = s->rd[i] == -1 ? t : (s->rd[i] == t ? t : -2);
    }
}
static void rc_span(int a, size_t first, size_t count, int write) {
    for (size_t k = 0; k < count; ++k) rc_touch(a, first + k, write);
}
#define RD(o, arr, i) (*(rc_touch(RC_##arr, (size_t)(i), 0), &(o)->arr[i]))
#define WR(o, arr, i) (*(rc_touch(RC_##arr, (size_t)(i), 1), &(o)->arr[i]))
#define RC_SPAN_W(o, arr, first, count) rc_span(RC_##arr, (size_t)(first), (size_t)(count), 1)
#else
#define RD(o, arr, i) ((o)->arr[i])
#define WR(o, arr, i) ((o)->arr[i])
#define RC_SPAN_W(o, arr, first, count) ((void)0)
#endif

static inline int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }
static inline int is_set(uint32_t v, int n) { return (int)((v >> n) & 1u); }

/* per-source precompute of H = Ks (R_rel - t_rel n^T / w) Kr^-1 = A - b m^T / w, APD.cu:334-394 */
static void precompute_homography(octx *o) {
    const apd_camera *r = &o->cam[0];
    double kr0 = r->K[0], kr2 = r->K[2], kr4 = r->K[4], kr5 = r->K[5];
    double Kri[9] = {1.0 / kr0, 0.0, -kr2 / kr0, 0.0, 1.0 / kr4, -kr5 / kr4, 0.0, 0.0, 1.0};
    o->ikx = (float)(1.0 / kr0);
    o->iky = (float)(1.0 / kr4);
    o->cxk = (float)(kr2 / kr0);
    o->cyk = (float)(kr5 / kr4);
    double rC[3];
    for (int j = 0; j < 3; ++j)
        rC[j] = -((double)r->R[j] * r->t[0] + (double)r->R[3 + j] * r->t[1] + (double)r->R[6 + j] * r->t[2]);
    for (int s = 0; s < o->NI; ++s) {
        const apd_camera *c = &o->cam[s];
        double sC[3], Crel[3], trel[3], Rrel[9];
        for (int j = 0; j < 3; ++j)
            sC[j] = -((double)c->R[j] * c->t[0] + (double)c->R[3 + j] * c->t[1] + (double)c->R[6 + j] * c->t[2]);
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j)
                Rrel[3 * i + j] = (double)c->R[3 * i] * r->R[3 * j] + (double)c->R[3 * i + 1] * r->R[3 * j + 1] +
                                  (double)c->R[3 * i + 2] * r->R[3 * j + 2];
        for (int j = 0; j < 3; ++j) Crel[j] = rC[j] - sC[j];
        for (int i = 0; i < 3; ++i)
            trel[i] = (double)c->R[3 * i] * Crel[0] + (double)c->R[3 * i + 1] * Crel[1] + (double)c->R[3 * i + 2] * Crel[2];
        double Ks[9] = {c->K[0], 0.0, c->K[2], 0.0, c->K[4], c->K[5], 0.0, 0.0, c->K[8]};
        double KR[9], A[9];
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j)
                KR[3 * i + j] = Ks[3 * i] * Rrel[j] + Ks[3 * i + 1] * Rrel[3 + j] + Ks[3 * i + 2] * Rrel[6 + j];
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j)
                A[3 * i + j] = KR[3 * i] * Kri[j] + KR[3 * i + 1] * Kri[3 + j] + KR[3 * i + 2] * Kri[6 + j];
        for (int k = 0; k < 9; ++k) o->A[s][k] = (float)A[k];
        for (int i = 0; i < 3; ++i)
            o->b[s][i] = (float)(Ks[3 * i] * trel[0] + Ks[3 * i + 1] * trel[1] + Ks[3 * i + 2] * trel[2]);
    }
}

static inline void homography(const octx *o, int s, f4 pl, float Hm[9]) {
    float m0 = pl.x * o->ikx;
    float m1 = pl.y * o->iky;
    float m2 = fmaf(-pl.y, o->cyk, fmaf(-pl.x, o->cxk, pl.z));
    float iw = FDIV(1.0f, pl.w);
    m0 *= iw; m1 *= iw; m2 *= iw;
    const float *A = o->A[s], *b = o->b[s];
    Hm[0] = fmaf(-b[0], m0, A[0]); Hm[1] = fmaf(-b[0], m1, A[1]); Hm[2] = fmaf(-b[0], m2, A[2]);
    Hm[3] = fmaf(-b[1], m0, A[3]); Hm[4] = fmaf(-b[1], m1, A[4]); Hm[5] = fmaf(-b[1], m2, A[5]);
    Hm[6] = fmaf(-b[2], m0, A[6]); Hm[7] = fmaf(-b[2], m1, A[7]); Hm[8] = fmaf(-b[2], m2, A[8]);
}

/* ComputeCorrespondingPoint, APD.cu:396-403 */
static inline void project(const float Hm[9], float x, float y, float *ox, float *oy) {
    float X = fmaf(Hm[1], y, fmaf(Hm[0], x, Hm[2]));
    float Y = fmaf(Hm[4], y, fmaf(Hm[3], x, Hm[5]));
    float Z = fmaf(Hm[7], y, fmaf(Hm[6], x, Hm[8]));
    float iz = FDIV(1.0f, Z);
    *ox = X * iz;
    *oy = Y * iz;
}

/* tex2D<float>(ref, x+0.5, y+0.5) at integer x,y: texel with clamp (APD.cu:483,520,531,632,687,2119) */
static inline float tex_ref(const octx *o, int x, int y) {
    return o->img[0][clampi(y, 0, o->H - 1) * o->W + clampi(x, 0, o->W - 1)];
}
/* tex2D<float>(src, x+0.5, y+0.5), linear filter (APD.cu:533,634,689) */
static inline float tex_bilinear(const octx *o, int v, float x, float y) {
    const float *T = o->img[v];
    const int W = o->W, H = o->H;
    x = fminf(fmaxf(x, -1.0f), (float)W);
    y = fminf(fmaxf(y, -1.0f), (float)H);
    int qx = (int)fmaf(x, 256.0f, 512.5f) - 512;
    int qy = (int)fmaf(y, 256.0f, 512.5f) - 512;
    int ix = ((qx + 512) >> 8) - 2, iy = ((qy + 512) >> 8) - 2;
    float a = (float)(qx & 255) * 0.00390625f;
    float b = (float)(qy & 255) * 0.00390625f;
    int x0 = clampi(ix, 0, W - 1), x1 = clampi(ix + 1, 0, W - 1);
    int y0 = clampi(iy, 0, H - 1), y1 = clampi(iy + 1, 0, H - 1);
    float t00 = T[y0 * W + x0], t10 = T[y0 * W + x1], t01 = T[y1 * W + x0], t11 = T[y1 * W + x1];
    float top = fmaf(a, t10 - t00, t00);
    float bot = fmaf(a, t11 - t01, t01);
    return fmaf(b, bot - top, top);
}
/* tex2D<float>(depth, (int)x + 0.5f, (int)y + 0.5f) (APD.cu:885, 2319) */
static inline int trunc_clamp(float x, int n) {
    x = fminf(fmaxf(x, -1.0f), (float)n);
    return clampi((int)x, 0, n - 1);
}

/* ------------------------------------------------------------------------------------------------
 * camera geometry, APD.cu:157-313, 405-423, 831-863
 * ----------------------------------------------------------------------------------------------*/
static inline void normalize3(f4 *v) { /* NormalizeVec3, APD.cu:157-164 */
    float ns = v->x * v->x + v->y * v->y + v->z * v->z;
    float inv = FRSQRT(ns);
    v->x *= inv; v->y *= inv; v->z *= inv;
}
static inline void normalize2(float *x, float *y) { /* NormalizeVec2, APD.cu:166-172 */
    float ns = *x * *x + *y * *y;
    float inv = FRSQRT(ns);
    *x *= inv; *y *= inv;
}
static inline void get3d(const apd_camera *c, float px, float py, float depth, float X[3]) { /* APD.cu:190-202 */
    X[0] = FDIV(depth * (px - c->K[2]), c->K[0]);
    X[1] = FDIV(depth * (py - c->K[5]), c->K[4]);
    X[2] = depth;
}
static inline f4 view_dir(const apd_camera *c, int px, int py, float depth) { /* APD.cu:204-216 */
    float X[3];
    get3d(c, (float)px, (float)py, depth, X);
    float norm = FSQRT(X[0] * X[0] + X[1] * X[1] + X[2] * X[2]);
    f4 v = {FDIV(X[0], norm), FDIV(X[1], norm), FDIV(X[2], norm), 0.0f};
    return v;
}
static inline float dist2origin(const apd_camera *c, int px, int py, float depth, f4 n) { /* APD.cu:218-223 */
    float X[3];
    get3d(c, (float)px, (float)py, depth, X);
    return -(n.x * X[0] + n.y * X[1] + n.z * X[2]);
}
static inline float depth_from_plane(const apd_camera *c, f4 pl, int px, int py) { /* APD.cu:237-240 */
    return FDIV(-pl.w * c->K[0],
                (((float)px - c->K[2]) * pl.x + FDIV(c->K[0], c->K[4]) * ((float)py - c->K[5]) * pl.y + c->K[0] * pl.z));
}
static f4 random_normal(const apd_camera *c, int px, int py, orng *g, float depth) { /* APD.cu:242-268 */
    float q1 = 1.0f, q2 = 1.0f, s = 2.0f;
    while (s >= 1.0f) {
        q1 = 2.0f * orng_uniform(g) - 1.0f;
        q2 = 2.0f * orng_uniform(g) - 1.0f;
        s = q1 * q1 + q2 * q2;
    }
    float sq = FSQRT(1.0f - s);
    f4 n = {2.0f * q1 * sq, 2.0f * q2 * sq, 1.0f - 2.0f * s, 0.0f};
    f4 vd = view_dir(c, px, py, depth);
    float dot = n.x * vd.x + n.y * vd.y + n.z * vd.z;
    if (dot > 0.0f) { n.x = -n.x; n.y = -n.y; n.z = -n.z; }
    normalize3(&n);
    return n;
}
static f4 perturbed_normal(const apd_camera *c, int px, int py, f4 n, orng *g, float pert) { /* APD.cu:270-305 */
    f4 vd = view_dir(c, px, py, 1.0f);
    float a1 = (orng_uniform(g) - 0.5f) * pert;
    float a2 = (orng_uniform(g) - 0.5f) * pert;
    float a3 = (orng_uniform(g) - 0.5f) * pert;
    float s1 = o_sinf(a1), s2 = o_sinf(a2), s3 = o_sinf(a3);
    float c1 = o_cosf(a1), c2 = o_cosf(a2), c3 = o_cosf(a3);
    float R[9];
    R[0] = c2 * c3;
    R[1] = c3 * s1 * s2 - c1 * s3;
    R[2] = s1 * s3 + c1 * c3 * s2;
    R[3] = c2 * s3;
    R[4] = c1 * c3 + s1 * s2 * s3;
    R[5] = c1 * s2 * s3 - c3 * s1;
    R[6] = -s2;
    R[7] = c2 * s1;
    R[8] = c1 * c2;
    f4 p = {R[0] * n.x + R[1] * n.y + R[2] * n.z, R[3] * n.x + R[4] * n.y + R[5] * n.z,
            R[6] * n.x + R[7] * n.y + R[8] * n.z, n.w};
    if (p.x * vd.x + p.y * vd.y + p.z * vd.z >= 0.0f) p = n;
    normalize3(&p);
    return p;
}
static inline f4 to_world(const apd_camera *c, f4 p) { /* TransformNormal, APD.cu:405-413 */
    f4 r = {c->R[0] * p.x + c->R[3] * p.y + c->R[6] * p.z, c->R[1] * p.x + c->R[4] * p.y + c->R[7] * p.z,
            c->R[2] * p.x + c->R[5] * p.y + c->R[8] * p.z, p.w};
    return r;
}
static inline f4 to_ref(const apd_camera *c, f4 p) { /* TransformNormal2RefCam, APD.cu:415-423 */
    f4 r = {c->R[0] * p.x + c->R[1] * p.y + c->R[2] * p.z, c->R[3] * p.x + c->R[4] * p.y + c->R[5] * p.z,
            c->R[6] * p.x + c->R[7] * p.y + c->R[8] * p.z, p.w};
    return r;
}
static inline void world_point(const apd_camera *c, float x, float y, float depth, float P[3]) { /* APD.cu:831-851 */
    float X0 = FDIV(depth * (x - c->K[2]), c->K[0]);
    float X1 = FDIV(depth * (y - c->K[5]), c->K[4]);
    float X2 = depth;
    float t0 = c->R[0] * X0 + c->R[3] * X1 + c->R[6] * X2;
    float t1 = c->R[1] * X0 + c->R[4] * X1 + c->R[7] * X2;
    float t2 = c->R[2] * X0 + c->R[5] * X1 + c->R[8] * X2;
    P[0] = t0 + c->c[0]; P[1] = t1 + c->c[1]; P[2] = t2 + c->c[2];
}
static inline void project_cam(const float P[3], const apd_camera *c, float *px, float *py, float *d) { /* APD.cu:853-863 */
    float t0 = c->R[0] * P[0] + c->R[1] * P[1] + c->R[2] * P[2] + c->t[0];
    float t1 = c->R[3] * P[0] + c->R[4] * P[1] + c->R[5] * P[2] + c->t[1];
    float t2 = c->R[6] * P[0] + c->R[7] * P[1] + c->R[8] * P[2] + c->t[2];
    float dd = c->K[6] * t0 + c->K[7] * t1 + c->K[8] * t2;
    *px = (c->K[0] * t0 + c->K[1] * t1 + c->K[2] * t2) / dd;
    *py = (c->K[3] * t0 + c->K[4] * t1 + c->K[5] * t2) / dd;
    *d = dd;
}

/* ------------------------------------------------------------------------------------------------
 * matching costs
 * ----------------------------------------------------------------------------------------------*/
static inline float ncc_finalize(float sr, float srr, float ss, float sss, float srs, float wsum) {
    float inv = FDIV(1.0f, wsum);
    sr *= inv; srr *= inv; ss *= inv; sss *= inv; srs *= inv;
    float var_ref = fmaf(-sr, sr, srr);
    float var_src = fmaf(-ss, ss, sss);
    if (var_ref < 1e-5f || var_src < 1e-5f) return COST_MAX;
    float covar = fmaf(-sr, ss, srs);
    float vrs = FSQRT(var_ref * var_src);
    return fmaxf(0.0f, fminf(COST_MAX, 1.0f - FDIV(covar, vrs)));
}

/* ComputeBilateralNCCOld, APD.cu:596-721 */
float o_ncc_old(const octx *o, int px, int py, int s, f4 pl) {
    const int W = o->W, H = o->H;
    float Hm[9];
    homography(o, s, pl, Hm);
    float ptx, pty;
    project(Hm, (float)px, (float)py, &ptx, &pty);
    if (ptx >= (float)W || ptx < 0.0f || pty >= (float)H || pty < 0.0f) return COST_MAX;
    const uint8_t cid = o->sa[py * W + px];
    int pidx = clampi((int)fmaf(pty, (float)W, ptx), 0, o->HW - 1);
    float sr = 0.0f, srr = 0.0f, ss = 0.0f, sss = 0.0f, srs = 0.0f, wsum = 0.0f;
    if (o->sa[pidx] == 0) {
        for (int i = -5; i <= 5; i += 2) {
            for (int j = -5; j <= 5; j += 2) {
                int rx = px + i, ry = py + j;
                float r = tex_ref(o, rx, ry);
                float sx, sy;
                project(Hm, (float)rx, (float)ry, &sx, &sy);
                float v = tex_bilinear(o, s, sx, sy);
                sr += r; srr = fmaf(r, r, srr);
                ss += v; sss = fmaf(v, v, sss);
                srs = fmaf(r, v, srs);
                wsum += 1.0f;
            }
        }
    } else {
        static const int sign[8] = {1, 1, -1, -1, 1, -1, -1, 1};
        static const int off[18] = {1, 1, 3, 1, 1, 3, 1, 5, 3, 3, 5, 1, 5, 3, 3, 5, 5, 5};
        for (int q = 0; q < 4; ++q) {
            for (int j = 0; j < 9; ++j) {
                int rx = px + off[2 * j] * sign[2 * q];
                int ry = py + off[2 * j + 1] * sign[2 * q + 1];
                if (rx < 0 || rx >= W || ry < 0 || ry >= H) continue;
                if (o->sa[ry * W + rx] != cid) break;
                float r = tex_ref(o, rx, ry);
                float sx, sy;
                project(Hm, (float)rx, (float)ry, &sx, &sy);
                float v = tex_bilinear(o, s, sx, sy);
                sr += r; srr = fmaf(r, r, srr);
                ss += v; sss = fmaf(v, v, sss);
                srs = fmaf(r, v, srs);
                wsum += 1.0f;
            }
        }
    }
    return ncc_finalize(sr, srr, ss, sss, srs, wsum);
}

static inline int16_t anchor_x(const octx *o, int pix, int k) { return RD(o, anchors, 2 * (RD(o, amap, pix) * ANCHOR_NUM + k)); }
static inline int16_t anchor_y(const octx *o, int pix, int k) { return RD(o, anchors, 2 * (RD(o, amap, pix) * ANCHOR_NUM + k) + 1); }

/* sa label at a possibly out-of-image linear index (APD.cu:494,527 read it unchecked): inside the
   H*W buffer -> that byte; outside -> treated as a label mismatch. Returns -1 for "outside". */
static inline int sa_at(const octx *o, int x, int y) {
    long idx = (long)y * o->W + x;
    if (idx < 0 || idx >= o->HW) return -1;
    return o->sa[idx];
}

/* Softmax, APD.cu:431-446 */
static void softmax(float *c, int n) {
    float mx = -1e10f;
    for (int i = 0; i < n; ++i) if (c[i] > mx) mx = c[i];
    float sum = 0.0f;
    for (int i = 0; i < n; ++i) { c[i] = o_expf(c[i] - mx); sum += c[i]; }
    for (int i = 0; i < n; ++i) c[i] /= sum;
}

/* ComputeBilateralNCCNew (deformable NCC with focal-weighted anchors), APD.cu:448-593 */
float o_ncc_new(const octx *o, int px, int py, int s, f4 pl) {
    const int W = o->W, H = o->H;
    const int center = px + py * W;
    const uint8_t cid = o->sa[center];
    const int use_sa = (cid != 0);
    float Hm[9];
    homography(o, s, pl, Hm);
    float ptx, pty;
    project(Hm, (float)px, (float)py, &ptx, &pty);
    if (ptx >= (float)W || ptx < 0.0f || pty >= (float)H || pty < 0.0f) return COST_MAX;
    if (RD(o, weak, center) != WEAK) return 0.0f; /* printf("error") branch, unreachable */
    float strong_costs[9];
    int ns = 0;
    float center_cost = 0.0f, strong_weight = 0.0f;
    for (int k = 0; k < ANCHOR_NUM; ++k) {
        int ax = anchor_x(o, center, k), ay = anchor_y(o, center, k);
        if (ax == -1 || ay == -1) continue;
        if (use_sa && sa_at(o, ax, ay) != cid) continue;
        float asx, asy;
        project(Hm, (float)ax, (float)ay, &asx, &asy);
        if (asx < 0 || asy < 0 || asx >= (float)W || asy >= (float)H) {
            if (k != 0) {
                if (is_set(RD(o, sel, ax + ay * W), s - 1)) { strong_costs[ns++] = COST_MAX; strong_weight += 1.0f; }
                continue;
            }
            return COST_MAX;
        }
        const int radius = 5, inc = (k == 0) ? 2 : 5;
        float sr = 0.0f, srr = 0.0f, ss = 0.0f, sss = 0.0f, srs = 0.0f, wsum = 0.0f;
        for (int i = -radius; i <= radius; i += inc) {
            for (int j = -radius; j <= radius; j += inc) {
                int rx = ax + i, ry = ay + j;
                if (use_sa && sa_at(o, rx, ry) != cid) continue;
                float r = tex_ref(o, rx, ry);
                float sx, sy;
                project(Hm, (float)rx, (float)ry, &sx, &sy);
                float v = tex_bilinear(o, s, sx, sy);
                sr += r; srr = fmaf(r, r, srr);
                ss += v; sss = fmaf(v, v, sss);
                srs = fmaf(r, v, srs);
                wsum += 1.0f;
            }
        }
        if (wsum == 0.0f) continue;
        float c = ncc_finalize(sr, srr, ss, sss, srs, wsum);
        if (k == 0) center_cost = c;
        else { strong_costs[ns++] = c; strong_weight += 1.0f; }
    }
    if (strong_weight <= 1e-6f) return center_cost;
    float w[9];
    for (int i = 0; i < ns; ++i) w[i] = strong_costs[i];
    softmax(w, ns);
    float sc = 0.0f;
    for (int i = 0; i < ns; ++i) sc = fmaf(w[i], strong_costs[i], sc);
    sc = CV_MIN(sc, COST_MAX);
    return (float)(0.25 * (double)center_cost + 0.75 * (double)sc);
}

/* ComputeGeomConsistencyCost, APD.cu:865-902 */
float o_geom_cost(const octx *o, int px, int py, int s, f4 pl) {
    const apd_camera *rc = &o->cam[0], *sc = &o->cam[s];
    float depth = depth_from_plane(rc, pl, px, py);
    float P[3];
    world_point(rc, (float)px, (float)py, depth, P);
    float sx, sy, sd;
    project_cam(P, sc, &sx, &sy, &sd);
    float src_depth = o->dep[s][trunc_clamp(sy, o->H) * o->W + trunc_clamp(sx, o->W)];
    if (src_depth == 0.0f) return 3.0f;
    float Q[3];
    world_point(sc, sx, sy, src_depth, Q);
    float bx, by, rd;
    project_cam(Q, rc, &bx, &by, &rd);
    float dx = (float)px - bx, dy = (float)py - by;
    float e = FSQRT(dx * dx + dy * dy);
    return fminf(3.0f, e);
}

/* ------------------------------------------------------------------------------------------------
 * kernels (one function per __global__ of APD.cu), pixel-level
 * ----------------------------------------------------------------------------------------------*/

/* RandomInitialization + ComputeMultiViewInitialCostandSelectedViews, APD.cu:919-948, 723-774 */
static void k_random_init(octx *o, int px, int py) {
    const int c = py * o->W + px;
    const apd_camera *cam = &o->cam[0];
    if (o->P.state == APD_FIRST_INIT) {
        orng g;
        orng_init(&g, o->seed, (uint32_t)c, ORD_INIT);
        float depth = orng_uniform(&g) * (o->P.depth_max - o->P.depth_min) + o->P.depth_min;
        f4 n = random_normal(cam, px, py, &g, depth);
        n.w = dist2origin(cam, px, py, depth, n);
        WR(o, plane, c) = n;
    } else {
        f4 n = to_ref(cam, RD(o, plane, c));
        float depth = n.w;
        n.w = dist2origin(cam, px, py, depth, n);
        WR(o, plane, c) = n;
    }
    f4 pl = RD(o, plane, c);
    const int N = o->N;
    const int use_new = o->P.use_APD && RD(o, weak, c) == WEAK;
    float cv[32], sorted[32];
    int nvalid = 0;
    for (int i = 1; i <= N; ++i) {
        float v = use_new ? o_ncc_new(o, px, py, i, pl) : o_ncc_old(o, px, py, i, pl);
        cv[i - 1] = v;
        sorted[i - 1] = v;
        if (v < COST_MAX) nvalid++;
    }
    /* sort_small, APD.cu:3-12 */
    for (int i = 1; i < N; ++i) {
        float t = sorted[i];
        int j;
        for (j = i; j >= 1 && t < sorted[j - 1]; j--) sorted[j] = sorted[j - 1];
        sorted[j] = t;
    }
    /* The reference writes selected_views[center] here while ComputeBilateralNCCNew of other WEAK pixels
       reads the anchors' selected_views in the same launch (APD.cu:502 vs 755-766): a race on
       uninitialised memory. Defined here as launch-start snapshot: results go to sel_next. */
    WR(o, sel_next, c) = 0;
    int top_k = nvalid < o->P.top_k ? nvalid : o->P.top_k;
    if (top_k > 0) {
        float cost = 0.0f;
        for (int i = 0; i < top_k; ++i) cost += sorted[i];
        float thr = sorted[top_k - 1];
        uint32_t sv = 0;
        for (int i = 0; i < N; ++i) if (cv[i] <= thr) sv |= (1u << i);
        WR(o, sel_next, c) = sv;
        WR(o, cost, c) = FDIV(cost, (float)top_k);
    } else {
        WR(o, cost, c) = COST_MAX;
    }
}

/* Multi-hypothesis joint view selection shared by the Strong/Weak sweeps, APD.cu:1339-1374 / 1505-1540 */
static void view_selection(const octx *o, float ca[8][32], const float *prior, int iter, orng *g, uint8_t *vw) {
    const int N = o->N;
    float thr = (float)(0.8 * (double)o_expf(FDIV((float)(iter * iter), (-90.0f))));
    float sp[32];
    for (int i = 0; i < N; ++i) {
        float count = 0.0f, tmpw = 0.0f;
        int cf = 0;
        for (int j = 0; j < 8; ++j) {
            float c = ca[j][i];
            if (c < thr) { tmpw += o_expf(FDIV(c * c, (-0.18f))); count += 1.0f; }
            if (c > 1.2f) cf++;
        }
        float p = 0.0f;
        if (count > 2 && cf < 3) p = FDIV(tmpw, count);
        else if (cf < 3) p = o_expf(FDIV(thr * thr, (-0.32f)));
        sp[i] = p * prior[i];
    }
    /* TransformPDFToCDF, APD.cu:174-188 */
    float sum = 0.0f;
    for (int i = 0; i < N; ++i) sum += sp[i];
    float inv = FDIV(1.0f, sum), cum = 0.0f;
    for (int i = 0; i < N; ++i) { cum = fmaf(sp[i], inv, cum); sp[i] = cum; }
    for (int i = 0; i < APD_MAX_IMAGES; ++i) vw[i] = 0;
    for (int smp = 0; smp < 15; ++smp) {
        float u = orng_uniform(g) - FLT_EPSILON;
        for (int i = 0; i < N; ++i) {
            if (sp[i] > u) { vw[i] += 1; break; }
        }
    }
}

/* PlaneHypothesisRefinementStrong / Weak candidate generation, APD.cu:961-980 / 1054-1067 */
static void refine_candidates(const octx *o, int px, int py, orng *g, f4 cur, float depth, float dcand[5], f4 ncand[5]) {
    const apd_camera *cam = &o->cam[0];
    const float dmin = o->P.depth_min, dmax = o->P.depth_max;
    float depth_rand = orng_uniform(g) * (dmax - dmin) + dmin;
    f4 nrand = random_normal(cam, px, py, g, depth);
    float dp = depth;
    const float dminp = (1 - 0.02f) * dp;
    const float dmaxp = (1 + 0.02f) * dp;
    int guard = 0;
    do {
        dp = orng_uniform(g) * (dmaxp - dminp) + dminp;
    } while (dp < dmin && dp > dmax && ++guard < 64);
    const float pert = (float)((double)0.02f * M_PI_D);
    f4 npert = perturbed_normal(cam, px, py, cur, g, pert);
    dcand[0] = depth_rand; dcand[1] = depth; dcand[2] = depth_rand; dcand[3] = depth; dcand[4] = dp;
    ncand[0] = cur; ncand[1] = nrand; ncand[2] = nrand; ncand[3] = npert; ncand[4] = cur;
}

/* CheckerboardPropagationStrong + PlaneHypothesisRefinementStrong, APD.cu:1098-1440, 950-1006 */
static void k_sweep_strong(octx *o, int px, int py, int iter) {
    const int W = o->W, H = o->H, N = o->N;
    const apd_camera *cam = &o->cam[0];
    const int c = py * W + px;
    float ca[8][32];
    memset(ca, 0, sizeof(ca));
    ca[0][0] = 2.0f; /* float cost_array[8][32] = {2.0f} */
    int flag[8] = {0};
    int pos[8];
    float cmin;
    int cminp;
    /* 0 up_near, 1 up_far, 2 down_near, 3 down_far, 4 left_near, 5 left_far, 6 right_near, 7 right_far */
    int up_near = c - W, up_far = c - 3 * W, down_near = c + W, down_far = c + 3 * W;
    int left_near = c - 1, left_far = c - 3, right_near = c + 1, right_far = c + 3;
    if (py > 2) {
        flag[1] = 1; cmin = RD(o, cost, up_far); cminp = up_far;
        for (int i = 1; i < 11; ++i)
            if (py > 2 + 2 * i) { int t = up_far - 2 * i * W; if (RD(o, cost, t) < cmin) { cmin = RD(o, cost, t); cminp = t; } }
        up_far = cminp;
    }
    if (py < H - 3) {
        flag[3] = 1; cmin = RD(o, cost, down_far); cminp = down_far;
        for (int i = 1; i < 11; ++i)
            if (py < H - 3 - 2 * i) { int t = down_far + 2 * i * W; if (RD(o, cost, t) < cmin) { cmin = RD(o, cost, t); cminp = t; } }
        down_far = cminp;
    }
    if (px > 2) {
        flag[5] = 1; cmin = RD(o, cost, left_far); cminp = left_far;
        for (int i = 1; i < 11; ++i)
            if (px > 2 + 2 * i) { int t = left_far - 2 * i; if (RD(o, cost, t) < cmin) { cmin = RD(o, cost, t); cminp = t; } }
        left_far = cminp;
    }
    if (px < W - 3) {
        flag[7] = 1; cmin = RD(o, cost, right_far); cminp = right_far;
        for (int i = 1; i < 11; ++i)
            if (px < W - 3 - 2 * i) { int t = right_far + 2 * i; if (RD(o, cost, t) < cmin) { cmin = RD(o, cost, t); cminp = t; } }
        right_far = cminp;
    }
    if (py > 0) {
        flag[0] = 1; cmin = RD(o, cost, up_near); cminp = up_near;
        for (int i = 0; i < 3; ++i) {
            if (py > 1 + i && px > i) { int t = up_near - (1 + i) * W - (i + 1); if (RD(o, cost, t) < cmin) { cmin = RD(o, cost, t); cminp = t; } }
            if (py > 1 + i && px < W - 1 - i) { int t = up_near - (1 + i) * W + (i + 1); if (RD(o, cost, t) < cmin) { cmin = RD(o, cost, t); cminp = t; } }
        }
        up_near = cminp;
    }
    if (py < H - 1) {
        flag[2] = 1; cmin = RD(o, cost, down_near); cminp = down_near;
        for (int i = 0; i < 3; ++i) {
            if (py < H - 2 - i && px > i) { int t = down_near + (1 + i) * W - (i + 1); if (RD(o, cost, t) < cmin) { cmin = RD(o, cost, t); cminp = t; } }
            if (py < H - 2 - i && px < W - 1 - i) { int t = down_near + (1 + i) * W + (i + 1); if (RD(o, cost, t) < cmin) { cmin = RD(o, cost, t); cminp = t; } }
        }
        down_near = cminp;
    }
    if (px > 0) {
        flag[4] = 1; cmin = RD(o, cost, left_near); cminp = left_near;
        for (int i = 0; i < 3; ++i) {
            if (px > 1 + i && py > i) { int t = left_near - (1 + i) - (i + 1) * W; if (RD(o, cost, t) < cmin) { cmin = RD(o, cost, t); cminp = t; } }
            if (px > 1 + i && py < H - 1 - i) { int t = left_near - (1 + i) + (i + 1) * W; if (RD(o, cost, t) < cmin) { cmin = RD(o, cost, t); cminp = t; } }
        }
        left_near = cminp;
    }
    if (px < W - 1) {
        flag[6] = 1; cmin = RD(o, cost, right_near); cminp = right_near;
        for (int i = 0; i < 3; ++i) {
            if (px < W - 2 - i && py > i) { int t = right_near + (1 + i) - (i + 1) * W; if (RD(o, cost, t) < cmin) { cmin = RD(o, cost, t); cminp = t; } }
            if (px < W - 2 - i && py < H - 1 - i) { int t = right_near + (1 + i) + (i + 1) * W; if (RD(o, cost, t) < cmin) { cmin = RD(o, cost, t); cminp = t; } }
        }
        right_near = cminp;
    }
    pos[0] = up_near; pos[1] = up_far; pos[2] = down_near; pos[3] = down_far;
    pos[4] = left_near; pos[5] = left_far; pos[6] = right_near; pos[7] = right_far;
    for (int j = 0; j < 8; ++j)
        if (flag[j])
            for (int i = 1; i <= N; ++i) ca[j][i - 1] = o_ncc_old(o, px, py, i, RD(o, plane, pos[j]));

    /* view selection priors, APD.cu:1323-1337 */
    float prior[32] = {0};
    const int nb[4] = {c - W, c + W, c - 1, c + 1};
    for (int i = 0; i < 4; ++i)
        if (flag[2 * i])
            for (int j = 0; j < N; ++j) prior[j] += is_set(RD(o, sel, nb[i]), j) ? 0.9f : 0.1f;
    orng g;
    orng_init(&g, o->seed, (uint32_t)c, ORD_STRONG(iter));
    uint8_t vw[APD_MAX_IMAGES];
    view_selection(o, ca, prior, iter, &g, vw);
    uint32_t tsel = 0;
    float wn = 0.0f;
    for (int i = 0; i < N; ++i) if (vw[i] > 0) { tsel |= 1u << i; wn += (float)vw[i]; }
    float fc[8];
    for (int j = 0; j < 8; ++j) {
        float acc = 0.0f;
        for (int i = 0; i < N; ++i) if (vw[i] > 0) acc = fmaf((float)vw[i], ca[j][i], acc);
        fc[j] = FDIV(acc, wn);
    }
    int mi = 0; /* FindMinCostIndex, APD.cu:60-71 */
    { float m = fc[0]; for (int j = 1; j < 8; ++j) if (fc[j] <= m) { m = fc[j]; mi = j; } }

    const int geom_imp = o->P.geom_consistency && o->P.use_impetus;
    const float gf = o->P.geom_factor;
    f4 cur = RD(o, plane, c);
    float cost_now = 0.0f;
    for (int i = 0; i < N; ++i) {
        float v = o_ncc_old(o, px, py, i + 1, cur);
        if (geom_imp) v = fmaf(gf, o_geom_cost(o, px, py, i + 1, cur), v);
        cost_now = fmaf((float)vw[i], v, cost_now);
    }
    cost_now /= wn;
    const float cost_init = cost_now;
    float depth_now = depth_from_plane(cam, cur, px, py);
    f4 pnow = cur;
    if (flag[mi]) {
        f4 cand = RD(o, plane, pos[mi]);
        float db = depth_from_plane(cam, cand, px, py);
        if (db >= o->P.depth_min && db <= o->P.depth_max && fc[mi] < cost_now) {
            depth_now = db; pnow = cand; cost_now = fc[mi];
            WR(o, sel, c) = tsel;
        }
    }
    /* PlaneHypothesisRefinementStrong, APD.cu:950-1006 */
    float dc[5];
    f4 nc[5];
    refine_candidates(o, px, py, &g, pnow, depth_now, dc, nc);
    for (int k = 0; k < 5; ++k) {
        f4 t = nc[k];
        t.w = dist2origin(cam, px, py, dc[k], t);
        float tc = 0.0f;
        for (int i = 0; i < N; ++i) {
            float v = o_ncc_old(o, px, py, i + 1, t);
            if (geom_imp) v = fmaf(gf, o_geom_cost(o, px, py, i + 1, t), v);
            tc = fmaf((float)vw[i], v, tc);
        }
        tc /= wn;
        float db = depth_from_plane(cam, t, px, py);
        if (db >= o->P.depth_min && db <= o->P.depth_max && tc < cost_now) {
            depth_now = db; pnow = t; cost_now = tc;
        }
    }
    if (o->P.state == APD_REFINE_INIT) {
        if ((double)cost_now < (double)cost_init - 0.1) { WR(o, cost, c) = cost_now; WR(o, plane, c) = pnow; }
        else WR(o, cost, c) = cost_init;
    } else {
        WR(o, cost, c) = cost_now; WR(o, plane, c) = pnow;
    }
    for (int i = 0; i < N; ++i) WR(o, vw, (size_t)i * o->HW + c) = vw[i];
}

#ifdef ORACLE_WEAK_STATS
/* Measurement build only (tools/weak_bound_stats.py): how many Weak-refinement evaluations lower
 * bounds could reject before the anchor windows. NCC-New = COST_MAX when the centre or its anchor
 * projects out of the source, else (float)(0.25 * cc + 0.75 * acc) with acc >= 0, so
 * lb = (float)(0.25 * (double)cc) (or COST_MAX) never exceeds it; fmaf(gf, geom, .) and the weighted
 * fmaf chain are monotone. */
static float o_ncc_new_centre_lb(const octx *o, int px, int py, int s, f4 pl) {
    const int W = o->W, H = o->H;
    const int center = px + py * W;
    float Hm[9];
    homography(o, s, pl, Hm);
    float ptx, pty;
    project(Hm, (float)px, (float)py, &ptx, &pty);
    if (ptx >= (float)W || ptx < 0.0f || pty >= (float)H || pty < 0.0f) return COST_MAX;
    int ax = anchor_x(o, center, 0), ay = anchor_y(o, center, 0);
    if (ax == -1 || ay == -1) return 0.0f;
    float asx, asy;
    project(Hm, (float)ax, (float)ay, &asx, &asy);
    if (asx < 0 || asy < 0 || asx >= (float)W || asy >= (float)H) return COST_MAX;
    float sr = 0.0f, srr = 0.0f, ss = 0.0f, sss = 0.0f, srs = 0.0f, wsum = 0.0f;
    for (int i = -5; i <= 5; i += 2)
        for (int j = -5; j <= 5; j += 2) {
            float r = tex_ref(o, ax + i, ay + j);
            float sx, sy;
            project(Hm, (float)(ax + i), (float)(ay + j), &sx, &sy);
            float v = tex_bilinear(o, s, sx, sy);
            sr += r; srr = fmaf(r, r, srr); ss += v; sss = fmaf(v, v, sss); srs = fmaf(r, v, srs); wsum += 1.0f;
        }
    return (float)(0.25 * (double)ncc_finalize(sr, srr, ss, sss, srs, wsum));
}
/* [0] candidates (fit + refinement), [1] weighted-view evaluations, [2] with the per-view prefix exit,
 * [3] rejected by the geometric bound, [4] by the centre + geometric bound, [5] anchor-window
 * evaluations left with the centre + geometric bound then the prefix exit, [6] candidates accepted */
static long long g_wstats[8];
long long oracle_weak_stats(int i) { return (i >= 0 && i < 8) ? g_wstats[i] : -1; }
void oracle_weak_stats_reset(void) { memset(g_wstats, 0, sizeof(g_wstats)); }
static void weak_stats(const octx *o, int px, int py, f4 t, const uint8_t *vw, float wn, float thr) {
    const int N = o->N, geom = o->P.geom_consistency;
    const float gf = o->P.geom_factor;
    long long st[8] = {0};
    float full[32], lbg[32], lbc[32];
    st[0] = 1;
    for (int i = 0; i < N; ++i) {
        if (!vw[i]) continue;
        const float g = geom ? o_geom_cost(o, px, py, i + 1, t) : 0.0f;
        const float nn = o_ncc_new(o, px, py, i + 1, t);
        full[i] = geom ? fmaf(gf, g, nn) : nn;
        lbg[i] = geom ? fmaf(gf, g, 0.0f) : 0.0f;
        const float lc = o_ncc_new_centre_lb(o, px, py, i + 1, t);
        lbc[i] = geom ? fmaf(gf, g, lc) : lc;
        st[1]++;
    }
    float P = 0.0f, Pg = 0.0f, Pc = 0.0f;
    int stop = 0;
    for (int i = 0; i < N; ++i) {
        if (!vw[i]) continue;
        if (!stop) { st[2]++; P = fmaf((float)vw[i], full[i], P); if (FDIV(P, wn) >= thr) stop = 1; }
        Pg = fmaf((float)vw[i], lbg[i], Pg);
        Pc = fmaf((float)vw[i], lbc[i], Pc);
    }
    if (FDIV(Pg, wn) >= thr) st[3] = 1;
    if (FDIV(Pc, wn) >= thr) st[4] = 1;
    else {  /* survivors: anchor windows with the prefix exit */
        float Q = 0.0f;
        for (int i = 0; i < N; ++i) {
            if (!vw[i]) continue;
            st[5]++;
            Q = fmaf((float)vw[i], full[i], Q);
            if (FDIV(Q, wn) >= thr) break;
        }
    }
    if (!stop) st[6] = 1;
#pragma omp critical
    for (int i = 0; i < 8; ++i) g_wstats[i] += st[i];
}
#endif

/* CheckerboardPropagationWeak + PlaneHypothesisRefinementWeak, APD.cu:1442-1615, 1008-1096 */
static void k_sweep_weak(octx *o, int px, int py, int iter) {
    const int W = o->W, N = o->N;
    const apd_camera *cam = &o->cam[0];
    const int c = py * W + px;
    float ca[8][32];
    memset(ca, 0, sizeof(ca));
    ca[0][0] = 2.0f;
    int flag[8] = {0}, pos[8] = {0};
    f4 newp[8];
    for (int i = 0; i < 8; ++i) {
        int ax = anchor_x(o, c, i + 1), ay = anchor_y(o, c, i + 1);
        if (ax == -1 || ay == -1 || RD(o, weak, ax + ay * W) != STRONG) continue;
        pos[i] = ax + ay * W;
        flag[i] = 1;
        for (int s = 1; s <= N; ++s) ca[i][s - 1] = o_ncc_new(o, px, py, s, RD(o, plane, pos[i]));
        newp[i] = RD(o, plane, pos[i]);
    }
    float prior[32] = {0};
    for (int i = 0; i < 8; ++i) {
        int ax = anchor_x(o, c, i + 1), ay = anchor_y(o, c, i + 1);
        if (ax == -1 || ay == -1) continue;
        for (int j = 0; j < N; ++j) prior[j] += is_set(RD(o, sel, ax + ay * W), j) ? 0.9f : 0.1f;
    }
    orng g;
    orng_init(&g, o->seed, (uint32_t)c, ORD_WEAK(iter));
    uint8_t vw[APD_MAX_IMAGES];
    view_selection(o, ca, prior, iter, &g, vw);
    uint32_t tsel = 0;
    float wn = 0.0f;
    for (int i = 0; i < N; ++i) if (vw[i] > 0) { tsel |= 1u << i; wn += (float)vw[i]; }
    const int geom = o->P.geom_consistency;
    const float gf = o->P.geom_factor;
    float fc[8];
    for (int j = 0; j < 8; ++j) {
        float acc = 0.0f;
        for (int i = 0; i < N; ++i) {
            if (vw[i] > 0) {
                float v = ca[j][i];
                if (geom) v = flag[j] ? fmaf(gf, o_geom_cost(o, px, py, i + 1, RD(o, plane, pos[j])), v) : fmaf(gf, 3.0f, v);
                acc = fmaf((float)vw[i], v, acc);
            }
        }
        fc[j] = FDIV(acc, wn);
    }
    int mi = 0;
    { float m = fc[0]; for (int j = 1; j < 8; ++j) if (fc[j] <= m) { m = fc[j]; mi = j; } }
    f4 cur = RD(o, plane, c);
    float cost_now = 0.0f;
    for (int i = 0; i < N; ++i) {
        float v = o_ncc_new(o, px, py, i + 1, cur);
        if (geom) v = fmaf(gf, o_geom_cost(o, px, py, i + 1, cur), v);
        cost_now = fmaf((float)vw[i], v, cost_now);
    }
    cost_now /= wn;
    const float cost_init = cost_now;
    float depth_now = depth_from_plane(cam, cur, px, py);
    f4 pnow = cur;
    if (flag[mi]) {
        float db = depth_from_plane(cam, newp[mi], px, py);
        if (db >= o->P.depth_min && db <= o->P.depth_max && fc[mi] < cost_now) {
            depth_now = db; pnow = newp[mi]; cost_now = fc[mi];
            WR(o, sel, c) = tsel;
        }
    }
    /* PlaneHypothesisRefinementWeak, APD.cu:1008-1096 */
    f4 fit = RD(o, fit, c);
    if (!(fit.x == 0 && fit.y == 0 && fit.z == 0)) {
#ifdef ORACLE_WEAK_STATS
        weak_stats(o, px, py, fit, vw, wn, cost_now);
#endif
        {
            float tc = 0.0f;
            for (int i = 0; i < N; ++i) {
                if (vw[i] > 0) {
                    float v = o_ncc_new(o, px, py, i + 1, fit);
                    if (geom) v = fmaf(gf, o_geom_cost(o, px, py, i + 1, fit), v);
                    tc = fmaf((float)vw[i], v, tc);
                }
            }
            tc /= wn;
            float db = depth_from_plane(cam, fit, px, py);
            if (db >= o->P.depth_min && db <= o->P.depth_max && tc < cost_now) { depth_now = db; pnow = fit; cost_now = tc; }
        }
        float dc[5];
        f4 nc[5];
        refine_candidates(o, px, py, &g, pnow, depth_now, dc, nc);
#ifdef ORACLE_WEAK_STATS
        const float thr5 = cost_now;  /* the GPU's exit threshold: the cost after the fit plane */
#endif
        for (int k = 0; k < 5; ++k) {
            f4 t = nc[k];
            t.w = dist2origin(cam, px, py, dc[k], t);
#ifdef ORACLE_WEAK_STATS
            weak_stats(o, px, py, t, vw, wn, thr5);
#endif
            float tc = 0.0f;
            for (int i = 0; i < N; ++i) {
                if (vw[i] > 0) {
                    float v = o_ncc_new(o, px, py, i + 1, t);
                    if (geom) v = fmaf(gf, o_geom_cost(o, px, py, i + 1, t), v);
                    tc = fmaf((float)vw[i], v, tc);
                }
            }
            tc /= wn;
            float db = depth_from_plane(cam, t, px, py);
            if (db >= o->P.depth_min && db <= o->P.depth_max && tc < cost_now) { depth_now = db; pnow = t; cost_now = tc; }
        }
    }
    if (o->P.state == APD_REFINE_INIT) {
        if ((double)cost_now < (double)cost_init - 0.1) { WR(o, cost, c) = cost_now; WR(o, plane, c) = pnow; }
        else WR(o, cost, c) = cost_init;
    } else {
        WR(o, cost, c) = cost_now; WR(o, plane, c) = pnow;
    }
    for (int i = 0; i < N; ++i) WR(o, vw, (size_t)i * o->HW + c) = vw[i];
}

/* PointinTriangle, APD.cu:122-143 */
static int point_in_triangle(int ax, int ay, int bx, int by, int cx, int cy, int px, int py) {
    float ABx = (float)(bx - ax), ABy = (float)(by - ay);
    float BCx = (float)(cx - bx), BCy = (float)(cy - by);
    float CAx = (float)(ax - cx), CAy = (float)(ay - cy);
    float AB = FSQRT(ABx * ABx + ABy * ABy), BC = FSQRT(BCx * BCx + BCy * BCy), CA = FSQRT(CAx * CAx + CAy * CAy);
    if (AB <= 2 || BC <= 2 || CA <= 2) return 0;
    if (!(AB + BC > CA && BC + CA > AB && AB + CA > BC)) return 0;
    float PAx = (float)(ax - px), PAy = (float)(ay - py);
    float PBx = (float)(bx - px), PBy = (float)(by - py);
    float PCx = (float)(cx - px), PCy = (float)(cy - py);
    float t1 = PAx * PBy - PAy * PBx;
    float t2 = PBx * PCy - PBy * PCx;
    float t3 = PCx * PAy - PCy * PAx;
    return t1 * t2 >= 0 && t1 * t3 >= 0;
}

/* FindNearestStrongPoint, APD.cu:2434-2484 (brute force, as the reference) */
static void k_find_nearest(octx *o, int px, int py) {
    const int W = o->W, H = o->H, c = px + py * W;
    int16_t *out = &o->nearest[2 * c];
    RC_SPAN_W(o, nearest, 2 * c, 2);
    out[0] = -1; out[1] = -1;
    const uint8_t cc = RD(o, conf, c);
    if (RD(o, weak, c) == WEAK || RD(o, weak, c) == UNKNOWN) {
        uint8_t bc = 0;
        int bx = -1, by = -1;
        float md = FLT_MAX;
        for (int x = -100; x <= 100; ++x) {
            for (int y = -100; y <= 100; ++y) {
                int tx = px + x, ty = py + y;
                if (tx < 0 || tx >= W || ty < 0 || ty >= H) continue;
                int t = tx + ty * W;
                if (RD(o, weak, t) != STRONG) continue;
                if (RD(o, conf, t) < cc) continue;
                float d = FSQRT((float)(x * x + y * y));
                if (d < md) { md = d; bx = tx; by = ty; bc = RD(o, conf, t); }
                else if (d == md) { if (RD(o, conf, t) > bc) { bx = tx; by = ty; bc = RD(o, conf, t); } }
            }
        }
        out[0] = (int16_t)bx; out[1] = (int16_t)by;
    } else if (RD(o, weak, c) == STRONG) {
        out[0] = (int16_t)px; out[1] = (int16_t)py;
    }
}

/* per-launch constants of GenAnchors computed in double like the reference (APD.cu:1897-1901) */
typedef struct { float cos_a, sin_a, thr; int shift; } anchor_consts;
static anchor_consts make_anchor_consts(int rotate_time) {
    anchor_consts k;
    float angle = FDIV(45.0f, (float)rotate_time);
    k.cos_a = (float)cos((double)angle * M_PI_D / 180.0f);
    k.sin_a = (float)sin((double)angle * M_PI_D / 180.0f);
    k.thr = (float)cos((double)(angle / 2.0f) * M_PI_D / 180.0f);
    int sr = (int)(tan((double)(angle / 2.0f) * M_PI_D / 180.0f) * 20);
    k.shift = CV_MAX(sr, 1);
    return k;
}

/* GenAnchors, APD.cu:1857-2082 */
static void k_gen_anchors(octx *o, int px, int py, anchor_consts K) {
    const int W = o->W, H = o->H, c = px + py * W;
    if (RD(o, weak, c) != WEAK) return;
    const int margin = 6;
    const float depth_diff = o->P.depth_max - o->P.depth_min;
    const apd_camera *cam = &o->cam[0];
    int16_t *anc = &o->anchors[2 * (RD(o, amap, c) * ANCHOR_NUM)];
    RC_SPAN_W(o, anchors, 2 * (RD(o, amap, c) * ANCHOR_NUM), 2 * ANCHOR_NUM);
    orng g;
    orng_init(&g, o->seed, (uint32_t)c, ORD_ANCHORS);
    for (int i = 0; i < ANCHOR_NUM; ++i) { anc[2 * i] = -1; anc[2 * i + 1] = -1; }
    anc[0] = (int16_t)px; anc[1] = (int16_t)py;
    int spx[32], spy[32], dvalid[32];
    for (int i = 0; i < 32; ++i) { spx[i] = -1; spy[i] = -1; dvalid[i] = 0; }
    int odi = -1, nsp = 0;
    const int rt = o->P.rotate_time;
    const unsigned shift = (unsigned)K.shift;
    for (int odx = -1; odx <= 1; ++odx) {
        for (int ody = -1; ody <= 1; ++ody) {
            if (odx == 0 && ody == 0) continue;
            float dx = (float)odx, dy = (float)ody;
            normalize2(&dx, &dy);
            odi++;
            for (int ri = 0; ri < rt; ++ri) {
                int di = odi * 4 + ri;
                for (int radius = 2; radius <= APD_MAX_SEARCH_RADIUS; radius = CV_MIN(radius * 2, radius + 25)) {
                    float tx = (float)px + dx * (float)radius, ty = (float)py + dy * (float)radius;
                    if (tx < 0 || ty < 0 || tx >= (float)W || ty >= (float)H) break;
                    for (int t = 0; t < 4; ++t) {
                        uint32_t sx = orng_u32(&g);
                        uint32_t mx = orng_u32(&g);
                        int rxs = (int)(((sx % 2u == 0) ? mx : (0u - mx)) % shift);
                        uint32_t sy = orng_u32(&g);
                        uint32_t my = orng_u32(&g);
                        int rys = (int)(((sy % 2u == 0) ? my : (0u - my)) % shift);
                        float ddx = dx * 20 + (float)rxs, ddy = dy * 20 + (float)rys;
                        normalize2(&ddx, &ddy);
                        int ax = (int16_t)(int)((float)px + ddx * (float)radius);
                        int ay = (int16_t)(int)((float)py + ddy * (float)radius);
                        if (ax < margin || ay < margin || ax >= W - margin || ay >= H - margin) continue;
                        int ac = ax + ay * W;
                        int nx = RD(o, nearest, 2 * ac), ny = RD(o, nearest, 2 * ac + 1);
                        if (nx == -1 || ny == -1) continue;
                        float tdx = (float)(nx - px), tdy = (float)(ny - py);
                        normalize2(&tdx, &tdy);
                        float ca = tdx * dx + tdy * dy;
                        if (ca > K.thr) { spx[di] = nx; spy[di] = ny; dvalid[di] = 1; nsp++; break; }
                    }
                    if (dvalid[di]) break;
                }
                float rx = dx * K.cos_a - dy * K.sin_a;
                float ry = dx * K.sin_a + dy * K.cos_a;
                normalize2(&rx, &ry);
                dx = rx; dy = ry;
            }
        }
    }
    if (nsp <= 3) { WR(o, reliable, c) = 0; return; }
    int vx[32], vy[32], vc = 0;
    float v3[32][3];
    float X[3];
    get3d(cam, (float)px, (float)py, RD(o, plane, c).w, X);
    float cw[3] = {X[0], X[1], X[2]};
    for (int i = 0; i < 32; ++i) {
        vx[i] = -1; vy[i] = -1;
        if (dvalid[i]) {
            int sc = spx[i] + spy[i] * W;
            vx[vc] = spx[i]; vy[vc] = spy[i];
            get3d(cam, (float)spx[i], (float)spy[i], RD(o, plane, sc).w, X);
            v3[vc][0] = X[0]; v3[vc][1] = X[1]; v3[vc][2] = X[2];
            vc++;
        }
    }
    f4 best = {0, 0, 0, 0};
    int ua = -1, ub = -1, uc = -1, has = 0;
    float min_cost = FLT_MAX;
    int max_count = 3;
    for (int it = 0; it < 50; ++it) {
        int a = (int)(orng_u32(&g) % (uint32_t)vc);
        int b = (int)(orng_u32(&g) % (uint32_t)vc);
        int cc = (int)(orng_u32(&g) % (uint32_t)vc);
        if (a == b || b == cc || a == cc) continue;
        if (!point_in_triangle(vx[a], vy[a], vx[b], vy[b], vx[cc], vy[cc], px, py)) continue;
        const float *A = v3[a], *B = v3[b], *C = v3[cc];
        float ACx = A[0] - C[0], ACy = A[1] - C[1], ACz = A[2] - C[2];
        float BCx = B[0] - C[0], BCy = B[1] - C[1], BCz = B[2] - C[2];
        f4 cr = {ACy * BCz - BCy * ACz, -(ACx * BCz - BCx * ACz), ACx * BCy - BCx * ACy, 0.0f};
        if ((cr.x == 0 && cr.y == 0 && cr.z == 0) || isnan(cr.x) || isnan(cr.y) || isnan(cr.z)) continue;
        normalize3(&cr);
        cr.w = -(cr.x * A[0] + cr.y * A[1] + cr.z * A[2]);
        int tcnt = 0;
        float sd = 0.0f;
        for (int k = 0; k < vc; ++k) {
            float d = fabsf(cr.x * v3[k][0] + cr.y * v3[k][1] + cr.z * v3[k][2] + cr.w);
            if (FDIV(d, depth_diff) < o->P.ransac_threshold) { tcnt++; sd += d; }
        }
        if (tcnt < 6) continue;
        if (tcnt > max_count) {
            max_count = tcnt;
            min_cost = fabsf(cr.x * cw[0] + cr.y * cw[1] + cr.z * cw[2] + cr.w);
            best = cr; has = 1; ua = a; ub = b; uc = cc;
        } else if (tcnt == max_count) {
            float cd = fabsf(cr.x * cw[0] + cr.y * cw[1] + cr.z * cw[2] + cr.w);
            if (cd < min_cost) { min_cost = cd; best = cr; ua = a; ub = b; uc = cc; }
        }
    }
    if (!has) { WR(o, reliable, c) = 0; return; }
    float wgt[32];
    for (int i = 0; i < vc; ++i) {
        float d = fabsf(best.x * v3[i][0] + best.y * v3[i][1] + best.z * v3[i][2] + best.w);
        if (FDIV(d, depth_diff) >= o->P.ransac_threshold) { vx[i] = -1; vy[i] = -1; wgt[i] = FLT_MAX; continue; }
        if (i == ua || i == ub || i == uc) d -= 1;
        wgt[i] = d;
    }
    /* sort_small_weighted, APD.cu:25-38 */
    for (int i = 1; i < vc; ++i) {
        int tx = vx[i], ty = vy[i];
        float tw = wgt[i];
        int j;
        for (j = i; j >= 1 && tw < wgt[j - 1]; j--) { vx[j] = vx[j - 1]; vy[j] = vy[j - 1]; wgt[j] = wgt[j - 1]; }
        vx[j] = tx; vy[j] = ty; wgt[j] = tw;
    }
    for (int i = 1; i < ANCHOR_NUM; ++i) { anc[2 * i] = (int16_t)vx[i - 1]; anc[2 * i + 1] = (int16_t)vy[i - 1]; }
    WR(o, reliable, c) = 1;
}

/* RANSACToGetFitPlane, APD.cu:2486-2598 */
static void k_ransac_fit(octx *o, int px, int py, int iter) {
    const int W = o->W, c = px + py * W;
    if (RD(o, weak, c) != WEAK) { WR(o, fit, c) = RD(o, plane, c); return; }
    const apd_camera *cam = &o->cam[0];
    int sx[8], sy[8], cnt = 0;
    float s3[8][3], X[3];
    for (int i = 1; i < ANCHOR_NUM; ++i) {
        int ax = anchor_x(o, c, i), ay = anchor_y(o, c, i);
        if (ax == -1 || ay == -1) continue;
        sx[cnt] = ax; sy[cnt] = ay;
        float d = depth_from_plane(cam, RD(o, plane, ax + ay * W), ax, ay);
        get3d(cam, (float)ax, (float)ay, d, X);
        s3[cnt][0] = X[0]; s3[cnt][1] = X[1]; s3[cnt][2] = X[2];
        cnt++;
    }
    if (cnt < 3) { WR(o, fit, c) = RD(o, plane, c); return; }
    orng g;
    orng_init(&g, o->seed, (uint32_t)c, ORD_FIT(iter));
    float min_cost = FLT_MAX;
    f4 best = {0, 0, 0, 0};
    int has = 0;
    for (int it = 0; it < 50; ++it) {
        int a = (int)(orng_u32(&g) % (uint32_t)cnt);
        int b = (int)(orng_u32(&g) % (uint32_t)cnt);
        int cc = (int)(orng_u32(&g) % (uint32_t)cnt);
        if (a == b || b == cc || a == cc) continue;
        if (!point_in_triangle(sx[a], sy[a], sx[b], sy[b], sx[cc], sy[cc], px, py)) continue;
        const float *A = s3[a], *B = s3[b], *C = s3[cc];
        float ACx = A[0] - C[0], ACy = A[1] - C[1], ACz = A[2] - C[2];
        float BCx = B[0] - C[0], BCy = B[1] - C[1], BCz = B[2] - C[2];
        f4 cr = {ACy * BCz - BCy * ACz, -(ACx * BCz - BCx * ACz), ACx * BCy - BCx * ACy, 0.0f};
        if ((cr.x == 0 && cr.y == 0 && cr.z == 0) || isnan(cr.x) || isnan(cr.y) || isnan(cr.z)) continue;
        normalize3(&cr);
        cr.w = -(cr.x * A[0] + cr.y * A[1] + cr.z * A[2]);
        float tc = 0.0f;
        for (int k = 0; k < cnt; ++k) {
            if (k == a || k == b || k == cc) continue;
            tc += fabsf(cr.x * s3[k][0] + cr.y * s3[k][1] + cr.z * s3[k][2] + cr.w);
        }
        if (tc < min_cost) { min_cost = tc; best = cr; has = 1; }
        if (min_cost == 0) break;
    }
    if (has) {
        float d = depth_from_plane(cam, RD(o, plane, c), px, py);
        f4 vd = view_dir(cam, px, py, d);
        float dot = best.x * vd.x + best.y * vd.y + best.z * vd.z;
        if (dot > 0) { best.x = -best.x; best.y = -best.y; best.z = -best.z; best.w = -best.w; }
        WR(o, fit, c) = best;
    } else {
        f4 z = {0, 0, 0, 0};
        WR(o, fit, c) = z;
    }
}

/* GetDepthandNormal, APD.cu:1694-1709 */
static void k_depth_normal(octx *o, int px, int py) {
    const int c = py * o->W + px;
    f4 p = RD(o, plane, c);
    p.w = depth_from_plane(&o->cam[0], p, px, py);
    WR(o, plane, c) = to_world(&o->cam[0], p);
}

/* CheckerboardFilterStrong, APD.cu:1711-1821 */
static void k_filter(octx *o, int px, int py) {
    const int W = o->W, H = o->H, c = py * W + px;
    float f[21];
    int n = 0;
    f[n++] = RD(o, plane, c).w;
    const int left = c - 1, leftleft = c - 3, up = c - W, upup = c - 3 * W;
    const int down = c + W, downdown = c + 3 * W, right = c + 1, rightright = c + 3;
    if (RD(o, cost, c) < 0.001f) return;
#define FADD(cond, idx) if ((cond) && RD(o, weak, (idx)) == STRONG) f[n++] = RD(o, plane, (idx)).w
    FADD(py > 0, up);
    FADD(py > 2, upup);
    FADD(py > 4, upup - W * 2);
    FADD(py < H - 1, down);
    FADD(py < H - 3, downdown);
    FADD(py < H - 5, downdown + W * 2);
    FADD(px > 0, left);
    FADD(px > 2, leftleft);
    FADD(px > 4, leftleft - 2);
    FADD(px < W - 1, right);
    FADD(px < W - 3, rightright);
    FADD(px < W - 5, rightright + 2);
    FADD(py > 0 && px < W - 2, up + 2);
    FADD(py < H - 1 && px < W - 2, down + 2);
    FADD(py > 0 && px > 1, up - 2);
    FADD(py < H - 1 && px > 1, down - 2);
    FADD(px > 0 && py > 2, left - W * 2);
    FADD(px < W - 1 && py > 2, right - W * 2);
    FADD(px > 0 && py < H - 2, left + W * 2);
    FADD(px < W - 1 && py < H - 2, right + W * 2);
#undef FADD
    for (int i = 1; i < n; ++i) {
        float t = f[i];
        int j;
        for (j = i; j >= 1 && t < f[j - 1]; j--) f[j] = f[j - 1];
        f[j] = t;
    }
    int m = n / 2;
    WR(o, plane, c).w = (n % 2 == 0) ? (f[m - 1] + f[m]) / 2 : f[m];
}

/* DepthToWeak's classification of a 61-sample cost curve (disparities -30..30), APD.cu:2200-2249:
   local minima ("peaks") at samples 2..58; WEAK unless the lowest one lies within weak_peak_radius of
   the centre and costs <= 0.5; then a single peak is STRONG iff it costs <= 0.15, several are STRONG
   iff the other peaks' cost spread sqrt(sum (c_i - c_min)^2) / (count - 1) exceeds 0.2. */
static int o_classify_curve(const float *pc, int weak_peak_radius) {
    int is_peak[61] = {0};
    int count = 0, min_peak = 0;
    float min_cost = 2.0f;
    for (int i = 2; i < 59; ++i) {
        if (pc[i - 1] > pc[i] && pc[i + 1] > pc[i]) {
            is_peak[i] = 1; count++;
            if (pc[i] < min_cost) { min_peak = i; min_cost = pc[i]; }
        }
    }
    if (abs(min_peak - 30) > weak_peak_radius || pc[min_peak] > 0.5f) return WEAK;
    if (count == 1) return (pc[min_peak] <= 0.15f) ? STRONG : WEAK;
    float var = 0.0f;
    for (int i = 2; i < 59; ++i) {
        if (is_peak[i] && i != min_peak) { float d = pc[i] - min_cost; var = fmaf(d, d, var); }
    }
    var = FSQRT(var);
    var /= (float)(count - 1);
    return (var > 0.2f) ? STRONG : WEAK;
}

/* DepthToWeak, APD.cu:2103-2250 */
static void k_depth_to_weak(octx *o, int px, int py) {
    const int W = o->W, H = o->H, c = px + py * W, N = o->N;
    if (px < 6 || py < 6 || px >= W - 6 || py >= H - 6) { WR(o, weak, c) = UNKNOWN; return; }
    const apd_camera *cam = &o->cam[0];
    f4 pl = to_ref(cam, RD(o, plane, c));
    float od = pl.w;
    if (od == 0) { WR(o, weak, c) = UNKNOWN; return; }
    const uint32_t sv = RD(o, sel, c);
    float base = 0.0f, wn = 0.0f;
    int valid = 0;
    for (int s = 1; s <= N; ++s) {
        if (is_set(sv, s - 1)) {
            wn += (float)RD(o, vw, (size_t)(s - 1) * o->HW + c);
            float d0 = cam->c[0] - o->cam[s].c[0], d1 = cam->c[1] - o->cam[s].c[1], d2 = cam->c[2] - o->cam[s].c[2];
            base += FSQRT(d0 * d0 + d1 * d1 + d2 * d2);
            valid++;
        }
    }
    if (valid == 0) { WR(o, weak, c) = UNKNOWN; return; }
    base /= (float)valid;
    float disp = FDIV(cam->K[0] * base, od);
    float pc[61];
    const int geom = o->P.geom_consistency;
    const float gf = o->P.geom_factor;
    for (int pd = -30; pd <= 30; ++pd) {
        float pdepth = FDIV(cam->K[0] * base, (disp + (float)pd));
        if (pdepth < o->P.depth_min || pdepth > o->P.depth_max) { pc[pd + 30] = 2.0f; continue; }
        f4 t = pl;
        t.w = dist2origin(cam, px, py, pdepth, t);
        float p = 0.0f;
        for (int s = 1; s <= N; ++s) {
            if (is_set(sv, s - 1)) {
                float tc = o_ncc_old(o, px, py, s, t);
                if (geom) tc = fmaf(gf, o_geom_cost(o, px, py, s, t), tc);
                p = fmaf(tc, (float)RD(o, vw, (size_t)(s - 1) * o->HW + c), p);
            }
        }
        p /= wn;
        pc[pd + 30] = CV_MIN(2.0f, p);
    }
    if (o->curve) {
        RC_SPAN_W(o, curve, (size_t)c * 61, 61);
        memcpy(&o->curve[(size_t)c * 61], pc, sizeof(pc));
    }
    WR(o, weak, c) = (uint8_t)o_classify_curve(pc, o->P.weak_peak_radius);
}

/* ConfidenceCompute, APD.cu:2282-2344 */
static void k_confidence(octx *o, int px, int py) {
    const int W = o->W, c = px + py * W;
    WR(o, conf, c) = 0;
    const apd_camera *rc = &o->cam[0];
    const uint32_t sv = RD(o, sel, c);
    const float rd = RD(o, plane, c).w;
    if (rd <= 0.0f) { WR(o, weak, c) = UNKNOWN; return; }
    float P[3];
    world_point(rc, (float)px, (float)py, rd, P);
    int nc = 1;
    for (int i = 0; i < o->N; ++i) {
        if (!is_set(sv, i)) continue;
        const int s = i + 1;
        const apd_camera *sc = &o->cam[s];
        float sx, sy, sd;
        project_cam(P, sc, &sx, &sy, &sd);
        float src_depth = o->dep[s][trunc_clamp(sy, o->H) * W + trunc_clamp(sx, W)];
        if (src_depth <= 0.0f) continue;
        nc += 1;
        float Q[3];
        world_point(sc, sx, sy, src_depth, Q);
        float bx, by, refd;
        project_cam(Q, rc, &bx, &by, &refd);
        float dx = (float)px - bx, dy = (float)py - by;
        if (FSQRT(dx * dx + dy * dy) <= 2.0f) nc += 2;
        if (FDIV(fabsf(rd - refd), rd) <= 0.02f) nc += 2;
    }
    if (nc > 255) nc = 255;
    WR(o, conf, c) = (uint8_t)nc;
}

/* LocalRefine, APD.cu:2346-2432 */
static void k_local_refine(octx *o, int px, int py) {
    const int W = o->W, c = px + py * W, N = o->N;
    const apd_camera *cam = &o->cam[0];
    f4 pl = to_ref(cam, RD(o, plane, c));
    float od = pl.w;
    if (od == 0) return;
    const uint32_t sv = RD(o, sel, c);
    const int geom = o->P.geom_consistency;
    const float gf = o->P.geom_factor;
    float cost_now = 0.0f, base = 0.0f, wn = 0.0f;
    int valid = 0;
    for (int s = 1; s <= N; ++s) {
        if (is_set(sv, s - 1)) {
            f4 t = pl;
            t.w = dist2origin(cam, px, py, od, t);
            float tc = o_ncc_old(o, px, py, s, t);
            if (geom) tc = fmaf(gf, o_geom_cost(o, px, py, s, t), tc);
            float w = (float)RD(o, vw, (size_t)(s - 1) * o->HW + c);
            cost_now = fmaf(tc, w, cost_now);
            wn += w;
            float d0 = cam->c[0] - o->cam[s].c[0], d1 = cam->c[1] - o->cam[s].c[1], d2 = cam->c[2] - o->cam[s].c[2];
            base += FSQRT(d0 * d0 + d1 * d1 + d2 * d2);
            valid++;
        }
    }
    if (wn == 0 || valid == 0) return;
    cost_now /= wn;
    base /= (float)valid;
    float disp = FDIV(cam->K[0] * base, od);
    float min_cost = 2.0f, best = od;
    for (int pd = -5; pd <= 5; ++pd) {
        float pdepth = FDIV(cam->K[0] * base, (disp + (float)pd));
        if (pdepth < o->P.depth_min || pdepth > o->P.depth_max) continue;
        f4 t = pl;
        t.w = dist2origin(cam, px, py, pdepth, t);
        float tc = 0.0f;
        for (int s = 1; s <= N; ++s) {
            if (is_set(sv, s - 1)) {
                float w = (float)RD(o, vw, (size_t)(s - 1) * o->HW + c);
                tc = fmaf(o_ncc_old(o, px, py, s, t), w, tc);
                if (geom) tc = fmaf(gf * o_geom_cost(o, px, py, s, t), w, tc);
            }
        }
        tc /= wn;
        if (tc < min_cost) { min_cost = tc; best = pdepth; }
    }
    if ((double)(cost_now - min_cost) > 0.1) WR(o, plane, c).w = best;
}

/* ------------------------------------------------------------------------------------------------
 * RunPatchMatch, APD.cu:2663-2737
 * ----------------------------------------------------------------------------------------------*/
#ifndef ORACLE_RACECHECK
#define FOR_ALL(o, body)                                                   \
    _Pragma("omp parallel for schedule(dynamic, 4)")                       \
    for (int py = 0; py < (o)->H; ++py)                                    \
        for (int px = 0; px < (o)->W; ++px) { body; }
#define FOR_COLOUR(o, colour, body)                                        \
    _Pragma("omp parallel for schedule(dynamic, 4)")                       \
    for (int py = 0; py < (o)->row_limit; ++py)                            \
        for (int px = ((py + (colour)) & 1); px < (o)->W; px += 2) { body; }
#else
/* one phase = one launch of the reference: fresh access sets, each pixel a task */
static void rc_phase(const octx *o, const char *fn, int line, int colour) {
    const size_t HW = (size_t)o->HW;
    for (int a = 0; a < RC_COUNT; ++a) {
        size_t n = HW;
        if (a == RC_vw) n = HW * (size_t)o->N;
        else if (a == RC_nearest) n = 2 * HW;
        else if (a == RC_anchors) n = (size_t)(o->weak_count > 0 ? o->weak_count : 1) * ANCHOR_NUM * 2;
        else if (a == RC_curve) n = o->curve ? HW * 61 : 0;
        rc_shadow *sh = &rc_sh[a];
        if (n > sh->cap) {
            free(sh->wr); free(sh->rd);
            sh->wr = (int32_t *)malloc((n ? n : 1) * sizeof(int32_t));
            sh->rd = (int32_t *)malloc((n ? n : 1) * sizeof(int32_t));
            sh->cap = n;
        }
        sh->n = n;
        memset(sh->wr, 0xff, n * sizeof(int32_t));
        memset(sh->rd, 0xff, n * sizeof(int32_t));
    }
    snprintf(rc_phase_name, sizeof rc_phase_name, "%s:%d%s", fn, line,
             colour < 0 ? "" : (colour ? " (colour 1)" : " (colour 0)"));
    rc_phases++;
}
#define FOR_ALL(o, body)                                                   \
    do {                                                                   \
        rc_phase((o), __func__, __LINE__, -1);                             \
        for (int py = 0; py < (o)->H; ++py)                                \
            for (int px = 0; px < (o)->W; ++px) {                          \
                rc_task = py * (o)->W + px;                                \
                body;                                                      \
            }                                                              \
        rc_task = -1;                                                      \
    } while (0)
#define FOR_COLOUR(o, colour, body)                                        \
    do {                                                                   \
        if (rc_merge_colours && (colour)) break;                           \
        rc_phase((o), __func__, __LINE__, rc_merge_colours ? -1 : (colour)); \
        for (int py = 0; py < (o)->row_limit; ++py)                        \
            for (int px = rc_merge_colours ? 0 : ((py + (colour)) & 1); px < (o)->W; \
                 px += rc_merge_colours ? 1 : 2) {                         \
                rc_task = py * (o)->W + px;                                \
                body;                                                      \
            }                                                              \
        rc_task = -1;                                                      \
    } while (0)
#endif

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

static void run_prepare(octx *o) {
    if (o->P.use_APD) {
        FOR_ALL(o, k_find_nearest(o, px, py));
        anchor_consts K = make_anchor_consts(o->P.rotate_time);
        FOR_ALL(o, k_gen_anchors(o, px, py, K));
        FOR_ALL(o, {
            int c = py * o->W + px;
            if (RD(o, weak, c) == WEAK && RD(o, reliable, c) != 1) WR(o, weak, c) = UNKNOWN;
        });
    }
    FOR_ALL(o, k_random_init(o, px, py));
    memcpy(o->sel, o->sel_next, (size_t)o->HW * sizeof(uint32_t));
}
static void run_iteration(octx *o, int it) {
    FOR_COLOUR(o, 0, if (RD(o, weak, py * o->W + px) != WEAK) k_sweep_strong(o, px, py, it));
    FOR_COLOUR(o, 1, if (RD(o, weak, py * o->W + px) != WEAK) k_sweep_strong(o, px, py, it));
    if (o->P.use_APD) {
        FOR_ALL(o, k_ransac_fit(o, px, py, it));
        FOR_COLOUR(o, 0, if (RD(o, weak, py * o->W + px) == WEAK) k_sweep_weak(o, px, py, it));
        FOR_COLOUR(o, 1, if (RD(o, weak, py * o->W + px) == WEAK) k_sweep_weak(o, px, py, it));
    }
}
static void run_finish(octx *o) {
    FOR_ALL(o, k_depth_normal(o, px, py));
    FOR_COLOUR(o, 0, if (RD(o, weak, py * o->W + px) != WEAK) k_filter(o, px, py));
    FOR_COLOUR(o, 1, if (RD(o, weak, py * o->W + px) != WEAK) k_filter(o, px, py));
    FOR_ALL(o, k_depth_to_weak(o, px, py));
    if (o->P.geom_consistency || o->P.use_APD) FOR_ALL(o, k_confidence(o, px, py));
    FOR_ALL(o, k_local_refine(o, px, py));
}

static int ctx_init(octx *o, const apd_problem *pb) {
    memset(o, 0, sizeof(*o));
    if (pb->num_images < 2 || pb->num_images > APD_MAX_IMAGES) return APD_ETOOMANYVIEWS;
    o->W = pb->width; o->H = pb->height; o->HW = o->W * o->H;
    o->NI = pb->num_images; o->N = o->NI - 1;
    o->P = pb->params;
    o->P.num_images = o->NI;
    o->seed = pb->seed;
    int hh = o->H / 2;
    int rl = 32 * ((hh + 15) / 16);
    o->row_limit = rl < o->H ? rl : o->H;
    for (int i = 0; i < o->NI; ++i) {
        o->img[i] = pb->images[i];
        o->cam[i] = pb->cameras[i];
        o->dep[i] = pb->depths ? pb->depths[i] : NULL;
    }
    precompute_homography(o);
    size_t HW = (size_t)o->HW;
    o->plane = (f4 *)calloc(HW, sizeof(f4));
    o->cost = (float *)calloc(HW, sizeof(float));
    o->sel = (uint32_t *)calloc(HW, sizeof(uint32_t));
    o->sel_next = (uint32_t *)calloc(HW, sizeof(uint32_t));
    o->vw = (uint8_t *)calloc(HW * (size_t)o->N, 1);
    o->weak = (uint8_t *)malloc(HW);
    o->conf = (uint8_t *)malloc(HW);
    o->sa_zero = (uint8_t *)calloc(HW, 1);
    o->amap = (int32_t *)malloc(HW * sizeof(int32_t));
    o->reliable = (uint8_t *)calloc(HW, 1);
    o->nearest = (int16_t *)calloc(HW * 2, sizeof(int16_t));
    o->fit = (f4 *)calloc(HW, sizeof(f4));
    if (!o->plane || !o->cost || !o->sel || !o->sel_next || !o->vw || !o->weak || !o->conf || !o->sa_zero || !o->amap ||
        !o->reliable || !o->nearest || !o->fit)
        return APD_ENOMEM;
    o->sa = pb->sa_mask ? pb->sa_mask : o->sa_zero;
    if (pb->params.use_APD && pb->weak_info) memcpy(o->weak, pb->weak_info, HW);
    else memset(o->weak, STRONG, HW);
    if (pb->params.use_APD && pb->confidence) memcpy(o->conf, pb->confidence, HW);
    else memset(o->conf, 1, HW);
    if (pb->params.state != APD_FIRST_INIT && pb->init_planes) memcpy(o->plane, pb->init_planes, HW * sizeof(f4));
    /* anchors_map = running row-major index of WEAK pixels (APD.cpp:627-640) */
    int32_t wc = 0;
    for (size_t i = 0; i < HW; ++i) WR(o, amap, i) = (o->P.use_APD && RD(o, weak, i) == WEAK) ? wc++ : -1;
    o->weak_count = wc;
    o->anchors = (int16_t *)calloc((size_t)(wc > 0 ? wc : 1) * ANCHOR_NUM * 2, sizeof(int16_t));
    if (!o->anchors) return APD_ENOMEM;
    if ((o->P.geom_consistency || o->P.use_APD) && !pb->depths) return APD_EINVAL;
    return APD_OK;
}
static void ctx_free(octx *o) {
    free(o->plane); free(o->cost); free(o->sel); free(o->sel_next); free(o->vw); free(o->weak); free(o->conf);
    free(o->sa_zero); free(o->amap); free(o->reliable); free(o->nearest); free(o->fit); free(o->anchors);
}
static void ctx_output(const octx *o, const apd_outputs *out) {
    size_t HW = (size_t)o->HW;
    if (out->planes) memcpy(out->planes, o->plane, HW * sizeof(f4));
    if (out->weak_info) memcpy(out->weak_info, o->weak, HW);
    if (out->confidence) memcpy(out->confidence, o->conf, HW);
    if (out->costs) memcpy(out->costs, o->cost, HW * sizeof(float));
    if (out->selected_views) memcpy(out->selected_views, o->sel, HW * sizeof(uint32_t));
    if (out->view_weights) memcpy(out->view_weights, o->vw, HW * (size_t)o->N);
    if (out->anchors && o->weak_count > 0) memcpy(out->anchors, o->anchors, (size_t)o->weak_count * ANCHOR_NUM * 2 * sizeof(int16_t));
    if (out->weak_count) *out->weak_count = o->weak_count;
}

/* Full RunPatchMatch on one problem. times (optional, seconds): [prepare, iterations, finish]. */
int oracle_run_patchmatch(const apd_problem *pb, const apd_outputs *out, int nthreads, double *times) {
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#else
    (void)nthreads;
#endif
#ifdef ORACLE_FASTMATH
    /* flush denormals (FTZ | DAZ) in this thread and in the OpenMP team, restored before returning:
       the process's other code (the parity oracle, numpy) shares the thread pool */
    const unsigned csr0 = _mm_getcsr();
    _mm_setcsr(csr0 | 0x8040u);
#ifdef _OPENMP
#pragma omp parallel
    _mm_setcsr(_mm_getcsr() | 0x8040u);
#endif
#endif
    octx *o = (octx *)malloc(sizeof(octx));
    if (!o) return APD_ENOMEM;
    int st = ctx_init(o, pb);
    if (st != APD_OK) { ctx_free(o); free(o); return st; }
    o->curve = out ? out->reliable_curve : NULL;
    double t0 = now_s();
    run_prepare(o);
    double t1 = now_s();
    for (int it = 0; it < o->P.max_iterations; ++it) run_iteration(o, it);
    double t2 = now_s();
    run_finish(o);
    double t3 = now_s();
    if (times) { times[0] = t1 - t0; times[1] = t2 - t1; times[2] = t3 - t2; }
    if (out) ctx_output(o, out);
    ctx_free(o);
    free(o);
#ifdef ORACLE_FASTMATH
#ifdef _OPENMP
#pragma omp parallel
    _mm_setcsr(_mm_getcsr() & ~0x8040u);
#endif
    _mm_setcsr(csr0);
#endif
    return APD_OK;
}

/* Bounded CPU-baseline sample: prepare, then `iters` sweep iterations over only the first
   `max_rows` rows' worth of pixels is not meaningful for a checkerboard, so the baseline instead runs
   the real sweep on the full image and reports per-iteration seconds in times[1]/iters. */
int oracle_time_iterations(const apd_problem *pb, int iters, int nthreads, double *times) {
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#else
    (void)nthreads;
#endif
    octx *o = (octx *)malloc(sizeof(octx));
    if (!o) return APD_ENOMEM;
    int st = ctx_init(o, pb);
    if (st != APD_OK) { ctx_free(o); free(o); return st; }
    double t0 = now_s();
    run_prepare(o);
    double t1 = now_s();
    for (int it = 0; it < iters; ++it) run_iteration(o, it % (o->P.max_iterations > 0 ? o->P.max_iterations : 1));
    double t2 = now_s();
    if (times) { times[0] = t1 - t0; times[1] = t2 - t1; }
    ctx_free(o);
    free(o);
    return APD_OK;
}

/* ---- single-function entry points for known-answer tests (tests/test_oracle_kat.py) ---- */
static int kat_ctx(octx *o, const apd_problem *pb) { return ctx_init(o, pb); }

float oracle_ncc_old(const apd_problem *pb, int px, int py, int src, const float *plane4) {
    octx *o = (octx *)malloc(sizeof(octx));
    float r = -1.0f;
    if (kat_ctx(o, pb) == APD_OK) { f4 p = {plane4[0], plane4[1], plane4[2], plane4[3]}; r = o_ncc_old(o, px, py, src, p); }
    ctx_free(o); free(o);
    return r;
}
float oracle_geom_cost(const apd_problem *pb, int px, int py, int src, const float *plane4) {
    octx *o = (octx *)malloc(sizeof(octx));
    float r = -1.0f;
    if (kat_ctx(o, pb) == APD_OK) { f4 p = {plane4[0], plane4[1], plane4[2], plane4[3]}; r = o_geom_cost(o, px, py, src, p); }
    ctx_free(o); free(o);
    return r;
}
void oracle_homography(const apd_problem *pb, int src, const float *plane4, float *H9) {
    octx *o = (octx *)malloc(sizeof(octx));
    if (kat_ctx(o, pb) == APD_OK) { f4 p = {plane4[0], plane4[1], plane4[2], plane4[3]}; homography(o, src, p, H9); }
    ctx_free(o); free(o);
}
float oracle_depth_from_plane(const apd_camera *cam, const float *plane4, int px, int py) {
    f4 p = {plane4[0], plane4[1], plane4[2], plane4[3]};
    return depth_from_plane(cam, p, px, py);
}
float oracle_dist2origin(const apd_camera *cam, int px, int py, float depth, const float *n4) {
    f4 n = {n4[0], n4[1], n4[2], n4[3]};
    return dist2origin(cam, px, py, depth, n);
}
float oracle_tex_bilinear(const float *img, int W, int H, float x, float y) {
    octx o;
    memset(&o, 0, sizeof(o));
    o.W = W; o.H = H; o.HW = W * H; o.img[1] = img;
    return tex_bilinear(&o, 1, x, y);
}
float oracle_expf(float x) { return o_expf(x); }
float oracle_sinf(float x) { return o_sinf(x); }
float oracle_cosf(float x) { return o_cosf(x); }
void oracle_philox(uint32_t *c4, uint32_t k0, uint32_t k1) { o_philox(c4, k0, k1); }

/* DepthToWeak's curve classification alone (APD.cu:2200-2249). */
int oracle_classify_curve(const float *pc61, int weak_peak_radius) { return o_classify_curve(pc61, weak_peak_radius); }

/* ComputeBilateralNCCNew (APD.cu:448-593) of one (pixel, source, plane) with caller-given anchors
   (9 x (x, y), anchor 0 first) and selected-view bitmasks (H*W); the problem must have use_APD set
   and the pixel WEAK in its weak_info. Returns -1 on a bad context. */
float oracle_ncc_new(const apd_problem *pb, int px, int py, int src, const float *plane4, const int16_t *anchors9,
                     const uint32_t *sel) {
    octx *o = (octx *)malloc(sizeof(octx));
    float r = -1.0f;
    if (kat_ctx(o, pb) == APD_OK && RD(o, amap, px + py * o->W) >= 0) {
        memcpy(&o->anchors[2 * (RD(o, amap, px + py * o->W) * ANCHOR_NUM)], anchors9, ANCHOR_NUM * 2 * sizeof(int16_t));
        if (sel) memcpy(o->sel, sel, (size_t)o->HW * sizeof(uint32_t));
        f4 p = {plane4[0], plane4[1], plane4[2], plane4[3]};
        r = o_ncc_new(o, px, py, src, p);
    }
    ctx_free(o); free(o);
    return r;
}

/* One stage of the post-processing / anchor preparation over the whole image on caller state, for
   the known-answer tests (tests/test_oracle_kat_apd.py). In/out arrays are H*W (planes: 4 floats per
   pixel, (world normal, depth) for stages 0/1 as after GetDepthandNormal):
     stage 0  CheckerboardFilterStrong, black then red non-WEAK pixels (APD.cu:1711-1855): planes
              (in/out), costs (in), weak (in);
     stage 1  ConfidenceCompute (APD.cu:2282-2344): planes (in), sel (in), pb->depths (in), conf
              (out), weak (in/out: UNKNOWN where depth <= 0);
     stage 2  FindNearestStrongPoint (APD.cu:2434-2484): weak, conf (in) -> nearest (out, x, y);
     stage 3  FindNearestStrongPoint + GenAnchors (APD.cu:1857-2082) + NeigbourUpdate
              (APD.cu:2084-2100): planes (in, as during the sweep), weak (in/out), conf (in) ->
              anchors (out, weak_count x 9 x (x, y), row-major WEAK order of the input), reliable (out).
   Returns APD_OK or a negative status. */
int oracle_kat_stage(const apd_problem *pb, int stage, const uint32_t *sel, const float *costs, float *planes,
                     uint8_t *weak, uint8_t *conf, int16_t *nearest, int16_t *anchors, uint8_t *reliable) {
    octx *o = (octx *)malloc(sizeof(octx));
    if (!o) return APD_ENOMEM;
    int st = kat_ctx(o, pb);
    if (st != APD_OK) { ctx_free(o); free(o); return st; }
    const size_t HW = (size_t)o->HW;
    if (planes) memcpy(o->plane, planes, HW * sizeof(f4));
    if (costs) memcpy(o->cost, costs, HW * sizeof(float));
    if (sel) memcpy(o->sel, sel, HW * sizeof(uint32_t));
    if (weak) memcpy(o->weak, weak, HW);
    if (conf) memcpy(o->conf, conf, HW);
    switch (stage) {
    case 0:
        FOR_COLOUR(o, 0, if (RD(o, weak, py * o->W + px) != WEAK) k_filter(o, px, py));
        FOR_COLOUR(o, 1, if (RD(o, weak, py * o->W + px) != WEAK) k_filter(o, px, py));
        break;
    case 1:
        FOR_ALL(o, k_confidence(o, px, py));
        break;
    case 2:
        FOR_ALL(o, k_find_nearest(o, px, py));
        break;
    case 3: {
        FOR_ALL(o, k_find_nearest(o, px, py));
        anchor_consts K = make_anchor_consts(o->P.rotate_time);
        FOR_ALL(o, k_gen_anchors(o, px, py, K));
        FOR_ALL(o, {
            int c = py * o->W + px;
            if (RD(o, weak, c) == WEAK && RD(o, reliable, c) != 1) WR(o, weak, c) = UNKNOWN;
        });
        break;
    }
    default:
        st = APD_EINVAL;
    }
    if (st == APD_OK) {
        if (planes) memcpy(planes, o->plane, HW * sizeof(f4));
        if (weak) memcpy(weak, o->weak, HW);
        if (conf) memcpy(conf, o->conf, HW);
        if (nearest) memcpy(nearest, o->nearest, HW * 2 * sizeof(int16_t));
        if (anchors && o->weak_count > 0) memcpy(anchors, o->anchors, (size_t)o->weak_count * ANCHOR_NUM * 2 * sizeof(int16_t));
        if (reliable) memcpy(reliable, o->reliable, HW);
    }
    ctx_free(o);
    free(o);
    return st;
}

#ifdef ORACLE_RACECHECK
/* access-set report since the last call (and reset): returns the number of conflicts; phases and
 * accesses counted, the first conflict described in `first`. merge_colours: the negative control
 * (see rc_merge_colours) for the runs that follow. */
int64_t oracle_racecheck_report(int merge_colours, int64_t *phases, int64_t *accesses, char *first, int first_len) {
    const int64_t c = rc_conflicts;
    if (phases) *phases = rc_phases;
    if (accesses) *accesses = rc_accesses;
    if (first && first_len > 0) snprintf(first, (size_t)first_len, "%s", rc_conflicts ? rc_first : "");
    rc_conflicts = rc_phases = rc_accesses = 0;
    rc_first[0] = 0;
    rc_merge_colours = merge_colours;
    return c;
}
#endif
