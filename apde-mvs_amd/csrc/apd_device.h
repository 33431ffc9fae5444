// apd_device.h — device building blocks of the MI355X PatchMatch engine (gfx950, wave64).
//
// Numerics contract (shared bit-for-bit with the CPU oracle, which restates it independently):
//   * compiled with -ffp-contract=off; the only fused multiply-adds are explicit fmaf() calls;
//   * IEEE division and sqrt (hipcc default -fhip-fp32-correctly-rounded-divide-sqrt);
//   * exp/sin/cos are the deterministic polynomials below, not the device libm;
//   * bilinear sampling is done in software on a "quad" layout (see sample_quad), with CUDA texture
//     semantics restated: 1/256 fixed-point coordinate, clamp-to-edge (APD.cpp:691-706).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <type_traits>

#define APD_COST_MAX 2.0f
#define APD_WEAK 0
#define APD_STRONG 1
#define APD_UNKNOWN 2
#define APD_FLT_EPSILON 1.19209290e-07f
#define APD_FLT_MAX 3.40282347e+38f

// Device pointers live in the global address space: without the qualifier every load through a
// struct member is a FLAT load (no scalar path, waits on both vmcnt and lgkmcnt).
// Per-problem tables no kernel writes (cameras, per-view homography terms) live in the constant
// address space: loads through them are invariant, so uniform ones become scalar loads even in
// kernels that store to global memory (the noclobber analysis cannot prove that for APD_G).
#if defined(__HIP_DEVICE_COMPILE__)
#define APD_G __attribute__((address_space(1)))
#define APD_C __attribute__((address_space(4)))
#else
#define APD_G
#define APD_C
#endif

namespace apd {

// launch ordinals of the RNG contract (identical to the oracle)
constexpr uint32_t ORD_ANCHORS = 1u;
constexpr uint32_t ORD_INIT = 2u;
__host__ __device__ constexpr uint32_t ord_strong(int i) { return 16u + 3u * (uint32_t)i; }
__host__ __device__ constexpr uint32_t ord_fit(int i) { return 17u + 3u * (uint32_t)i; }
__host__ __device__ constexpr uint32_t ord_weak(int i) { return 18u + 3u * (uint32_t)i; }
constexpr uint32_t RNG_TAG = 0x41504421u;

struct Cam {  // the float part of apd_camera / Camera (main.h:50-61)
    float K[9], R[9], t[3], c[3];
};

struct SrcView {  // H = A - b (n^T Kr^-1)/w   (APD.cu:334-394, regrouped)
    float A[9];
    float b[3];
};

// Kernel arguments: scalars + device pointers. Passed by value (well under the kernarg limit).
struct Args {
    int W, H, HW, N, row_limit, state;
    float dmin, dmax, gf, ransac_thr;
    int geom, impetus, use_apd, peak_radius, rotate_time, sa_any, top_k;
    uint32_t seed_lo, seed_hi;
    float ikx, iky, cxk, cyk;              // Kr^-1 pieces: 1/fx, 1/fy, cx/fx, cy/fy
    float anc_cos, anc_sin, anc_thr;       // GenAnchors per-launch constants (APD.cu:1897-1901)
    int anc_shift;
    // GenAnchors inlier test d / (dmax - dmin) < ransac_thr as d < anc_dlim (d >= 0): the smallest d
    // whose IEEE quotient reaches the threshold, found on the host (the quotient is monotone in d)
    float anc_dlim;
    int anc_dlim_ok;
    size_t qstride;                        // float4 elements per source quad image ((W+1)*(H+1))
    const APD_G float *ref;                // reference image, H*W
    const APD_G float4 *quad;              // source images 1..N in quad layout, view v at (v-1)*qstride
    const APD_G uint32_t *pairs;           // or in fp16 vertical-pair layout (tex_f16), same stride
    int tex_f16;
    int force_slow;                        // test hook: route every NCC-Old window through ncc_old_slow
    const APD_G float *depth;              // [N+1][H*W] depth maps (geom / APD)
    const APD_C SrcView *views;            // [N+1]
    const APD_C Cam *cams;                 // [N+1]
    APD_G float4 *plane;
    APD_G float *cost;
    APD_G uint32_t *sel;
    APD_G uint32_t *sel_next;              // RandomInitialization output (launch-start snapshot of sel)
    APD_G uint8_t *vw;                     // view-major [N][H*W]
    APD_G uint8_t *weak;
    APD_G uint8_t *conf;
    const APD_G uint8_t *sa;
    const APD_G int *amap;
    APD_G short2 *anchors;                 // weak_count*9
    APD_G uint8_t *reliable;
    APD_G short2 *nearest;
    APD_G float4 *fit;
    APD_G float *curve;                    // optional H*W*61
    const APD_G short2 *near_offsets;      // 201*201 offsets sorted by (d^2, x, y)
    const APD_G struct Args *self;         // this struct in device memory, for out-of-line callees
    APD_G unsigned long long *evals;       // profiling only (else null): the APD_PROF_COUNTERS device counters (apd_hip.h)
    // DepthToWeak -> LocalRefine hand-over (view-major kernels; null = off): the NCC-Old and geometric
    // terms of DepthToWeak's samples p_disp = -5..5, which are LocalRefine's, [11][N][tile slots]
    APD_G float *lr_ncc;
    APD_G float *lr_geo;
    // RandomInitialization -> first Weak sweep (null = off): each WEAK pixel's NCC-New of its initial
    // plane per view, [N][H*W], NaN where it read an anchor's selected views
    APD_G float *wcur;
    // anchor-window reference records (APD passes): per pixel q, [0] the 3x3 / step-5 window around q
    // unfiltered, [1] filtered by q's own SA label (when the problem has labels): taps, tap mask and
    // ncc_finalize's reference-side terms -- see AncRec in apd_kernels.hip
    const APD_G uint4 *arec;
    // DepthToWeak's pre-differenced fp16 texels (tex_f16 problems; null = off, see FastTexD): per padded
    // pair position k, {pairs[k], (pairs[k + 1] - pairs[k]) / 256}, same stride as pairs
    const APD_G uint2 *dpairs;
};

// ---------------------------------------------------------------------------------------------
// deterministic math
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ float d_expf(float x) {
    if (x != x) return x;
    if (x > 88.7228394f) return __int_as_float(0x7f800000);
    if (x < -103.972084f) return 0.0f;
    float kf = floorf(fmaf(x, 1.44269502f, 0.5f));
    int k = (int)kf;
    float r = fmaf(kf, -0.693145752f, x);
    r = fmaf(kf, -1.42860677e-06f, r);
    float p = 1.98412698e-04f;
    p = fmaf(p, r, 1.38888889e-03f);
    p = fmaf(p, r, 8.33333333e-03f);
    p = fmaf(p, r, 4.16666667e-02f);
    p = fmaf(p, r, 1.66666667e-01f);
    p = fmaf(p, r, 0.5f);
    p = fmaf(p, r, 1.0f);
    p = fmaf(p, r, 1.0f);
    int k1 = k / 2, k2 = k - k1;
    p *= __int_as_float((k1 + 127) << 23);
    p *= __int_as_float((k2 + 127) << 23);
    return p;
}
__device__ __forceinline__ float d_sinf(float x) {
    float s2 = x * x;
    float p = -2.50521084e-08f;
    p = fmaf(p, s2, 2.75573192e-06f);
    p = fmaf(p, s2, -1.98412698e-04f);
    p = fmaf(p, s2, 8.33333333e-03f);
    p = fmaf(p, s2, -1.66666667e-01f);
    return fmaf(x * s2, p, x);
}
__device__ __forceinline__ float d_cosf(float x) {
    float s2 = x * x;
    float p = 2.08767570e-09f;
    p = fmaf(p, s2, -2.75573192e-07f);
    p = fmaf(p, s2, 2.48015873e-05f);
    p = fmaf(p, s2, -1.38888889e-03f);
    p = fmaf(p, s2, 4.16666667e-02f);
    p = fmaf(p, s2, -0.5f);
    return fmaf(s2, p, 1.0f);
}

// ---------------------------------------------------------------------------------------------
// RNG contract: Philox4x32-10, counter (pixel, ordinal, block, TAG), key = seed
// (replaces curand_init(clock64(), y, x) + XORWOW, APD.cu:904-917)
// ---------------------------------------------------------------------------------------------
struct Rng {
    uint32_t k0, k1, c0, c1, n;
    uint32_t b0, b1, b2, b3;

    __device__ __forceinline__ Rng(uint32_t slo, uint32_t shi, uint32_t pixel, uint32_t ordinal)
        : k0(slo), k1(shi), c0(pixel), c1(ordinal), n(0), b0(0), b1(0), b2(0), b3(0) {}

    __device__ __forceinline__ void refill() {
        uint32_t x0 = c0, x1 = c1, x2 = n >> 2, x3 = RNG_TAG;
        uint32_t key0 = k0, key1 = k1;
#pragma unroll
        for (int r = 0; r < 10; ++r) {
            // (one 32x32 -> 64-bit product each: v_mad_u64_u32 instead of v_mul_lo + v_mul_hi)
            const uint64_t p0 = (uint64_t)0xD2511F53u * x0, p1 = (uint64_t)0xCD9E8D57u * x2;
            const uint32_t lo0 = (uint32_t)p0, hi0 = (uint32_t)(p0 >> 32);
            const uint32_t lo1 = (uint32_t)p1, hi1 = (uint32_t)(p1 >> 32);
            uint32_t n0 = hi1 ^ x1 ^ key0, n2 = hi0 ^ x3 ^ key1;
            x0 = n0; x1 = lo1; x2 = n2; x3 = lo0;
            key0 += 0x9E3779B9u; key1 += 0xBB67AE85u;
        }
        b0 = x0; b1 = x1; b2 = x2; b3 = x3;
    }
    // block `blk` of this stream (draws 4*blk .. 4*blk+3), state untouched
    __device__ __forceinline__ uint4 block(uint32_t blk) const {
        uint32_t x0 = c0, x1 = c1, x2 = blk, x3 = RNG_TAG;
        uint32_t key0 = k0, key1 = k1;
#pragma unroll
        for (int r = 0; r < 10; ++r) {
            // (one 32x32 -> 64-bit product each: v_mad_u64_u32 instead of v_mul_lo + v_mul_hi)
            const uint64_t p0 = (uint64_t)0xD2511F53u * x0, p1 = (uint64_t)0xCD9E8D57u * x2;
            const uint32_t lo0 = (uint32_t)p0, hi0 = (uint32_t)(p0 >> 32);
            const uint32_t lo1 = (uint32_t)p1, hi1 = (uint32_t)(p1 >> 32);
            uint32_t n0 = hi1 ^ x1 ^ key0, n2 = hi0 ^ x3 ^ key1;
            x0 = n0; x1 = lo1; x2 = n2; x3 = lo0;
            key0 += 0x9E3779B9u; key1 += 0xBB67AE85u;
        }
        return make_uint4(x0, x1, x2, x3);
    }
    // curand()
    __device__ __forceinline__ uint32_t u32() {
        uint32_t j = n & 3u;
        if (j == 0) refill();
        n++;
        return j == 0 ? b0 : (j == 1 ? b1 : (j == 2 ? b2 : b3));
    }
    // curand_uniform(): (0,1]
    __device__ __forceinline__ float uniform() { return (float)((u32() >> 8) + 1u) * 5.96046448e-08f; }
};

// ---------------------------------------------------------------------------------------------
// geometry (APD.cu:157-313, 405-423, 831-863) — same operation order as the oracle
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ void normalize3(float4 &v) {
    float ns = v.x * v.x + v.y * v.y + v.z * v.z;
    float inv = 1.0f / sqrtf(ns);
    v.x *= inv; v.y *= inv; v.z *= inv;
}
__device__ __forceinline__ void normalize2(float &x, float &y) {
    float ns = x * x + y * y;
    float inv = 1.0f / sqrtf(ns);
    x *= inv; y *= inv;
}
__device__ __forceinline__ void get3d(const APD_C Cam &c, float px, float py, float depth, float X[3]) {
    X[0] = depth * (px - c.K[2]) / c.K[0];
    X[1] = depth * (py - c.K[5]) / c.K[4];
    X[2] = depth;
}
__device__ __forceinline__ float4 view_dir(const APD_C Cam &c, int px, int py, float depth) {
    float X[3];
    get3d(c, (float)px, (float)py, depth, X);
    float norm = sqrtf(X[0] * X[0] + X[1] * X[1] + X[2] * X[2]);
    return make_float4(X[0] / norm, X[1] / norm, X[2] / norm, 0.0f);
}
__device__ __forceinline__ float dist2origin(const APD_C Cam &c, int px, int py, float depth, float4 n) {
    float X[3];
    get3d(c, (float)px, (float)py, depth, X);
    return -(n.x * X[0] + n.y * X[1] + n.z * X[2]);
}
__device__ __forceinline__ float depth_from_plane(const APD_C Cam &c, float4 pl, int px, int py) {
    return -pl.w * c.K[0] /
           (((float)px - c.K[2]) * pl.x + (c.K[0] / c.K[4]) * ((float)py - c.K[5]) * pl.y + c.K[0] * pl.z);
}
__device__ __forceinline__ float4 random_normal(const APD_C Cam &c, int px, int py, Rng &g, float depth) {
    float q1 = 1.0f, q2 = 1.0f, s = 2.0f;
    while (s >= 1.0f) {
        q1 = 2.0f * g.uniform() - 1.0f;
        q2 = 2.0f * g.uniform() - 1.0f;
        s = q1 * q1 + q2 * q2;
    }
    float sq = sqrtf(1.0f - s);
    float4 n = make_float4(2.0f * q1 * sq, 2.0f * q2 * sq, 1.0f - 2.0f * s, 0.0f);
    float4 vd = view_dir(c, px, py, depth);
    float dot = n.x * vd.x + n.y * vd.y + n.z * vd.z;
    if (dot > 0.0f) { n.x = -n.x; n.y = -n.y; n.z = -n.z; }
    normalize3(n);
    return n;
}
__device__ __forceinline__ float4 perturbed_normal(const APD_C Cam &c, int px, int py, float4 n, Rng &g, float pert) {
    float4 vd = view_dir(c, px, py, 1.0f);
    float a1 = (g.uniform() - 0.5f) * pert;
    float a2 = (g.uniform() - 0.5f) * pert;
    float a3 = (g.uniform() - 0.5f) * pert;
    float s1 = d_sinf(a1), s2 = d_sinf(a2), s3 = d_sinf(a3);
    float c1 = d_cosf(a1), c2 = d_cosf(a2), c3 = d_cosf(a3);
    float R0 = c2 * c3;
    float R1 = c3 * s1 * s2 - c1 * s3;
    float R2 = s1 * s3 + c1 * c3 * s2;
    float R3 = c2 * s3;
    float R4 = c1 * c3 + s1 * s2 * s3;
    float R5 = c1 * s2 * s3 - c3 * s1;
    float R6 = -s2;
    float R7 = c2 * s1;
    float R8 = c1 * c2;
    float4 p = make_float4(R0 * n.x + R1 * n.y + R2 * n.z, R3 * n.x + R4 * n.y + R5 * n.z,
                           R6 * n.x + R7 * n.y + R8 * n.z, n.w);
    if (p.x * vd.x + p.y * vd.y + p.z * vd.z >= 0.0f) p = n;
    normalize3(p);
    return p;
}
__device__ __forceinline__ float4 to_world(const APD_C Cam &c, float4 p) {
    return make_float4(c.R[0] * p.x + c.R[3] * p.y + c.R[6] * p.z, c.R[1] * p.x + c.R[4] * p.y + c.R[7] * p.z,
                       c.R[2] * p.x + c.R[5] * p.y + c.R[8] * p.z, p.w);
}
__device__ __forceinline__ float4 to_ref(const APD_C Cam &c, float4 p) {
    return make_float4(c.R[0] * p.x + c.R[1] * p.y + c.R[2] * p.z, c.R[3] * p.x + c.R[4] * p.y + c.R[5] * p.z,
                       c.R[6] * p.x + c.R[7] * p.y + c.R[8] * p.z, p.w);
}
__device__ __forceinline__ void world_point(const APD_C Cam &c, float x, float y, float depth, float P[3]) {
    float X0 = depth * (x - c.K[2]) / c.K[0];
    float X1 = depth * (y - c.K[5]) / c.K[4];
    float X2 = depth;
    float t0 = c.R[0] * X0 + c.R[3] * X1 + c.R[6] * X2;
    float t1 = c.R[1] * X0 + c.R[4] * X1 + c.R[7] * X2;
    float t2 = c.R[2] * X0 + c.R[5] * X1 + c.R[8] * X2;
    P[0] = t0 + c.c[0]; P[1] = t1 + c.c[1]; P[2] = t2 + c.c[2];
}
__device__ __forceinline__ void project_cam(const float P[3], const APD_C Cam &c, float &px, float &py, float &d) {
    float t0 = c.R[0] * P[0] + c.R[1] * P[1] + c.R[2] * P[2] + c.t[0];
    float t1 = c.R[3] * P[0] + c.R[4] * P[1] + c.R[5] * P[2] + c.t[1];
    float t2 = c.R[6] * P[0] + c.R[7] * P[1] + c.R[8] * P[2] + c.t[2];
    float dd = c.K[6] * t0 + c.K[7] * t1 + c.K[8] * t2;
    px = (c.K[0] * t0 + c.K[1] * t1 + c.K[2] * t2) / dd;
    py = (c.K[3] * t0 + c.K[4] * t1 + c.K[5] * t2) / dd;
    d = dd;
}

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }
__device__ __forceinline__ int trunc_clamp(float x, int n) {
    x = fminf(fmaxf(x, -1.0f), (float)n);
    return clampi((int)x, 0, n - 1);
}

// ---------------------------------------------------------------------------------------------
// homography + projection
// ---------------------------------------------------------------------------------------------
struct Hom { float h[9]; };

// The view-independent part of the homography, n^T Kr^-1 / w (a kernel that evaluates one plane
// in several views may compute it once), and the per-view part H = A - b m.
template <class AT>
__device__ __forceinline__ float3 plane_terms(const AT &a, float4 pl) {
    float m0 = pl.x * a.ikx;
    float m1 = pl.y * a.iky;
    float m2 = fmaf(-pl.y, a.cyk, fmaf(-pl.x, a.cxk, pl.z));
    float iw = 1.0f / pl.w;
    m0 *= iw; m1 *= iw; m2 *= iw;
    return make_float3(m0, m1, m2);
}
template <class AT>
__device__ __forceinline__ Hom homography_terms(const AT &a, int s, float3 m) {
    const APD_C SrcView &V = a.views[s];
    Hom H;
    H.h[0] = fmaf(-V.b[0], m.x, V.A[0]); H.h[1] = fmaf(-V.b[0], m.y, V.A[1]); H.h[2] = fmaf(-V.b[0], m.z, V.A[2]);
    H.h[3] = fmaf(-V.b[1], m.x, V.A[3]); H.h[4] = fmaf(-V.b[1], m.y, V.A[4]); H.h[5] = fmaf(-V.b[1], m.z, V.A[5]);
    H.h[6] = fmaf(-V.b[2], m.x, V.A[6]); H.h[7] = fmaf(-V.b[2], m.y, V.A[7]); H.h[8] = fmaf(-V.b[2], m.z, V.A[8]);
    return H;
}
template <class AT>
__device__ __forceinline__ Hom homography(const AT &a, int s, float4 pl) {
    return homography_terms(a, s, plane_terms(a, pl));
}
__device__ __forceinline__ void project(const Hom &H, float x, float y, float &ox, float &oy) {
    float X = fmaf(H.h[1], y, fmaf(H.h[0], x, H.h[2]));
    float Y = fmaf(H.h[4], y, fmaf(H.h[3], x, H.h[5]));
    float Z = fmaf(H.h[7], y, fmaf(H.h[6], x, H.h[8]));
    float iz = 1.0f / Z;
    ox = X * iz;
    oy = Y * iz;
}

// ---------------------------------------------------------------------------------------------
// texture sampling
// ---------------------------------------------------------------------------------------------
template <class AT>
__device__ __forceinline__ float tex_ref(const AT &a, int x, int y) {
    return a.ref[clampi(y, 0, a.H - 1) * a.W + clampi(x, 0, a.W - 1)];
}
// Quad layout: Q[(iy+1)*(W+1) + (ix+1)] = {T(ix,iy), T(ix+1,iy), T(ix,iy+1), T(ix+1,iy+1)} with
// clamp-to-edge, for ix in [-1, W-1], iy in [-1, H-1] — one 16-byte gather per bilinear sample.
// One bilinear tap: quad index + 1/256 fractions. The coordinate is clamped to [-1, W-1] x [-1, H-1];
// this is bit-identical to clamp-to-edge over [-1, W] x [-1, H] (the oracle's statement), because past
// the last texel both taps of the lerp hold the same texel and fmaf(a, 0, t) == t for any fraction a.
struct QuadTap {
    uint32_t idx;
    float ax, ay;
};
__device__ __forceinline__ QuadTap quad_tap(float Wm1, float Hm1, uint32_t W1, float x, float y) {
    x = fminf(fmaxf(x, -1.0f), Wm1);
    y = fminf(fmaxf(y, -1.0f), Hm1);
    const int qx = (int)fmaf(x, 256.0f, 512.5f);  // floor(256 x + 0.5) + 512, always >= 256
    const int qy = (int)fmaf(y, 256.0f, 512.5f);
    QuadTap t;
    t.idx = __umul24((uint32_t)((qy >> 8) - 1), W1) + (uint32_t)((qx >> 8) - 1);
    t.ax = (float)(qx & 255) * 0.00390625f;
    t.ay = (float)(qy & 255) * 0.00390625f;
    return t;
}
__device__ __forceinline__ float bilerp(const float4 q, float ax, float ay) {
    const float top = fmaf(ax, q.y - q.x, q.x);
    const float bot = fmaf(ax, q.w - q.z, q.z);
    return fmaf(ay, bot - top, top);
}
// Source-image storage, selected per problem by the host:
//  F16 = true : "vertical fp16 pairs", P[(iy+1)*(W+2) + (ix+1)] = {half T(ix,iy), half T(ix,iy+1)}
//               (clamp-to-edge, ix in [-1, W], iy in [-1, H-1]); ONE 8-byte load at tap index idx
//               returns the 2x2 footprint. 4 bytes per texel. Used when every source texel is
//               exactly representable in fp16 (8-bit images and their dyadic INTER_LINEAR
//               downscales are), so the fp32 arithmetic after the exact conversion is unchanged.
//  F16 = false: fp32 quads, Q[(iy+1)*(W+1) + (ix+1)] = {T00, T10, T01, T11}, 16 bytes per texel.
typedef _Float16 apd_h2 __attribute__((ext_vector_type(2)));
struct __attribute__((aligned(4))) apd_u2_a4 { uint32_t x, y; };  // 8-byte load at 4-byte alignment
template <bool F16>
struct SrcTex {
    const APD_G void *base;
    template <class AT>
    __device__ __forceinline__ SrcTex(const AT &a, int s) {
        if constexpr (F16) base = (const APD_G void *)(a.pairs + (size_t)(s - 1) * a.qstride);
        else base = (const APD_G void *)(a.quad + (size_t)(s - 1) * a.qstride);
    }
    static __device__ __forceinline__ uint32_t pitch(int W) { return (uint32_t)(F16 ? W + 2 : W + 1); }
    __device__ __forceinline__ float4 fetch(uint32_t idx) const {
        if constexpr (F16) {
            const apd_u2_a4 v = *(const APD_G apd_u2_a4 *)((const APD_G uint32_t *)base + idx);
            const apd_h2 c0 = __builtin_bit_cast(apd_h2, v.x);  // {T(ix,iy), T(ix,iy+1)}
            const apd_h2 c1 = __builtin_bit_cast(apd_h2, v.y);  // {T(ix+1,iy), T(ix+1,iy+1)}
            return make_float4((float)c0.x, (float)c1.x, (float)c0.y, (float)c1.y);
        } else {
            return ((const APD_G float4 *)base)[idx];
        }
    }
};
template <bool F16>
__device__ __forceinline__ float sample_src(const SrcTex<F16> &T, int W, int H, float x, float y) {
    const QuadTap t = quad_tap((float)(W - 1), (float)(H - 1), SrcTex<F16>::pitch(W), x, y);
    return bilerp(T.fetch(t.idx), t.ax, t.ay);
}

__device__ __forceinline__ float ncc_finalize(float sr, float srr, float ss, float sss, float srs, float wsum) {
    float inv = 1.0f / wsum;
    sr *= inv; srr *= inv; ss *= inv; sss *= inv; srs *= inv;
    float var_ref = fmaf(-sr, sr, srr);
    float var_src = fmaf(-ss, ss, sss);
    if (var_ref < 1e-5f || var_src < 1e-5f) return APD_COST_MAX;
    float covar = fmaf(-sr, ss, srs);
    float vrs = sqrtf(var_ref * var_src);
    return fmaxf(0.0f, fminf(APD_COST_MAX, 1.0f - covar / vrs));
}
// ncc_finalize with its reference-side statements done beforehand (inv = 1 / wsum, srp = sr * inv,
// var_ref = fmaf(-srp, srp, srr * inv)): the same values
__device__ __forceinline__ float ncc_finalize_pre(float inv, float srp, float var_ref, float ss, float sss, float srs) {
    ss *= inv; sss *= inv; srs *= inv;
    float var_src = fmaf(-ss, ss, sss);
    if (var_ref < 1e-5f || var_src < 1e-5f) return APD_COST_MAX;
    float covar = fmaf(-srp, ss, srs);
    float vrs = sqrtf(var_ref * var_src);
    return fmaxf(0.0f, fminf(APD_COST_MAX, 1.0f - covar / vrs));
}

// Reference-side window of ComputeBilateralNCCOld (6x6, radius 5, step 2): fixed per pixel, so it is
// gathered once per pixel into LDS (one copy per pixel, each of the pixel's N lanes fetching a share)
// and read back by broadcast across all 14*N NCC evaluations of a sweep.
// SA quadrant window of ComputeBilateralNCCOld (APD.cu:664-719) for one reference pixel: which of the
// 36 visiting slots (quadrant-major, see sa_dx/sa_dy) the branch visits -- it depends only on the
// image bounds and the SA labels around the pixel -- and its reference moments in visiting order.
struct alignas(16) SaWin {
    uint32_t mlo, mhi;  // visited slots: bit k of (mhi:mlo)
    float sr, srr;      // sum r, sum r*r over the visited slots, in visiting order
};
// RT: the reference taps' storage type in LDS -- float, or _Float16 where the images are exactly
// fp16-representable (the Strong sweep's taps; every read converts exactly to the same fp32 value)
template <class RT = float>
struct RefWinT {
    const RT *r;       // 36 values in LDS, column-major (i*6 + j), element k at r[k * stride]
    float mean, var;   // sum_ref/36 and sum_ref_ref/36 - mean^2, same op order as the oracle
    const SaWin *sa = nullptr;  // view-major kernels with SA masks: the pixel's SaWin in LDS
};
using RefWin = RefWinT<float>;
// mean / variance of a reference window already in LDS (element k at r[k * RS])
template <int RS, class RT = float>
__device__ __forceinline__ RefWinT<RT> refwin_from_lds(const RT *r) {
    float sr = 0.0f, srr = 0.0f;
#pragma unroll
    for (int k = 0; k < 36; ++k) {
        const float x = (float)r[k * RS];
        sr += x;
        srr = fmaf(x, x, srr);
    }
    const float inv = 1.0f / 36.0f;
    sr *= inv;
    srr *= inv;
    RefWinT<RT> w;
    w.r = r;
    w.mean = sr;
    w.var = fmaf(-sr, sr, srr);
    return w;
}

// Visiting slot k (0..35) of the SA branch: quadrant q = k / 9 with signs (+,+), (-,-), (+,-), (-,+)
// (sign[] of APD.cu:664-719), tap j = k % 9 at the odd offsets off[] of that branch.
__host__ __device__ constexpr int sa_off(int j, int c) {
    constexpr int off[18] = {1, 1, 3, 1, 1, 3, 1, 5, 3, 3, 5, 1, 5, 3, 3, 5, 5, 5};
    return off[2 * j + c];
}
__host__ __device__ constexpr int sa_dx(int k) { return sa_off(k % 9, 0) * ((k / 9 == 0 || k / 9 == 2) ? 1 : -1); }
__host__ __device__ constexpr int sa_dy(int k) { return sa_off(k % 9, 1) * ((k / 9 == 0 || k / 9 == 3) ? 1 : -1); }
// grid index (i*6 + j) of slot k in the 6x6 NCC-Old reference window
__host__ __device__ constexpr int sa_grid(int k) { return ((sa_dx(k) + 5) / 2) * 6 + (sa_dy(k) + 5) / 2; }

template <class AT>
__device__ __forceinline__ SaWin sa_window(const AT &a, int px, int py) {
    const uint8_t cid = a.sa[py * a.W + px];
    uint64_t m = 0;
    float sr = 0.0f, srr = 0.0f;
    for (int q = 0; q < 4; ++q) {
        for (int j = 0; j < 9; ++j) {
            const int k = q * 9 + j;
            const int rx = px + sa_dx(k), ry = py + sa_dy(k);
            if (rx < 0 || rx >= a.W || ry < 0 || ry >= a.H) continue;
            if (a.sa[ry * a.W + rx] != cid) break;
            const float r = tex_ref(a, rx, ry);
            sr += r;
            srr = fmaf(r, r, srr);
            m |= 1ull << k;
        }
    }
    SaWin w;
    w.mlo = (uint32_t)m;
    w.mhi = (uint32_t)(m >> 32);
    w.sr = sr;
    w.srr = srr;
    return w;
}

// SA quadrant branch of ComputeBilateralNCCOld (APD.cu:664-719), IEEE taps: out of line (ncc_old_slow).
template <bool F16>
__device__ __forceinline__ float ncc_old_sa(const APD_G Args *ap, int px, int py, int s, const Hom &H, uint8_t cid) {
    const APD_G Args &a = *ap;
    const int sign[8] = {1, 1, -1, -1, 1, -1, -1, 1};
    const int off[18] = {1, 1, 3, 1, 1, 3, 1, 5, 3, 3, 5, 1, 5, 3, 3, 5, 5, 5};
    const SrcTex<F16> Q(a, s);
    float sr = 0.0f, srr = 0.0f, ss = 0.0f, sss = 0.0f, srs = 0.0f, wsum = 0.0f;
    for (int q = 0; q < 4; ++q) {
        for (int j = 0; j < 9; ++j) {
            int rx = px + off[2 * j] * sign[2 * q];
            int ry = py + off[2 * j + 1] * sign[2 * q + 1];
            if (rx < 0 || rx >= a.W || ry < 0 || ry >= a.H) continue;
            if (a.sa[ry * a.W + rx] != cid) break;
            float r = tex_ref(a, rx, ry);
            float sx, sy;
            project(H, (float)rx, (float)ry, sx, sy);
            float v = sample_src(Q, a.W, a.H, sx, sy);
            sr += r; srr = fmaf(r, r, srr);
            ss += v; sss = fmaf(v, v, sss);
            srs = fmaf(r, v, srs);
            wsum += 1.0f;
        }
    }
    return ncc_finalize(sr, srr, ss, sss, srs, wsum);
}

// ---------------------------------------------------------------------------------------------
// Fast window taps. Same arithmetic as project() + quad_tap() + bilerp(), restated for throughput:
//   * 1/Z = v_rcp_f32 + one Newton step, r' = fma(fma(-Z, r, 1), r, r). tools/rcp_exhaustive.hip
//     checks on gfx950 that this equals the IEEE quotient 1.0f/Z for EVERY significand and both signs
//     over the exponent range the window guard below admits, so it is the same value, not an
//     approximation. Windows the guard rejects (Z near 0 or huge anywhere in the window) take the
//     IEEE path (ncc_old_ieee).
//   * (X, Y) pairs, the 1/256 fixed-point step and the bilinear lerps use packed fp32 (v_pk_fma_f32,
//     v_pk_mul_f32, v_pk_add_f32): per-component IEEE results identical to the scalar ops.
//   * the tap address is a 32-bit byte offset from the (wave-uniform) texel base: the -1 of the
//     quad index is folded into the per-view offset.
// ---------------------------------------------------------------------------------------------
typedef float apd_f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ apd_f2 pk_fma(apd_f2 a, apd_f2 b, apd_f2 c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ float rcp_newton(float z) {
    const float r = __builtin_amdgcn_rcpf(z);
    return fmaf(fmaf(-z, r, 1.0f), r, r);
}
// true iff every tap Z of the window [x0, x0+10] x [y0, y0+10] is provably in the range where
// rcp_newton is exact: corners of one sign with |Z| >= max(2^-100, 2^-16 S) and S <= 2^100, S being a
// bound on the magnitude of the terms of Z (rounding error of any tap's Z is < 2^-21 S, and Z is
// affine, so every tap's computed Z keeps the corners' sign and |Z| >= 2^-101); and |h0..h5| <= 2^100
// so X, Y are finite. NaN -> false.
// (window_rcp_ok_box: the same proof for every tap in the box [x0, x1] x [y0, y1], e.g. the bounding
// box of all windows of one NCC-New evaluation: the corners' Z bound every tap's, as Z is affine)
__device__ __forceinline__ bool window_rcp_ok_box(const Hom &Hm, float x0, float y0, float x1, float y1) {
    const float z00 = fmaf(Hm.h[7], y0, fmaf(Hm.h[6], x0, Hm.h[8]));
    const float z10 = fmaf(Hm.h[7], y0, fmaf(Hm.h[6], x1, Hm.h[8]));
    const float z01 = fmaf(Hm.h[7], y1, fmaf(Hm.h[6], x0, Hm.h[8]));
    const float z11 = fmaf(Hm.h[7], y1, fmaf(Hm.h[6], x1, Hm.h[8]));
    const float S = fmaf(fabsf(Hm.h[6]), fmaxf(fabsf(x0), fabsf(x1)),
                         fmaf(fabsf(Hm.h[7]), fmaxf(fabsf(y0), fabsf(y1)), fabsf(Hm.h[8])));
    const float lo = fmaxf(0x1p-100f, S * 0x1p-16f);
    const float mn = fminf(fminf(z00, z10), fminf(z01, z11));
    const float mx = fmaxf(fmaxf(z00, z10), fmaxf(z01, z11));
    // X and Y finite at every tap (so X/Z is never NaN and the med3 clamp below is exact)
    const float hm = fmaxf(fmaxf(fmaxf(fabsf(Hm.h[0]), fabsf(Hm.h[1])), fmaxf(fabsf(Hm.h[2]), fabsf(Hm.h[3]))),
                           fmaxf(fabsf(Hm.h[4]), fabsf(Hm.h[5])));
    return (mn >= lo || mx <= -lo) && S <= 0x1p100f && hm <= 0x1p100f;
}
__device__ __forceinline__ bool window_rcp_ok(const Hom &Hm, float x0, float y0) {
    return window_rcp_ok_box(Hm, x0, y0, x0 + 10.0f, y0 + 10.0f);
}
// v_fma_mix_f32 with both fp16 operands taken from the low (lo) / high (hi) halves: fma(a, (float)b,
// (float)c) in fp32 with exact fp16->fp32 conversions. Written as inline asm because the SLP
// vectoriser otherwise converts all four halves and packs the two FMAs (more instructions).
__device__ __forceinline__ float fma_mix_lo(float a, apd_h2 b, apd_h2 c) {
    float d;
    asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel_hi:[0,1,1]" : "=v"(d) : "v"(a), "v"(b), "v"(c));
    return d;
}
__device__ __forceinline__ float fma_mix_hi(float a, apd_h2 b, apd_h2 c) {
    float d;
    asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel:[0,1,1] op_sel_hi:[0,1,1]" : "=v"(d) : "v"(a), "v"(b), "v"(c));
    return d;
}
// UNI: the source view is wave-uniform (view-major kernels) -> its base folds into the SGPR pointer.
template <bool F16, bool UNI>
struct FastTex {
    const APD_G char *base;  // wave-uniform: a.pairs / a.quad (+ the view's offset when UNI)
    uint32_t vbase;          // byte offset of view s (0 when UNI), minus one row and one texel of the pitch
    uint32_t W1;             // pitch in texels
    float Wm1, Hm1;
    static constexpr uint32_t SHIFT = F16 ? 2u : 4u;  // log2 bytes per texel
    template <class AT>
    __device__ __forceinline__ FastTex(const AT &a, int s) {
        base = F16 ? (const APD_G char *)a.pairs : (const APD_G char *)a.quad;
        W1 = SrcTex<F16>::pitch(a.W);
        const uint32_t vb = (uint32_t)(((uint32_t)(s - 1) * (uint32_t)a.qstride - W1 - 1u) << SHIFT);
        if constexpr (UNI) {
            base = (const APD_G char *)((F16 ? (const APD_G char *)a.pairs : (const APD_G char *)a.quad) +
                                        ((int64_t)(s - 1) * (int64_t)a.qstride - (int64_t)W1 - 1) * (1 << SHIFT));
            vbase = 0u;
        } else {
            vbase = vb;
        }
        Wm1 = (float)(a.W - 1);
        Hm1 = (float)(a.H - 1);
    }
    // one bilinear sample at (X/Z, Y/Z) given iz = 1/Z: identical to sample_src(X*iz, Y*iz).
    // Clamp with v_med3_f32: equal to fminf(fmaxf(x, -1), Wm1) for every non-NaN x (window_rcp_ok
    // guarantees X, Y finite and Z finite non-zero, so X*iz is never NaN).
    struct Tap { uint32_t off; apd_f2 f; };
    __device__ __forceinline__ Tap tap(apd_f2 XY, float iz) const {
        apd_f2 p = XY * iz;
        p.x = __builtin_amdgcn_fmed3f(p.x, -1.0f, Wm1);
        p.y = __builtin_amdgcn_fmed3f(p.y, -1.0f, Hm1);
        const apd_f2 q = pk_fma(p, (apd_f2){256.0f, 256.0f}, (apd_f2){512.5f, 512.5f});
        const int qx = (int)q.x, qy = (int)q.y;
        Tap t;
#ifdef APD_ABLATE_ONEROW  // timing-only build: every tap of a wave in 1-2 texel rows, wrong values
        // padded rows 1..2, columns 1..32 of view s: inside the view for W >= 30 (vbase removes one row
        // and one texel of the pitch)
        t.off = ((__umul24((((uint32_t)qy >> 8) & 1u) + 1u, W1) + (((uint32_t)qx >> 8) & 31u) + 1u) << SHIFT) + vbase;
#else
        t.off = ((__umul24((uint32_t)qy >> 8, W1) + ((uint32_t)qx >> 8)) << SHIFT) + vbase;
#endif
        t.f = (apd_f2){(float)(qx & 255), (float)(qy & 255)} * 0.00390625f;
#ifdef APD_ABLATE_VALU  // timing-only build: APD_ABLATE_VALU extra (dead) VALU instructions per tap, same values
#pragma unroll
        for (int i = 0; i < APD_ABLATE_VALU; ++i) {
            float d;
            asm volatile("v_mov_b32 %0, %1" : "=v"(d) : "v"(p.x));
        }
#endif
        return t;
    }
    using Raw = typename std::conditional<F16, apd_u2_a4, float4>::type;
#ifdef APD_ABLATE_DWORD  // timing-only build: 4-byte instead of 8-byte gathers, wrong values
    __device__ __forceinline__ Raw load(const Tap &t) const {
        if constexpr (F16) {
            const uint32_t x = *(const APD_G uint32_t *)(base + t.off);
            return Raw{x, x};
        } else {
            return *(const APD_G Raw *)(base + t.off);
        }
    }
#else
    __device__ __forceinline__ Raw load(const Tap &t) const { return *(const APD_G Raw *)(base + t.off); }
#endif
    __device__ __forceinline__ float finish(const Tap &t, const Raw &v) const {
        if constexpr (F16) {
            // F16 storage is only selected for quarter-integer texels in [0, 256) (see apd_set_problem):
            // the horizontal differences T10-T00, T11-T01 are then exact in fp16, so they are taken with
            // one v_pk_add_f16 and fed to v_fma_mix_f32 (fp16 operands converted exactly) -- the same
            // fp32 values and FMAs as bilerp() on the converted texels.
            const apd_h2 c0 = __builtin_bit_cast(apd_h2, v.x);  // {T00, T01}
            const apd_h2 c1 = __builtin_bit_cast(apd_h2, v.y);  // {T10, T11}
            const apd_h2 dd = c1 - c0;
            const float top = fma_mix_lo(t.f.x, dd, c0);  // fma(ax, T10 - T00, T00)
            const float bot = fma_mix_hi(t.f.x, dd, c0);  // fma(ax, T11 - T01, T01)
            return fmaf(t.f.y, bot - top, top);
        } else {
            const float4 q = v;
            // top = fma(ax, T10 - T00, T00), bot = fma(ax, T11 - T01, T01), v = fma(ay, bot - top, top)
            const apd_f2 lo = (apd_f2){q.x, q.z}, hi = (apd_f2){q.y, q.w};
            const apd_f2 tb = pk_fma((apd_f2){t.f.x, t.f.x}, hi - lo, lo);
            return fmaf(t.f.y, tb.y - tb.x, tb.x);
        }
    }
    __device__ __forceinline__ float sample(const Tap &t) const { return finish(t, load(t)); }
};

// FastTex over pre-differenced fp16 texels (F16 problems; DepthToWeak): the 8-byte record at the tap's
// base position holds the vertical pair {T(ix,iy), T(ix,iy+1)} and the horizontal differences
// {(T(ix+1,iy) - T(ix,iy)) / 256, (T(ix+1,iy+1) - T(ix,iy+1)) / 256}, all exact in fp16 (quarter-
// integer texels in [0, 256): the differences are multiples of 2^-10 below 1 in magnitude, normal
// fp16). The lerp takes the x fraction as the integer 256 * ax: fma(256 ax, dd / 256, T00) has the
// exact product ax * dd of fma(ax, dd, T00), hence the same single rounding -- bit-identical to
// FastTex<true>::finish -- without FastTex's per-tap v_pk_add_f16 for the differences (and the x
// fraction's 1/256 multiply). Twice the bytes per texel position; for the VALU-bound kernels.
template <bool UNI>
struct FastTexD {
    const APD_G char *base;
    uint32_t vbase;
    uint32_t W1;
    float Wm1, Hm1;
    static constexpr uint32_t SHIFT = 3u;
    template <class AT>
    __device__ __forceinline__ FastTexD(const AT &a, int s) {
        W1 = SrcTex<true>::pitch(a.W);
        const int64_t off = ((int64_t)(s - 1) * (int64_t)a.qstride - (int64_t)W1 - 1) * (1 << SHIFT);
        if constexpr (UNI) {
            base = (const APD_G char *)a.dpairs + off;
            vbase = 0u;
        } else {
            base = (const APD_G char *)a.dpairs;
            vbase = (uint32_t)off;
        }
        Wm1 = (float)(a.W - 1);
        Hm1 = (float)(a.H - 1);
    }
    struct Tap { uint32_t off; apd_f2 f; };  // f = {256 ax, ay}
    __device__ __forceinline__ Tap tap(apd_f2 XY, float iz) const {
        apd_f2 p = XY * iz;
        p.x = __builtin_amdgcn_fmed3f(p.x, -1.0f, Wm1);
        p.y = __builtin_amdgcn_fmed3f(p.y, -1.0f, Hm1);
        const apd_f2 q = pk_fma(p, (apd_f2){256.0f, 256.0f}, (apd_f2){512.5f, 512.5f});
        const int qx = (int)q.x, qy = (int)q.y;
        Tap t;
        t.off = ((__umul24((uint32_t)qy >> 8, W1) + ((uint32_t)qx >> 8)) << SHIFT) + vbase;
        t.f = (apd_f2){(float)(qx & 255), (float)(qy & 255) * 0.00390625f};
        return t;
    }
    using Raw = uint2;
    __device__ __forceinline__ Raw load(const Tap &t) const { return *(const APD_G uint2 *)(base + t.off); }
    __device__ __forceinline__ float finish(const Tap &t, const Raw &v) const {
        const apd_h2 c0 = __builtin_bit_cast(apd_h2, v.x);  // {T00, T01}
        const apd_h2 dd = __builtin_bit_cast(apd_h2, v.y);  // {(T10 - T00) / 256, (T11 - T01) / 256}
        const float top = fma_mix_lo(t.f.x, dd, c0);      // fma(ax, T10 - T00, T00)
        const float bot = fma_mix_hi(t.f.x, dd, c0);      // fma(ax, T11 - T01, T01)
        return fmaf(t.f.y, bot - top, top);
    }
    __device__ __forceinline__ float sample(const Tap &t) const { return finish(t, load(t)); }
};

// The 36 taps of a ComputeBilateralNCCOld window (6x6, step 2) and their moments, for a texel source
// TT with the FastTex interface (tap / load / finish). Accumulation order = the reference's (i outer,
// j inner). (Factored out of ncc_old_fast; the Strong sweep measured 3 % faster with this form.)
template <class TT, int RS, class RW>
__device__ __forceinline__ void ncc_old_taps(const TT &T, const Hom &Hm, int px, int py, const RW &rw, float &ss,
                                             float &sss, float &srs) {
        using FT = TT;
        auto column = [&](int i, typename FT::Tap *t) {
            const float x = (float)(px - 5 + 2 * i);
            const apd_f2 cxy = {fmaf(Hm.h[0], x, Hm.h[2]), fmaf(Hm.h[3], x, Hm.h[5])};
            const float cz = fmaf(Hm.h[6], x, Hm.h[8]);
#pragma unroll
            for (int j = 0; j < 6; ++j) {
                const float y = (float)(py - 5 + 2 * j);
                const apd_f2 XY = pk_fma((apd_f2){Hm.h[1], Hm.h[4]}, (apd_f2){y, y}, cxy);
                const float Z = fmaf(Hm.h[7], y, cz);
                t[j] = T.tap(XY, rcp_newton(Z));
            }
        };
        auto consume = [&](int i, const typename FT::Tap *t, const typename FT::Raw *q) {
#pragma unroll
            for (int j = 0; j < 6; ++j) {
                const float v = T.finish(t[j], q[j]);
                ss += v;
                // (sss, srs) = (fma(v, v, sss), fma(r, v, srs))
                const apd_f2 acc = pk_fma((apd_f2){v, (float)rw.r[(i * 6 + j) * RS]}, (apd_f2){v, v}, (apd_f2){sss, srs});
                sss = acc.x;
                srs = acc.y;
            }
        };
#ifndef APD_NCC_NOPIPE
        // software pipeline: column i+1's gathers are in flight while column i is consumed
        typename FT::Tap ta[6], tb[6];
        typename FT::Raw qa[6], qb[6];
        column(0, ta);
#pragma unroll
        for (int j = 0; j < 6; ++j) qa[j] = T.load(ta[j]);
#pragma unroll
        for (int i = 0; i < 6; i += 2) {
            if (i + 1 < 6) {
                column(i + 1, tb);
#pragma unroll
                for (int j = 0; j < 6; ++j) qb[j] = T.load(tb[j]);
            }
            consume(i, ta, qa);
            if (i + 2 < 6) {
                column(i + 2, ta);
#pragma unroll
                for (int j = 0; j < 6; ++j) qa[j] = T.load(ta[j]);
            }
            if (i + 1 < 6) consume(i + 1, tb, qb);
        }
#else
        // One window column (6 taps) per step: all 6 gathers are issued before the first is consumed.
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            typename FT::Tap t[6];
            typename FT::Raw q[6];
            column(i, t);
#pragma unroll
            for (int j = 0; j < 6; ++j) q[j] = T.load(t[j]);
            consume(i, t, q);
        }
#endif
}

// The SA quadrant branch's source moments on the fast taps: all 36 slots in visiting order (groups of
// 6, software-pipelined as ncc_old_taps), the slots the pixel's SaWin does not visit contributing
// exact zeros: the partial sums start at +0 and are never -0, so x + (+-0) == x bit-for-bit.
// Same (X, Y, Z) expressions as project().
template <class TT, int RS, class RT>
__device__ __forceinline__ void ncc_old_sa_taps(const TT &T, const Hom &Hm, int px, int py, const RT *r,
                                                const SaWin &w, float &ss, float &sss, float &srs) {
    auto group = [&](int g, typename TT::Tap *t) {
#pragma unroll
        for (int j = 0; j < 6; ++j) {
            const int k = 6 * g + j;
            const float x = (float)(px + sa_dx(k)), y = (float)(py + sa_dy(k));
            const apd_f2 cxy = {fmaf(Hm.h[0], x, Hm.h[2]), fmaf(Hm.h[3], x, Hm.h[5])};
            const apd_f2 XY = pk_fma((apd_f2){Hm.h[1], Hm.h[4]}, (apd_f2){y, y}, cxy);
            const float Z = fmaf(Hm.h[7], y, fmaf(Hm.h[6], x, Hm.h[8]));
            t[j] = T.tap(XY, rcp_newton(Z));
        }
    };
    auto consume = [&](int g, const typename TT::Tap *t, const typename TT::Raw *q) {
#pragma unroll
        for (int j = 0; j < 6; ++j) {
            const int k = 6 * g + j;
            const uint32_t on = k < 32 ? (w.mlo >> k) & 1u : (w.mhi >> (k - 32)) & 1u;
            const float v = on ? T.finish(t[j], q[j]) : 0.0f;
            ss += v;
            const apd_f2 acc = pk_fma((apd_f2){v, (float)r[sa_grid(k) * RS]}, (apd_f2){v, v}, (apd_f2){sss, srs});
            sss = acc.x;
            srs = acc.y;
        }
    };
    typename TT::Tap ta[6], tb[6];
    typename TT::Raw qa[6], qb[6];
    group(0, ta);
#pragma unroll
    for (int j = 0; j < 6; ++j) qa[j] = T.load(ta[j]);
#pragma unroll
    for (int g = 0; g < 6; g += 2) {
        group(g + 1, tb);
#pragma unroll
        for (int j = 0; j < 6; ++j) qb[j] = T.load(tb[j]);
        consume(g, ta, qa);
        if (g + 2 < 6) {
            group(g + 2, ta);
#pragma unroll
            for (int j = 0; j < 6; ++j) qa[j] = T.load(ta[j]);
        }
        consume(g + 1, tb, qb);
    }
}

// IEEE-division statement of the ComputeBilateralNCCOld window sum (taken only for windows that
// window_rcp_ok rejects).
template <bool F16, class RT = float>
__device__ __forceinline__ apd_f2 ncc_old_ieee(const APD_G Args *ap, int px, int py, int s, const Hom &Hm,
                                               const RT *r, int rs, float *sss_out) {
    const APD_G Args &a = *ap;
    const SrcTex<F16> Q(a, s);
    const float Wm1 = (float)(a.W - 1), Hm1 = (float)(a.H - 1);
    const uint32_t W1 = SrcTex<F16>::pitch(a.W);
    float ss = 0.0f, sss = 0.0f, srs = 0.0f;
    for (int i = 0; i < 6; ++i) {
        const float x = (float)(px - 5 + 2 * i);
        const float cx = fmaf(Hm.h[0], x, Hm.h[2]);
        const float cy = fmaf(Hm.h[3], x, Hm.h[5]);
        const float cz = fmaf(Hm.h[6], x, Hm.h[8]);
        for (int j = 0; j < 6; ++j) {
            const float y = (float)(py - 5 + 2 * j);
            const float X = fmaf(Hm.h[1], y, cx);
            const float Y = fmaf(Hm.h[4], y, cy);
            const float Z = fmaf(Hm.h[7], y, cz);
            const float iz = 1.0f / Z;
            const QuadTap t = quad_tap(Wm1, Hm1, W1, X * iz, Y * iz);
            const float v = bilerp(Q.fetch(t.idx), t.ax, t.ay);
            ss += v;
            sss = fmaf(v, v, sss);
            srs = fmaf((float)r[(i * 6 + j) * rs], v, srs);
        }
    }
    *sss_out = sss;
    return (apd_f2){ss, srs};
}

__device__ __forceinline__ float ncc_old_finish(float ss, float sss, float srs, float mean, float var) {
    const float inv = 1.0f / 36.0f;
    ss *= inv; sss *= inv; srs *= inv;
    float var_src = fmaf(-ss, ss, sss);
    if (var < 1e-5f || var_src < 1e-5f) return APD_COST_MAX;
    float covar = fmaf(-mean, ss, srs);
    float vrs = sqrtf(var * var_src);
    return fmaxf(0.0f, fminf(APD_COST_MAX, 1.0f - covar / vrs));
}

// Out-of-line ComputeBilateralNCCOld for the windows ncc_old_fast hands back: the SA quadrant
// variant, or windows whose taps need the IEEE reciprocal. Everything arrives by value (the
// homography is recomputed from the plane), so the hot path never spills a homography to the stack.
template <bool F16, class RT = float>
__device__ __noinline__ float ncc_old_slow(const APD_G Args *ap, int px, int py, int s, float4 pl, const RT *r,
                                           int rs, float mean, float var) {
    const APD_G Args &a = *ap;
    const Hom Hm = homography(a, s, pl);
    float ptx, pty;
    project(Hm, (float)px, (float)py, ptx, pty);
    if (ptx >= (float)a.W || ptx < 0.0f || pty >= (float)a.H || pty < 0.0f) return APD_COST_MAX;
    if (a.sa_any) {
        int pidx = clampi((int)fmaf(pty, (float)a.W, ptx), 0, a.HW - 1);
        if (a.sa[pidx] != 0) return ncc_old_sa<F16>(ap, px, py, s, Hm, a.sa[py * a.W + px]);
    }
    float sss;
    const apd_f2 rr = ncc_old_ieee<F16, RT>(ap, px, py, s, Hm, r, rs, &sss);
    return ncc_old_finish(rr.x, sss, rr.y, mean, var);
}

// ComputeBilateralNCCOld (APD.cu:596-721) for source view s (1..N), plane in the ref frame: the
// call-free fast path. Returns the cost, or sets `slow` when the window needs ncc_old_slow (SA mask
// hit at the projected centre, or a Z the Newton reciprocal is not proven for); the returned value
// is then meaningless (the taps ran on a dummy homography that keeps every address in bounds).
// RS = LDS stride of the reference window (1: per-pixel contiguous; 64: [k][pixel] layout).
// (ncc_old_fast_h: the same with the window's homography given, e.g. from precomputed plane_terms)
template <bool F16, int RS = 1, bool DP = false, class RW = RefWin>
__device__ __forceinline__ float ncc_old_fast_h(const Args &a, int px, int py, int s, Hom Hm, const RW &rw,
                                                bool &slow) {
    // DP: the taps over the pre-differenced texels (FastTexD, F16 problems with a.dpairs)
    using TT = typename std::conditional<DP && F16, FastTexD<(RS > 1)>, FastTex<F16, (RS > 1)>>::type;
    const int W = a.W, H = a.H;
    float ptx, pty;
    project(Hm, (float)px, (float)py, ptx, pty);
    slow = false;
    if (ptx >= (float)W || ptx < 0.0f || pty >= (float)H || pty < 0.0f) return APD_COST_MAX;
    bool sa_win = false;  // SA quadrant branch on the fast taps (view-major kernels: rw.sa set)
    if (a.sa_any) {
        int pidx = clampi((int)fmaf(pty, (float)W, ptx), 0, a.HW - 1);
        if (a.sa[pidx] != 0) {
            if (RS > 1 && rw.sa != nullptr) sa_win = true;
            else slow = true;
        }
    }
#ifdef APD_ABLATE_NCC  // timing-only build: skeleton without the window sums
    return fabsf(Hm.h[0] + Hm.h[8]) * 0.001f;
#endif
    if (!window_rcp_ok(Hm, (float)(px - 5), (float)(py - 5)) || a.force_slow) slow = true;
    if (slow) {
#pragma unroll
        for (int k = 0; k < 9; ++k) Hm.h[k] = (k == 8) ? 1.0f : 0.0f;  // every tap -> texel (0, 0)
    }
    float ss = 0.0f, sss = 0.0f, srs = 0.0f;
    const TT T(a, s);
    if constexpr (RS > 1) {
        if (rw.sa != nullptr) {
            // each branch runs only if some lane of the wave needs it
            if (__builtin_amdgcn_ballot_w64(!sa_win)) ncc_old_taps<TT, RS>(T, Hm, px, py, rw, ss, sss, srs);
            if (__builtin_amdgcn_ballot_w64(sa_win)) {
                const SaWin w = *rw.sa;
                float s2 = 0.0f, ss2 = 0.0f, rs2 = 0.0f;
                ncc_old_sa_taps<TT, RS>(T, Hm, px, py, rw.r, w, s2, ss2, rs2);
                if (sa_win) return ncc_finalize(w.sr, w.srr, s2, ss2, rs2, (float)(__popc(w.mlo) + __popc(w.mhi)));
            }
            return ncc_old_finish(ss, sss, srs, rw.mean, rw.var);
        }
    }
    ncc_old_taps<TT, RS>(T, Hm, px, py, rw, ss, sss, srs);
    return ncc_old_finish(ss, sss, srs, rw.mean, rw.var);
}
template <bool F16, int RS = 1, class RW = RefWin>
__device__ __forceinline__ float ncc_old_fast(const Args &a, int px, int py, int s, float4 pl, const RW &rw,
                                              bool &slow) {
    return ncc_old_fast_h<F16, RS, false, RW>(a, px, py, s, homography(a, s, pl), rw, slow);
}




// ComputeGeomConsistencyCost (APD.cu:865-902). geom_cost_p: from the view-independent world point
// P = world_point(ref, depth_from_plane(plane)) onwards (a kernel scoring one plane in several views
// computes P once); geom_cost: the whole statement sequence.
__device__ __forceinline__ void geom_point(const Args &a, int px, int py, float4 pl, float P[3]) {
    const APD_C Cam &rc = a.cams[0];
    float depth = depth_from_plane(rc, pl, px, py);
    world_point(rc, (float)px, (float)py, depth, P);
}
__device__ __forceinline__ float geom_cost_p(const Args &a, int px, int py, int s, const float P[3]) {
    const APD_C Cam &rc = a.cams[0];
    const APD_C Cam &sc = a.cams[s];
    float sx, sy, sd;
    project_cam(P, sc, sx, sy, sd);
    float src_depth = a.depth[(size_t)s * a.HW + trunc_clamp(sy, a.H) * a.W + trunc_clamp(sx, a.W)];
    if (src_depth == 0.0f) return 3.0f;
    float Q[3];
    world_point(sc, sx, sy, src_depth, Q);
    float bx, by, rd;
    project_cam(Q, rc, bx, by, rd);
    float dx = (float)px - bx, dy = (float)py - by;
    float e = sqrtf(dx * dx + dy * dy);
    return fminf(3.0f, e);
}
// geom_cost_p in two halves around its one gather (the source depth), so that a caller scoring
// several planes can issue all the gathers before consuming any: the same statements.
struct GeomHead { size_t idx; float sx, sy; };
__device__ __forceinline__ GeomHead geom_head(const Args &a, int s, const float P[3]) {
    const APD_C Cam &sc = a.cams[s];
    GeomHead h;
    float sd;
    project_cam(P, sc, h.sx, h.sy, sd);
    h.idx = (size_t)s * a.HW + trunc_clamp(h.sy, a.H) * a.W + trunc_clamp(h.sx, a.W);
    return h;
}
__device__ __forceinline__ float geom_tail(const Args &a, int px, int py, int s, const GeomHead &h, float src_depth) {
    if (src_depth == 0.0f) return 3.0f;
    const APD_C Cam &rc = a.cams[0];
    const APD_C Cam &sc = a.cams[s];
    float Q[3];
    world_point(sc, h.sx, h.sy, src_depth, Q);
    float bx, by, rd;
    project_cam(Q, rc, bx, by, rd);
    float dx = (float)px - bx, dy = (float)py - by;
    float e = sqrtf(dx * dx + dy * dy);
    return fminf(3.0f, e);
}
__device__ __forceinline__ float geom_cost(const Args &a, int px, int py, int s, float4 pl) {
    float P[3];
    geom_point(a, px, py, pl, P);
    return geom_cost_p(a, px, py, s, P);
}

}  // namespace apd
