// apd_fusion.hip — device half of depth-map fusion (include/apd_fusion.h) for gfx950.
//
// Three per-pixel kernels over HBM-resident views. Each is a gather kernel: one lane per reference
// pixel, N projections per lane into source depth/normal maps (random but spatially coherent
// reads, L2-resident for neighbouring lanes). No LDS, no MFMA: the arithmetic is a few dozen
// float/double ops per (pixel, source), the bound is the gather traffic.
//
// Numerics contract with the host restatement (oracle/fusion_oracle.c) and the reference's host
// code (APD.cpp:866-910, compiled for x86-64 without FMA): -ffp-contract=off, float ops in source
// order, double where C++ promotes (cv::norm, pow(float, int), M_PI), and float->int conversion
// with x86 cvttss2si semantics (NaN / out of range -> INT_MIN) for `int(point.y + 0.5f)`.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/apd_fusion.h"

namespace {

struct V3 {
    float x, y, z;
};

// Get3DPointonWorld (APD.cpp:866-889): float ops in the reference's order.
__device__ __host__ inline V3 point_on_world(int x, int y, float depth, const apd_camera &cam) {
    V3 p, t, c;
    p.x = depth * ((float)x - cam.K[2]) / cam.K[0];
    p.y = depth * ((float)y - cam.K[5]) / cam.K[4];
    p.z = depth;
    t.x = cam.R[0] * p.x + cam.R[3] * p.y + cam.R[6] * p.z;
    t.y = cam.R[1] * p.x + cam.R[4] * p.y + cam.R[7] * p.z;
    t.z = cam.R[2] * p.x + cam.R[5] * p.y + cam.R[8] * p.z;
    c.x = -(cam.R[0] * cam.t[0] + cam.R[3] * cam.t[1] + cam.R[6] * cam.t[2]);
    c.y = -(cam.R[1] * cam.t[0] + cam.R[4] * cam.t[1] + cam.R[7] * cam.t[2]);
    c.z = -(cam.R[2] * cam.t[0] + cam.R[5] * cam.t[1] + cam.R[8] * cam.t[2]);
    return V3{t.x + c.x, t.y + c.y, t.z + c.z};
}

// ProjectCamera (APD.cpp:891-900).
__device__ inline void project(const V3 &X, const apd_camera &cam, float &px, float &py, float &depth) {
    const float tx = cam.R[0] * X.x + cam.R[1] * X.y + cam.R[2] * X.z + cam.t[0];
    const float ty = cam.R[3] * X.x + cam.R[4] * X.y + cam.R[5] * X.z + cam.t[1];
    const float tz = cam.R[6] * X.x + cam.R[7] * X.y + cam.R[8] * X.z + cam.t[2];
    depth = cam.K[6] * tx + cam.K[7] * ty + cam.K[8] * tz;
    px = (cam.K[0] * tx + cam.K[1] * ty + cam.K[2] * tz) / depth;
    py = (cam.K[3] * tx + cam.K[4] * ty + cam.K[5] * tz) / depth;
}

// int(v) as x86-64 cvttss2si: truncation, INT_MIN for NaN and out-of-range values.
__device__ inline int trunc_x86(float v) {
    if (!(v >= -2147483648.0f && v < 2147483648.0f)) return INT32_MIN;
    return (int)v;
}

// q of GetAngle (APD.cpp:902-910): float dot over double cv::norm product (normL2Sqr<float,double>).
__device__ inline float angle_q(float a0, float a1, float a2, float b0, float b1, float b2) {
    const float dot = a0 * b0 + a1 * b1 + a2 * b2;
    const double na = __builtin_sqrt(((double)a0 * (double)a0 + (double)a1 * (double)a1) + (double)a2 * (double)a2);
    const double nb = __builtin_sqrt(((double)b0 * (double)b0 + (double)b1 * (double)b1) + (double)b2 * (double)b2);
    return (float)((double)dot / (na * nb));
}
__device__ inline bool in_unit(float q) { return q >= -1.0f && q <= 1.0f; }

// confidences[i].at<float>(r, c) on a CV_8UC1 Mat (APD.cpp:1010-1011): 4 bytes from r*W + 4c.
// The device copy is padded with zeros past W*H (see apd_fusion.h).
__device__ inline float conf_as_float(const uint8_t *conf, int W, int r, int c) {
    const size_t o = (size_t)r * W + 4 * (size_t)c;
    const uint32_t u = (uint32_t)conf[o] | (uint32_t)conf[o + 1] << 8 | (uint32_t)conf[o + 2] << 16 |
                       (uint32_t)conf[o + 3] << 24;
    return __uint_as_float(u);
}

struct DevView {
    int W, H;
    const float *depth;
    const float *normal;
    const uint8_t *weak;
    const uint8_t *conf;
};

// XCD-aware block order: the dispatcher deals blocks round-robin to the 8 XCDs, so block b runs on
// XCD b % 8; give each XCD a contiguous range of pixel blocks (neighbouring rows share L2 lines of the
// source maps). Bijective for any block count.
__device__ inline int xcd_block(int b, int nb) {
    const int q = nb / 8, rem = nb % 8;
    const int x = b % 8, i = b / 8;
    return x * q + (x < rem ? x : rem) + i;
}

constexpr int kWeak = 0, kStrong = 1;  // PixelState, main.h:74-78

__global__ void __launch_bounds__(256) k_weak_filter(const DevView *views, const apd_camera *cams, int nv, int ref,
                                                    float q_view, uint8_t *skip) {
    const DevView rv = views[ref];
    const int npx = rv.W * rv.H;
    const int p = xcd_block(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x;
    if (p >= npx) return;
    const int r = p / rv.W, c = p - r * rv.W;
    uint8_t out = 0;
    if (rv.weak[p] == kWeak) {
        const apd_camera &rc = cams[ref];
        const float ref_depth = rv.depth[p];
        const V3 X = point_on_world(c, r, ref_depth, rc);
        const float ref_conf = conf_as_float(rv.conf, rv.W, r, c);
        int strong = 0, weak = 0;
        for (int s = 0; s < nv; ++s) {
            if (s == ref) continue;
            const apd_camera &sc = cams[s];
            const float q = angle_q(rc.c[0] - X.x, rc.c[1] - X.y, rc.c[2] - X.z, sc.c[0] - X.x, sc.c[1] - X.y,
                                    sc.c[2] - X.z);
            if (in_unit(q) && q < q_view) continue;  // angle > 80 degrees
            float px, py, pd;
            project(X, sc, px, py, pd);
            if (pd <= 0.0f) continue;
            const int sr = trunc_x86(py + 0.5f), scol = trunc_x86(px + 0.5f);
            const DevView sv = views[s];
            if (scol >= 0 && scol < sv.W && sr >= 0 && sr < sv.H) {
                const int sp = sr * sv.W + scol;
                const float sd = sv.depth[sp];
                const uint8_t st = sv.weak[sp];
                if (st == kStrong) {
                    if (pd < sd - 0.01f * sd) ++strong;
                } else if (st == kWeak) {
                    if (conf_as_float(sv.conf, sv.W, sr, scol) < ref_conf && pd < sd - 0.01f * sd) ++weak;
                }
            }
        }
        out = (strong >= 2 || weak >= 4) ? 1 : 0;
    }
    skip[p] = out;
}

// Shared geometry of RunFusion and the TAT variants (APD.cpp:1166-1187 / 1360-1381): returns false
// when the candidate does not reach the cost computation (out of bounds or source depth <= 0).
__device__ inline bool candidate(const DevView &rv, const apd_camera &rc, int r, int c, float ref_depth, const V3 &X,
                                 float n0, float n1, float n2, const DevView &sv, const apd_camera &scam, int &sp,
                                 float &err, float &rel, float &q) {
    float px, py, pd;
    project(X, scam, px, py, pd);
    const int sr = trunc_x86(py + 0.5f), scol = trunc_x86(px + 0.5f);
    if (!(scol >= 0 && scol < sv.W && sr >= 0 && sr < sv.H)) return false;
    sp = sr * sv.W + scol;
    const float sd = sv.depth[sp];
    if (sd <= 0.0f) return false;
    const float m0 = sv.normal[3 * (size_t)sp], m1 = sv.normal[3 * (size_t)sp + 1], m2 = sv.normal[3 * (size_t)sp + 2];
    const V3 Y = point_on_world(scol, sr, sd, scam);
    float tx, ty, td;
    project(Y, rc, tx, ty, td);
    const double dx = (double)((float)c - tx), dy = (double)((float)r - ty);
    err = (float)__builtin_sqrt(dx * dx + dy * dy);
    rel = fabsf(td - ref_depth) / ref_depth;
    q = angle_q(n0, n1, n2, m0, m1, m2);
    return true;
}

struct SrcList {
    int n;
    int idx[APD_MAX_IMAGES];
};

__global__ void __launch_bounds__(256) k_consistency(const DevView *views, const apd_camera *cams, int ref, SrcList src,
                                                    float q_angle, int32_t *src_pix, float *err_rel, float *cos_angle) {
    const DevView rv = views[ref];
    const int npx = rv.W * rv.H;
    const int p = xcd_block(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x;
    if (p >= npx) return;
    const int r = p / rv.W, c = p - r * rv.W;
    const apd_camera &rc = cams[ref];
    const float d = rv.depth[p];
    const size_t o = (size_t)p * src.n;
    if (d <= 0.0f) {  // `ref_depth <= 0.0` (APD.cpp:1157): NaN depths are processed
        for (int j = 0; j < src.n; ++j) src_pix[o + j] = -1;
        return;
    }
    const V3 X = point_on_world(c, r, d, rc);
    const float n0 = rv.normal[3 * (size_t)p], n1 = rv.normal[3 * (size_t)p + 1], n2 = rv.normal[3 * (size_t)p + 2];
    for (int j = 0; j < src.n; ++j) {
        const int s = src.idx[j];
        int sp = -1;
        float err = 0.f, rel = 0.f, q = 0.f;
        bool ok = candidate(rv, rc, r, c, d, X, n0, n1, n2, views[s], cams[s], sp, err, rel, q);
        ok = ok && err < 2.0f && rel < 0.01f && (!in_unit(q) || q > q_angle);
        src_pix[o + j] = ok ? sp : -1;
        err_rel[o + j] = err + 200.0f * rel;
        cos_angle[o + j] = q;
    }
}

struct LevelCuts {
    float q[APD_MAX_IMAGES + 1];
};

__global__ void __launch_bounds__(256) k_tat_levels(const DevView *views, const apd_camera *cams, int ref, SrcList src,
                                                   float dist_base, float depth_base, int use_angle, LevelCuts cuts,
                                                   int32_t *src_pix, uint8_t *level) {
    const DevView rv = views[ref];
    const int npx = rv.W * rv.H;
    const int p = xcd_block(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x;
    if (p >= npx) return;
    const int r = p / rv.W, c = p - r * rv.W;
    const apd_camera &rc = cams[ref];
    const float d = rv.depth[p];
    const size_t o = (size_t)p * src.n;
    if (d <= 0.0f) {  // `ref_depth <= 0.0` (APD.cpp:1157): NaN depths are processed
        for (int j = 0; j < src.n; ++j) { src_pix[o + j] = -1; level[o + j] = 255; }
        return;
    }
    const V3 X = point_on_world(c, r, d, rc);
    const float n0 = rv.normal[3 * (size_t)p], n1 = rv.normal[3 * (size_t)p + 1], n2 = rv.normal[3 * (size_t)p + 2];
    for (int j = 0; j < src.n; ++j) {
        const int s = src.idx[j];
        int sp = -1;
        float err = 0.f, rel = 0.f, q = 0.f;
        uint8_t lv = 255;
        if (candidate(rv, rc, r, c, d, X, n0, n1, n2, views[s], cams[s], sp, err, rel, q)) {
            const bool any_angle = !in_unit(q);  // NaN acosf -> angle 0 (APD.cpp:906-907)
            for (int k = 2; k <= src.n; ++k) {
                if (err < (float)k * dist_base && rel < (float)k * depth_base &&
                    (!use_angle || any_angle || q > cuts.q[k])) {
                    lv = (uint8_t)k;
                    break;
                }
            }
        } else {
            sp = -1;
        }
        src_pix[o + j] = sp;
        level[o + j] = lv;
    }
}

}  // namespace

struct apd_fusion_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    std::string err;
    std::vector<void *> bufs;  // per-view device arrays
    DevView *d_views = nullptr;
    apd_camera *d_cams = nullptr;
    std::vector<DevView> views;
    void *out_buf = nullptr;
    size_t out_bytes = 0;
};

#define FUS_OK(ctx, call)                                                                          \
    do {                                                                                           \
        hipError_t e_ = (call);                                                                    \
        if (e_ != hipSuccess) {                                                                    \
            (ctx)->err = std::string(#call) + ": " + hipGetErrorString(e_);                        \
            return APD_EDEVICE;                                                                    \
        }                                                                                          \
    } while (0)

static void release_views(apd_fusion_ctx *ctx) {
    for (void *p : ctx->bufs) (void)hipFree(p);
    ctx->bufs.clear();
    if (ctx->d_views) (void)hipFree(ctx->d_views);
    if (ctx->d_cams) (void)hipFree(ctx->d_cams);
    ctx->d_views = nullptr;
    ctx->d_cams = nullptr;
    ctx->views.clear();
}

static int ensure_out(apd_fusion_ctx *ctx, size_t bytes) {
    if (ctx->out_bytes >= bytes) return APD_OK;
    if (ctx->out_buf) (void)hipFree(ctx->out_buf);
    ctx->out_buf = nullptr;
    ctx->out_bytes = 0;
    FUS_OK(ctx, hipMalloc(&ctx->out_buf, bytes));
    ctx->out_bytes = bytes;
    return APD_OK;
}

static int check_srcs(apd_fusion_ctx *ctx, int ref, int num_src, const int32_t *src, SrcList &sl) {
    const int nv = (int)ctx->views.size();
    if (nv == 0) { ctx->err = "apd_fusion: no views loaded"; return APD_ESTATE; }
    if (ref < 0 || ref >= nv) { ctx->err = "apd_fusion: reference view out of range"; return APD_EINVAL; }
    if (num_src < 0 || num_src > APD_MAX_IMAGES || (num_src > 0 && !src)) {
        ctx->err = "apd_fusion: bad source list";
        return num_src > APD_MAX_IMAGES ? APD_ETOOMANYVIEWS : APD_EINVAL;
    }
    sl.n = num_src;
    for (int j = 0; j < num_src; ++j) {
        if (src[j] < 0 || src[j] >= nv) { ctx->err = "apd_fusion: source view out of range"; return APD_EINVAL; }
        sl.idx[j] = src[j];
    }
    return APD_OK;
}

extern "C" {

apd_fusion_ctx *apd_fusion_create(int32_t device) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) return nullptr;
    if (hipSetDevice(device) != hipSuccess) return nullptr;
    auto *ctx = new apd_fusion_ctx();
    ctx->device = device;
    if (hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess) {
        delete ctx;
        return nullptr;
    }
    return ctx;
}

void apd_fusion_destroy(apd_fusion_ctx *ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    release_views(ctx);
    if (ctx->out_buf) (void)hipFree(ctx->out_buf);
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;
}

const char *apd_fusion_last_error(const apd_fusion_ctx *ctx) {
    return ctx ? ctx->err.c_str() : "apd_fusion_create failed (no such HIP device)";
}

int32_t apd_fusion_set_views(apd_fusion_ctx *ctx, int32_t num_views, const apd_fusion_view *views) {
    if (!ctx) return APD_EINVAL;
    FUS_OK(ctx, hipSetDevice(ctx->device));
    release_views(ctx);
    if (num_views <= 0 || !views) { ctx->err = "apd_fusion_set_views: no views"; return APD_EINVAL; }
    std::vector<apd_camera> cams(num_views);
    for (int i = 0; i < num_views; ++i) {
        const apd_fusion_view &v = views[i];
        if (v.width <= 0 || v.height <= 0 || !v.depth || !v.normal || !v.weak ||
            (int64_t)v.width * v.height > (int64_t)1 << 30) {
            ctx->err = "apd_fusion_set_views: view " + std::to_string(i) + " has a bad size or a NULL map";
            return APD_EINVAL;
        }
        const size_t npx = (size_t)v.width * v.height;
        // confidence: W*H bytes + the zero tail read by at<float>(r, c) for the last row (<= 4W+4)
        const size_t conf_bytes = npx + 4 * (size_t)v.width + 8;
        void *dd = nullptr, *dn = nullptr, *dw = nullptr, *dc = nullptr;
        FUS_OK(ctx, hipMalloc(&dd, npx * 4));
        ctx->bufs.push_back(dd);
        FUS_OK(ctx, hipMalloc(&dn, npx * 12));
        ctx->bufs.push_back(dn);
        FUS_OK(ctx, hipMalloc(&dw, npx));
        ctx->bufs.push_back(dw);
        FUS_OK(ctx, hipMalloc(&dc, conf_bytes));
        ctx->bufs.push_back(dc);
        FUS_OK(ctx, hipMemcpyAsync(dd, v.depth, npx * 4, hipMemcpyHostToDevice, ctx->stream));
        FUS_OK(ctx, hipMemcpyAsync(dn, v.normal, npx * 12, hipMemcpyHostToDevice, ctx->stream));
        FUS_OK(ctx, hipMemcpyAsync(dw, v.weak, npx, hipMemcpyHostToDevice, ctx->stream));
        FUS_OK(ctx, hipMemsetAsync(dc, 0, conf_bytes, ctx->stream));
        if (v.confidence) FUS_OK(ctx, hipMemcpyAsync(dc, v.confidence, npx, hipMemcpyHostToDevice, ctx->stream));
        ctx->views.push_back(DevView{v.width, v.height, (const float *)dd, (const float *)dn, (const uint8_t *)dw,
                                     (const uint8_t *)dc});
        cams[i] = v.camera;
    }
    FUS_OK(ctx, hipMalloc(&ctx->d_views, sizeof(DevView) * num_views));
    FUS_OK(ctx, hipMalloc(&ctx->d_cams, sizeof(apd_camera) * num_views));
    FUS_OK(ctx, hipMemcpyAsync(ctx->d_views, ctx->views.data(), sizeof(DevView) * num_views, hipMemcpyHostToDevice,
                               ctx->stream));
    FUS_OK(ctx, hipMemcpyAsync(ctx->d_cams, cams.data(), sizeof(apd_camera) * num_views, hipMemcpyHostToDevice,
                               ctx->stream));
    FUS_OK(ctx, hipStreamSynchronize(ctx->stream));
    return APD_OK;
}

int32_t apd_fusion_weak_filter(apd_fusion_ctx *ctx, int32_t ref, float q_view, uint8_t *skip) {
    if (!ctx) return APD_EINVAL;
    SrcList sl;
    int st = check_srcs(ctx, ref, 0, nullptr, sl);
    if (st) return st;
    if (!skip) { ctx->err = "apd_fusion_weak_filter: NULL output"; return APD_EINVAL; }
    FUS_OK(ctx, hipSetDevice(ctx->device));
    const DevView &rv = ctx->views[ref];
    const size_t npx = (size_t)rv.W * rv.H;
    if ((st = ensure_out(ctx, npx))) return st;
    const int blocks = (int)((npx + 255) / 256);
    hipLaunchKernelGGL(k_weak_filter, dim3(blocks), dim3(256), 0, ctx->stream, ctx->d_views, ctx->d_cams,
                       (int)ctx->views.size(), ref, q_view, (uint8_t *)ctx->out_buf);
    FUS_OK(ctx, hipGetLastError());
    FUS_OK(ctx, hipMemcpyAsync(skip, ctx->out_buf, npx, hipMemcpyDeviceToHost, ctx->stream));
    FUS_OK(ctx, hipStreamSynchronize(ctx->stream));
    return APD_OK;
}

int32_t apd_fusion_consistency(apd_fusion_ctx *ctx, int32_t ref, int32_t num_src, const int32_t *src, float q_angle,
                               int32_t *src_pix, float *err_rel, float *cos_angle) {
    if (!ctx) return APD_EINVAL;
    SrcList sl;
    int st = check_srcs(ctx, ref, num_src, src, sl);
    if (st) return st;
    if (!src_pix || !err_rel || !cos_angle) { ctx->err = "apd_fusion_consistency: NULL output"; return APD_EINVAL; }
    FUS_OK(ctx, hipSetDevice(ctx->device));
    const DevView &rv = ctx->views[ref];
    const size_t npx = (size_t)rv.W * rv.H, n = npx * (size_t)num_src;
    if (n == 0) return APD_OK;
    if ((st = ensure_out(ctx, n * 12))) return st;
    int32_t *d_pix = (int32_t *)ctx->out_buf;
    float *d_er = (float *)(d_pix + n), *d_q = d_er + n;
    const int blocks = (int)((npx + 255) / 256);
    hipLaunchKernelGGL(k_consistency, dim3(blocks), dim3(256), 0, ctx->stream, ctx->d_views, ctx->d_cams, ref, sl,
                       q_angle, d_pix, d_er, d_q);
    FUS_OK(ctx, hipGetLastError());
    FUS_OK(ctx, hipMemcpyAsync(src_pix, d_pix, n * 4, hipMemcpyDeviceToHost, ctx->stream));
    FUS_OK(ctx, hipMemcpyAsync(err_rel, d_er, n * 4, hipMemcpyDeviceToHost, ctx->stream));
    FUS_OK(ctx, hipMemcpyAsync(cos_angle, d_q, n * 4, hipMemcpyDeviceToHost, ctx->stream));
    FUS_OK(ctx, hipStreamSynchronize(ctx->stream));
    return APD_OK;
}

int32_t apd_fusion_tat_levels(apd_fusion_ctx *ctx, int32_t ref, int32_t num_src, const int32_t *src, float dist_base,
                              float depth_base, const float *q_k, int32_t *src_pix, uint8_t *level) {
    if (!ctx) return APD_EINVAL;
    SrcList sl;
    int st = check_srcs(ctx, ref, num_src, src, sl);
    if (st) return st;
    if (!src_pix || !level) { ctx->err = "apd_fusion_tat_levels: NULL output"; return APD_EINVAL; }
    FUS_OK(ctx, hipSetDevice(ctx->device));
    LevelCuts cuts{};
    if (q_k)
        for (int k = 0; k <= num_src; ++k) cuts.q[k] = q_k[k];
    const DevView &rv = ctx->views[ref];
    const size_t npx = (size_t)rv.W * rv.H, n = npx * (size_t)num_src;
    if (n == 0) return APD_OK;
    if ((st = ensure_out(ctx, n * 5))) return st;
    int32_t *d_pix = (int32_t *)ctx->out_buf;
    uint8_t *d_lv = (uint8_t *)(d_pix + n);
    const int blocks = (int)((npx + 255) / 256);
    hipLaunchKernelGGL(k_tat_levels, dim3(blocks), dim3(256), 0, ctx->stream, ctx->d_views, ctx->d_cams, ref, sl,
                       dist_base, depth_base, q_k ? 1 : 0, cuts, d_pix, d_lv);
    FUS_OK(ctx, hipGetLastError());
    FUS_OK(ctx, hipMemcpyAsync(src_pix, d_pix, n * 4, hipMemcpyDeviceToHost, ctx->stream));
    FUS_OK(ctx, hipMemcpyAsync(level, d_lv, n, hipMemcpyDeviceToHost, ctx->stream));
    FUS_OK(ctx, hipStreamSynchronize(ctx->stream));
    return APD_OK;
}

}  // extern "C"
