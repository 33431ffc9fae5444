/*
 * fusion_oracle.c — CPU restatement of the reference's depth-map fusion, for parity tests ONLY.
 *
 * TEST INFRASTRUCTURE: only tests/ (and bench.py's cpu_baseline leg) load this. The product
 * fusion is apde-mvs_amd/host/fusion.cpp + the HIP kernels of apde-mvs_amd/csrc/apd_fusion.hip,
 * which never call into oracle/.
 *
 * A literal restatement of the loops of
 *   WeakVisFilter    APD.cpp:962-1049
 *   RunFusion        APD.cpp:1051-1227   (variant 0: DTU / ETH3D / default)
 *   RunFusion_TAT_I  APD.cpp:1229-1432   (variant 1)
 *   RunFusion_TAT_A  APD.cpp:1433-1608   (variant 2)
 * with the helpers Get3DPointonWorld (:866-889), ProjectCamera (:891-900) and GetAngle (:902-910).
 * Same order of pixels, views and float operations; no restructuring. Arithmetic types follow the
 * C++ the reference is written in: cv::norm(Vec3f) accumulates and returns double, pow(float, 2)
 * promotes to double, `angle * 180.0f / M_PI` divides in double, `exp(float)` resolves to the
 * float overload (expf) through libstdc++'s <math.h>, acosf is glibc's. Compiled with
 * -ffp-contract=off (the reference's host code is plain x86-64 SSE: no FMA).
 *
 * Parity: unpinned against the reference binary (it needs CUDA + OpenCV + Boost, none of which
 * exist here, and the reference ships no fusion fixtures). Two reference behaviours are undefined
 * and are pinned to a definition here and in the product alike:
 *   - `confidences[i].at<float>(r, c)` on a CV_8UC1 Mat (APD.cpp:1010-1011) reads the 4 bytes at
 *     r*W + 4c; bytes past the W*H buffer read as 0 (the reference reads adjacent heap memory);
 *   - `int(point.y + 0.5f)` of NaN / out-of-range values is INT_MIN (x86 cvttss2si), so such
 *     projections are out of bounds.
 * The TAT variants' per-image cost cache (`diff`, declared once per image at :1347) is NOT reset
 * between pixels: an unusable source keeps the last usable pixel's cost and source pixel. Kept.
 */
#include <float.h>
#include <limits.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/apd_hip.h"

#ifndef M_PI
#define M_PI 3.14159265358979323846
#endif

typedef struct oracle_fusion_view {
    int32_t width, height;          /* depth-map size */
    apd_camera camera;              /* after RescaleImageAndCamera (APD.cpp:844-864) */
    const float *depth;             /* H*W   */
    const float *normal;            /* H*W*3 */
    const uint8_t *weak;            /* H*W   */
    const uint8_t *confidence;      /* H*W   (NULL: zeros) */
    const uint8_t *bgr;             /* H*W*3 colour image at depth-map size */
    int32_t ref_id;                 /* problem of this index (problems[i], pair.txt order) */
    int32_t num_src;
    const int32_t *src_ids;
} oracle_fusion_view;

typedef struct { float x, y, z; } f3;

static f3 get_3d_point_on_world(int x, int y, float depth, const apd_camera *cam) {
    f3 p, t, c, o;
    p.x = depth * (x - cam->K[2]) / cam->K[0];
    p.y = depth * (y - cam->K[5]) / cam->K[4];
    p.z = depth;
    t.x = cam->R[0] * p.x + cam->R[3] * p.y + cam->R[6] * p.z;
    t.y = cam->R[1] * p.x + cam->R[4] * p.y + cam->R[7] * p.z;
    t.z = cam->R[2] * p.x + cam->R[5] * p.y + cam->R[8] * p.z;
    c.x = -(cam->R[0] * cam->t[0] + cam->R[3] * cam->t[1] + cam->R[6] * cam->t[2]);
    c.y = -(cam->R[1] * cam->t[0] + cam->R[4] * cam->t[1] + cam->R[7] * cam->t[2]);
    c.z = -(cam->R[2] * cam->t[0] + cam->R[5] * cam->t[1] + cam->R[8] * cam->t[2]);
    o.x = t.x + c.x;
    o.y = t.y + c.y;
    o.z = t.z + c.z;
    return o;
}

static void project_camera(f3 X, const apd_camera *cam, float *px, float *py, float *depth) {
    float tx = cam->R[0] * X.x + cam->R[1] * X.y + cam->R[2] * X.z + cam->t[0];
    float ty = cam->R[3] * X.x + cam->R[4] * X.y + cam->R[5] * X.z + cam->t[1];
    float tz = cam->R[6] * X.x + cam->R[7] * X.y + cam->R[8] * X.z + cam->t[2];
    *depth = cam->K[6] * tx + cam->K[7] * ty + cam->K[8] * tz;
    *px = (cam->K[0] * tx + cam->K[1] * ty + cam->K[2] * tz) / *depth;
    *py = (cam->K[3] * tx + cam->K[4] * ty + cam->K[5] * tz) / *depth;
}

static double cv_norm3(const float *v) {
    double s = 0;
    for (int i = 0; i < 3; ++i) {
        double x = v[i];
        s += x * x;
    }
    return sqrt(s);
}

static float get_angle(const float *v1, const float *v2) {
    float dot_product = v1[0] * v2[0] + v1[1] * v2[1] + v1[2] * v2[2];
    float angle = acosf((float)(dot_product / (cv_norm3(v1) * cv_norm3(v2))));
    if (angle != angle) return 0.0f;
    return angle;
}

static int int_x86(float v) {
    if (!(v >= -2147483648.0f && v < 2147483648.0f)) return INT_MIN;
    return (int)v;
}

static float conf_at_float(const oracle_fusion_view *v, int r, int c) {
    const size_t n = (size_t)v->width * v->height;
    const size_t o = (size_t)r * v->width + 4 * (size_t)c;
    uint8_t b[4];
    for (int k = 0; k < 4; ++k) b[k] = (v->confidence && o + k < n) ? v->confidence[o + k] : 0;
    uint32_t u = (uint32_t)b[0] | (uint32_t)b[1] << 8 | (uint32_t)b[2] << 16 | (uint32_t)b[3] << 24;
    float f;
    memcpy(&f, &u, 4);
    return f;
}

/* imageIdToindexMap: emplace keeps the first index of an id; operator[] on a missing id inserts 0. */
static int index_of(int n, const oracle_fusion_view *v, int id) {
    for (int i = 0; i < n; ++i)
        if (v[i].ref_id == id) return i;
    return 0;
}

enum { WEAK = 0, STRONG = 1 };

/* WeakVisFilter, APD.cpp:972-1026 (per reference view; the reference runs views on a thread pool). */
void oracle_weak_vis_filter(int n, const oracle_fusion_view *v, int ref_index, uint8_t *skip) {
    const int width = v[ref_index].width, height = v[ref_index].height;
    memset(skip, 0, (size_t)width * height);
    for (int r = 0; r < height; ++r) {
        for (int c = 0; c < width; ++c) {
            if (v[ref_index].weak[(size_t)r * width + c] != WEAK) continue;
            float ref_depth = v[ref_index].depth[(size_t)r * width + c];
            f3 PointX = get_3d_point_on_world(c, r, ref_depth, &v[ref_index].camera);
            int strong_occluded = 0, weak_occluded = 0;
            for (int src_index = 0; src_index < n; ++src_index) {
                const apd_camera *ref_cam = &v[ref_index].camera, *src_cam = &v[src_index].camera;
                if (ref_index == src_index) continue;
                float a[3] = {ref_cam->c[0] - PointX.x, ref_cam->c[1] - PointX.y, ref_cam->c[2] - PointX.z};
                float b[3] = {src_cam->c[0] - PointX.x, src_cam->c[1] - PointX.y, src_cam->c[2] - PointX.z};
                float angle = get_angle(a, b);
                angle = (float)(angle * 180.0f / M_PI);
                if (angle > 80.0f) continue;
                float px, py, proj_depth;
                project_camera(PointX, src_cam, &px, &py, &proj_depth);
                if (proj_depth <= 0.0f) continue;
                int src_r = int_x86(py + 0.5f), src_c = int_x86(px + 0.5f);
                const int src_cols = v[src_index].width, src_rows = v[src_index].height;
                if (src_c >= 0 && src_c < src_cols && src_r >= 0 && src_r < src_rows) {
                    const size_t sp = (size_t)src_r * src_cols + src_c;
                    float src_depth = v[src_index].depth[sp];
                    if (v[src_index].weak[sp] == STRONG) {
                        if (proj_depth < src_depth - 0.01f * src_depth) strong_occluded++;
                    } else if (v[src_index].weak[sp] == WEAK) {
                        if (conf_at_float(&v[src_index], src_r, src_c) < conf_at_float(&v[ref_index], r, c)) {
                            if (proj_depth < src_depth - 0.01f * src_depth) weak_occluded++;
                        }
                    }
                }
            }
            if (strong_occluded >= 2 || weak_occluded >= 4) skip[(size_t)r * width + c] = 1;
        }
    }
}

/* Per-(pixel, source) quantities of RunFusion / RunFusion_TAT_* (APD.cpp:1166-1187) for view `ref`
   against source VIEW INDICES src[0..num_src), without masks: out index p*num_src + j.
   sp = source pixel (-1: out of bounds or source depth <= 0); dist = reproj_error,
   rel = relative_depth_diff, angle = GetAngle, q = its acosf argument. Unset for depth <= 0. */
void oracle_fusion_candidates(const oracle_fusion_view *v, int ref, int num_src, const int32_t *src, int32_t *sp_out,
                              float *dist_out, float *rel_out, float *angle_out, float *q_out) {
    const oracle_fusion_view *rv = &v[ref];
    for (int r = 0; r < rv->height; ++r)
        for (int c = 0; c < rv->width; ++c) {
            const size_t p = (size_t)r * rv->width + c;
            float ref_depth = rv->depth[p];
            for (int j = 0; j < num_src; ++j) sp_out[p * num_src + j] = -1;
            if (ref_depth <= 0.0) continue;
            const float *ref_normal = rv->normal + 3 * p;
            f3 PointX = get_3d_point_on_world(c, r, ref_depth, &rv->camera);
            for (int j = 0; j < num_src; ++j) {
                const oracle_fusion_view *sv = &v[src[j]];
                float px, py, proj_depth;
                project_camera(PointX, &sv->camera, &px, &py, &proj_depth);
                int src_r = int_x86(py + 0.5f), src_c = int_x86(px + 0.5f);
                if (!(src_c >= 0 && src_c < sv->width && src_r >= 0 && src_r < sv->height)) continue;
                const size_t spx = (size_t)src_r * sv->width + src_c;
                float src_depth = sv->depth[spx];
                if (src_depth <= 0.0) continue;
                const float *src_normal = sv->normal + 3 * spx;
                f3 tmp_X = get_3d_point_on_world(src_c, src_r, src_depth, &sv->camera);
                float tx, ty;
                project_camera(tmp_X, &rv->camera, &tx, &ty, &proj_depth);
                const size_t o = p * num_src + j;
                sp_out[o] = (int32_t)spx;
                dist_out[o] = (float)sqrt(pow(c - tx, 2) + pow(r - ty, 2));
                rel_out[o] = fabsf(proj_depth - ref_depth) / ref_depth;
                angle_out[o] = get_angle(ref_normal, src_normal);
                float dot = ref_normal[0] * src_normal[0] + ref_normal[1] * src_normal[1] + ref_normal[2] * src_normal[2];
                q_out[o] = (float)(dot / (cv_norm3(ref_normal) * cv_norm3(src_normal)));
            }
        }
}

typedef struct {
    float *xyz, *bgr;
    int64_t count, cap;
} cloud;

static void emit(cloud *pc, f3 p, const float col[3]) {
    if (pc->count < pc->cap) {
        pc->xyz[3 * pc->count] = p.x;
        pc->xyz[3 * pc->count + 1] = p.y;
        pc->xyz[3 * pc->count + 2] = p.z;
        pc->bgr[3 * pc->count] = col[0];
        pc->bgr[3 * pc->count + 1] = col[1];
        pc->bgr[3 * pc->count + 2] = col[2];
    }
    pc->count++;
}

static const uint8_t *bgr_at(const oracle_fusion_view *v, int r, int c) {
    return v->bgr + 3 * ((size_t)r * v->width + c);
}

/* RunFusion core loop, APD.cpp:1140-1222. */
static void run_fusion_default(int n, const oracle_fusion_view *v, uint8_t **masks, uint8_t **skip, cloud *pc) {
    for (int i = 0; i < n; ++i) {
        int ref_index = index_of(n, v, v[i].ref_id);
        const oracle_fusion_view *rv = &v[ref_index];
        const int cols = rv->width, rows = rv->height;
        int num_ngb = v[i].num_src;
        int *used_c = malloc(sizeof(int) * (num_ngb > 0 ? num_ngb : 1));
        int *used_r = malloc(sizeof(int) * (num_ngb > 0 ? num_ngb : 1));
        for (int r = 0; r < rows; ++r) {
            for (int c = 0; c < cols; ++c) {
                const size_t p = (size_t)r * cols + c;
                if (masks[ref_index][p] == 1) continue;
                if (skip[ref_index][p] == 1) continue;
                float ref_depth = rv->depth[p];
                if (ref_depth <= 0.0) continue;
                const float *ref_normal = rv->normal + 3 * p;
                f3 PointX = get_3d_point_on_world(c, r, ref_depth, &rv->camera);
                f3 consistent_Point = PointX;
                int num_consistent = 0;
                float dynamic_consistency = 0.0f;
                for (int j = 0; j < num_ngb; ++j) used_c[j] = used_r[j] = -1;
                for (int j = 0; j < num_ngb; ++j) {
                    int src_index = index_of(n, v, v[i].src_ids[j]);
                    const oracle_fusion_view *sv = &v[src_index];
                    const int src_cols = sv->width, src_rows = sv->height;
                    float px, py, proj_depth;
                    project_camera(PointX, &sv->camera, &px, &py, &proj_depth);
                    int src_r = int_x86(py + 0.5f), src_c = int_x86(px + 0.5f);
                    if (src_c >= 0 && src_c < src_cols && src_r >= 0 && src_r < src_rows) {
                        const size_t sp = (size_t)src_r * src_cols + src_c;
                        if (masks[src_index][sp] == 1) continue;
                        float src_depth = sv->depth[sp];
                        if (src_depth <= 0.0) continue;
                        const float *src_normal = sv->normal + 3 * sp;
                        f3 tmp_X = get_3d_point_on_world(src_c, src_r, src_depth, &sv->camera);
                        float tx, ty;
                        project_camera(tmp_X, &rv->camera, &tx, &ty, &proj_depth);
                        float reproj_error = (float)sqrt(pow(c - tx, 2) + pow(r - ty, 2));
                        float relative_depth_diff = fabsf(proj_depth - ref_depth) / ref_depth;
                        float angle = get_angle(ref_normal, src_normal);
                        if (reproj_error < 2.0f && relative_depth_diff < 0.01f && angle < 0.174533f) {
                            used_c[j] = src_c;
                            used_r[j] = src_r;
                            float tmp_index = reproj_error + 200 * relative_depth_diff + angle * 10;
                            dynamic_consistency += expf(-tmp_index);
                            num_consistent++;
                        }
                    }
                }
                float factor = (rv->weak[p] == WEAK ? 0.45f : 0.3f);
                if (num_consistent >= 1 && (dynamic_consistency > factor * num_consistent)) {
                    const uint8_t *rc = bgr_at(rv, r, c);
                    float col[3] = {(float)rc[0], (float)rc[1], (float)rc[2]};
                    for (int j = 0; j < num_ngb; ++j) {
                        if (used_c[j] == -1) continue;
                        int src_index = index_of(n, v, v[i].src_ids[j]);
                        masks[src_index][(size_t)used_r[j] * v[src_index].width + used_c[j]] = 1;
                        const uint8_t *sc = bgr_at(&v[src_index], used_r[j], used_c[j]);
                        col[0] += sc[0];
                        col[1] += sc[1];
                        col[2] += sc[2];
                    }
                    col[0] /= (num_consistent + 1);
                    col[1] /= (num_consistent + 1);
                    col[2] /= (num_consistent + 1);
                    emit(pc, consistent_Point, col);
                }
            }
        }
        free(used_c);
        free(used_r);
    }
}

typedef struct {
    float dist, depth, angle;
    int src_r, src_c;
    int use;
} cost_data;

/* RunFusion_TAT_I (variant 1, APD.cpp:1338-1428) / RunFusion_TAT_A (variant 2, :1534-1603). */
static void run_fusion_tat(int variant, int n, const oracle_fusion_view *v, uint8_t **masks, uint8_t **skip,
                           cloud *pc, int64_t *skip_weak_counts) {
    const float dist_base = 0.25f;
    const float depth_base = variant == 1 ? 1.0f / 3500.0f : 1.0f / 3000.0f;
    const float angle_base = 0.06981317007977318f;
    const float angle_grad = 0.05235987755982988f;
    for (int i = 0; i < n; ++i) {
        int ref_index = index_of(n, v, v[i].ref_id);
        const oracle_fusion_view *rv = &v[ref_index];
        const int cols = rv->width, rows = rv->height;
        int num_ngb = v[i].num_src;
        cost_data *diff = malloc(sizeof(cost_data) * (num_ngb > 0 ? num_ngb : 1));
        for (int j = 0; j < num_ngb; ++j) {
            diff[j].dist = FLT_MAX;
            diff[j].depth = FLT_MAX;
            diff[j].angle = FLT_MAX;
            diff[j].src_r = diff[j].src_c = 0;
            diff[j].use = 0;
        }
        int64_t skip_weak = 0;
        for (int r = 0; r < rows; ++r) {
            for (int c = 0; c < cols; ++c) {
                const size_t p = (size_t)r * cols + c;
                if (skip[ref_index][p] == 1) {
                    skip_weak++;
                    continue;
                }
                float ref_depth = rv->depth[p];
                if (ref_depth <= 0.0) continue;
                const float *ref_normal = rv->normal + 3 * p;
                f3 PointX = get_3d_point_on_world(c, r, ref_depth, &rv->camera);
                f3 consistent_Point = PointX;
                for (int j = 0; j < num_ngb; ++j) {
                    int src_index = index_of(n, v, v[i].src_ids[j]);
                    const oracle_fusion_view *sv = &v[src_index];
                    const int src_cols = sv->width, src_rows = sv->height;
                    float px, py, proj_depth;
                    project_camera(PointX, &sv->camera, &px, &py, &proj_depth);
                    int src_r = int_x86(py + 0.5f), src_c = int_x86(px + 0.5f);
                    if (src_c >= 0 && src_c < src_cols && src_r >= 0 && src_r < src_rows) {
                        const size_t sp = (size_t)src_r * src_cols + src_c;
                        if (masks[src_index][sp] == 1) continue;
                        float src_depth = sv->depth[sp];
                        if (src_depth <= 0.0) continue;
                        const float *src_normal = sv->normal + 3 * sp;
                        f3 tmp_X = get_3d_point_on_world(src_c, src_r, src_depth, &sv->camera);
                        float tx, ty;
                        project_camera(tmp_X, &rv->camera, &tx, &ty, &proj_depth);
                        float reproj_error = (float)sqrt(pow(c - tx, 2) + pow(r - ty, 2));
                        float relative_depth_diff = fabsf(proj_depth - ref_depth) / ref_depth;
                        float angle = get_angle(ref_normal, src_normal);
                        diff[j].dist = reproj_error;
                        diff[j].depth = relative_depth_diff;
                        diff[j].angle = angle;
                        diff[j].src_r = src_r;
                        diff[j].src_c = src_c;
                    }
                }
                for (int k = 2; k <= num_ngb; ++k) {
                    int count = 0;
                    for (int j = 0; j < num_ngb; ++j) {
                        diff[j].use = 0;
                        int pass = diff[j].dist < k * dist_base && diff[j].depth < k * depth_base;
                        if (variant == 1) pass = pass && diff[j].angle < (k * angle_grad + angle_base);
                        if (pass) {
                            count++;
                            diff[j].use = 1;
                        }
                    }
                    if (count >= k) {
                        const uint8_t *rc = bgr_at(rv, r, c);
                        float col[3] = {(float)rc[0], (float)rc[1], (float)rc[2]};
                        if (variant == 1) {
                            for (int j = 0; j < num_ngb; ++j) {
                                if (!diff[j].use) continue;
                                int src_index = index_of(n, v, v[i].src_ids[j]);
                                const uint8_t *sc = bgr_at(&v[src_index], diff[j].src_r, diff[j].src_c);
                                col[0] += (float)sc[0];
                                col[1] += (float)sc[1];
                                col[2] += (float)sc[2];
                            }
                            col[0] /= (count + 1.0f);
                            col[1] /= (count + 1.0f);
                            col[2] /= (count + 1.0f);
                        }
                        emit(pc, consistent_Point, col);
                        masks[ref_index][p] = 1;
                        break;
                    }
                }
            }
        }
        if (skip_weak_counts) skip_weak_counts[i] = skip_weak;
        free(diff);
    }
}

/* Whole fusion. skip_out[i] (may be NULL) receives view i's WeakVisFilter flags; skip_weak_counts
   (TAT_A's printed "skip_weak" per image, may be NULL). Returns the number of points (only the first
   `cap` are stored; colours are the float values before the PLY's uchar cast). */
int64_t oracle_fusion(int variant, int n, const oracle_fusion_view *v, int weak_filter, uint8_t **skip_out,
                      float *xyz, float *bgr, int64_t cap, int64_t *skip_weak_counts) {
    uint8_t **masks = calloc((size_t)n, sizeof(uint8_t *));
    uint8_t **skip = calloc((size_t)n, sizeof(uint8_t *));
    for (int i = 0; i < n; ++i) {
        masks[i] = calloc((size_t)v[i].width * v[i].height, 1);
        skip[i] = calloc((size_t)v[i].width * v[i].height, 1);
    }
    if (weak_filter) {
#pragma omp parallel for schedule(dynamic, 1)
        for (int i = 0; i < n; ++i) oracle_weak_vis_filter(n, v, i, skip[i]);
    }
    if (skip_out)
        for (int i = 0; i < n; ++i)
            if (skip_out[i]) memcpy(skip_out[i], skip[i], (size_t)v[i].width * v[i].height);
    cloud pc = {xyz, bgr, 0, cap};
    if (variant == 0)
        run_fusion_default(n, v, masks, skip, &pc);
    else
        run_fusion_tat(variant, n, v, masks, skip, &pc, skip_weak_counts);
    for (int i = 0; i < n; ++i) {
        free(masks[i]);
        free(skip[i]);
    }
    free(masks);
    free(skip);
    return pc.count;
}
