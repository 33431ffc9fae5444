/*
 * apd_fusion.h — C-ABI of the device half of depth-map fusion (libapd_hip.so).
 *
 * The reference fuses the per-view depth maps into APD.ply on the CPU, single-threaded except for
 * the weak-pixel visibility filter:
 *
 *   reference                                                   this ABI
 *   ----------------------------------------------------------  ------------------------------------
 *   WeakVisFilter                      APD.cpp:962-1049          apd_fusion_weak_filter()
 *   RunFusion   per-(pixel, source) reprojection test
 *                                      APD.cpp:1160-1197         apd_fusion_consistency()
 *   RunFusion_TAT_I / RunFusion_TAT_A  per-(pixel, source) cost + the k-level test
 *                                      APD.cpp:1355-1395, 1559-1583   apd_fusion_tat_levels()
 *   (loaded once: images' depth/normal/weak/confidence + cameras, APD.cpp:1071-1133)
 *                                                                 apd_fusion_set_views()
 *
 * What stays on the host (apde-mvs_amd/host/fusion.cpp): the ordered commit. In RunFusion a
 * consistent pixel marks its source pixels in masks[src] (APD.cpp:1209) and every LATER pixel —
 * of the same view too — skips masked source pixels, so acceptance is inherently sequential in
 * (view, row, column) order. The kernels therefore compute only the mask-independent part of every
 * (pixel, source) test; the host walks pixels in the reference's order, applies the masks, and
 * evaluates acosf/expf (glibc) only for the candidates that passed. In the TAT variants the
 * per-view cost cache `diff` is NOT reset between pixels (APD.cpp:1347), so an unusable source
 * keeps the previous pixel's cost; the host replays that cache from the kernels' per-candidate
 * levels.
 *
 * Angle tests never call acosf on the device: GetAngle (APD.cpp:902-910) is
 *     q = (float)(dot_f32 / ((double)|a| * (double)|b|)),  angle = isnan(acosf(q)) ? 0 : acosf(q)
 * and acosf is monotone, so "angle < T" is "q outside [-1,1] (angle 0) or q > q_T" for the float
 * q_T the host finds by bisection over glibc acosf (fusion.cpp: angle_cut). The kernels take those
 * cuts as arguments and compute q bit-exactly (float dot, double norms, -ffp-contract=off).
 *
 * Conventions as in apd_hip.h: plain C types, APD_OK or a negative apd_status, never exit().
 */
#ifndef APD_FUSION_H_
#define APD_FUSION_H_

#include <stdint.h>
#include "apd_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

/* One view as RunFusion holds it after loading (APD.cpp:1081-1133): depth-map resolution, the
   camera after RescaleImageAndCamera (APD.cpp:844-864), and the four bin-mats of APD/<id>/. */
typedef struct apd_fusion_view {
    int32_t width, height;
    apd_camera camera;
    const float *depth;          /* H*W            depths.bin      CV_32FC1 */
    const float *normal;         /* H*W*3          normals.bin     CV_32FC3 */
    const uint8_t *weak;         /* H*W            weak.bin        CV_8UC1 (PixelState) */
    const uint8_t *confidence;   /* H*W            confidence.bin  CV_8UC1; may be NULL (zeros) */
} apd_fusion_view;

typedef struct apd_fusion_ctx apd_fusion_ctx;

apd_fusion_ctx *apd_fusion_create(int32_t device);
void apd_fusion_destroy(apd_fusion_ctx *ctx);
const char *apd_fusion_last_error(const apd_fusion_ctx *ctx);

/* Upload every view once (all resident in HBM for the whole fusion). */
int32_t apd_fusion_set_views(apd_fusion_ctx *ctx, int32_t num_views, const apd_fusion_view *views);

/* WeakVisFilter for view `ref` (APD.cpp:972-1026): skip[p] = 1 for WEAK pixels occluded in >= 2
   STRONG or >= 4 WEAK views among ALL other views, else 0. `q_view` is the cut for the 80 degree
   view-angle test: a source is ignored iff q in [-1,1] and q < q_view. The confidence comparison
   reproduces the reference's `confidences[i].at<float>(r, c)` on a CV_8UC1 Mat: the float whose
   4 little-endian bytes start at byte r*W + 4*c; bytes past the W*H buffer read as 0 (the
   reference reads whatever follows the allocation there). */
int32_t apd_fusion_weak_filter(apd_fusion_ctx *ctx, int32_t ref, float q_view, uint8_t *skip);

/* RunFusion's reprojection test for view `ref` against sources src[0..num_src) (view indices):
   for every pixel p and source j, out index p*num_src + j:
     src_pix   = sr*W_src + sc of the rounded projection if the source pixel is in bounds, has
                 depth > 0 and passes reproj_error < 2, relative depth < 0.01 and angle < 0.174533
                 (angle test: q outside [-1,1] or q > q_angle); else -1
     err_rel   = reproj_error + 200 * relative_depth_diff (float, the first two terms of tmp_index)
     cos_angle = q of GetAngle(ref_normal, src_normal)
   The masks are NOT applied (host). Values for pixels with depth <= 0 are unspecified. */
int32_t apd_fusion_consistency(apd_fusion_ctx *ctx, int32_t ref, int32_t num_src, const int32_t *src,
                               float q_angle, int32_t *src_pix, float *err_rel, float *cos_angle);

/* TAT_I / TAT_A per-candidate levels for view `ref`: out index p*num_src + j:
     src_pix = sr*W_src + sc if the projection is in bounds and the source depth > 0 (the candidate
               would overwrite diff[j], masks permitting), else -1
     level   = smallest k in [2, num_src] with dist < k*dist_base && depth < k*depth_base
               (&& angle < k*angle_grad + angle_base when q_k != NULL: q outside [-1,1] or
               q > q_k[k]); 255 if none. q_k has num_src+1 entries (index k). */
int32_t apd_fusion_tat_levels(apd_fusion_ctx *ctx, int32_t ref, int32_t num_src, const int32_t *src,
                              float dist_base, float depth_base, const float *q_k, int32_t *src_pix,
                              uint8_t *level);

#ifdef __cplusplus
}
#endif

#endif /* APD_FUSION_H_ */
