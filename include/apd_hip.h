/*
 * apd_hip.h — C-ABI of the MI355X-native PatchMatch depth engine (libapd_hip.so).
 *
 * This is the drop-in boundary for the per-reference-view PatchMatch hot path of APDe-MVS.
 * It replaces the in-process `class APD` lifecycle of the reference:
 *
 *   reference (APD.h:88-190, APD.cpp:458-842, APD.cu:2663-2737)      this ABI
 *   ---------------------------------------------------------------  -----------------------------
 *   APD::APD(const Problem&)                   APD.cpp:458             apd_create()
 *   APD::InuputInitialization()                APD.cpp:501-685  \
 *   APD::CudaSpaceInitialization()             APD.cpp:687-788   >     apd_set_problem()
 *   APD::SetDataPassHelperInCuda()             APD.cpp:790-814  /
 *   APD::RunPatchMatch()                       APD.cu:2663-2737        apd_run_patchmatch()
 *   APD::GetPlaneHypothesis / GetPixelStates / GetConfidence
 *                                              APD.cpp:816-826         apd_get_results()
 *   APD::~APD()                                APD.cpp:463-499         apd_destroy()
 *   CudaSafeCall / exit(EXIT_FAILURE)          APD.cpp:417-450         return codes + apd_last_error()
 *
 * Host-side file I/O (cv::imread, cv::resize, pair.txt / cam.txt parsing, bin-mat writing) stays
 * outside the library, in the `apd` driver (apde-mvs_amd/host), exactly as it lives outside the
 * CUDA kernels in the reference (APD.cpp:501-685, main.cpp).
 *
 * Conventions
 *  - Plain C types only: pointers + sizes; no torch / HIP types in any signature.
 *  - Images are H*W row-major float32 gray values (already resized to the pass resolution),
 *    index 0 = reference view, 1..N = source views (N <= 31, MAX_IMAGES 32, main.h:40).
 *  - Planes ("plane hypotheses") are float4 {x,y,z,w}: on input (init_planes) and output they are
 *    {world-frame normal, depth} exactly like plane_hypotheses_host after GetDepthandNormal
 *    (APD.cu:1694-1709, APD.cpp:661-683).
 *  - Every entry point returns APD_OK (0) or a negative apd_status; it never calls exit().
 *  - One apd_ctx per device; a ctx is bound to one HIP stream and is not thread-safe. Several ctxs
 *    (one per GPU) may run concurrently from different threads / processes.
 */
#ifndef APD_HIP_H_
#define APD_HIP_H_

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define APD_ABI_VERSION 3  /* 2: apd_timing.lists_ms / pairs_ms, 9 profiling counters, kinds 4-7;
                                  3: apd_timing.join_ms / prepare_ms, apd_get_prepare_timing */
#define APD_MAX_IMAGES 32          /* main.h:40  MAX_IMAGES            */
#define APD_ANCHOR_NUM 9           /* main.h:41  ANCHOR_NUM            */
#define APD_MAX_SEARCH_RADIUS 4096 /* main.h:42  MAX_SEARCH_RADIUS     */
#define APD_CURVE_SAMPLES 61       /* main.h:45  RELIABLE_CURVE_SAMPLE_NUM */

typedef enum apd_status {
    APD_OK = 0,
    APD_EINVAL = -1,          /* bad argument / unsupported parameter value            */
    APD_ENOMEM = -2,          /* device or host allocation failed                      */
    APD_EDEVICE = -3,         /* HIP runtime error (launch, copy, no device)           */
    APD_ETOOMANYVIEWS = -4,   /* num_images > APD_MAX_IMAGES (APD.cpp:528-531 exits)    */
    APD_ESTATE = -5           /* call out of lifecycle order (e.g. run before set)     */
} apd_status;

/* RunState, main.h:68-72 */
enum { APD_FIRST_INIT = 0, APD_REFINE_INIT = 1, APD_REFINE_ITER = 2 };
/* PixelState, main.h:74-78 */
enum { APD_WEAK = 0, APD_STRONG = 1, APD_UNKNOWN = 2 };

/* Byte-compatible with `struct Camera` (main.h:50-61): 120 bytes. */
typedef struct apd_camera {
    float K[9];
    float R[9];
    float t[3];
    float c[3];           /* camera centre in world coords (APD.cpp:114-119) */
    int32_t height;
    int32_t width;
    float depth_min;
    float depth_max;
    float interval;
    float depth_num;
} apd_camera;

/* Mirrors `struct PatchMatchParams` (main.h:80-100). The reference's `bool` members are int32 here
 * so the ABI has no implementation-defined layout. depth_min/depth_max are the *already scaled*
 * range (cam.depth_min*0.6, cam.depth_max*1.2, APD.cpp:554-555). strong/weak radius/increment must
 * be the reference defaults (5/2 and 5/5; main.cpp never changes them): the kernels are
 * specialised for those window shapes and apd_set_problem rejects anything else with APD_EINVAL. */
typedef struct apd_params {
    int32_t max_iterations;   /* 3   */
    int32_t num_images;       /* ref + src, <= 32 */
    int32_t top_k;            /* 4   */
    float depth_min;
    float depth_max;
    int32_t geom_consistency; /* bool */
    int32_t use_impetus;      /* bool */
    int32_t strong_radius;    /* 5   */
    int32_t strong_increment; /* 2   */
    int32_t weak_radius;      /* 5   */
    int32_t weak_increment;   /* 5   */
    int32_t use_APD;          /* bool */
    int32_t use_sa;           /* bool (host-side only: decides whether sa_mask is passed) */
    int32_t weak_peak_radius; /* 2..6 */
    int32_t rotate_time;      /* 1, 2 or 4 */
    float ransac_threshold;
    float geom_factor;        /* 0.2 ETH/DTU/General, 0.05 TaT (main.cpp:293-299) */
    int32_t state;            /* APD_FIRST_INIT / APD_REFINE_INIT / APD_REFINE_ITER */
} apd_params;

/* One Problem (main.h:102-115) at its pass resolution, with every input the reference reads in
 * InuputInitialization (APD.cpp:501-685), already decoded/resized by the host. */
typedef struct apd_problem {
    int32_t width;
    int32_t height;
    int32_t num_images;                /* ref + src                                          */
    const float *const *images;        /* [num_images] -> H*W float32                         */
    const apd_camera *cameras;         /* [num_images], K already scaled (APD.cpp:580-585)    */
    apd_params params;
    /* geom_consistency || use_APD: [num_images] -> H*W depth maps (index 0 = own prior),
       already resized INTER_NEAREST (APD.cpp:592-610). NULL otherwise. */
    const float *const *depths;
    /* state != FIRST_INIT: H*W*4 floats {world normal xyz, depth} (APD.cpp:661-683). */
    const float *init_planes;
    /* use_APD: H*W PixelState bytes and confidence bytes (APD.cpp:614-626); NULL otherwise
       (then every pixel is STRONG and confidence 1, APD.cpp:655-658). */
    const uint8_t *weak_info;
    const uint8_t *confidence;
    /* use_APD && use_sa && mask present: H*W segment labels (APD.cpp:641-652); NULL = all 0. */
    const uint8_t *sa_mask;
    /* Deterministic RNG contract (replaces curand_init(clock64(),...), APD.cu:904-917). */
    uint64_t seed;
    /* Problem::export_reliable_curve (main.h:111): keep DepthToWeak's 61-sample cost curves so
       apd_get_results can return them in apd_outputs.reliable_curve (APD.cu:2713-2724). */
    int32_t export_reliable_curve;
} apd_problem;

/* Caller-allocated outputs (D2H of APD.cu:2731-2736). Any pointer may be NULL to skip it. */
typedef struct apd_outputs {
    float *planes;             /* H*W*4: {world normal xyz, depth} (after GetDepthandNormal, filter, LocalRefine) */
    uint8_t *weak_info;        /* H*W PixelState after DepthToWeak / ConfidenceCompute */
    uint8_t *confidence;       /* H*W (valid iff geom_consistency || use_APD)         */
    float *costs;              /* H*W final matching cost                            */
    uint32_t *selected_views;  /* H*W view bitmask                                   */
    uint8_t *view_weights;     /* N*H*W (view-major) sampled view weights, N = num_images-1 */
    int16_t *anchors;          /* weak_count*9*2 (x,y) anchors, APD.cu:2614-2626 export   */
    int32_t *weak_count;       /* out: number of WEAK pixels in the input weak_info       */
    float *reliable_curve;     /* H*W*61 DepthToWeak cost curves (APD.cu:2188-2198), optional */
} apd_outputs;

/* Device-time breakdown of the last apd_run_patchmatch (HIP events on the ctx stream), ms. */
typedef struct apd_timing {
    float total_ms;            /* whole RunPatchMatch bracket (main.cpp:157-159 equivalent) */
    float init_ms;             /* RandomInitialization (beside the lists and the pair table
                                  on a side stream, so the phases may sum to more than total) */
    float anchors_ms;          /* FindNearestStrongPoint + GenAnchors + NeigbourUpdate      */
    float sweep_ms;            /* all sweep iterations (Strong + RANSAC fit + Weak)         */
    float post_ms;             /* GetDepthandNormal + filter + DepthToWeak + Confidence + LocalRefine */
    float iter_ms[8];          /* per-iteration sweep time (first 8 iterations)             */
    int32_t iterations;
    float lists_ms;            /* the sweeps' pixel lists (after NeigbourUpdate)            */
    float pairs_ms;            /* the Weak candidates' image-wide pair table (APD passes) and
                                  the anchor-window records it reads                         */
    float join_ms;             /* the wait for RandomInitialization after the pair table    */
    float prepare_ms;          /* apd_stage_prepare's bracket: anchors .. join               */
    /* Serial ctx (APD_NO_OVERLAP=1): total_ms == anchors_ms + lists_ms + pairs_ms + init_ms
       + sweep_ms + post_ms. Overlapped (default): RandomInitialization runs on a side stream from
       the end of the anchors, so prepare_ms == anchors_ms + lists_ms + pairs_ms + join_ms and
       total_ms == prepare_ms + sweep_ms + post_ms; init_ms is then RandomInitialization's own
       span, overlapping lists_ms + pairs_ms. */
} apd_timing;

typedef struct apd_ctx apd_ctx;

/* Library / device queries. */
int32_t apd_abi_version(void);
int32_t apd_device_count(void);

/* apd_create: bind a new context to HIP device `device` (cudaSetDevice, main.cpp:264). Returns
   NULL on failure; the reason is available from apd_last_error(NULL). */
apd_ctx *apd_create(int32_t device);
void apd_destroy(apd_ctx *ctx);
const char *apd_last_error(const apd_ctx *ctx);

/* Upload one problem: images (plus the LDS/quad gather layout built on device), cameras, priors,
   masks, params. Device buffers are reused across problems of the same or smaller size. Every array
   pointer of the problem (images, depths, init_planes, weak_info, confidence, sa_mask) may be a host
   pointer or a device pointer on the ctx's device (the copies use hipMemcpyDefault): a caller that
   keeps a scan's images and depth maps resident in HBM passes device pointers and nothing crosses
   PCIe. The per-problem statistics (WEAK count, largest confidence, SA labels present, fp16-texel
   eligibility) are computed on the device. */
int32_t apd_set_problem(apd_ctx *ctx, const apd_problem *problem);

/* Run the full RunPatchMatch kernel sequence (APD.cu:2663-2737) on the loaded problem. */
int32_t apd_run_patchmatch(apd_ctx *ctx);

/* Fine-grained stages of the same sequence, for benchmarking the per-iteration metric:
   apd_stage_prepare = InitRandomStates..RandomInitialization (APD.cu:2685-2697);
   apd_stage_iteration(i) = loop body i (APD.cu:2700-2707);
   apd_stage_finish = GetDepthandNormal..LocalRefine (APD.cu:2710-2729).
   prepare + iteration(0..max_iterations-1) + finish == apd_run_patchmatch. */
int32_t apd_stage_prepare(apd_ctx *ctx);
int32_t apd_stage_iteration(apd_ctx *ctx, int32_t iter);
int32_t apd_stage_finish(apd_ctx *ctx);

/* Block until every launch on the ctx stream completed. */
int32_t apd_synchronize(apd_ctx *ctx);

/* Copy results out (GetPlaneHypothesis/GetPixelStates/GetConfidence, APD.cpp:816-826); every
   output pointer may be a host buffer or a device buffer on the ctx's device. */
int32_t apd_get_results(apd_ctx *ctx, const apd_outputs *out);

/* Device timing of the last apd_run_patchmatch. */
int32_t apd_get_timing(apd_ctx *ctx, apd_timing *timing);

/* The prepare-phase fields (anchors_ms, lists_ms, pairs_ms, init_ms, join_ms, prepare_ms) of the
   last apd_stage_prepare, whether or not apd_run_patchmatch ran it; the other fields are zero.
   Waits for the ctx stream. bench.py charges pairs_ms to the iterations of a staged pass. */
int32_t apd_get_prepare_timing(apd_ctx *ctx, apd_timing *timing);

/* Profiling of the loop-body kernels (APD.cu:2699-2708), used by bench.py for roofline.achieved.
   apd_profile_reset(ctx, 1) clears and enables it: every later launch of the kinds below is
   bracketed by HIP events on the ctx stream, and the device counters below are accumulated.
   apd_profile_kernel: total duration (ms), launch count and pixels covered by the launches of one
   kind since the reset. apd_profile_query == apd_profile_kernel(APD_PROF_STRONG_SWEEP). */
#define APD_PROF_STRONG_SWEEP 0 /* k_sweep_strong_vm (CheckerboardPropagationStrong, APD.cu:1098-1440) */
#define APD_PROF_RANSAC_FIT 1   /* k_ransac_fit (RANSACToGetFitPlane, APD.cu:2486-2598)             */
#define APD_PROF_WEAK_CAND 2    /* the Weak sweep's anchor candidates: the SUM of the kernel brackets
                                   of k_gp_cost + k_weak_cand_g + k_weak_cand_comb (the image-wide pair
                                   table). k_gp_cost runs on side stream 1 beside k_weak_cand_g, so
                                   with overlap this counts the overlapped time twice: it is not an
                                   elapsed time -- rate math uses APD_PROF_WEAK_PATH              */
#define APD_PROF_WEAK_SWEEP 3   /* k_sweep_weak_vm (CheckerboardPropagationWeak, APD.cu:1442-1615)   */
#define APD_PROF_DEPTH_TO_WEAK 4 /* k_depth_to_weak_vm (DepthToWeak, APD.cu:2103-2250)                */
#define APD_PROF_GP_COST 5      /* k_gp_cost alone (pair windows, inside APD_PROF_WEAK_CAND)         */
#define APD_PROF_WEAK_CAND_G 6  /* k_weak_cand_g alone (centre windows, inside APD_PROF_WEAK_CAND)    */
#define APD_PROF_WEAK_CAND_COMB 7 /* k_weak_cand_comb alone (focal combination, inside WEAK_CAND)   */
#define APD_PROF_WEAK_PATH 8    /* wall time from the end of the Strong sweeps to the end of the Weak
                                   sweeps: RANSAC and k_gp_cost run on side streams beside the
                                   candidate kernels, so the kernels' own brackets overlap           */
int32_t apd_profile_reset(apd_ctx *ctx, int32_t enable);
int32_t apd_profile_kernel(apd_ctx *ctx, int32_t kind, double *ms_total, int64_t *launches,
                           int64_t *pixels);
int32_t apd_profile_query(apd_ctx *ctx, double *sweep_ms_total, int64_t *sweep_launches,
                          int64_t *sweep_pixels);
/* Device counters since the reset, so bench.py prices roofline.achieved on work done, not on an
   upper bound. counts[0..n-1] (n <= APD_PROF_COUNTERS; extra entries are zeroed):
   [0] NCC-Old evaluations the Strong sweep launches issued (valid propagation candidates + current
       plane + refinement candidates of views with weight > 0);
   [1] NCC-New evaluations of the Weak sweep: valid anchor candidates x N + current plane x views
       with weight > 0 (the values CheckerboardPropagationWeak needs, however the engine obtained
       them: the image-wide pair table, RandomInitialization's kept costs, or the
       sweep itself), plus the fit-plane and refinement-candidate evaluations of views with weight
       > 0 the sweep actually issued (those its exact early exit proves unnecessary are not counted);
   [2] geometric-consistency terms of the same evaluations (APD.cu:1561, 1583, 1037, 1079);
   [3] NCC-Old evaluations DepthToWeak issued (APD.cu:2155-2186: active pixel x disparity in range x
       selected view; disparities 0 and 60 only with the curve export);
   [4] geometric-consistency terms DepthToWeak issued;
   The rest count what the Weak path's kernels actually evaluated (device-issued work, as opposed to
   [1], the work the reference's CheckerboardPropagationWeak would do):
   [5] 3x3 pair windows k_gp_cost evaluated (pair x view, window inside the source image);
   [6] 6x6 centre windows k_weak_cand_g evaluated;
   [7] 6x6 centre windows k_sweep_weak_vm evaluated itself (current plane, fit plane, refinement
       candidates, and the anchor candidates when no candidate kernel ran);
   [8] 3x3 anchor windows k_sweep_weak_vm evaluated itself.
   apd_profile_evaluations(ctx, &n) == apd_profile_counters(ctx, &n, 1). */
#define APD_PROF_COUNTERS 9
int32_t apd_profile_counters(apd_ctx *ctx, int64_t *counts, int32_t n);
int32_t apd_profile_evaluations(apd_ctx *ctx, int64_t *ncc_evaluations);

/* Device memory for hosts that keep a scan resident in HBM without linking HIP themselves (the `apd`
   binary; APD.cpp:687-788 re-uploads every image and prior per problem instead). Allocations live on
   the ctx's device; copies go in any direction (hipMemcpyDefault) and return when done. */
int32_t apd_device_alloc(apd_ctx *ctx, size_t bytes, void **ptr);
int32_t apd_device_free(apd_ctx *ctx, void *ptr);
int32_t apd_device_copy(apd_ctx *ctx, void *dst, const void *src, size_t bytes);
/* Free and total bytes of the ctx's device (hipMemGetInfo): the `apd` binary sizes its
   device-resident store from it, leaving room for the library's per-problem buffers. */
/* Device memory the ctx's own buffers hold (bytes): the `apd` binary sizes its device store from it. */
int32_t apd_device_bytes(apd_ctx *ctx, size_t *bytes);

/* Copy `bytes` from device memory of src_ctx's device to device memory of dst_ctx's device (the same
   device, or a peer over xGMI with peer access enabled on first use); waits for the copy. The `apd`
   binary moves a Jacobi pass's new view maps between its contexts' device stores with it. */
int32_t apd_device_copy_peer(apd_ctx *dst_ctx, void *dst, apd_ctx *src_ctx, const void *src, size_t bytes);

int32_t apd_device_mem_info(apd_ctx *ctx, size_t *free_bytes, size_t *total_bytes);
/* cv::resize INTER_NEAREST (the priors' resize, APD.cpp:605-672) from a device buffer of sw x sh
   elements of elem_bytes to one of dw x dh, with the host library's index arithmetic. */
int32_t apd_device_resize_nearest(apd_ctx *ctx, const void *src, int32_t sw, int32_t sh, void *dst,
                                  int32_t dw, int32_t dh, int32_t elem_bytes);
/* The last run's results after ProcessProblem's epilogue (main.cpp:168-178), on the device: depth
   (H*W fp32; 0 outside [depth_min, depth_max], as apd_epilogue) and/or planes (H*W x (normal xyz,
   that depth)) -- exactly the depths.bin and the (normals.bin, depths.bin) pair the next pass reads
   as priors. Either pointer may be NULL. */
int32_t apd_result_device(apd_ctx *ctx, float *depth_dev, float *planes_dev);

/* Host epilogue of ProcessProblem (main.cpp:168-178): depth = plane.w clipped to
   [depth_min, depth_max] (else 0 and PixelState UNKNOWN), normal = plane.xyz. Pure host code. */
int32_t apd_epilogue(int32_t width, int32_t height, const float *planes, float depth_min,
                     float depth_max, float *depth_out, float *normal_out, uint8_t *weak_inout);

#ifdef __cplusplus
}
#endif

#endif /* APD_HIP_H_ */
