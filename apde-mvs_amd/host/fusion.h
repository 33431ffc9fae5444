// fusion.h — depth-map fusion of the `apd` driver: RunFusion / RunFusion_TAT_I / RunFusion_TAT_A
// (APD.cpp:1051-1608) with WeakVisFilter (APD.cpp:962-1049) and the PLY writer (APD.cpp:316-356).
//
// Split: the per-(pixel, source) reprojection tests run on the GPU (include/apd_fusion.h); this file
// loads the views, derives the exact angle cuts the kernels compare against, and replays the
// reference's ordered commit (masks, the TAT cost cache, colours, point order) on the host.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "io.h"

namespace apdhost {

struct FusionOptions {
    std::string dense_folder;
    std::string dataset = "DTU";  // "TaT_a" -> RunFusion_TAT_A, "TaT_i" -> RunFusion_TAT_I, else RunFusion
    bool weak_filter = true;
    bool export_color = true;
    int device = 0;
    std::string name = "APD.ply";
};

struct FusionReport {
    int64_t points = 0;
    double load_ms = 0, upload_ms = 0, filter_ms = 0, fuse_ms = 0, write_ms = 0;
    double gpu_ms = 0;     // sum of the device calls (kernel + copy) inside filter/fuse
    double term_ms = 0;    // parallel host evaluation of the candidates' exp terms (RunFusion)
    double commit_ms = 0;  // sequential ordered commit
};

// Runs the whole fusion and writes <dense>/APD/<name> (+ APD/<id>/skip.png with the weak filter).
bool run_fusion(const std::vector<Problem> &problems, const FusionOptions &opt, MatStore &store, FusionReport &rep,
                std::string &err);

// Exact q-space cuts of GetAngle (APD.cpp:902-910) for the kernels, from glibc acosf:
//   angle_cut_lt(T): largest float q in [-1,1] with acosf(q) >= T   ("angle < T" <=> q > cut)
//   view_cut_deg(D): smallest float q in [-1,1] with deg(q) <= D, deg(q) = (float)(acosf(q)*180.0f / M_PI)
//                    ("angle_deg > D" <=> q < cut)
// Both verify monotonicity over a window around the cut and throw std::runtime_error otherwise.
float angle_cut_lt(float T);
float view_cut_deg(float D);

void write_ply(const std::string &path, const std::vector<float> &xyz, const std::vector<float> &bgr,
               bool export_color);

}  // namespace apdhost
