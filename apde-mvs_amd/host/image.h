// image.h — host-side image input of the `apd` driver (replaces the OpenCV calls of the reference's
// host code: cv::imread(IMREAD_GRAYSCALE) + convertTo(CV_32F) in ReadImage (APD.cpp:137-160) and
// cv::resize INTER_LINEAR / INTER_NEAREST in InuputInitialization (APD.cpp:562-672)).
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace apdhost {

struct Gray8 {
    int width = 0, height = 0;
    std::vector<uint8_t> px;  // row-major
};

// Decode an 8-bit image file to gray. Supported: PNG (8-bit gray / gray+alpha / RGB / RGBA /
// palette, non-interlaced; colour converted like OpenCV's BGR2GRAY fixed-point path), baseline
// JPEG (luma plane = libjpeg's JCS_GRAYSCALE output, islow IDCT), binary PGM/PPM. Returns false and
// fills `err` on anything else.
bool read_gray8(const std::string &path, Gray8 &out, std::string &err);
bool decode_png_gray(const std::vector<uint8_t> &file, Gray8 &out, std::string &err);
bool decode_jpeg_gray(const std::vector<uint8_t> &file, Gray8 &out, std::string &err);
bool decode_pnm_gray(const std::vector<uint8_t> &file, Gray8 &out, std::string &err);

// Colour image, BGR interleaved (cv::imread(IMREAD_COLOR), used by fusion: APD.cpp:1077).
struct Bgr8 {
    int width = 0, height = 0;
    std::vector<uint8_t> px;  // row-major B,G,R
};
// PNG (gray/RGB/palette, alpha stripped), baseline JPEG (libjpeg-turbo default decode: islow IDCT,
// fancy chroma upsampling, jdcolor.c YCbCr->RGB tables), binary PGM/PPM.
bool read_bgr8(const std::string &path, Bgr8 &out, std::string &err);
bool decode_png_bgr(const std::vector<uint8_t> &file, Bgr8 &out, std::string &err);
bool decode_jpeg_bgr(const std::vector<uint8_t> &file, Bgr8 &out, std::string &err);
bool decode_pnm_bgr(const std::vector<uint8_t> &file, Bgr8 &out, std::string &err);
// cv::imwrite of an 8-bit gray image as PNG (skip.png, APD.cpp:1036-1037).
bool write_png_gray8(const std::string &path, const uint8_t *px, int w, int h);
// cv::resize INTER_LINEAR on CV_8UC3 (RescaleImageAndCamera, APD.cpp:857); fixed-point path.
void resize_linear_u8c3(const uint8_t *src, int sw, int sh, uint8_t *dst, int dw, int dh);

// cv::resize(src, dst, Size(dw, dh), 0, 0, INTER_LINEAR) on a CV_32FC1 image (OpenCV 4.x rules:
// half-pixel centres, clamped borders, exact 2x downscale handled as INTER_AREA).
void resize_linear_f32(const float *src, int sw, int sh, float *dst, int dw, int dh);
// cv::resize(..., INTER_NEAREST) for any element size (bytes per pixel = elem).
void resize_nearest(const void *src, int sw, int sh, void *dst, int dw, int dh, int elem);

}  // namespace apdhost
