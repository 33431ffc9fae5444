// capi.cpp -- C entry points over the host helpers (image decode, OpenCV-rule resize, cam.txt / pair.txt
// parsing) as libapdhost.so: used by the multi-process scan runner (apde-mvs_amd/scan_runner.py) and by
// the CPU tests (tests/test_host.py).
#include <cstring>
#include <string>

#include "image.h"
#include "io.h"

using namespace apdhost;

extern "C" {
// decode an image file to gray; returns width*height (copied into out if out_cap suffices) or < 0
long apdhost_read_gray8(const char *path, unsigned char *out, long out_cap, int *w, int *h) {
    Gray8 g;
    std::string err;
    if (!read_gray8(path, g, err)) return -1;
    *w = g.width;
    *h = g.height;
    const long n = (long)g.px.size();
    if (out && out_cap >= n) memcpy(out, g.px.data(), n);
    return n;
}
void apdhost_resize_linear_f32(const float *src, int sw, int sh, float *dst, int dw, int dh) {
    resize_linear_f32(src, sw, sh, dst, dw, dh);
}
void apdhost_resize_nearest(const void *src, int sw, int sh, void *dst, int dw, int dh, int elem) {
    resize_nearest(src, sw, sh, dst, dw, dh, elem);
}
int apdhost_read_camera(const char *path, apd_camera *cam) { return read_camera(path, *cam) ? 0 : -1; }
// ReadBinMat (APD.cpp:18-56): payload bytes (copied into out if out_cap suffices) or -1 when the file
// is missing, malformed or truncated (then no Mat at all, not a partly filled one)
long apdhost_read_binmat(const char *path, void *out, long out_cap, int *rows, int *cols, int *type) {
    Mat m;
    if (!read_binmat_file(path, m)) return m.empty() ? -1 : -2;
    *rows = m.rows;
    *cols = m.cols;
    *type = m.type;
    const long n = (long)m.size_bytes();
    if (out && out_cap >= n) memcpy(out, m.bytes(), n);
    return n;
}
}

#include "fusion.h"
extern "C" {
// cv::imread(IMREAD_COLOR): BGR bytes; same return convention as apdhost_read_gray8
long apdhost_read_bgr8(const char *path, unsigned char *out, long out_cap, int *w, int *h) {
    Bgr8 g;
    std::string err;
    if (!read_bgr8(path, g, err)) return -1;
    *w = g.width;
    *h = g.height;
    const long n = (long)g.px.size();
    if (out && out_cap >= n) memcpy(out, g.px.data(), n);
    return n;
}
void apdhost_resize_linear_u8c3(const unsigned char *src, int sw, int sh, unsigned char *dst, int dw, int dh) {
    resize_linear_u8c3(src, sw, sh, dst, dw, dh);
}
int apdhost_write_png_gray8(const char *path, const unsigned char *px, int w, int h) {
    return write_png_gray8(path, px, w, h) ? 0 : -1;
}
float apdhost_angle_cut_lt(float t) { return angle_cut_lt(t); }
float apdhost_view_cut_deg(float d) { return view_cut_deg(d); }
}
