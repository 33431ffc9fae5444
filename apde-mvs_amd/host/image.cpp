// image.cpp — gray image decoding and OpenCV-semantics resizing for the `apd` driver.
//
// The reference reads every image with cv::imread(IMREAD_GRAYSCALE) and converts it to CV_32F
// (APD.cpp:137-160), then cv::resize(INTER_LINEAR) to the pass resolution (APD.cpp:562-590) and
// cv::resize(INTER_NEAREST) for the priors (APD.cpp:592-672). OpenCV is not available here, so the
// three operations are restated:
//   * PNG  : zlib inflate + the five PNG filters; colour -> gray with libpng's rgb_to_gray weights
//            (0.299, 0.587 in 1/32768 fixed point), which is what OpenCV's PNG decoder requests.
//   * JPEG : baseline sequential Huffman; the luma component is what libjpeg hands OpenCV for
//            JCS_GRAYSCALE output, reconstructed with libjpeg's "islow" integer IDCT (LL&M, 13-bit
//            constants, 2 pass-1 bits) and its post-IDCT range-limit table.
//   * resize: OpenCV 4.x INTER_LINEAR coefficient rules (half-pixel centres, borders clamped with a
//            zero fraction), exact 2x downscales routed to INTER_AREA as cv::resize does.
// Parity with OpenCV is unpinned for colour PNG/JPEG and for non-integer float resize inputs
// (OpenCV's SIMD paths may contract multiply-adds); gray 8-bit inputs and the 2^-k pyramid are exact.
#include "image.h"

#include <zlib.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <fstream>

#include <sys/stat.h>

namespace apdhost {

static bool read_file(const std::string &path, std::vector<uint8_t> &data) {
    struct stat st;
    if (stat(path.c_str(), &st) != 0 || !S_ISREG(st.st_mode)) return false;  // directories throw in the reads
    std::ifstream f(path, std::ios::binary);
    if (!f) return false;
    data.resize((size_t)st.st_size);
    f.read(reinterpret_cast<char *>(data.data()), (std::streamsize)data.size());
    data.resize((size_t)f.gcount());
    return true;
}

static uint8_t rgb_to_gray(int r, int g, int b) {
    // libpng png_do_rgb_to_gray, 8-bit, no gamma: (rc*R + gc*G + bc*B) >> 15 with rc = 9798,
    // gc = 19235, bc = 32768 - rc - gc; identical channels pass through unchanged.
    if (r == g && r == b) return (uint8_t)r;
    return (uint8_t)((9798 * r + 19235 * g + 3735 * b) >> 15);
}

// ----------------------------------------------------------------------------------------------
// PNG
// ----------------------------------------------------------------------------------------------
static uint32_t be32(const uint8_t *p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; }

namespace {
struct PngRaw {
    int w = 0, h = 0, ctype = 0, ch = 0;
    std::vector<uint8_t> img, plte;  // unfiltered 8-bit samples, w*ch per row
};
}  // namespace

static bool png_raw(const std::vector<uint8_t> &file, PngRaw &png, std::string &err) {
    static const uint8_t sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
    if (file.size() < 8 || memcmp(file.data(), sig, 8) != 0) { err = "not a PNG file"; return false; }
    size_t pos = 8;
    int w = 0, h = 0, depth = 0, ctype = 0, interlace = 0;
    std::vector<uint8_t> idat, plte;
    while (pos + 12 <= file.size()) {
        const uint32_t len = be32(&file[pos]);
        const std::string type(reinterpret_cast<const char *>(&file[pos + 4]), 4);
        if (pos + 12 + (size_t)len > file.size()) { err = "truncated PNG chunk"; return false; }
        const uint8_t *d = &file[pos + 8];
        if (type == "IHDR") {
            if (len < 13) { err = "bad PNG IHDR"; return false; }
            w = (int)be32(d); h = (int)be32(d + 4); depth = d[8]; ctype = d[9]; interlace = d[12];
        } else if (type == "PLTE") {
            plte.assign(d, d + len);
        } else if (type == "IDAT") {
            idat.insert(idat.end(), d, d + len);
        } else if (type == "IEND") {
            break;
        }
        pos += 12 + len;
    }
    if (w <= 0 || h <= 0) { err = "PNG without IHDR"; return false; }
    if ((size_t)w * (size_t)h > ((size_t)1 << 28)) { err = "unsupported PNG size"; return false; }
    if (depth != 8) { err = "only 8-bit PNG is supported"; return false; }
    if (interlace) { err = "interlaced PNG is not supported"; return false; }
    int ch;
    switch (ctype) {
        case 0: ch = 1; break;  // gray
        case 2: ch = 3; break;  // RGB
        case 3: ch = 1; break;  // palette
        case 4: ch = 2; break;  // gray + alpha
        case 6: ch = 4; break;  // RGBA
        default: err = "unsupported PNG colour type"; return false;
    }
    const size_t stride = (size_t)w * ch;
    std::vector<uint8_t> raw((stride + 1) * (size_t)h);
    z_stream zs;
    memset(&zs, 0, sizeof(zs));
    if (inflateInit(&zs) != Z_OK) { err = "inflateInit failed"; return false; }
    zs.next_in = idat.data();
    zs.avail_in = (uInt)idat.size();
    zs.next_out = raw.data();
    zs.avail_out = (uInt)raw.size();
    const int zr = inflate(&zs, Z_FINISH);
    inflateEnd(&zs);
    if (zr != Z_STREAM_END && !(zr == Z_BUF_ERROR && zs.avail_out == 0)) { err = "PNG inflate failed"; return false; }
    // unfilter in place (bytes-per-pixel = ch for 8-bit)
    std::vector<uint8_t> img(stride * (size_t)h);
    for (int y = 0; y < h; ++y) {
        const uint8_t ft = raw[(stride + 1) * y];
        const uint8_t *src = &raw[(stride + 1) * y + 1];
        uint8_t *cur = &img[stride * y];
        const uint8_t *prev = y ? &img[stride * (y - 1)] : nullptr;
        for (size_t i = 0; i < stride; ++i) {
            const int a = i >= (size_t)ch ? cur[i - ch] : 0;
            const int b = prev ? prev[i] : 0;
            const int c = (prev && i >= (size_t)ch) ? prev[i - ch] : 0;
            int v = src[i];
            switch (ft) {
                case 0: break;
                case 1: v += a; break;
                case 2: v += b; break;
                case 3: v += (a + b) >> 1; break;
                case 4: {
                    const int p = a + b - c, pa = std::abs(p - a), pb = std::abs(p - b), pc = std::abs(p - c);
                    v += (pa <= pb && pa <= pc) ? a : (pb <= pc ? b : c);
                    break;
                }
                default: err = "bad PNG filter type"; return false;
            }
            cur[i] = (uint8_t)v;
        }
    }
    png.w = w;
    png.h = h;
    png.ctype = ctype;
    png.ch = ch;
    png.img.swap(img);
    png.plte.swap(plte);
    return true;
}

bool decode_png_gray(const std::vector<uint8_t> &file, Gray8 &out, std::string &err) {
    PngRaw png;
    if (!png_raw(file, png, err)) return false;
    const int w = png.w, h = png.h, ctype = png.ctype, ch = png.ch;
    const std::vector<uint8_t> &img = png.img, &plte = png.plte;
    out.width = w;
    out.height = h;
    out.px.resize((size_t)w * h);
    for (size_t i = 0; i < (size_t)w * h; ++i) {
        const uint8_t *p = &img[i * ch];
        switch (ctype) {
            case 0: case 4: out.px[i] = p[0]; break;
            case 2: case 6: out.px[i] = rgb_to_gray(p[0], p[1], p[2]); break;
            case 3: {
                const size_t k = (size_t)p[0] * 3;
                if (k + 2 >= plte.size()) { err = "PNG palette index out of range"; return false; }
                out.px[i] = rgb_to_gray(plte[k], plte[k + 1], plte[k + 2]);
                break;
            }
        }
    }
    return true;
}

// ----------------------------------------------------------------------------------------------
// PGM / PPM (binary)
// ----------------------------------------------------------------------------------------------
bool decode_pnm_gray(const std::vector<uint8_t> &file, Gray8 &out, std::string &err) {
    if (file.size() < 3 || file[0] != 'P' || (file[1] != '5' && file[1] != '6')) { err = "not a binary PGM/PPM"; return false; }
    const int ch = file[1] == '5' ? 1 : 3;
    size_t pos = 2;
    int vals[3], nv = 0;
    while (nv < 3 && pos < file.size()) {
        while (pos < file.size() && (isspace(file[pos]) || file[pos] == '#')) {
            if (file[pos] == '#') while (pos < file.size() && file[pos] != '\n') ++pos;
            else ++pos;
        }
        int v = 0;
        bool any = false;
        while (pos < file.size() && isdigit(file[pos])) { v = v * 10 + (file[pos++] - '0'); any = true; }
        if (!any) { err = "bad PNM header"; return false; }
        vals[nv++] = v;
    }
    ++pos;  // single whitespace after maxval
    if (nv < 3 || vals[2] != 255) { err = "only 8-bit PNM is supported"; return false; }
    const int w = vals[0], h = vals[1];
    if (pos + (size_t)w * h * ch > file.size()) { err = "truncated PNM"; return false; }
    out.width = w;
    out.height = h;
    out.px.resize((size_t)w * h);
    for (size_t i = 0; i < (size_t)w * h; ++i) {
        const uint8_t *p = &file[pos + i * ch];
        out.px[i] = ch == 1 ? p[0] : rgb_to_gray(p[0], p[1], p[2]);
    }
    return true;
}

// ----------------------------------------------------------------------------------------------
// baseline JPEG, luma only
// ----------------------------------------------------------------------------------------------
namespace {
const int kZigzag[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33, 40, 48,
                         41, 34, 27, 20, 13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23,
                         30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

struct Huff {
    bool present = false;
    // canonical decoding tables (JPEG Annex F.2.2.3)
    int maxcode[18], valptr[17], mincode[17];
    uint8_t vals[256];
};

struct Comp {
    int id, h, v, tq, td = 0, ta = 0, pred = 0;
    int bw, bh;                  // blocks per line / column in the component (padded to MCUs)
    std::vector<int16_t> coef;   // bw*bh*64, natural order (component 0, or all when decoding colour)
};

struct BitReader {
    const uint8_t *d;
    size_t n, pos;
    uint32_t acc = 0;
    int bits = 0;
    bool marker_hit = false;
    int fill_byte() {
        if (marker_hit || pos >= n) return 0;
        uint8_t b = d[pos];
        if (b == 0xFF) {
            const uint8_t nx = pos + 1 < n ? d[pos + 1] : 0;
            if (nx == 0x00) { pos += 2; return 0xFF; }
            marker_hit = true;  // a marker: feed zeros (libjpeg does the same)
            return 0;
        }
        ++pos;
        return b;
    }
    int bit() {
        if (bits == 0) { acc = (uint32_t)fill_byte(); bits = 8; }
        --bits;
        return (acc >> bits) & 1;
    }
    int get(int k) {
        int v = 0;
        for (int i = 0; i < k; ++i) v = (v << 1) | bit();
        return v;
    }
    void reset() { bits = 0; }
};

int huff_decode(BitReader &br, const Huff &h) {
    int code = br.bit();
    int l = 1;
    while (l <= 16 && code > h.maxcode[l]) { code = (code << 1) | br.bit(); ++l; }
    if (l > 16) return -1;
    return h.vals[h.valptr[l] + code - h.mincode[l]];
}
int extend(int v, int s) { return s == 0 ? 0 : (v < (1 << (s - 1)) ? v - (1 << s) + 1 : v); }

// libjpeg jidctint.c (islow) arithmetic, with the post-IDCT range-limit table of jdmaster.c.
void idct_islow(const int16_t *coef, const uint16_t *q, uint8_t *out, int ostride) {
    const int CONST_BITS = 13, PASS1_BITS = 2;
    auto DESCALE = [](int64_t x, int n) { return (int32_t)((x + ((int64_t)1 << (n - 1))) >> n); };
    const int32_t F0_298 = 2446, F0_390 = 3196, F0_541 = 4433, F0_765 = 6270, F0_899 = 7373, F1_175 = 9633,
                  F1_501 = 12299, F1_847 = 15137, F1_961 = 16069, F2_053 = 16819, F2_562 = 20995, F3_072 = 25172;
    int32_t ws[64];
    for (int c = 0; c < 8; ++c) {
        const int16_t *in = coef + c;
        const uint16_t *qt = q + c;
        bool ac_zero = true;
        for (int r = 1; r < 8; ++r) if (in[8 * r] != 0) { ac_zero = false; break; }
        if (ac_zero) {
            const int32_t dc = ((int32_t)in[0] * qt[0]) * (1 << PASS1_BITS);
            for (int r = 0; r < 8; ++r) ws[8 * r + c] = dc;
            continue;
        }
        int64_t z2 = (int32_t)in[16] * qt[16], z3 = (int32_t)in[48] * qt[48];
        int64_t z1 = (z2 + z3) * F0_541;
        int64_t tmp2 = z1 + z3 * (-F1_847);
        int64_t tmp3 = z1 + z2 * F0_765;
        z2 = (int32_t)in[0] * qt[0];
        z3 = (int32_t)in[32] * qt[32];
        int64_t tmp0 = (z2 + z3) * (1 << CONST_BITS);
        int64_t tmp1 = (z2 - z3) * (1 << CONST_BITS);
        const int64_t tmp10 = tmp0 + tmp3, tmp13 = tmp0 - tmp3, tmp11 = tmp1 + tmp2, tmp12 = tmp1 - tmp2;
        tmp0 = (int32_t)in[56] * qt[56];
        tmp1 = (int32_t)in[40] * qt[40];
        tmp2 = (int32_t)in[24] * qt[24];
        tmp3 = (int32_t)in[8] * qt[8];
        z1 = tmp0 + tmp3;
        z2 = tmp1 + tmp2;
        z3 = tmp0 + tmp2;
        int64_t z4 = tmp1 + tmp3;
        const int64_t z5 = (z3 + z4) * F1_175;
        tmp0 *= F0_298; tmp1 *= F2_053; tmp2 *= F3_072; tmp3 *= F1_501;
        z1 *= -F0_899; z2 *= -F2_562; z3 *= -F1_961; z4 *= -F0_390;
        z3 += z5; z4 += z5;
        tmp0 += z1 + z3; tmp1 += z2 + z4; tmp2 += z2 + z3; tmp3 += z1 + z4;
        const int S = CONST_BITS - PASS1_BITS;
        ws[8 * 0 + c] = DESCALE(tmp10 + tmp3, S);
        ws[8 * 7 + c] = DESCALE(tmp10 - tmp3, S);
        ws[8 * 1 + c] = DESCALE(tmp11 + tmp2, S);
        ws[8 * 6 + c] = DESCALE(tmp11 - tmp2, S);
        ws[8 * 2 + c] = DESCALE(tmp12 + tmp1, S);
        ws[8 * 5 + c] = DESCALE(tmp12 - tmp1, S);
        ws[8 * 3 + c] = DESCALE(tmp13 + tmp0, S);
        ws[8 * 4 + c] = DESCALE(tmp13 - tmp0, S);
    }
    // post-IDCT range limit: v = x & 1023 -> x+128 (0..127), 255 (128..511), 0 (512..895), v-896 (896..1023)
    auto limit = [](int32_t x) -> uint8_t {
        const int v = x & 1023;
        if (v < 128) return (uint8_t)(v + 128);
        if (v < 512) return 255;
        if (v < 896) return 0;
        return (uint8_t)(v - 896);
    };
    for (int r = 0; r < 8; ++r) {
        const int32_t *w = ws + 8 * r;
        uint8_t *o = out + (size_t)r * ostride;
        bool ac_zero = true;
        for (int k = 1; k < 8; ++k) if (w[k] != 0) { ac_zero = false; break; }
        const int S = CONST_BITS + PASS1_BITS + 3;
        if (ac_zero) {
            const uint8_t dc = limit(DESCALE(w[0], PASS1_BITS + 3));
            for (int k = 0; k < 8; ++k) o[k] = dc;
            continue;
        }
        int64_t z2 = w[2], z3 = w[6];
        int64_t z1 = (z2 + z3) * F0_541;
        int64_t tmp2 = z1 + z3 * (-F1_847);
        int64_t tmp3 = z1 + z2 * F0_765;
        int64_t tmp0 = ((int64_t)w[0] + w[4]) * (1 << CONST_BITS);
        int64_t tmp1 = ((int64_t)w[0] - w[4]) * (1 << CONST_BITS);
        const int64_t tmp10 = tmp0 + tmp3, tmp13 = tmp0 - tmp3, tmp11 = tmp1 + tmp2, tmp12 = tmp1 - tmp2;
        tmp0 = w[7]; tmp1 = w[5]; tmp2 = w[3]; tmp3 = w[1];
        z1 = tmp0 + tmp3; z2 = tmp1 + tmp2; z3 = tmp0 + tmp2;
        int64_t z4 = tmp1 + tmp3;
        const int64_t z5 = (z3 + z4) * F1_175;
        tmp0 *= F0_298; tmp1 *= F2_053; tmp2 *= F3_072; tmp3 *= F1_501;
        z1 *= -F0_899; z2 *= -F2_562; z3 *= -F1_961; z4 *= -F0_390;
        z3 += z5; z4 += z5;
        tmp0 += z1 + z3; tmp1 += z2 + z4; tmp2 += z2 + z3; tmp3 += z1 + z4;
        o[0] = limit(DESCALE(tmp10 + tmp3, S));
        o[7] = limit(DESCALE(tmp10 - tmp3, S));
        o[1] = limit(DESCALE(tmp11 + tmp2, S));
        o[6] = limit(DESCALE(tmp11 - tmp2, S));
        o[2] = limit(DESCALE(tmp12 + tmp1, S));
        o[5] = limit(DESCALE(tmp12 - tmp1, S));
        o[3] = limit(DESCALE(tmp13 + tmp0, S));
        o[4] = limit(DESCALE(tmp13 - tmp0, S));
    }
}
}  // namespace

// Entropy decode + islow IDCT of every needed component into padded sample planes.
struct JpegPlanes {
    int W = 0, H = 0, hmax = 1, vmax = 1;
    bool jfif = false;
    int adobe_transform = -1;  // APP14 "Adobe" transform flag, -1 if absent
    struct Plane {
        int id, h, v, pw, ph;  // sampling factors, padded plane size (blocks * 8)
        std::vector<uint8_t> px;
    };
    std::vector<Plane> planes;
};

static bool jpeg_decode(const std::vector<uint8_t> &f, bool all_comps, JpegPlanes &res, std::string &err) {
    if (f.size() < 4 || f[0] != 0xFF || f[1] != 0xD8) { err = "not a JPEG file"; return false; }
    uint16_t qt[4][64];
    bool qt_ok[4] = {false, false, false, false};
    Huff hdc[4], hac[4];
    std::vector<Comp> comps;
    int W = 0, H = 0, hmax = 1, vmax = 1, restart = 0, mcux = 0, mcuy = 0;
    bool sof = false, done = false;
    size_t pos = 2;
    while (pos + 4 <= f.size() && !done) {
        if (f[pos] != 0xFF) { ++pos; continue; }
        const uint8_t m = f[pos + 1];
        if (m == 0xFF) { ++pos; continue; }
        pos += 2;
        if (m == 0xD8 || (m >= 0xD0 && m <= 0xD7) || m == 0x01) continue;
        if (m == 0xD9) break;
        const size_t len = (size_t)f[pos] << 8 | f[pos + 1];
        if (len < 2) { err = "bad JPEG segment length"; return false; }
        if (pos + len > f.size()) { err = "truncated JPEG segment"; return false; }
        const uint8_t *d = &f[pos + 2];
        const size_t dl = len - 2;
        if (m == 0xE0 && dl >= 5 && memcmp(d, "JFIF", 5) == 0) {
            res.jfif = true;
        } else if (m == 0xEE && dl >= 12 && memcmp(d, "Adobe", 5) == 0) {
            res.adobe_transform = d[11];
        } else if (m == 0xDB) {  // DQT
            size_t i = 0;
            while (i < dl) {
                const int pq = d[i] >> 4, tq = d[i] & 15;
                ++i;
                if (tq > 3 || i + (pq ? 128 : 64) > dl) { err = "bad DQT"; return false; }
                for (int k = 0; k < 64; ++k) {
                    uint16_t v = pq ? (uint16_t)(d[i] << 8 | d[i + 1]) : d[i];
                    i += pq ? 2 : 1;
                    qt[tq][kZigzag[k]] = v;
                }
                qt_ok[tq] = true;
            }
        } else if (m == 0xC4) {  // DHT
            size_t i = 0;
            while (i < dl) {
                const int tc = d[i] >> 4, th = d[i] & 15;
                ++i;
                if (th > 3 || i + 16 > dl) { err = "bad DHT"; return false; }
                Huff &h = tc ? hac[th] : hdc[th];
                int counts[17] = {0};
                int total = 0;
                for (int l = 1; l <= 16; ++l) { counts[l] = d[i + l - 1]; total += counts[l]; }
                i += 16;
                if (total > 256 || i + (size_t)total > dl) { err = "bad DHT"; return false; }
                memcpy(h.vals, &d[i], total);
                i += total;
                int code = 0, k = 0;
                for (int l = 1; l <= 16; ++l) {
                    h.valptr[l] = k;
                    h.mincode[l] = code;
                    code += counts[l];
                    k += counts[l];
                    h.maxcode[l] = counts[l] ? code - 1 : -1;
                    code <<= 1;
                }
                h.maxcode[17] = 0x7FFFFFFF;
                h.present = true;
            }
        } else if (m == 0xDD) {  // DRI
            if (dl < 2) { err = "bad DRI"; return false; }
            restart = d[0] << 8 | d[1];
        } else if (m == 0xC0 || m == 0xC1) {  // baseline / extended sequential Huffman
            if (dl < 6) { err = "bad SOF"; return false; }
            if (d[0] != 8) { err = "only 8-bit JPEG is supported"; return false; }
            H = d[1] << 8 | d[2];
            W = d[3] << 8 | d[4];
            const int nc = d[5];
            // corrupt headers must not index tables out of range or size huge buffers
            if (nc < 1 || nc > 4 || dl < 6 + 3 * (size_t)nc) { err = "bad SOF"; return false; }
            if (W < 1 || H < 1 || (size_t)W * H > ((size_t)1 << 28)) { err = "unsupported JPEG size"; return false; }
            comps.resize(nc);
            for (int c = 0; c < nc; ++c) {
                comps[c].id = d[6 + 3 * c];
                comps[c].h = d[7 + 3 * c] >> 4;
                comps[c].v = d[7 + 3 * c] & 15;
                comps[c].tq = d[8 + 3 * c];
                if (comps[c].h < 1 || comps[c].h > 4 || comps[c].v < 1 || comps[c].v > 4 || comps[c].tq > 3) {
                    err = "bad SOF component";
                    return false;
                }
                hmax = std::max(hmax, comps[c].h);
                vmax = std::max(vmax, comps[c].v);
            }
            mcux = (W + 8 * hmax - 1) / (8 * hmax);
            mcuy = (H + 8 * vmax - 1) / (8 * vmax);
            for (auto &c : comps) {
                c.bw = mcux * c.h;
                c.bh = mcuy * c.v;
            }
            if (comps[0].h != hmax || comps[0].v != vmax) { err = "subsampled luma is not supported"; return false; }
            for (size_t c = 0; c < comps.size(); ++c)
                if (c == 0 || all_comps) comps[c].coef.assign((size_t)comps[c].bw * comps[c].bh * 64, 0);
            sof = true;
        } else if (m >= 0xC2 && m <= 0xCF && m != 0xC4 && m != 0xC8 && m != 0xCC) {
            err = "progressive / arithmetic / lossless JPEG is not supported";
            return false;
        } else if (m == 0xDA) {  // SOS
            if (!sof) { err = "SOS before SOF"; return false; }
            const int ns = d[0];
            if (ns < 1 || ns > 4 || dl < 1 + 2 * (size_t)ns) { err = "bad SOS"; return false; }
            std::vector<int> sc(ns);
            for (int k = 0; k < ns; ++k) {
                const int cid = d[1 + 2 * k];
                int idx = -1;
                for (size_t c = 0; c < comps.size(); ++c) if (comps[c].id == cid) idx = (int)c;
                if (idx < 0) { err = "SOS references unknown component"; return false; }
                sc[k] = idx;
                comps[idx].td = d[2 + 2 * k] >> 4;
                comps[idx].ta = d[2 + 2 * k] & 15;
                if (comps[idx].td > 3 || comps[idx].ta > 3) { err = "bad SOS table index"; return false; }
                comps[idx].pred = 0;
            }
            pos += len;
            BitReader br{f.data(), f.size(), pos};
            int16_t blk[64];
            auto decode_block = [&](Comp &c, int bx, int by) -> bool {
                memset(blk, 0, sizeof(blk));
                const Huff &dc = hdc[c.td], &ac = hac[c.ta];
                if (!dc.present || !ac.present) return false;
                const int t = huff_decode(br, dc);
                if (t < 0 || t > 15) return false;  // DC categories are <= 11 for 8-bit data
                c.pred = (int)((unsigned)c.pred + (unsigned)extend(br.get(t), t));  // wraps, never UB
                blk[0] = (int16_t)c.pred;
                for (int k = 1; k < 64;) {
                    const int rs = huff_decode(br, ac);
                    if (rs < 0) return false;
                    const int r = rs >> 4, s = rs & 15;
                    if (s == 0) {
                        if (r != 15) break;
                        k += 16;
                        continue;
                    }
                    k += r;
                    if (k > 63) return false;
                    blk[kZigzag[k]] = (int16_t)extend(br.get(s), s);
                    ++k;
                }
                if (!c.coef.empty() && bx < c.bw && by < c.bh)
                    memcpy(&c.coef[((size_t)by * c.bw + bx) * 64], blk, sizeof(blk));
                return true;
            };
            auto handle_restart = [&]() {
                br.reset();
                // skip to and past the RSTn marker
                while (br.pos + 1 < br.n && !(br.d[br.pos] == 0xFF && br.d[br.pos + 1] >= 0xD0 && br.d[br.pos + 1] <= 0xD7)) ++br.pos;
                if (br.pos + 1 < br.n) br.pos += 2;
                br.marker_hit = false;
                for (int k : sc) comps[k].pred = 0;
            };
            int units = 0;
            if (ns == 1) {  // non-interleaved: blocks of the component in raster order
                Comp &c = comps[sc[0]];
                const int cw = (W * c.h + 8 * hmax - 1) / (8 * hmax), ch = (H * c.v + 8 * vmax - 1) / (8 * vmax);
                for (int by = 0; by < ch; ++by)
                    for (int bx = 0; bx < cw; ++bx) {
                        if (restart && units && units % restart == 0) handle_restart();
                        if (!decode_block(c, bx, by)) { err = "corrupt JPEG entropy data"; return false; }
                        ++units;
                    }
            } else {
                for (int my = 0; my < mcuy; ++my)
                    for (int mx = 0; mx < mcux; ++mx) {
                        if (restart && units && units % restart == 0) handle_restart();
                        for (int k : sc) {
                            Comp &c = comps[k];
                            for (int v = 0; v < c.v; ++v)
                                for (int u = 0; u < c.h; ++u)
                                    if (!decode_block(c, mx * c.h + u, my * c.v + v)) {
                                        err = "corrupt JPEG entropy data";
                                        return false;
                                    }
                        }
                        ++units;
                    }
            }
            // continue after the entropy-coded segment
            pos = br.pos;
            continue;
        }
        pos += len;
    }
    if (!sof) { err = "JPEG without SOF"; return false; }
    res.W = W;
    res.H = H;
    res.hmax = hmax;
    res.vmax = vmax;
    for (size_t c = 0; c < comps.size(); ++c) {
        Comp &y = comps[c];
        if (y.coef.empty()) continue;
        if (!qt_ok[y.tq]) { err = "missing quantisation table"; return false; }
        JpegPlanes::Plane pl{y.id, y.h, y.v, y.bw * 8, y.bh * 8, {}};
        pl.px.resize((size_t)pl.pw * pl.ph);
        for (int by = 0; by < y.bh; ++by)
            for (int bx = 0; bx < y.bw; ++bx)
                idct_islow(&y.coef[((size_t)by * y.bw + bx) * 64], qt[y.tq], &pl.px[(size_t)by * 8 * pl.pw + bx * 8],
                           pl.pw);
        res.planes.push_back(std::move(pl));
    }
    return true;
}

bool decode_jpeg_gray(const std::vector<uint8_t> &f, Gray8 &out, std::string &err) {
    JpegPlanes jp;
    if (!jpeg_decode(f, false, jp, err)) return false;
    const JpegPlanes::Plane &y = jp.planes[0];
    out.width = jp.W;
    out.height = jp.H;
    out.px.resize((size_t)jp.W * jp.H);
    for (int r = 0; r < jp.H; ++r) memcpy(&out.px[(size_t)r * jp.W], &y.px[(size_t)r * y.pw], jp.W);
    return true;
}

bool read_gray8(const std::string &path, Gray8 &out, std::string &err) {
    std::vector<uint8_t> data;
    if (!read_file(path, data)) { err = "cannot open " + path; return false; }
    if (data.size() >= 8 && data[0] == 137 && data[1] == 'P') return decode_png_gray(data, out, err);
    if (data.size() >= 2 && data[0] == 0xFF && data[1] == 0xD8) return decode_jpeg_gray(data, out, err);
    if (data.size() >= 2 && data[0] == 'P') return decode_pnm_gray(data, out, err);
    err = "unsupported image format: " + path;
    return false;
}

// ----------------------------------------------------------------------------------------------
// colour: cv::imread(IMREAD_COLOR) for fusion (RunFusion, APD.cpp:1077)
// ----------------------------------------------------------------------------------------------
bool decode_png_bgr(const std::vector<uint8_t> &file, Bgr8 &out, std::string &err) {
    PngRaw png;
    if (!png_raw(file, png, err)) return false;
    out.width = png.w;
    out.height = png.h;
    out.px.resize((size_t)png.w * png.h * 3);
    for (size_t i = 0; i < (size_t)png.w * png.h; ++i) {
        const uint8_t *p = &png.img[i * png.ch];
        uint8_t *o = &out.px[3 * i];
        switch (png.ctype) {
            case 0: case 4: o[0] = o[1] = o[2] = p[0]; break;  // png_set_gray_to_rgb, alpha stripped
            case 2: case 6: o[0] = p[2]; o[1] = p[1]; o[2] = p[0]; break;
            case 3: {
                const size_t k = (size_t)p[0] * 3;
                if (k + 2 >= png.plte.size()) { err = "PNG palette index out of range"; return false; }
                o[0] = png.plte[k + 2]; o[1] = png.plte[k + 1]; o[2] = png.plte[k];
                break;
            }
        }
    }
    return true;
}

bool decode_pnm_bgr(const std::vector<uint8_t> &file, Bgr8 &out, std::string &err) {
    Gray8 g;
    if (file.size() >= 2 && file[1] == '5') {
        if (!decode_pnm_gray(file, g, err)) return false;
        out.width = g.width;
        out.height = g.height;
        out.px.resize(g.px.size() * 3);
        for (size_t i = 0; i < g.px.size(); ++i) out.px[3 * i] = out.px[3 * i + 1] = out.px[3 * i + 2] = g.px[i];
        return true;
    }
    // P6: parse the header with the gray decoder's rules, then copy RGB -> BGR
    if (!decode_pnm_gray(file, g, err)) return false;
    const size_t n = (size_t)g.width * g.height;
    const size_t start = file.size() - n * 3;  // the decoder checked the payload fits; P6 data ends the file
    out.width = g.width;
    out.height = g.height;
    out.px.resize(n * 3);
    for (size_t i = 0; i < n; ++i) {
        const uint8_t *p = &file[start + 3 * i];
        out.px[3 * i] = p[2];
        out.px[3 * i + 1] = p[1];
        out.px[3 * i + 2] = p[0];
    }
    return true;
}

namespace {
// libjpeg-turbo jdsample.c with do_fancy_upsampling (the default): upsample one component plane to
// (hmax/h) x (vmax/v) of its downsampled size (dw x dh real samples; edges replicate, as the
// context rows of jdmainct.c and the first/last-column special cases do).
std::vector<uint8_t> upsample_plane(const JpegPlanes::Plane &pl, int dw, int dh, int fx, int fy, int &ow, int &oh) {
    ow = dw * fx;
    oh = dh * fy;
    std::vector<uint8_t> o((size_t)ow * oh);
    auto at = [&](int r, int c) -> int {
        r = r < 0 ? 0 : (r >= dh ? dh - 1 : r);
        c = c < 0 ? 0 : (c >= dw ? dw - 1 : c);
        return pl.px[(size_t)r * pl.pw + c];
    };
    const bool fancy_h = dw > 2;
    if (fx == 2 && fy == 1) {
        for (int r = 0; r < dh; ++r)
            for (int c = 0; c < dw; ++c) {
                const int v = at(r, c);
                uint8_t *d = &o[(size_t)r * ow + 2 * c];
                if (fancy_h) {  // h2v1_fancy_upsample
                    d[0] = (uint8_t)(c == 0 ? v : (v * 3 + at(r, c - 1) + 1) >> 2);
                    d[1] = (uint8_t)(c == dw - 1 ? v : (v * 3 + at(r, c + 1) + 2) >> 2);
                } else {
                    d[0] = d[1] = (uint8_t)v;
                }
            }
    } else if (fx == 1 && fy == 2) {  // h1v2_fancy_upsample
        for (int r = 0; r < dh; ++r)
            for (int c = 0; c < dw; ++c) {
                const int v3 = at(r, c) * 3;
                o[(size_t)(2 * r) * ow + c] = (uint8_t)((v3 + at(r - 1, c) + 1) >> 2);
                o[(size_t)(2 * r + 1) * ow + c] = (uint8_t)((v3 + at(r + 1, c) + 2) >> 2);
            }
    } else if (fx == 2 && fy == 2 && fancy_h) {  // h2v2_fancy_upsample
        for (int r = 0; r < dh; ++r)
            for (int v = 0; v < 2; ++v) {
                const int rn = v == 0 ? r - 1 : r + 1;
                auto colsum = [&](int c) { return at(r, c) * 3 + at(rn, c); };
                uint8_t *d = &o[(size_t)(2 * r + v) * ow];
                for (int c = 0; c < dw; ++c) {
                    const int t = colsum(c);
                    d[2 * c] = (uint8_t)(c == 0 ? (t * 4 + 8) >> 4 : (t * 3 + colsum(c - 1) + 8) >> 4);
                    d[2 * c + 1] = (uint8_t)(c == dw - 1 ? (t * 4 + 7) >> 4 : (t * 3 + colsum(c + 1) + 7) >> 4);
                }
            }
    } else {  // h2v1/h2v2 with narrow planes and every other integral ratio: replication (int_upsample)
        for (int r = 0; r < oh; ++r)
            for (int c = 0; c < ow; ++c) o[(size_t)r * ow + c] = (uint8_t)at(r / fy, c / fx);
    }
    return o;
}
}  // namespace

bool decode_jpeg_bgr(const std::vector<uint8_t> &f, Bgr8 &out, std::string &err) {
    JpegPlanes jp;
    if (!jpeg_decode(f, true, jp, err)) return false;
    const int W = jp.W, H = jp.H;
    out.width = W;
    out.height = H;
    out.px.resize((size_t)W * H * 3);
    if (jp.planes.size() == 1) {  // gray_rgb_convert
        const JpegPlanes::Plane &y = jp.planes[0];
        for (int r = 0; r < H; ++r)
            for (int c = 0; c < W; ++c) {
                uint8_t *o = &out.px[3 * ((size_t)r * W + c)];
                o[0] = o[1] = o[2] = y.px[(size_t)r * y.pw + c];
            }
        return true;
    }
    if (jp.planes.size() != 3) { err = "only 1- and 3-component JPEG is supported"; return false; }
    std::vector<std::vector<uint8_t>> full(3);
    std::vector<int> fw(3);
    for (int k = 0; k < 3; ++k) {
        const JpegPlanes::Plane &pl = jp.planes[k];
        if (jp.hmax % pl.h || jp.vmax % pl.v) { err = "non-integral JPEG sampling ratio"; return false; }
        const int dw = (W * pl.h + jp.hmax - 1) / jp.hmax, dh = (H * pl.v + jp.vmax - 1) / jp.vmax;  // jdinput.c
        int ow, oh;
        full[k] = upsample_plane(pl, dw, dh, jp.hmax / pl.h, jp.vmax / pl.v, ow, oh);
        fw[k] = ow;
    }
    // jdapimin.c default_decompress_parms: JFIF -> YCbCr; Adobe transform 0 -> RGB; else by ids
    bool rgb = false;
    if (!jp.jfif) {
        if (jp.adobe_transform >= 0) rgb = jp.adobe_transform == 0;
        else rgb = jp.planes[0].id == 82 && jp.planes[1].id == 71 && jp.planes[2].id == 66;
    }
    // jdcolor.c build_ycc_rgb_table / ycc_rgb_convert (SCALEBITS 16)
    static int cr_r[256], cb_b[256], cr_g[256], cb_g[256];
    static bool init = false;
    if (!init) {
        auto FIX = [](double x) { return (int)(x * 65536.0 + 0.5); };
        for (int i = 0; i < 256; ++i) {
            const int x = i - 128;
            cr_r[i] = (FIX(1.40200) * x + (1 << 15)) >> 16;
            cb_b[i] = (FIX(1.77200) * x + (1 << 15)) >> 16;
            cr_g[i] = -FIX(0.71414) * x;
            cb_g[i] = -FIX(0.34414) * x + (1 << 15);
        }
        init = true;
    }
    auto clamp8 = [](int v) { return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v)); };
    for (int r = 0; r < H; ++r)
        for (int c = 0; c < W; ++c) {
            const int y = full[0][(size_t)r * fw[0] + c], cb = full[1][(size_t)r * fw[1] + c],
                      cr = full[2][(size_t)r * fw[2] + c];
            uint8_t *o = &out.px[3 * ((size_t)r * W + c)];
            if (rgb) {
                o[0] = (uint8_t)cr; o[1] = (uint8_t)cb; o[2] = (uint8_t)y;
            } else {
                o[2] = clamp8(y + cr_r[cr]);
                o[1] = clamp8(y + ((cb_g[cb] + cr_g[cr]) >> 16));
                o[0] = clamp8(y + cb_b[cb]);
            }
        }
    return true;
}

bool read_bgr8(const std::string &path, Bgr8 &out, std::string &err) {
    std::vector<uint8_t> data;
    if (!read_file(path, data)) { err = "cannot open " + path; return false; }
    if (data.size() >= 8 && data[0] == 137 && data[1] == 'P') return decode_png_bgr(data, out, err);
    if (data.size() >= 2 && data[0] == 0xFF && data[1] == 0xD8) return decode_jpeg_bgr(data, out, err);
    if (data.size() >= 2 && data[0] == 'P') return decode_pnm_bgr(data, out, err);
    err = "unsupported image format: " + path;
    return false;
}

bool write_png_gray8(const std::string &path, const uint8_t *px, int w, int h) {
    std::vector<uint8_t> raw(((size_t)w + 1) * h);
    for (int r = 0; r < h; ++r) {
        raw[((size_t)w + 1) * r] = 0;  // filter: none
        memcpy(&raw[((size_t)w + 1) * r + 1], px + (size_t)r * w, w);
    }
    uLongf zlen = compressBound((uLong)raw.size());
    std::vector<uint8_t> z(zlen);
    if (compress2(z.data(), &zlen, raw.data(), (uLong)raw.size(), 1) != Z_OK) return false;
    z.resize(zlen);
    std::ofstream o(path, std::ios::binary);
    if (!o) return false;
    auto put32 = [&](std::vector<uint8_t> &v, uint32_t x) {
        v.push_back(x >> 24); v.push_back(x >> 16); v.push_back(x >> 8); v.push_back(x);
    };
    auto chunk = [&](const char *type, const std::vector<uint8_t> &data) {
        std::vector<uint8_t> c;
        put32(c, (uint32_t)data.size());
        c.insert(c.end(), type, type + 4);
        c.insert(c.end(), data.begin(), data.end());
        put32(c, (uint32_t)crc32(0, c.data() + 4, (uInt)(c.size() - 4)));
        o.write(reinterpret_cast<const char *>(c.data()), (std::streamsize)c.size());
    };
    static const uint8_t sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
    o.write(reinterpret_cast<const char *>(sig), 8);
    std::vector<uint8_t> ihdr;
    put32(ihdr, (uint32_t)w);
    put32(ihdr, (uint32_t)h);
    ihdr.insert(ihdr.end(), {8, 0, 0, 0, 0});  // 8-bit gray, deflate, adaptive filter, no interlace
    chunk("IHDR", ihdr);
    chunk("IDAT", z);
    chunk("IEND", {});
    return (bool)o;
}

// ----------------------------------------------------------------------------------------------
// resize
// ----------------------------------------------------------------------------------------------
namespace {
struct LinTab {
    std::vector<int> ofs;
    std::vector<float> a0, a1;
    int lim = 0;  // first index that has only one tap (right border)
};
// OpenCV resize() coefficient loop for INTER_LINEAR (ksize 2), per axis. Along x the tap and its
// weight are clamped at the borders; along y (clamp = false) only the ROWS are clamped later
// (resizeGeneric_Invoker clips sy to [0, H-1]) and the weights keep fy.
LinTab linear_table(int ssz, int dsz, bool clamp = true) {
    LinTab t;
    const double scale = 1.0 / ((double)dsz / ssz);  // hal::resize: scale_x = 1./inv_scale_x
    t.ofs.resize(dsz);
    t.a0.resize(dsz);
    t.a1.resize(dsz);
    t.lim = dsz;
    for (int d = 0; d < dsz; ++d) {
        float fx = (float)((d + 0.5) * scale - 0.5);
        int sx = (int)std::floor(fx);
        fx -= (float)sx;
        if (clamp) {
            if (sx < 0) { fx = 0.0f; sx = 0; }
            if (sx + 1 >= ssz) {
                t.lim = std::min(t.lim, d);
                if (sx >= ssz - 1) { fx = 0.0f; sx = ssz - 1; }
            }
        }
        t.ofs[d] = sx;
        t.a0[d] = 1.0f - fx;
        t.a1[d] = fx;
    }
    return t;
}
inline int clip_row(int y, int h) { return y < 0 ? 0 : (y >= h ? h - 1 : y); }
}  // namespace

void resize_linear_f32(const float *src, int sw, int sh, float *dst, int dw, int dh) {
    if (sw == dw && sh == dh) {
        memcpy(dst, src, sizeof(float) * sw * sh);
        return;
    }
    const double sx = 1.0 / ((double)dw / sw), sy = 1.0 / ((double)dh / sh);
    const int isx = (int)std::lround(sx), isy = (int)std::lround(sy);
    if (std::fabs(sx - isx) < 2.220446049250313e-16 && std::fabs(sy - isy) < 2.220446049250313e-16 && isx == 2 &&
        isy == 2) {
        // INTER_LINEAR with an exact 2x downscale is INTER_AREA (resizeAreaFast): mean of the 2x2 block
        for (int y = 0; y < dh; ++y)
            for (int x = 0; x < dw; ++x) {
                const float *s0 = src + (size_t)(2 * y) * sw + 2 * x, *s1 = s0 + sw;
                const float sum = ((s0[0] + s0[1]) + (s1[0] + s1[1]));
                dst[(size_t)y * dw + x] = sum * 0.25f;
            }
        return;
    }
    const LinTab tx = linear_table(sw, dw), ty = linear_table(sh, dh, false);
    std::vector<float> r0(dw), r1(dw);
    auto hpass = [&](int row, std::vector<float> &o) {
        const float *s = src + (size_t)row * sw;
        for (int x = 0; x < dw; ++x) {
            const int k = tx.ofs[x];
            if (x < tx.lim) {
                const float p = s[k] * tx.a0[x];
                const float q = s[k + 1] * tx.a1[x];
                o[x] = p + q;
            } else {
                o[x] = s[k] * tx.a0[x];
            }
        }
    };
    for (int y = 0; y < dh; ++y) {
        const int k = ty.ofs[y];
        hpass(clip_row(k, sh), r0);
        hpass(clip_row(k + 1, sh), r1);
        const float b0 = ty.a0[y], b1 = ty.a1[y];
        for (int x = 0; x < dw; ++x) {
            const float p = r0[x] * b0;
            const float q = r1[x] * b1;
            dst[(size_t)y * dw + x] = p + q;
        }
    }
}

// cv::resize INTER_LINEAR on CV_8UC3, OpenCV 4.x fixed-point path (INTER_RESIZE_COEF_BITS 11):
// HResizeLinear<uchar,int,short> is exact integer arithmetic; VResizeLinear is taken as the x86
// SIMD kernel (VResizeLinearVec_32s8u: ((S0>>4)*b0 >> 16) + ((S1>>4)*b1 >> 16), then (+2) >> 2,
// 16- then 8-byte blocks at 128-bit width) with the scalar FixedPtCast tail ((S0*b0 + S1*b1 + 2^21) >> 22). Exact 2x
// downscales take INTER_AREA's resizeAreaFast ((a+b+c+d+2) >> 2).
void resize_linear_u8c3(const uint8_t *src, int sw, int sh, uint8_t *dst, int dw, int dh) {
    const int cn = 3;
    if (sw == dw && sh == dh) {
        memcpy(dst, src, (size_t)sw * sh * cn);
        return;
    }
    const double sx = 1.0 / ((double)dw / sw), sy = 1.0 / ((double)dh / sh);
    const int isx = (int)std::lround(sx), isy = (int)std::lround(sy);
    if (std::fabs(sx - isx) < 2.220446049250313e-16 && std::fabs(sy - isy) < 2.220446049250313e-16 && isx == 2 &&
        isy == 2) {
        for (int y = 0; y < dh; ++y)
            for (int x = 0; x < dw; ++x)
                for (int k = 0; k < cn; ++k) {
                    const uint8_t *s0 = src + ((size_t)(2 * y) * sw + 2 * x) * cn + k, *s1 = s0 + (size_t)sw * cn;
                    dst[((size_t)y * dw + x) * cn + k] = (uint8_t)((s0[0] + s0[cn] + s1[0] + s1[cn] + 2) >> 2);
                }
        return;
    }
    auto to_short = [](float v) { return (int)std::nearbyint(v); };  // saturate_cast<short>(float)
    const LinTab tx = linear_table(sw, dw), ty = linear_table(sh, dh, false);
    std::vector<int> ax0(dw), ax1(dw);
    for (int x = 0; x < dw; ++x) {
        ax0[x] = to_short(tx.a0[x] * 2048.0f);
        ax1[x] = to_short(tx.a1[x] * 2048.0f);
    }
    const int width = dw * cn;
    std::vector<int> r0(width), r1(width);
    auto hpass = [&](int row, std::vector<int> &o) {
        const uint8_t *s = src + (size_t)row * sw * cn;
        for (int x = 0; x < dw; ++x)
            for (int k = 0; k < cn; ++k) {
                const int j = tx.ofs[x] * cn + k;
                o[x * cn + k] = x < tx.lim ? s[j] * ax0[x] + s[j + cn] * ax1[x] : s[j] * 2048;
            }
    };
    for (int y = 0; y < dh; ++y) {
        hpass(clip_row(ty.ofs[y], sh), r0);
        hpass(clip_row(ty.ofs[y] + 1, sh), r1);
        const int b0 = to_short(ty.a0[y] * 2048.0f), b1 = to_short(ty.a1[y] * 2048.0f);
        uint8_t *d = dst + (size_t)y * width;
        auto simd = [&](int x) {
            const int v = (((r0[x] >> 4) * b0) >> 16) + (((r1[x] >> 4) * b1) >> 16);
            const int o = (v + 2) >> 2;
            d[x] = (uint8_t)(o < 0 ? 0 : (o > 255 ? 255 : o));
        };
        int x = 0;
        for (; x <= width - 16; x += 16)  // v_uint8 blocks
            for (int k = 0; k < 16; ++k) simd(x + k);
        for (; x < width - 8; x += 8)  // v_int16 blocks (strict <, as in the source)
            for (int k = 0; k < 8; ++k) simd(x + k);
        for (; x < width; ++x) {
            const int o = (r0[x] * b0 + r1[x] * b1 + (1 << 21)) >> 22;
            d[x] = (uint8_t)(o < 0 ? 0 : (o > 255 ? 255 : o));
        }
    }
}

void resize_nearest(const void *src, int sw, int sh, void *dst, int dw, int dh, int elem) {
    const double ifx = 1.0 / ((double)dw / sw), ify = 1.0 / ((double)dh / sh);
    const uint8_t *s = static_cast<const uint8_t *>(src);
    uint8_t *d = static_cast<uint8_t *>(dst);
    std::vector<int> xo(dw);
    for (int x = 0; x < dw; ++x) xo[x] = std::min((int)std::floor(x * ifx), sw - 1);
    for (int y = 0; y < dh; ++y) {
        const int sy = std::min((int)std::floor(y * ify), sh - 1);
        for (int x = 0; x < dw; ++x)
            memcpy(d + ((size_t)y * dw + x) * elem, s + ((size_t)sy * sw + xo[x]) * elem, elem);
    }
}

}  // namespace apdhost
