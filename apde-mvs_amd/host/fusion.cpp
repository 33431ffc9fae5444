// fusion.cpp — see fusion.h. Reference: APD.cpp:316-356 (ExportPointCloud), 844-864
// (RescaleImageAndCamera), 866-910 (geometry helpers), 962-1049 (WeakVisFilter), 1051-1608
// (RunFusion, RunFusion_TAT_I, RunFusion_TAT_A).
#include "fusion.h"

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <atomic>
#include <future>
#include <iomanip>
#include <iostream>
#include <stdexcept>
#include <thread>

#include "../../include/apd_fusion.h"
#include "image.h"

namespace apdhost {

namespace {

using Clock = std::chrono::steady_clock;
double ms_since(Clock::time_point t) { return std::chrono::duration<double, std::milli>(Clock::now() - t).count(); }

struct F3 {
    float x, y, z;
};

// Get3DPointonWorld (APD.cpp:866-889) — the same float sequence as the kernels and the oracle.
F3 point_on_world(int x, int y, float depth, const apd_camera &cam) {
    float px = depth * ((float)x - cam.K[2]) / cam.K[0];
    float py = depth * ((float)y - cam.K[5]) / cam.K[4];
    float pz = depth;
    float tx = cam.R[0] * px + cam.R[3] * py + cam.R[6] * pz;
    float ty = cam.R[1] * px + cam.R[4] * py + cam.R[7] * pz;
    float tz = cam.R[2] * px + cam.R[5] * py + cam.R[8] * pz;
    float cx = -(cam.R[0] * cam.t[0] + cam.R[3] * cam.t[1] + cam.R[6] * cam.t[2]);
    float cy = -(cam.R[1] * cam.t[0] + cam.R[4] * cam.t[1] + cam.R[7] * cam.t[2]);
    float cz = -(cam.R[2] * cam.t[0] + cam.R[5] * cam.t[1] + cam.R[8] * cam.t[2]);
    return F3{tx + cx, ty + cy, tz + cz};
}

// GetAngle from its q (APD.cpp:904-909): NaN (q outside [-1,1] or NaN) -> 0.
inline float angle_of_q(float q) {
    const float a = acosf(q);
    return a != a ? 0.0f : a;
}

// Ordered float keys for bisection over the floats of [-1, 1].
int64_t fkey(float f) {
    uint32_t u;
    memcpy(&u, &f, 4);
    return (u >> 31) ? -(int64_t)(u & 0x7fffffffu) : (int64_t)u;
}
float from_key(int64_t k) {
    const uint32_t u = k < 0 ? (uint32_t)(-k) | 0x80000000u : (uint32_t)k;
    float f;
    memcpy(&f, &u, 4);
    return f;
}

// Largest q in [-1,1] with pred(q) true, for pred true on a prefix; verified on a window.
template <class P> float last_true(P pred, const char *what) {
    int64_t lo = fkey(-1.0f), hi = fkey(1.0f);
    if (!pred(from_key(lo))) return std::nextafter(-1.0f, -2.0f);  // pred false everywhere
    if (pred(from_key(hi))) return 1.0f;
    while (hi - lo > 1) {  // invariant: pred(lo) && !pred(hi)
        const int64_t mid = lo + (hi - lo) / 2;
        (pred(from_key(mid)) ? lo : hi) = mid;
    }
    for (int64_t k = std::max(fkey(-1.0f), lo - 65536); k <= std::min(fkey(1.0f), lo + 65536); ++k)
        if (pred(from_key(k)) != (k <= lo))
            throw std::runtime_error(std::string("fusion: acosf is not monotone around the ") + what + " cut");
    return from_key(lo);
}

}  // namespace

float angle_cut_lt(float T) {
    return last_true([T](float q) { return acosf(q) >= T; }, "angle");
}

float view_cut_deg(float D) {
    // deg(q) > D on a prefix of [-1,1]; the cut is the first q with deg(q) <= D
    const float last = last_true([D](float q) { return (float)(acosf(q) * 180.0f / M_PI) > D; }, "view-angle");
    return std::nextafter(last, 2.0f);
}

void write_ply(const std::string &path, const std::vector<float> &xyz, const std::vector<float> &bgr,
               bool export_color) {
    std::ofstream out(path, std::ios::binary);
    const size_t n = xyz.size() / 3;
    out << "ply\n";
    out << "format binary_little_endian 1.0\n";
    out << "element vertex " << int(n) << "\n";
    out << "property float x\n";
    out << "property float y\n";
    out << "property float z\n";
    if (export_color) {
        out << "property uchar blue\n";
        out << "property uchar green\n";
        out << "property uchar red\n";
    }
    out << "end_header\n";
    const size_t rec = export_color ? 15 : 12;
    std::vector<char> buf(rec * n);
    for (size_t i = 0; i < n; ++i) {
        char *b = &buf[rec * i];
        memcpy(b, &xyz[3 * i], 12);
        if (export_color)
            for (int k = 0; k < 3; ++k) b[12 + k] = (char)static_cast<uint8_t>(bgr[3 * i + k]);
    }
    out.write(buf.data(), (std::streamsize)buf.size());
}

namespace {

struct View {
    int id = 0;
    apd_camera cam{};
    Mat depth, normal, weak, conf;
    Bgr8 color;  // at depth-map size
    uint8_t *mask = nullptr;  // into the global mask array (all views, concatenated)
    size_t off = 0;           // this view's first pixel in the global arrays
    std::vector<uint8_t> skip;
};

// One view as RunFusion loads it (APD.cpp:1071-1133).
bool load_view(const std::string &dense, const Problem &pb, MatStore &store, View &v, std::string &err) {
    v.id = pb.ref_image_id;
    const std::string img = dense + "/images/" + format_index(pb.ref_image_id) + pb.img_ext;
    const std::string cam = dense + "/cams/" + format_index(pb.ref_image_id) + "_cam.txt";
    const std::string res = dense + "/APD/" + format_index(pb.ref_image_id);
    Bgr8 src;
    if (!read_bgr8(img, src, err)) return false;
    if (!read_camera(cam, v.cam)) { err = "cannot read " + cam; return false; }
    if (!store.read(res + "/depths.bin", v.depth) || !store.read(res + "/normals.bin", v.normal) ||
        !store.read(res + "/weak.bin", v.weak) || !store.read(res + "/confidence.bin", v.conf)) {
        err = "missing depth-stage outputs under " + res;
        return false;
    }
    const int W = v.depth.cols, H = v.depth.rows;
    if (v.depth.type != CV_32FC1 || v.normal.type != CV_32FC3 || v.weak.type != CV_8UC1 || v.conf.type != CV_8UC1) {
        err = "unexpected bin-mat types under " + res;
        return false;
    }
    // APD.cpp:1105-1116 prints and `continue`s here, which leaves imageIdToindexMap pointing past
    // the loaded vectors (undefined); refuse instead.
    if (v.normal.cols != W || v.normal.rows != H) { err = "Error: normal size is not equal to depth size"; return false; }
    if (v.weak.cols != W || v.weak.rows != H) { err = "Error: weak size is not equal to depth size"; return false; }
    if (v.conf.cols != W || v.conf.rows != H) { err = "Error: confidence size is not equal to depth size"; return false; }
    // RescaleImageAndCamera (APD.cpp:844-864)
    if (src.width == W && src.height == H) {
        v.color = std::move(src);
    } else {
        const float scale_x = W / static_cast<float>(src.width);
        const float scale_y = H / static_cast<float>(src.height);
        v.color.width = W;
        v.color.height = H;
        v.color.px.resize((size_t)W * H * 3);
        resize_linear_u8c3(src.px.data(), src.width, src.height, v.color.px.data(), W, H);
        v.cam.K[0] *= scale_x;
        v.cam.K[2] *= scale_x;
        v.cam.K[4] *= scale_y;
        v.cam.K[5] *= scale_y;
        v.cam.width = W;
        v.cam.height = H;
    }
    v.skip.assign((size_t)W * H, 0);
    return true;
}

struct Fuser {
    apd_fusion_ctx *ctx = nullptr;
    std::vector<View> &views;
    const std::vector<Problem> &problems;
    std::vector<float> xyz, bgr;
    double gpu_ms = 0;
    std::string err;

    Fuser(std::vector<View> &v, const std::vector<Problem> &p) : views(v), problems(p) {}

    // imageIdToindexMap (APD.cpp:1072): first index of an id; a missing id reads as 0 (operator[]).
    int index_of(int id) const {
        for (size_t i = 0; i < views.size(); ++i)
            if (views[i].id == id) return (int)i;
        return 0;
    }
    std::vector<int32_t> src_list(int i) const {
        std::vector<int32_t> s;
        for (int id : problems[i].src_image_ids) s.push_back(index_of(id));
        return s;
    }
    bool dev(int32_t st, const char *what) {
        if (st == APD_OK) return true;
        err = std::string(what) + ": " + apd_fusion_last_error(ctx);
        return false;
    }
    void emit(const F3 &p, const float col[3]) {
        xyz.push_back(p.x);
        xyz.push_back(p.y);
        xyz.push_back(p.z);
        bgr.push_back(col[0]);
        bgr.push_back(col[1]);
        bgr.push_back(col[2]);
    }
    const uint8_t *color_at(int v, int pix) const { return &views[v].color.px[3 * (size_t)pix]; }

    // Device half of one image of RunFusion: mask-independent candidate records.
    struct Cands {
        // device records, compacted per pixel by consistency(): slot m < cnt[p] of pixel p holds the
        // m-th consistent source (in j order): global target index tgt (view offset + source pixel),
        // its exp term, and j
        std::vector<int32_t> tgt;
        std::vector<float> er, term;
        std::vector<uint8_t> cnt, jj;
    };
    double term_ms = 0, commit_ms = 0;
    int threads = 1;
    bool consistency(int i, float q_angle, Cands &c) {
        const int ref = index_of(problems[i].ref_image_id);
        const std::vector<int32_t> src = src_list(i);
        const size_t npx = (size_t)views[ref].depth.rows * views[ref].depth.cols, N = src.size(), n = npx * N;
        c.tgt.resize(n);
        c.er.resize(n);
        c.term.resize(n);
        c.jj.resize(n);
        c.cnt.resize(npx);
        auto t0 = Clock::now();
        const bool ok = dev(apd_fusion_consistency(ctx, ref, (int32_t)N, src.data(), q_angle, c.tgt.data(),
                                                   c.er.data(), c.term.data()),
                            "apd_fusion_consistency");
        gpu_ms += ms_since(t0);
        if (!ok) return false;
        // Mask-independent work in parallel: the exp(-tmp_index) term of every consistent candidate
        // (APD.cpp:1192-1193, glibc acosf/expf like the reference) and the per-pixel compaction;
        // skipped pixels (WeakVisFilter) get no candidates.
        t0 = Clock::now();
        const View &rv = views[ref];
        std::vector<size_t> soff(N);
        for (size_t j = 0; j < N; ++j) soff[j] = views[src[j]].off;
        std::vector<std::thread> th;
        const size_t chunk = (npx + threads - 1) / threads;
        for (int t = 0; t < threads; ++t)
            th.emplace_back([&, t]() {
                const size_t e = std::min(npx, (t + 1) * chunk);
                for (size_t p = t * chunk; p < e; ++p) {
                    const size_t o = p * N;
                    int m = 0;
                    if (rv.skip[p] != 1)
                        for (size_t j = 0; j < N; ++j) {
                            const int32_t sp = c.tgt[o + j];
                            if (sp < 0) continue;
                            const float tmp_index = c.er[o + j] + angle_of_q(c.term[o + j]) * 10;
                            c.tgt[o + m] = (int32_t)(soff[j] + (size_t)sp);
                            c.term[o + m] = expf(-tmp_index);
                            c.jj[o + m] = (uint8_t)j;
                            ++m;
                        }
                    c.cnt[p] = (uint8_t)m;
                }
            });
        for (auto &t : th) t.join();
        term_ms += ms_since(t0);
        return true;
    }

    // RunFusion ordered commit (APD.cpp:1147-1219) over the compacted candidates. A pixel without
    // consistent candidates can never be accepted and has no side effect, so it is passed over.
    void commit_default(int i, const Cands &cd, uint8_t *gmask) {
        const int ref = index_of(problems[i].ref_image_id);
        View &rv = views[ref];
        const std::vector<int32_t> src = src_list(i);
        const int N = (int)src.size(), W = rv.depth.cols, H = rv.depth.rows;
        const float *depth = rv.depth.ptr<float>();
        const uint8_t *weak = rv.weak.ptr<uint8_t>();
        int32_t used[APD_MAX_IMAGES];
        for (int r = 0; r < H; ++r)
            for (int c = 0; c < W; ++c) {
                const size_t p = (size_t)r * W + c;
                const int m = cd.cnt[p];
                if (m == 0 || rv.mask[p] == 1) continue;
                const size_t o = p * N;
                int num_consistent = 0;
                float dynamic_consistency = 0.0f;
                for (int k = 0; k < m; ++k) {
                    const int32_t t = cd.tgt[o + k];
                    used[k] = -1;
                    if (gmask[t] == 1) continue;
                    used[k] = t;
                    dynamic_consistency += cd.term[o + k];
                    num_consistent++;
                }
                const float factor = (weak[p] == APD_WEAK ? 0.45f : 0.3f);
                if (num_consistent >= 1 && (dynamic_consistency > factor * num_consistent)) {
                    const uint8_t *rc = color_at(ref, (int)p);
                    float col[3] = {(float)rc[0], (float)rc[1], (float)rc[2]};
                    for (int k = 0; k < m; ++k) {
                        if (used[k] == -1) continue;
                        gmask[used[k]] = 1;
                        const int sv = src[cd.jj[o + k]];
                        const uint8_t *sc = color_at(sv, (int)(used[k] - (int64_t)views[sv].off));
                        col[0] += sc[0];
                        col[1] += sc[1];
                        col[2] += sc[2];
                    }
                    col[0] /= (num_consistent + 1);
                    col[1] /= (num_consistent + 1);
                    col[2] /= (num_consistent + 1);
                    emit(point_on_world(c, r, depth[p], rv.cam), col);
                }
            }
    }

    struct Levels {
        std::vector<int32_t> pix;
        std::vector<uint8_t> lv;
    };
    bool levels(int i, bool tat_i, const std::vector<float> &qk, Levels &l) {
        const int ref = index_of(problems[i].ref_image_id);
        const std::vector<int32_t> src = src_list(i);
        const size_t n = (size_t)views[ref].depth.rows * views[ref].depth.cols * src.size();
        l.pix.resize(n);
        l.lv.resize(n);
        const float dist_base = 0.25f;
        const float depth_base = tat_i ? 1.0f / 3500.0f : 1.0f / 3000.0f;
        const auto t0 = Clock::now();
        const bool ok = dev(apd_fusion_tat_levels(ctx, ref, (int32_t)src.size(), src.data(), dist_base, depth_base,
                                                  tat_i ? qk.data() : nullptr, l.pix.data(), l.lv.data()),
                            "apd_fusion_tat_levels");
        gpu_ms += ms_since(t0);
        return ok;
    }

    // RunFusion_TAT_I / _A ordered commit (APD.cpp:1347-1427, 1541-1603). The per-image cost cache
    // `diff` becomes (level, source pixel) per source, refreshed only by usable candidates; a pixel's
    // outcome depends on the cache state and masks[src], and writes only masks[ref] at itself. So when
    // no source is the reference view itself (masks[src] are then fixed during this image), the scan
    // splits exactly into row chunks: (1) each chunk's last cache update per source, in parallel,
    // (2) the incoming cache of every chunk by a prefix fold, (3) each chunk replayed in parallel.
    struct TatChunk {
        std::vector<uint8_t> last_lv;
        std::vector<int32_t> last_pix;
        std::vector<float> xyz, bgr;
        int64_t skip_weak = 0;
    };
    int64_t commit_tat(int i, bool tat_i, const Levels &l) {
        const int ref = index_of(problems[i].ref_image_id);
        View &rv = views[ref];
        const std::vector<int32_t> src = src_list(i);
        const int N = (int)src.size(), W = rv.depth.cols, H = rv.depth.rows;
        const float *depth = rv.depth.ptr<float>();
        bool self_src = false;
        for (int s : src) self_src |= s == ref;
        const int nch = self_src ? 1 : std::max(1, std::min(threads * 4, H));
        std::vector<TatChunk> ch(nch);
        auto rows_of = [&](int k, int &r0, int &r1) {
            r0 = (int)((int64_t)H * k / nch);
            r1 = (int)((int64_t)H * (k + 1) / nch);
        };
        auto usable = [&](size_t p) { return rv.skip[p] != 1 && !(depth[p] <= 0.0f); };  // NaN depths are processed
        auto par = [&](auto fn) {
            if (nch == 1) { fn(0); return; }
            std::vector<std::thread> th;
            std::atomic<int> next{0};
            for (int t = 0; t < std::min(threads, nch); ++t)
                th.emplace_back([&]() {
                    for (int k; (k = next++) < nch;) fn(k);
                });
            for (auto &t : th) t.join();
        };
        // (1) last usable update per source in each chunk (255 = none in this chunk)
        par([&](int k) {
            TatChunk &C = ch[k];
            C.last_lv.assign(N, 255);
            C.last_pix.assign(N, -1);
            int r0, r1;
            rows_of(k, r0, r1);
            for (size_t p = (size_t)r0 * W; p < (size_t)r1 * W; ++p) {
                if (!usable(p)) continue;
                const size_t o = p * N;
                for (int j = 0; j < N; ++j) {
                    const int32_t sp = l.pix[o + j];
                    if (sp < 0 || views[src[j]].mask[sp] == 1) continue;
                    C.last_lv[j] = l.lv[o + j];
                    C.last_pix[j] = sp;
                }
            }
        });
        // (2) incoming cache per chunk: the image starts with FLT_MAX costs (level 255)
        std::vector<std::vector<uint8_t>> in_lv(nch, std::vector<uint8_t>(N, 255));
        std::vector<std::vector<int32_t>> in_pix(nch, std::vector<int32_t>(N, 0));
        for (int k = 1; k < nch; ++k)
            for (int j = 0; j < N; ++j) {
                const bool upd = ch[k - 1].last_pix[j] >= 0;
                in_lv[k][j] = upd ? ch[k - 1].last_lv[j] : in_lv[k - 1][j];
                in_pix[k][j] = upd ? ch[k - 1].last_pix[j] : in_pix[k - 1][j];
            }
        // (3) replay every chunk from its incoming cache
        par([&](int k) {
            TatChunk &C = ch[k];
            std::vector<uint8_t> cur_lv = in_lv[k];
            std::vector<int32_t> cur_pix = in_pix[k];
            int r0, r1;
            rows_of(k, r0, r1);
            for (int r = r0; r < r1; ++r)
                for (int c = 0; c < W; ++c) {
                    const size_t p = (size_t)r * W + c;
                    if (rv.skip[p] == 1) {
                        C.skip_weak++;
                        continue;
                    }
                    const float ref_depth = depth[p];
                    if (ref_depth <= 0.0) continue;
                    const size_t o = p * N;
                    for (int j = 0; j < N; ++j) {
                        const int32_t sp = l.pix[o + j];
                        if (sp < 0 || views[src[j]].mask[sp] == 1) continue;
                        cur_lv[j] = l.lv[o + j];
                        cur_pix[j] = sp;
                    }
                    // count(k) = #{j : level_j <= k}: levels are monotone in k (thresholds grow with k)
                    int hist[APD_MAX_IMAGES + 2] = {0};
                    for (int j = 0; j < N; ++j) hist[cur_lv[j] <= N ? cur_lv[j] : N + 1]++;
                    int count = 0;
                    for (int kk = 2; kk <= N; ++kk) {
                        count += hist[kk];
                        if (count >= kk) {
                            const uint8_t *rc = color_at(ref, (int)p);
                            float col[3] = {(float)rc[0], (float)rc[1], (float)rc[2]};
                            if (tat_i) {
                                for (int j = 0; j < N; ++j) {
                                    if (cur_lv[j] > kk) continue;
                                    const uint8_t *sc = color_at(src[j], cur_pix[j]);
                                    col[0] += (float)sc[0];
                                    col[1] += (float)sc[1];
                                    col[2] += (float)sc[2];
                                }
                                col[0] /= (count + 1.0f);
                                col[1] /= (count + 1.0f);
                                col[2] /= (count + 1.0f);
                            }
                            const F3 pt = point_on_world(c, r, ref_depth, rv.cam);
                            C.xyz.insert(C.xyz.end(), {pt.x, pt.y, pt.z});
                            C.bgr.insert(C.bgr.end(), {col[0], col[1], col[2]});
                            rv.mask[p] = 1;
                            break;
                        }
                    }
                }
        });
        // points in the reference's order: chunk by chunk
        int64_t skip_weak = 0;
        std::vector<size_t> at(nch + 1, xyz.size());
        for (int k = 0; k < nch; ++k) {
            at[k + 1] = at[k] + ch[k].xyz.size();
            skip_weak += ch[k].skip_weak;
        }
        xyz.resize(at[nch]);
        bgr.resize(at[nch]);
        par([&](int k) {
            std::copy(ch[k].xyz.begin(), ch[k].xyz.end(), xyz.begin() + at[k]);
            std::copy(ch[k].bgr.begin(), ch[k].bgr.end(), bgr.begin() + at[k]);
        });
        return skip_weak;
    }
};

}  // namespace

bool run_fusion(const std::vector<Problem> &problems, const FusionOptions &opt, MatStore &store, FusionReport &rep,
                std::string &err) {
    const int n = (int)problems.size();
    if (n == 0) { err = "fusion: no problems"; return false; }
    for (const Problem &pb : problems)
        if ((int)pb.src_image_ids.size() > APD_MAX_IMAGES) { err = "fusion: too many source views"; return false; }
    auto t0 = Clock::now();
    std::vector<View> views(n);
    {
        // decode/read views in parallel (the reference reads them one by one, APD.cpp:1073-1133)
        std::vector<std::string> errs(n);
        std::vector<char> ok(n, 0);
        const int nt = std::max(1, std::min(n, (int)std::min(16u, std::max(1u, std::thread::hardware_concurrency()))));
        std::vector<std::thread> th;
        std::atomic<int> next{0};
        for (int t = 0; t < nt; ++t)
            th.emplace_back([&]() {
                for (int i; (i = next++) < n;) ok[i] = load_view(opt.dense_folder, problems[i], store, views[i], errs[i]);
            });
        for (auto &t : th) t.join();
        for (int i = 0; i < n; ++i) {
            std::cout << "Reading image " << std::setw(8) << std::setfill('0') << i << "..." << std::endl;
            if (!ok[i]) { err = errs[i]; return false; }
        }
    }
    rep.load_ms = ms_since(t0);

    size_t total_px = 0;
    for (View &v : views) {
        v.off = total_px;
        total_px += (size_t)v.depth.cols * v.depth.rows;
    }
    if (total_px >= ((size_t)1 << 31)) { err = "fusion: more than 2^31 pixels in the scan"; return false; }
    std::vector<uint8_t> gmask(total_px, 0);
    for (View &v : views) v.mask = gmask.data() + v.off;
    Fuser fu(views, problems);
    fu.xyz.reserve(3 * total_px);  // at most one point per pixel; untouched pages cost nothing
    fu.bgr.reserve(3 * total_px);
    fu.threads = (int)std::min(16u, std::max(1u, std::thread::hardware_concurrency()));
    fu.ctx = apd_fusion_create(opt.device);
    if (!fu.ctx) { err = std::string("fusion: ") + apd_fusion_last_error(nullptr); return false; }
    struct CtxGuard {
        apd_fusion_ctx *c;
        ~CtxGuard() { apd_fusion_destroy(c); }
    } guard{fu.ctx};
    t0 = Clock::now();
    {
        std::vector<apd_fusion_view> fv(n);
        for (int i = 0; i < n; ++i) {
            View &v = views[i];
            fv[i] = apd_fusion_view{v.depth.cols, v.depth.rows, v.cam, v.depth.ptr<float>(), v.normal.ptr<float>(),
                                    v.weak.ptr<uint8_t>(), v.conf.ptr<uint8_t>()};
        }
        if (!fu.dev(apd_fusion_set_views(fu.ctx, n, fv.data()), "apd_fusion_set_views")) { err = fu.err; return false; }
    }
    rep.upload_ms = ms_since(t0);

    t0 = Clock::now();
    if (opt.weak_filter) {
        const float q_view = view_cut_deg(80.0f);
        for (int i = 0; i < n; ++i) {
            const auto tg = Clock::now();
            if (!fu.dev(apd_fusion_weak_filter(fu.ctx, i, q_view, views[i].skip.data()), "apd_fusion_weak_filter")) {
                err = fu.err;
                return false;
            }
            fu.gpu_ms += ms_since(tg);
            std::vector<uint8_t> img(views[i].skip.size());
            for (size_t p = 0; p < img.size(); ++p) img[p] = views[i].skip[p] == 1 ? 255 : 0;
            const std::string path = opt.dense_folder + "/APD/" + format_index(problems[i].ref_image_id) + "/skip.png";
            write_png_gray8(path, img.data(), views[i].depth.cols, views[i].depth.rows);
            printf("filter for image %d done\n", problems[i].ref_image_id);
        }
    }
    rep.filter_ms = ms_since(t0);

    t0 = Clock::now();
    if (opt.dataset == "TaT_a" || opt.dataset == "TaT_i") {
        const bool tat_i = opt.dataset == "TaT_i";
        const float angle_base = 0.06981317007977318f, angle_grad = 0.05235987755982988f;
        std::vector<float> qk(APD_MAX_IMAGES + 1, 1.0f);
        if (tat_i)
            for (int k = 2; k <= APD_MAX_IMAGES; ++k) qk[k] = angle_cut_lt(k * angle_grad + angle_base);
        // the kernel half of image i+1 overlaps the host commit of image i (levels are mask-free)
        Fuser::Levels cur, nxt;
        if (!fu.levels(0, tat_i, qk, cur)) { err = fu.err; return false; }
        for (int i = 0; i < n; ++i) {
            std::cout << "Fusing image " << std::setw(8) << std::setfill('0') << i << "..." << std::endl;
            std::future<bool> pre;
            if (i + 1 < n) pre = std::async(std::launch::async, [&, i]() { return fu.levels(i + 1, tat_i, qk, nxt); });
            const auto tc = Clock::now();
            const int64_t sw = fu.commit_tat(i, tat_i, cur);
            fu.commit_ms += ms_since(tc);
            if (!tat_i) printf("skip_weak: %lld\n", (long long)sw);
            if (pre.valid() && !pre.get()) { err = fu.err; return false; }
            std::swap(cur, nxt);
        }
    } else {
        const float q_angle = angle_cut_lt(0.174533f);
        Fuser::Cands cur, nxt;
        if (!fu.consistency(0, q_angle, cur)) { err = fu.err; return false; }
        for (int i = 0; i < n; ++i) {
            std::cout << "Fusing image " << std::setw(8) << std::setfill('0') << i << "..." << std::endl;
            std::future<bool> pre;
            if (i + 1 < n) pre = std::async(std::launch::async, [&, i]() { return fu.consistency(i + 1, q_angle, nxt); });
            const auto tc = Clock::now();
            fu.commit_default(i, cur, gmask.data());
            fu.commit_ms += ms_since(tc);
            if (pre.valid() && !pre.get()) { err = fu.err; return false; }
            std::swap(cur, nxt);
        }
    }
    rep.fuse_ms = ms_since(t0);
    rep.gpu_ms = fu.gpu_ms;
    rep.term_ms = fu.term_ms;
    rep.commit_ms = fu.commit_ms;

    t0 = Clock::now();
    write_ply(opt.dense_folder + "/APD/" + opt.name, fu.xyz, fu.bgr, opt.export_color);
    rep.write_ms = ms_since(t0);
    rep.points = (int64_t)(fu.xyz.size() / 3);
    return true;
}

}  // namespace apdhost
