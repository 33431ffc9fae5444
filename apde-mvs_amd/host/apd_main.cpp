// apd_main.cpp — the `apd` depth binary: drop-in for the reference's `APD` executable (main.cpp),
// driving libapd_hip.so through the C ABI of include/apd_hip.h.
//
// Same flags, defaults, bool-word parsing, exit codes and stdout lines as main.cpp:9-40 / 210-400
// (run.py:104-119 builds the command line), the same per-problem host work as
// APD::InuputInitialization (APD.cpp:501-685) and ProcessProblem (main.cpp:148-191), and the same
// round schedule (main.cpp:290-367). Additions (all optional):
//   --gpus LIST          comma-separated HIP devices; views of a pass are dealt to the devices by a
//                        dynamic work queue (one thread + one apd_ctx per device)
//   --ordering MODE      sequential (reference order: a view sees the current pass's depth maps of
//                        the views processed before it) | jacobi (every view of a pass reads the
//                        previous pass's maps; required for > 1 GPU, results independent of the
//                        device count and of the processing order)
//   --seed N             base of the deterministic per-problem RNG seed
// Fusion (RunFusion / RunFusion_TAT_I / RunFusion_TAT_A + WeakVisFilter, APD.cpp:962-1608) runs in
// fusion.cpp: per-(pixel, source) tests on the GPU, the ordered commit on the host.
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iomanip>
#include <iostream>
#include <map>
#include <set>
#include <memory>
#include <mutex>
#include <sstream>
#include <string>
#include <thread>
#include <tuple>
#include <vector>

#include "fusion.h"

#include "../../include/apd_hip.h"
#include "image.h"
#include "io.h"

using namespace apdhost;

namespace {

std::mutex g_print;
#define SAY(expr)                                      \
    do {                                               \
        std::lock_guard<std::mutex> _g(g_print);       \
        std::cout << expr << std::endl;                \
    } while (0)

// ------------------------------------------------------------------------------------------------
// arguments (boost::program_options semantics of main.cpp:6-40)
// ------------------------------------------------------------------------------------------------
struct Opt {
    const char *name, *shortname, *defval, *help;
    bool is_bool;
};
const Opt kOpts[] = {
    {"dense_folder", "d", nullptr, "path to dense folder", false},
    {"gpu_index", "g", "0", "gpu index", false},
    {"dataset", "D", "DTU", "dataset name, DTU, ETH3D or Tanks and Temples", false},
    {"only_fuse", "f", "false", "only fuse depths", true},
    {"no_fuse", "F", "false", "skip fuse", true},
    {"memory_cache", "m", "true", "use memory cache", true},
    {"use_sa", "s", "true", "use segment anything results", true},
    {"use_impetus", "i", "true", "use impetus", true},
    {"weak_filter", "w", "true", "use weak filter", true},
    {"flush", nullptr, "false", "Flush mat to disk", true},
    {"export_anchor", "n", "false", "Export anchor points to disk", true},
    {"export_curve", "r", "false", "Export reliable curve to disk", true},
    {"export_color", "c", "true", "Export ply with color", true},
    {"gpus", nullptr, "", "comma-separated HIP devices (default: gpu_index)", false},
    {"ordering", nullptr, "", "sequential | jacobi (default: sequential on 1 GPU, jacobi on more)", false},
    {"seed", nullptr, "24301", "base RNG seed of the deterministic PatchMatch RNG", false},
};

void usage() {
    std::cout << "Allowed options:\n";
    for (const Opt &o : kOpts) {
        std::string n = std::string("  ") + (o.shortname ? std::string("-") + o.shortname + " [ --" : "--") + o.name +
                        (o.shortname ? " ]" : "") + " arg";
        std::cout << std::left << std::setw(34) << n << o.help;
        if (o.defval && *o.defval) std::cout << " (=" << o.defval << ")";
        std::cout << "\n";
    }
    std::cout << "  -h [ --help ]                   produce help message\n";
}

bool parse_bool(const std::string &v, bool &b) {
    std::string s;
    for (char c : v) s += (char)tolower(c);
    if (s == "true" || s == "1" || s == "yes" || s == "on") { b = true; return true; }
    if (s == "false" || s == "0" || s == "no" || s == "off") { b = false; return true; }
    return false;
}

std::map<std::string, std::string> parse_args(int argc, char **argv) {
    std::map<std::string, std::string> vals;
    for (const Opt &o : kOpts)
        if (o.defval) vals[o.name] = o.defval;
    auto fail = [](const std::string &msg) {
        std::cout << "Error: " << msg << std::endl;
        usage();
        exit(-1);
    };
    for (int i = 1; i < argc; ++i) {
        std::string a = argv[i];
        if (a == "-h" || a == "--help") {
            usage();
            exit(0);
        }
        const Opt *opt = nullptr;
        std::string value;
        bool have_value = false;
        if (a.rfind("--", 0) == 0) {
            std::string n = a.substr(2);
            const size_t eq = n.find('=');
            if (eq != std::string::npos) { value = n.substr(eq + 1); n = n.substr(0, eq); have_value = true; }
            for (const Opt &o : kOpts) if (n == o.name) opt = &o;
        } else if (a.size() >= 2 && a[0] == '-') {
            const std::string n = a.substr(1, 1);
            for (const Opt &o : kOpts) if (o.shortname && n == o.shortname) opt = &o;
            if (a.size() > 2) { value = a.substr(2); have_value = true; }
        }
        if (!opt) fail("unrecognised option '" + a + "'");
        if (!have_value) {
            if (i + 1 >= argc) fail(std::string("the required argument for option '--") + opt->name + "' is missing");
            value = argv[++i];
        }
        if (opt->is_bool) {
            bool b;
            if (!parse_bool(value, b))
                fail(std::string("the argument ('") + value + "') for option '--" + opt->name + "' is invalid");
        }
        vals[opt->name] = value;
    }
    if (!vals.count("dense_folder")) fail("the option '--dense_folder' is required but missing");
    return vals;
}

bool as_bool(const std::map<std::string, std::string> &v, const char *k) {
    bool b = false;
    parse_bool(v.at(k), b);
    return b;
}

// ------------------------------------------------------------------------------------------------
// per-problem state (main.h:80-115)
// ------------------------------------------------------------------------------------------------
struct Job {
    Problem pb;
    apd_params params{};
    int scale_size = 1;
    int iteration = 0;
    bool export_anchor = false, export_curve = false;
    long used_ms = 0;
};

// Decoded and rescaled images shared by every problem of the run. The reference decodes and
// resizes all N+1 images again for each problem of each pass (APD.cpp:508-590): a 9-view 3024x2016
// scan spent 41 of its 93 s there. Here each file is decoded once and each (file, scale, size)
// resized once; the pixels are the ones the per-problem path produces (same decoder, same resize).
struct ImageCache {
    struct Decoded {
        std::once_flag once;
        bool ok = false;
        Gray8 g;
    };
    struct Scaled {
        std::once_flag once;
        std::vector<float> img;
        int w = 0, h = 0;
    };
    std::mutex mu;
    std::map<std::string, std::shared_ptr<Decoded>> decoded;
    std::map<std::string, std::shared_ptr<Scaled>> scaled;

    std::shared_ptr<Decoded> decode(const std::string &path) {
        std::shared_ptr<Decoded> e;
        {
            std::lock_guard<std::mutex> g(mu);
            auto &slot = decoded[path];
            if (!slot) slot = std::make_shared<Decoded>();
            e = slot;
        }
        std::call_once(e->once, [&] {
            std::string err;
            e->ok = read_gray8(path, e->g, err);
            if (!e->ok) SAY("Error opening file: \"" << path << "\" (" << err << ")");
        });
        return e;
    }
    // convertTo(CV_32FC1) of the file, resized with INTER_LINEAR to round(src * 1/scale) when
    // scale != 1, src_w x src_h being the size the reference resizes from (the ref image's, APD.cpp:567)
    std::shared_ptr<Scaled> image(const std::string &path, int scale, int src_w, int src_h, const Gray8 &g) {
        const std::string key = path + "|" + std::to_string(scale) + "|" + std::to_string(src_w) + "x" + std::to_string(src_h);
        std::shared_ptr<Scaled> e;
        {
            std::lock_guard<std::mutex> l(mu);
            auto &slot = scaled[key];
            if (!slot) slot = std::make_shared<Scaled>();
            e = slot;
        }
        std::call_once(e->once, [&] {
            std::vector<float> f(g.px.size());
            for (size_t i = 0; i < g.px.size(); ++i) f[i] = (float)g.px[i];
            if (scale == 1) {
                e->img.swap(f);
                e->w = g.width;
                e->h = g.height;
                return;
            }
            const float factor = 1.0f / (float)scale;
            e->w = (int)std::round(src_w * factor);
            e->h = (int)std::round(src_h * factor);
            e->img.resize((size_t)e->w * e->h);
            resize_linear_f32(f.data(), src_w, src_h, e->img.data(), e->w, e->h);
        });
        return e;
    }
    void drop_scaled() {  // a new round: the previous scale is not used again
        std::lock_guard<std::mutex> l(mu);
        scaled.clear();
    }
};

// run f(0..n-1) on up to `threads` host threads
template <class F>
void parallel_for(size_t n, unsigned threads, F f) {
    threads = std::max(1u, std::min<unsigned>(threads, (unsigned)n));
    std::atomic<size_t> next{0};
    auto body = [&] {
        for (size_t i; (i = next.fetch_add(1)) < n;) f(i);
    };
    std::vector<std::thread> th;
    for (unsigned t = 1; t < threads; ++t) th.emplace_back(body);
    body();
    for (auto &t : th) t.join();
}
unsigned host_threads() {
    const unsigned hw = std::thread::hardware_concurrency();
    return std::max(1u, std::min(16u, hw ? hw : 4u));
}

struct Pending {  // Jacobi ordering: outputs committed at the end of the pass
    std::string path;
    Mat mat;
};

// Device-resident view state (one per context): the round's images and every view's last depth and
// (normal, depth) planes stay in HBM between problems. The reference re-reads and re-uploads all of
// them per problem (APD.cpp:508-684): at 6048x4032 with 10 sources that is 2.5 GB of uploads per
// problem. The files are still written (fusion and later runs read them) and the maps here hold the
// same values: depth = the epilogue's depth, planes = (normals.bin, depths.bin) interleaved, the
// INTER_NEAREST resize to a new round's size done by the same index map on the device. A view whose
// map is not here (none yet) falls back to the store.
struct DevStore {
    struct Map {
        void *p = nullptr;
        int w = 0, h = 0;
        size_t bytes = 0;
    };
    apd_ctx *ctx = nullptr;
    std::map<std::string, Map> images;          // this round's images, by path
    std::map<int, Map> depth, planes;           // committed maps, by view id
    std::map<int, Map> pend_depth, pend_planes;  // Jacobi: this pass's outputs until commit()
    std::set<int> fresh;                         // views whose pending maps this pass wrote (commit() clears;
                                                 // after a commit the pending slots hold recycled buffers)
    Map scratch;                                 // resized priors of one problem
    long uploaded = 0;                           // bytes copied from the host (images)
    // bytes held; an allocation that fails (or would pass APD_DEVICE_STATE_CAP_MB, a test hook) makes
    // the caller fall back to the host path for that image / problem / view
    size_t used = 0, cap = (size_t)-1;
    int share = 1;             // contexts on this store's device (they share its free memory)
    size_t lib_peak = 0;       // the most device memory the library's own buffers held after a problem
    bool cap_fixed = false;    // APD_DEVICE_STATE_CAP_MB (test hook): the cap is not resized
    // After a problem: the cap follows the real footprint -- what the store holds plus this context's
    // share of the free memory, less room for the library's buffers to grow on later problems (half
    // of their peak, at least 2 GiB: the pair table and the hand-over vary with the WEAK fraction)
    void resize_cap() {
        size_t lb = 0, fb = 0, tb = 0;
        if (cap_fixed || apd_device_bytes(ctx, &lb) != APD_OK || apd_device_mem_info(ctx, &fb, &tb) != APD_OK) return;
        lib_peak = std::max(lib_peak, lb);
        const size_t margin = std::max<size_t>((size_t)2 << 30, lib_peak / 2);
        const size_t avail = fb / (size_t)std::max(1, share);
        cap = used + (avail > margin ? avail - margin : 0);
    }

    bool reserve(Map &m, size_t bytes) {
        if (m.p && m.bytes >= bytes) return true;
        release(m);
        if (used + bytes > cap || apd_device_alloc(ctx, bytes, &m.p) != APD_OK) {
            m = Map{};
            return false;
        }
        m.bytes = bytes;
        used += bytes;
        return true;
    }
    void release(Map &m) {
        if (m.p) {
            apd_device_free(ctx, m.p);
            used -= m.bytes;
        }
        m = Map{};
    }
    void release_all(std::map<int, Map> &ms) {
        for (auto &kv : ms) release(kv.second);
        ms.clear();
    }
    // the round image in HBM; nullptr with *failed false: no room (the caller uploads it per problem),
    // with *failed true: the copy itself failed (an error, the buffer is released)
    const float *image(const std::string &key, const ImageCache::Scaled &s, bool *failed) {
        *failed = false;
        Map &m = images[key];
        if (!m.p) {
            const size_t b = (size_t)s.w * s.h * sizeof(float);
            if (!reserve(m, b)) return nullptr;
            if (apd_device_copy(ctx, m.p, s.img.data(), b) != APD_OK) {
                release(m);
                *failed = true;
                return nullptr;
            }
            m.w = s.w;
            m.h = s.h;
            uploaded += (long)b;
        }
        return static_cast<const float *>(m.p);
    }
    void drop_images() {
        for (auto &kv : images) release(kv.second);
        images.clear();
    }
    // the map of view `id` at w x h: the committed map itself, or its nearest resize into `dst`
    const void *fitted(const Map &m, int w, int h, int elem, uint8_t *dst) {
        if (m.w == w && m.h == h) return m.p;
        if (apd_device_resize_nearest(ctx, m.p, m.w, m.h, dst, w, h, elem) != APD_OK) return nullptr;
        return dst;
    }
    // view `id` leaves the device state (HBM exhausted): every later problem reads its priors from
    // the store, which always holds the same values (the files are written either way)
    void forget(int id) {
        fresh.erase(id);
        for (auto *ms : {&depth, &planes, &pend_depth, &pend_planes}) {
            auto it = ms->find(id);
            if (it != ms->end()) {
                release(it->second);
                ms->erase(it);
            }
        }
    }
    // device buffers for view `id`'s new maps at w x h (false: no room, the view was forgotten)
    bool output(int id, bool pending, int w, int h, float **d, float **pl) {
        Map &md = (pending ? pend_depth : depth)[id], &mp = (pending ? pend_planes : planes)[id];
        const size_t n = (size_t)w * h;
        if (!reserve(md, n * sizeof(float)) || !reserve(mp, n * 4 * sizeof(float))) {
            forget(id);
            return false;
        }
        md.w = mp.w = w;
        md.h = mp.h = h;
        if (pending) fresh.insert(id);
        *d = static_cast<float *>(md.p);
        *pl = static_cast<float *>(mp.p);
        return true;
    }
    void commit() {
        for (auto pair : {std::make_pair(&pend_depth, &depth), std::make_pair(&pend_planes, &planes)})
            for (auto &kv : *pair.first)
                if (fresh.count(kv.first)) std::swap((*pair.second)[kv.first], kv.second);  // the old buffer serves the next pass
        fresh.clear();
    }
    // Jacobi over several contexts: view `id`'s new maps, produced by another context, into this
    // store's pending maps, device to device (apd_device_copy_peer: xGMI between GPUs, a device copy
    // between two contexts of one GPU). False (the view forgotten here) when there is no room.
    struct Source {  // a snapshot of another store's pending maps of one view (taken before the pulls)
        int id;
        DevStore *from;   // nullptr: no store holds the view's new maps
        const void *d, *pl;
        int w, h;
    };
    bool pull(const Source &v) {
        float *d = nullptr, *pl = nullptr;
        if (!output(v.id, true, v.w, v.h, &d, &pl)) return false;
        if (apd_device_copy_peer(ctx, d, v.from->ctx, v.d, (size_t)v.w * v.h * sizeof(float)) != APD_OK ||
            apd_device_copy_peer(ctx, pl, v.from->ctx, v.pl, (size_t)v.w * v.h * 4 * sizeof(float)) != APD_OK) {
            forget(v.id);
            return false;
        }
        return true;
    }
    bool pending_of(int id) const { return fresh.count(id) != 0; }
    ~DevStore() {
        if (!ctx) return;
        drop_images();
        release_all(depth);
        release_all(planes);
        release_all(pend_depth);
        release_all(pend_planes);
        release(scratch);
    }
};

struct Driver {
    std::string dense;
    bool use_sa = true, flush = false;
    uint64_t seed = 24301;
    bool jacobi = false;
    MatStore *store = nullptr;
    ImageCache images;
    // one device store per context (each holds every view's maps on its own device; a Jacobi pass's
    // new maps are exchanged between them at the commit), or none (APD_DEVICE_STATE=0)
    std::vector<apd_ctx *> ctxs;
    std::vector<std::unique_ptr<DevStore>> devs;
    std::unique_ptr<DevStore> &store_for(apd_ctx *ctx) {
        static std::unique_ptr<DevStore> none;
        for (size_t k = 0; k < ctxs.size(); ++k)
            if (ctxs[k] == ctx && k < devs.size()) return devs[k];
        none.reset();
        return none;
    }
    std::vector<int> pass_views;  // the views of the current pass (the commit exchanges their maps)
    std::mutex pend_mu;
    std::vector<Pending> pending;

    // INTER_NEAREST resizes of priors (APD.cpp:605-609, 619-625, 669-673) at a round's first pass: every
    // problem that reads view j's map resizes the same Mat to the same size, so each (Mat, size) is
    // resized once per pass (entries keep their source alive, so a buffer address is never reused
    // while it is a key; cleared at every pass).
    std::mutex fit_mu;
    std::map<std::tuple<const uint8_t *, int, int>, std::pair<Mat, Mat>> fitted;
    Mat fit_cached(const Mat &m, int w, int h) {
        // the key (buffer address) is stable only when reads are served from the MemoryCache: without
        // it every read returns a fresh buffer, nothing would hit, and the map would pin every prior
        if (!store->cached()) return resize_nearest(m, w, h);
        const auto key = std::make_tuple(m.bytes(), w, h);
        {
            std::lock_guard<std::mutex> g(fit_mu);
            auto it = fitted.find(key);
            if (it != fitted.end()) return it->second.second;
        }
        Mat r = resize_nearest(m, w, h);
        std::lock_guard<std::mutex> g(fit_mu);
        return fitted.emplace(key, std::make_pair(m, r)).first->second.second;
    }
    void emit(const std::string &path, const Mat &m) {
        if (jacobi) {
            std::lock_guard<std::mutex> g(pend_mu);
            pending.push_back({path, m});
        } else {
            store->write(path, m, flush);
        }
    }
    void commit() {
        for (auto &p : pending) store->write(p.path, p.mat, flush);
        pending.clear();
        exchange_maps();
        for (auto &d : devs)
            if (d) d->commit();
        std::lock_guard<std::mutex> g(fit_mu);
        fitted.clear();
    }
    // Jacobi over several contexts (after the pass's workers joined): every store gets every view's new
    // maps. A view that no store holds (its context's store ran out of room or was released) is
    // forgotten everywhere: the previous pass's map would be stale, and the files hold the new one.
    // Each destination store pulls on its own thread (its own device and stream).
    void exchange_maps() {
        std::vector<DevStore *> live;
        for (auto &d : devs)
            if (d) live.push_back(d.get());
        if (live.size() < 2 && live.size() == devs.size()) return;  // one context: nothing to exchange
        // the sources, read here before any store changes its maps (each pulling thread then writes
        // only its own store's maps)
        std::vector<DevStore::Source> src;
        for (int id : pass_views) {
            DevStore::Source v{id, nullptr, nullptr, nullptr, 0, 0};
            for (DevStore *d : live)
                if (d->pending_of(id)) {
                    const DevStore::Map &md = d->pend_depth.at(id), &mp = d->pend_planes.at(id);
                    v = DevStore::Source{id, d, md.p, mp.p, md.w, md.h};
                    break;
                }
            src.push_back(v);
        }
        std::vector<std::thread> th;
        for (DevStore *to : live)
            th.emplace_back([&src, to]() {
                for (const auto &v : src) {
                    if (v.from == to) continue;
                    if (!v.from) { to->forget(v.id); continue; }
                    if (!to->pull(v))
                        SAY("device state full: view " << v.id << " falls back to the host store on one context");
                }
            });
        for (auto &t : th) t.join();
    }
    void new_round() {  // each round uses one scale
        images.drop_scaled();
        for (auto &d : devs)
            if (d) d->drop_images();
    }

    // APD::InuputInitialization + CudaSpaceInitialization + RunPatchMatch + ProcessProblem
    bool process(apd_ctx *ctx, Job &job);
    // decode (once) and resize (once per round) every image the round's problems read, on host
    // threads in parallel; process() then finds them in the ImageCache. Same decoder and resize, so
    // the same pixels; a file that fails to decode is reported by process() as before.
    void prefetch_round(int scale, const std::vector<Problem> &problems) {
        std::vector<std::pair<int, std::string>> files;  // (id, extension of the problem naming it)
        std::map<int, bool> seen;
        for (const Problem &p : problems) {
            std::vector<int> ids{p.ref_image_id};
            ids.insert(ids.end(), p.src_image_ids.begin(), p.src_image_ids.end());
            for (int id : ids)
                if (!seen[id]) { seen[id] = true; files.push_back({id, p.img_ext}); }
        }
        parallel_for(files.size(), host_threads(), [&](size_t k) {
            const std::string path = dense + "/images/" + format_index(files[k].first) + files[k].second;
            auto d = images.decode(path);
            if (!d->ok) return;
            // every image of a problem is resized from the reference image's size (APD.cpp:567), and
            // all images of a scan have one size (CheckImages), so (own size) is the key process() uses
            images.image(path, scale, d->g.width, d->g.height, d->g);
        });
    }
};

bool Driver::process(apd_ctx *ctx, Job &job) {
    const Problem &pb = job.pb;
    std::unique_ptr<DevStore> &dev = store_for(ctx);  // (this context's store; only its worker uses it)
    const std::string result_folder = dense + "/APD/" + format_index(pb.ref_image_id);
    SAY("Processing image: " << format_index(pb.ref_image_id) << "...");
    const auto start = std::chrono::steady_clock::now();
    // ---- images (APD.cpp:508-533), decoded once per run (ImageCache)
    std::vector<int> ids{pb.ref_image_id};
    ids.insert(ids.end(), pb.src_image_ids.begin(), pb.src_image_ids.end());
    std::vector<std::shared_ptr<ImageCache::Decoded>> dec;
    for (size_t i = 0; i < ids.size(); ++i) {
        dec.push_back(images.decode(dense + "/images/" + format_index(ids[i]) + pb.img_ext));
        if (!dec.back()->ok) return false;
    }
    int width = dec[0]->g.width, height = dec[0]->g.height;
    for (size_t i = 1; i < dec.size(); ++i)
        if (dec[i]->g.width != width || dec[i]->g.height != height) {
            SAY("Image size mismatch: " << format_index(ids[i]) << " is " << dec[i]->g.width << "x" << dec[i]->g.height
                                        << ", the reference image " << width << "x" << height);
            return false;
        }
    if (dec.size() > APD_MAX_IMAGES) {
        SAY("Can't process so much images: " << dec.size());
        exit(EXIT_FAILURE);
    }
    const int NI = (int)dec.size();
    // ---- cameras (APD.cpp:536-556)
    std::vector<apd_camera> cams(NI);
    for (int i = 0; i < NI; ++i) {
        if (!read_camera(dense + "/cams/" + format_index(ids[i]) + "_cam.txt", cams[i])) {
            SAY("Error opening file: " << dense << "/cams/" << format_index(ids[i]) << "_cam.txt");
            return false;
        }
        cams[i].width = width;
        cams[i].height = height;
    }
    apd_params P = job.params;
    P.depth_min = cams[0].depth_min * 0.6f;
    P.depth_max = cams[0].depth_max * 1.2f;
    P.num_images = NI;
    {
        std::lock_guard<std::mutex> g(g_print);
        std::cout << "Read images and camera done\n";
        std::cout << "Depth range: " << P.depth_min << " " << P.depth_max << std::endl;
        std::cout << "Num images: " << P.num_images << std::endl;
    }
    // ---- scale (APD.cpp:562-590): every image is resized from the reference's size
    std::vector<std::shared_ptr<ImageCache::Scaled>> scaled;
    for (int i = 0; i < NI; ++i) {
        scaled.push_back(images.image(dense + "/images/" + format_index(ids[i]) + pb.img_ext, job.scale_size, width,
                                      height, dec[i]->g));
        if (job.scale_size != 1) {
            const float scale_x = scaled[i]->w / (float)width, scale_y = scaled[i]->h / (float)height;
            cams[i].K[0] *= scale_x;
            cams[i].K[2] *= scale_x;
            cams[i].K[4] *= scale_y;
            cams[i].K[5] *= scale_y;
            cams[i].width = scaled[i]->w;
            cams[i].height = scaled[i]->h;
        }
    }
    if (job.scale_size != 1) {
        width = cams[0].width;
        height = cams[0].height;
        SAY("Scale images and cameras done");
    }
    SAY("Image size: " << width << " * " << height);
    const size_t HW = (size_t)width * height;
    auto fit = [&](Mat m) { return (m.cols != width || m.rows != height) ? fit_cached(m, width, height) : m; };
    // device-resident inputs: every image, and every depth / plane prior this problem reads when the
    // DevStore holds all of them (else the priors come from the store as below)
    const bool need_depths = P.geom_consistency || P.use_APD, need_planes = P.state != APD_FIRST_INIT;
    std::vector<const float *> img_ptrs(NI), dep_ptrs(NI);
    const float *dev_planes = nullptr;
    bool dev_priors = false;
    if (dev) {
        for (int i = 0; i < NI; ++i) {
            bool failed = false;
            img_ptrs[i] = dev->image(dense + "/images/" + format_index(ids[i]) + pb.img_ext, *scaled[i], &failed);
            if (failed) { SAY("device upload failed: " << apd_last_error(ctx)); return false; }
            if (!img_ptrs[i]) {  // no room in HBM: this image is uploaded per problem, as the reference does
                dev->images.erase(dense + "/images/" + format_index(ids[i]) + pb.img_ext);
                img_ptrs[i] = scaled[i]->img.data();
            }
        }
        auto held = [](const std::map<int, DevStore::Map> &ms, int id) {
            auto it = ms.find(id);
            return it != ms.end() && it->second.p;
        };
        dev_priors = need_depths || need_planes;
        for (int i = 0; i < NI && dev_priors && need_depths; ++i) dev_priors = held(dev->depth, ids[i]);
        if (dev_priors && need_planes) dev_priors = held(dev->planes, ids[0]);
        if (dev_priors) {
            const size_t slots = need_depths ? (size_t)NI : 0;
            // (no room for the resized priors in HBM: this problem reads them from the store)
            if (!dev->reserve(dev->scratch, HW * sizeof(float) * (slots + 4))) dev_priors = false;
            uint8_t *s = static_cast<uint8_t *>(dev->scratch.p);
            for (size_t i = 0; i < slots && dev_priors; ++i) {
                dep_ptrs[i] = static_cast<const float *>(
                    dev->fitted(dev->depth[ids[i]], width, height, 4, s + i * HW * sizeof(float)));
                if (!dep_ptrs[i]) { SAY("device resize failed: " << apd_last_error(ctx)); return false; }
            }
            if (need_planes && dev_priors) {
                dev_planes = static_cast<const float *>(
                    dev->fitted(dev->planes[ids[0]], width, height, 16, s + slots * HW * sizeof(float)));
                if (!dev_planes) { SAY("device resize failed: " << apd_last_error(ctx)); return false; }
            }
        }
    }
    const auto t_img = std::chrono::steady_clock::now();
    // ---- priors (APD.cpp:592-684)
    std::vector<Mat> depths;
    if (need_depths && !dev_priors) {
        Mat d;
        store->read(result_folder + "/depths.bin", d);
        depths.push_back(fit(d));
        for (int id : pb.src_image_ids) {
            Mat s;
            store->read(dense + "/APD/" + format_index(id) + "/depths.bin", s);
            depths.push_back(fit(s));
        }
        for (auto &m : depths)
            if (m.empty() || m.type != CV_32FC1) { SAY("Error: missing depth prior"); return false; }
    }
    Mat weak, conf, sa, anchors_map;
    int weak_count = 0;
    if (P.use_APD) {
        store->read(result_folder + "/weak.bin", weak);
        store->read(result_folder + "/confidence.bin", conf);
        if (weak.empty() || conf.empty()) { SAY("Error: missing weak/confidence prior"); return false; }
        if (weak.cols != width || weak.rows != height) { SAY("resize weak info to target size"); weak = fit(weak); }
        if (conf.cols != width || conf.rows != height) { SAY("resize confidence to target size"); conf = fit(conf); }
        // anchors_map (APD.cpp:627-640) is built on the device; the host copy only feeds --export_anchor
        const uint8_t *wp = weak.ptr<uint8_t>();
        if (job.export_anchor) {
            anchors_map = Mat(height, width, CV_32SC1);
            for (size_t i = 0; i < HW; ++i) anchors_map.ptr<int32_t>()[i] = wp[i] == APD_WEAK ? weak_count++ : -1;
        } else {
            const size_t chunk = 1 << 20, nc = (HW + chunk - 1) / chunk;
            std::vector<int> part(nc, 0);
            parallel_for(nc, host_threads(), [&](size_t b) {
                int c = 0;
                for (size_t i = b * chunk, e = std::min(HW, i + chunk); i < e; ++i) c += wp[i] == APD_WEAK;
                part[b] = c;
            });
            for (int c : part) weak_count += c;
        }
        if (P.use_sa) {
            const std::string sa_dir = dense + "/sa_masks";
            if (file_exists(sa_dir)) {
                store->read(sa_dir + "/" + format_index(pb.ref_image_id) + ".bin", sa);
                if (!sa.empty() && (sa.cols != width || sa.rows != height)) { SAY("resize sa mask to target size"); sa = fit(sa); }
            } else {
                SAY("Can't find sa mask folder: \"" << sa_dir << "\"");
            }
        }
        SAY("Weak count: " << weak_count << " / " << HW << " = " << (float)weak_count / (float)HW * 100 << "%");
    }
    std::shared_ptr<uint8_t[]> init_planes;  // pooled, not zero-filled: every element is written below
    if (need_planes && !dev_priors) {
        Mat d, n;
        store->read(result_folder + "/depths.bin", d);
        store->read(result_folder + "/normals.bin", n);
        if (d.empty() || n.empty()) { SAY("Error: missing depth/normal prior"); return false; }
        if (d.cols != width || d.rows != height || n.cols != width || n.rows != height) {
            SAY("resize depth and normal to target size");
            d = fit(d);
            n = fit(n);
        }
        init_planes = pool_buffer(HW * 4 * sizeof(float));
        float *ip = reinterpret_cast<float *>(init_planes.get());
        const float *np_ = n.ptr<float>(), *dp = d.ptr<float>();
        const size_t chunk = 1 << 18;
        parallel_for((HW + chunk - 1) / chunk, host_threads(), [&](size_t b) {
            for (size_t i = b * chunk, e = std::min(HW, i + chunk); i < e; ++i) {
                ip[4 * i + 0] = np_[3 * i + 0];
                ip[4 * i + 1] = np_[3 * i + 1];
                ip[4 * i + 2] = np_[3 * i + 2];
                ip[4 * i + 3] = dp[i];
            }
        });
    }
    const auto t_pri = std::chrono::steady_clock::now();
    // ---- device (CudaSpaceInitialization + RunPatchMatch)
    if (!dev)
        for (int i = 0; i < NI; ++i) img_ptrs[i] = scaled[i]->img.data();
    if (!dev_priors)
        for (size_t i = 0; i < depths.size(); ++i) dep_ptrs[i] = depths[i].ptr<float>();
    apd_problem prob{};
    prob.width = width;
    prob.height = height;
    prob.num_images = NI;
    prob.images = img_ptrs.data();
    prob.cameras = cams.data();
    prob.params = P;
    prob.depths = need_depths ? dep_ptrs.data() : nullptr;
    prob.init_planes = dev_priors ? dev_planes : reinterpret_cast<const float *>(init_planes.get());
    prob.weak_info = P.use_APD ? weak.ptr<uint8_t>() : nullptr;
    prob.confidence = P.use_APD ? conf.ptr<uint8_t>() : nullptr;
    prob.sa_mask = (P.use_APD && !sa.empty()) ? sa.ptr<uint8_t>() : nullptr;
    prob.seed = seed ^ ((uint64_t)(uint32_t)job.iteration << 32) ^ (uint64_t)(uint32_t)pb.ref_image_id;
    prob.export_reliable_curve = job.export_curve ? 1 : 0;
    int st = apd_set_problem(ctx, &prob);
    if (dev && st == APD_OK) {  // test hook: the k-th problem with the device store finds HBM exhausted
        static std::atomic<int> n_dev_problems{0};
        const char *e = getenv("APD_TEST_ENOMEM_AT");
        if (e && ++n_dev_problems == atoi(e)) st = APD_ENOMEM;
    }
    auto t0 = std::chrono::steady_clock::now();
    if (st == APD_OK) {
        t0 = std::chrono::steady_clock::now();
        st = apd_run_patchmatch(ctx);
    }
    const auto t1 = std::chrono::steady_clock::now();
    if (st == APD_ENOMEM && dev) {
        // the library's own per-problem buffers did not fit next to the device-resident store: the
        // store is released (its maps hold the same values as the files, pending ones are committed
        // from the host side at the pass end) and the run continues on the host store, starting with
        // this problem
        SAY("device memory exhausted (" << apd_last_error(ctx) << "): device-resident state released, "
                                         "the run continues from the host store");
        dev.reset();
        return process(ctx, job);
    }
    if (st != APD_OK) { SAY("RunPatchMatch failed: " << apd_last_error(ctx)); return false; }
    if (dev) dev->resize_cap();
    const long ms = (long)std::chrono::duration_cast<std::chrono::milliseconds>(t1 - t0).count();
    {
        std::lock_guard<std::mutex> g(g_print);
        printf("RunPatchMatch time: %ld ms\n", ms);
        fflush(stdout);
    }
    job.used_ms += ms;
    // ---- results
    std::shared_ptr<uint8_t[]> planes_buf = pool_buffer(HW * 4 * sizeof(float));  // filled by apd_get_results
    float *planes = reinterpret_cast<float *>(planes_buf.get());
    Mat depth(height, width, CV_32FC1), normal(height, width, CV_32FC3), states(height, width, CV_8UC1),
        confidence(height, width, CV_8UC1);
    std::vector<int16_t> anchors;
    std::vector<float> curve;
    int32_t wc = 0;
    apd_outputs out{};
    out.planes = planes;
    out.weak_info = states.ptr<uint8_t>();
    out.confidence = confidence.ptr<uint8_t>();
    out.weak_count = &wc;
    if (job.export_anchor && P.use_APD) {
        anchors.resize((size_t)std::max(weak_count, 1) * APD_ANCHOR_NUM * 2);
        out.anchors = anchors.data();
    }
    if (job.export_curve) {
        curve.resize(HW * APD_CURVE_SAMPLES);
        out.reliable_curve = curve.data();
    }
    const auto t_run = std::chrono::steady_clock::now();
    st = apd_get_results(ctx, &out);
    if (st == APD_ENOMEM && dev) {
        // the anchors export's staging buffer did not fit next to the store: release the store (as
        // above) and read the results again -- the ctx still holds them
        SAY("device memory exhausted (" << apd_last_error(ctx) << "): device-resident state released, "
                                         "the run continues from the host store");
        dev.reset();
        st = apd_get_results(ctx, &out);
    }
    const auto t_get = std::chrono::steady_clock::now();
    if (st != APD_OK) { SAY("apd_get_results failed: " << apd_last_error(ctx)); return false; }
    if (dev) {  // this view's next priors, kept in HBM (Jacobi: visible after the pass, as the files)
        float *dd = nullptr, *dp = nullptr;
        if (!dev->output(pb.ref_image_id, jacobi, width, height, &dd, &dp)) {
            // HBM exhausted: the view's later priors come from the store (dev->forget)
            SAY("device state full: view " << pb.ref_image_id << " falls back to the host store");
        } else if (apd_result_device(ctx, dd, dp) != APD_OK) {
            SAY("apd_result_device failed: " << apd_last_error(ctx));
            return false;
        }
    }
    if (!(P.geom_consistency || P.use_APD)) memset(confidence.bytes(), 1, confidence.size_bytes());
    {  // the epilogue is element-wise: row chunks on host threads
        const int rows = 64;
        parallel_for((size_t)(height + rows - 1) / rows, host_threads(), [&](size_t b) {
            const int r0 = (int)b * rows, nr = std::min(rows, height - r0);
            const size_t o = (size_t)r0 * width;
            apd_epilogue(width, nr, planes + 4 * o, P.depth_min, P.depth_max, depth.ptr<float>() + o,
                         normal.ptr<float>() + 3 * o, states.ptr<uint8_t>() + o);
        });
    }
    // ---- exports (APD.cu:2614-2626, 2649-2660); written immediately, they are not priors
    if (job.export_anchor && P.use_APD) {
        write_binmat_file(result_folder + "/anchors_map.bin", anchors_map);
        FILE *fa = fopen((result_folder + "/anchors.bin").c_str(), "wb");
        if (fa) {
            const int32_t n = wc, k = APD_ANCHOR_NUM;
            fwrite(&n, 4, 1, fa);
            fwrite(&k, 4, 1, fa);
            fwrite(anchors.data(), sizeof(int16_t) * 2, (size_t)wc * APD_ANCHOR_NUM, fa);
            fclose(fa);
        }
    }
    if (job.export_curve) {
        FILE *fc = fopen((result_folder + "/reliable_curve.bin").c_str(), "wb");
        if (fc) {
            const int32_t w32 = width, h32 = height, ns = APD_CURVE_SAMPLES;
            fwrite(&w32, 4, 1, fc);
            fwrite(&h32, 4, 1, fc);
            fwrite(&ns, 4, 1, fc);
            fwrite(curve.data(), sizeof(float), curve.size(), fc);
            fclose(fc);
        }
    }
    const auto t_epi = std::chrono::steady_clock::now();
    emit(result_folder + "/depths.bin", depth);
    emit(result_folder + "/normals.bin", normal);
    emit(result_folder + "/weak.bin", states);
    if (P.geom_consistency || P.use_APD) emit(result_folder + "/confidence.bin", confidence);
    const auto end = std::chrono::steady_clock::now();
    if (getenv("APD_HOST_TIMING")) {  // host-side breakdown of one problem (ms)
        auto ms_ = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
        std::lock_guard<std::mutex> g(g_print);
        printf("HostTiming images %.1f priors %.1f set+run %.1f (run %ld) results %.1f epilogue %.1f emit %.1f\n",
               ms_(start, t_img), ms_(t_img, t_pri), ms_(t_pri, t_run), ms, ms_(t_run, t_get), ms_(t_get, t_epi),
               ms_(t_epi, end));
    }
    if (getenv("APD_PHASE_TIMING")) {  // the library's phase split of this RunPatchMatch (device events, ms)
        apd_timing tm{};
        if (apd_get_timing(ctx, &tm) == APD_OK) {
            std::lock_guard<std::mutex> g(g_print);
            printf("PhaseTiming %d %d iters %d weak %d total %.3f anchors %.3f lists %.3f pairs %.3f init %.3f "
                   "sweep %.3f post %.3f\n", width, height, tm.iterations, weak_count, tm.total_ms, tm.anchors_ms,
                   tm.lists_ms, tm.pairs_ms, tm.init_ms, tm.sweep_ms, tm.post_ms);
        }
    }
    {
        std::lock_guard<std::mutex> g(g_print);
        std::cout << "Processing image: " << format_index(pb.ref_image_id) << " done!" << std::endl;
        std::cout << "Cost time: " << std::chrono::duration_cast<std::chrono::milliseconds>(end - start).count()
                  << " ms" << std::endl;
    }
    return true;
}

}  // namespace

int main(int argc, char **argv) {
    auto vm = parse_args(argc, argv);
    const std::string dense = vm["dense_folder"];
    const int gpu_index = std::atoi(vm["gpu_index"].c_str());
    const std::string dataset = vm["dataset"];
    const bool only_fuse = as_bool(vm, "only_fuse");
    const bool no_fuse = as_bool(vm, "no_fuse");
    bool use_memory_cache = as_bool(vm, "memory_cache");
    const bool use_sa = as_bool(vm, "use_sa");
    const bool use_impetus = as_bool(vm, "use_impetus");
    const bool weak_filter = as_bool(vm, "weak_filter");
    bool flush = as_bool(vm, "flush");
    const bool export_anchor = as_bool(vm, "export_anchor");
    const bool export_curve = as_bool(vm, "export_curve");
    const bool export_color = as_bool(vm, "export_color");
    if (only_fuse) use_memory_cache = false;
    if (no_fuse) flush = true;
    std::vector<int> gpus;
    {
        std::stringstream ss(vm["gpus"]);
        std::string tok;
        while (std::getline(ss, tok, ',')) if (!tok.empty()) gpus.push_back(std::atoi(tok.c_str()));
        if (gpus.empty()) gpus.push_back(gpu_index);
    }
    std::string ordering = vm["ordering"];
    if (ordering.empty()) ordering = gpus.size() > 1 ? "jacobi" : "sequential";
    if (ordering != "sequential" && ordering != "jacobi") {
        std::cout << "Error: --ordering must be sequential or jacobi" << std::endl;
        return -1;
    }
    if (gpus.size() > 1 && ordering != "jacobi") {
        std::cout << "Error: more than one GPU requires --ordering jacobi" << std::endl;
        return -1;
    }
    std::cout << "========================== Config ==========================" << std::endl;
    std::cout << "dense_folder : " << dense << std::endl;
    std::cout << "gpu_index    : " << gpu_index << std::endl;
    std::cout << "dataset      : " << dataset << std::endl;
    std::cout << "only_fuse    : " << only_fuse << std::endl;
    std::cout << "no_fuse      : " << no_fuse << std::endl;
    std::cout << "memory_cache : " << use_memory_cache << std::endl;
    std::cout << "use_sa       : " << use_sa << std::endl;
    std::cout << "use_impetus  : " << use_impetus << std::endl;
    std::cout << "weak_filter  : " << weak_filter << std::endl;
    std::cout << "flush        : " << flush << std::endl;
    std::cout << "export_anchor: " << export_anchor << std::endl;
    std::cout << "export_curve : " << export_curve << std::endl;
    std::cout << "export_color : " << export_color << std::endl;
    std::cout << "gpus         : " << vm["gpus"] << std::endl;
    std::cout << "ordering     : " << ordering << std::endl;
    std::cout << "============================================================" << std::endl;
    if (use_memory_cache) printf("Use memory cache!\n");
    MatStore store(use_memory_cache);
    make_dir(dense + "/APD");
    std::vector<Problem> problems;
    std::string err;
    if (!read_pair_file(dense, problems, err)) {
        std::cout << "Error: " << err << std::endl;
        return -1;
    }
    for (auto &p : problems) make_dir(dense + "/APD/" + format_index(p.ref_image_id));
    Driver drv;
    // CheckImages (main.cpp:104-127) + ComputeRoundNum (main.cpp:129-146). The reference decodes every
    // reference image here and again per problem; the decodes go to the run's ImageCache instead
    // (host threads in parallel), so the schedule below never decodes a reference image again.
    int W0 = 0, H0 = 0;
    if (problems.empty()) {
        std::cout << "Images may error, check it!\n";
        return EXIT_FAILURE;
    }
    {
        std::vector<std::shared_ptr<ImageCache::Decoded>> dec(problems.size());
        parallel_for(problems.size(), host_threads(), [&](size_t i) {
            dec[i] = drv.images.decode(dense + "/images/" + format_index(problems[i].ref_image_id) + problems[i].img_ext);
        });
        for (size_t i = 0; i < problems.size(); ++i) {
            if (!dec[i]->ok || (i > 0 && (dec[i]->g.width != W0 || dec[i]->g.height != H0))) {
                std::cout << "Images may error, check it!\n";
                return EXIT_FAILURE;
            }
            W0 = dec[i]->g.width;
            H0 = dec[i]->g.height;
        }
    }
    std::cout << "There are " << problems.size() << " problems needed to be processed!" << std::endl;
    auto fuse = [&]() -> bool {
        FusionOptions fo;
        fo.dense_folder = dense;
        fo.dataset = dataset;
        fo.weak_filter = weak_filter;
        fo.export_color = export_color;
        fo.device = gpus[0];
        FusionReport rep;
        std::string ferr;
        if (!run_fusion(problems, fo, store, rep, ferr)) {
            std::cout << "Error: " << ferr << std::endl;
            return false;
        }
        printf("Fusion: %lld points, load %.0f ms, upload %.0f ms, weak filter %.0f ms, fuse %.0f ms (device %.0f ms, "
               "terms %.0f ms, commit %.0f ms), write %.0f ms\n",
               (long long)rep.points, rep.load_ms, rep.upload_ms, rep.filter_ms, rep.fuse_ms, rep.gpu_ms, rep.term_ms,
               rep.commit_ms, rep.write_ms);
        return true;
    };
    if (only_fuse) {
        if (!fuse()) return EXIT_FAILURE;
        printf("Fusion done!\n");
        return EXIT_SUCCESS;
    }
    int max_size = std::max(W0, H0), round_num = 1;
    while (max_size > 800) {
        max_size /= 2;
        round_num++;
    }
    std::cout << "Round nums: " << round_num << std::endl;
    const float geom_factor = (dataset == "TaT_a" || dataset == "TaT_i") ? 0.05f : 0.2f;

    drv.dense = dense;
    drv.use_sa = use_sa;
    drv.flush = flush;
    drv.seed = std::strtoull(vm["seed"].c_str(), nullptr, 10);
    drv.jacobi = ordering == "jacobi";
    drv.store = &store;
    std::vector<apd_ctx *> &ctxs = drv.ctxs;
    for (int d : gpus) {
        apd_ctx *c = apd_create(d);
        if (!c) {
            std::cout << "apd_create(" << d << ") failed: " << apd_last_error(nullptr) << std::endl;
            return EXIT_FAILURE;
        }
        ctxs.push_back(c);
    }
    if (!(getenv("APD_DEVICE_STATE") && std::string(getenv("APD_DEVICE_STATE")) == "0")) {
        // one store per context. Default cap: the device's free memory less room for the library's
        // per-problem buffers (≈ 40 GB at C3 with the pair table and the DepthToWeak hand-over; a quarter
        // of the free memory, at least 16 GiB), shared by the contexts on that device; a problem that
        // still runs out releases its context's store (process())
        std::map<int, int> per_dev;
        for (int d : gpus) per_dev[d]++;
        auto share_of = [&](int dev_id) { return per_dev[dev_id]; };
        for (size_t k = 0; k < ctxs.size(); ++k) {
            auto d = std::make_unique<DevStore>();
            d->ctx = ctxs[k];
            size_t fb = 0, tb = 0;
            if (apd_device_mem_info(ctxs[k], &fb, &tb) == APD_OK) {
                const int share = per_dev[gpus[k]];
                const size_t room = std::max<size_t>((size_t)16 << 30, fb / 4) * share;
                d->cap = fb > room ? (fb - room) / share : 0;
            }
            d->share = share_of(gpus[k]);
            if (const char *e = getenv("APD_DEVICE_STATE_CAP_MB")) {
                d->cap = (size_t)std::max(0L, atol(e)) << 20;
                d->cap_fixed = true;
            }
            drv.devs.push_back(std::move(d));
        }
    }
    for (auto &p : problems) drv.pass_views.push_back(p.ref_image_id);
    std::vector<Job> jobs(problems.size());
    for (size_t i = 0; i < problems.size(); ++i) jobs[i].pb = problems[i];
    bool ok = true;
    // one pass over all views: dynamic work queue over the devices
    auto run_pass = [&]() {
        std::atomic<size_t> next{0};
        std::atomic<bool> good{true};
        auto worker = [&](apd_ctx *ctx) {
            for (size_t k; good && (k = next.fetch_add(1)) < jobs.size();)
                if (!drv.process(ctx, jobs[k])) good = false;
        };
        if (ctxs.size() == 1) {
            worker(ctxs[0]);
        } else {
            std::vector<std::thread> th;
            for (apd_ctx *c : ctxs) th.emplace_back(worker, c);
            for (auto &t : th) t.join();
        }
        drv.commit();
        return (bool)good;
    };
    auto base_params = [&]() {
        apd_params p{};
        p.max_iterations = 3;
        p.top_k = 4;
        p.use_impetus = use_impetus;
        p.strong_radius = 5;
        p.strong_increment = 2;
        p.weak_radius = 5;
        p.weak_increment = 5;
        p.use_sa = use_sa;
        p.weak_peak_radius = 6;
        p.rotate_time = 4;
        p.ransac_threshold = 0.005f;
        p.geom_factor = geom_factor;
        return p;
    };
    // round schedule (main.cpp:290-367)
    int iteration_index = 0;
    const int geom_iteration = 3;
    const auto start = std::chrono::steady_clock::now();
    for (int i = 0; i < round_num && ok; ++i) {
        drv.new_round();
        drv.prefetch_round((int)std::pow(2, round_num - 1 - i), problems);
        std::cout << "========================== Round " << i << " ==========================" << std::endl;
        std::cout << "======== iteration " << iteration_index << "========" << std::endl;
        for (auto &job : jobs) {
            apd_params p = base_params();
            if (i == 0) {
                p.state = APD_FIRST_INIT;
                p.use_APD = 0;
            } else {
                p.state = APD_REFINE_INIT;
                p.use_APD = 1;
                p.ransac_threshold = (float)(0.01 - i * 0.00125);
                p.rotate_time = std::min((int)std::pow(2, i), 4);
            }
            p.geom_consistency = 0;
            p.weak_peak_radius = 6;
            job.params = p;
            job.iteration = iteration_index;
            job.scale_size = (int)std::pow(2, round_num - 1 - i);
        }
        ok = run_pass();
        iteration_index++;
        for (int j = 0; j < geom_iteration && ok; ++j) {
            std::cout << "======== iteration " << iteration_index << "========" << std::endl;
            const bool is_last = (i == round_num - 1 && j == geom_iteration - 1);
            for (auto &job : jobs) {
                apd_params p = base_params();
                p.state = APD_REFINE_ITER;
                if (i == 0) {
                    p.use_APD = 0;
                } else {
                    p.use_APD = 1;
                    p.ransac_threshold = (float)(0.01 - i * 0.00125);
                    p.rotate_time = std::min((int)std::pow(2, i), 4);
                }
                p.geom_consistency = 1;
                p.weak_peak_radius = std::max(4 - 2 * j, 2);
                job.params = p;
                job.export_anchor = is_last && export_anchor;
                job.export_curve = is_last && export_curve;
                job.iteration = iteration_index;
                job.scale_size = (int)std::pow(2, round_num - 1 - i);
            }
            ok = run_pass();
            iteration_index++;
        }
        std::cout << "=============================================================" << std::endl;
    }
    {
        long up = 0;
        bool any = false;
        for (auto &d : drv.devs)
            if (d) { up += d->uploaded; any = true; }
        if (any) printf("Device-resident state: %.1f MB of image uploads\n", up / 1048576.0);
    }
    drv.devs.clear();  // their buffers belong to the contexts
    for (apd_ctx *c : ctxs) apd_destroy(c);
    if (!ok) return EXIT_FAILURE;
    const auto end = std::chrono::steady_clock::now();
    std::cout << "Cost time: " << std::chrono::duration_cast<std::chrono::milliseconds>(end - start).count() << " ms"
              << std::endl;
    long avg = 0;
    for (auto &j : jobs) avg += j.used_ms;
    avg /= (long)jobs.size();
    std::cout << "Average used time: " << avg << " ms" << std::endl;
    if (use_memory_cache && flush) {
        printf("Write memory cache to disk!\n");
        store.flush_all();
        printf("All done!\n");
    }
    store.drain();
    if (store.failed_writes()) {
        std::cout << "Error: " << store.failed_writes() << " result file(s) could not be written" << std::endl;
        return EXIT_FAILURE;
    }
    if (no_fuse) {
        printf("Skip fusion, all done!\n");
        return EXIT_SUCCESS;
    }
    std::cout << "Run fusion\n";
    if (!fuse()) return EXIT_FAILURE;
    std::cout << "All done\n";
    return EXIT_SUCCESS;
}
