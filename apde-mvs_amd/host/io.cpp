// io.cpp — bin-mat / cam.txt / pair.txt I/O of the `apd` driver (see io.h for the reference lines).
#include "io.h"

#include <map>
#include <mutex>

#include <sys/stat.h>

#include <cstdio>
#include <cstring>
#include <fstream>
#include <iomanip>
#include <iostream>
#include <sstream>

#include "image.h"

namespace apdhost {

int cv_elem_size(int type) {
    switch (type) {
        case CV_8UC1: return 1;
        case CV_32SC1: return 4;
        case CV_32FC1: return 4;
        case CV_32FC3: return 12;
        default: return 0;
    }
}

namespace {
struct BufferPool {
    std::mutex mu;
    std::multimap<size_t, uint8_t *> free_;
    size_t pooled = 0;
    static constexpr size_t kCap = (size_t)8 << 30;   // bytes kept for reuse
    static constexpr size_t kMin = (size_t)1 << 20;   // smaller buffers use plain new/delete
    uint8_t *take(size_t n) {
        std::lock_guard<std::mutex> g(mu);
        auto it = free_.find(n);
        if (it == free_.end()) return nullptr;
        uint8_t *p = it->second;
        free_.erase(it);
        pooled -= n;
        return p;
    }
    void give(uint8_t *p, size_t n) {
        {
            std::lock_guard<std::mutex> g(mu);
            if (pooled + n <= kCap) {
                free_.emplace(n, p);
                pooled += n;
                return;
            }
        }
        delete[] p;
    }
};
BufferPool &pool() {
    static BufferPool *p = new BufferPool();  // never destroyed: buffers may be released at exit
    return *p;
}
}  // namespace

std::shared_ptr<uint8_t[]> pool_buffer(size_t bytes) {
    if (bytes < BufferPool::kMin) return std::shared_ptr<uint8_t[]>(new uint8_t[bytes]);
    uint8_t *p = pool().take(bytes);
    if (!p) p = new uint8_t[bytes];
    return std::shared_ptr<uint8_t[]>(p, [bytes](uint8_t *q) { pool().give(q, bytes); });
}

Mat resize_nearest(const Mat &m, int w, int h) {
    Mat o(h, w, m.type);
    resize_nearest(m.bytes(), m.cols, m.rows, o.bytes(), w, h, cv_elem_size(m.type));
    return o;
}

bool read_binmat_file(const std::string &path, Mat &m) {
    std::ifstream in(path, std::ios::binary);
    if (!in) return false;
    int32_t hdr[4];
    in.read(reinterpret_cast<char *>(hdr), sizeof(hdr));
    if (!in || hdr[0] != 1) return false;
    const int es = cv_elem_size(hdr[3]);
    if (es == 0 || hdr[1] < 0 || hdr[2] < 0) return false;
    // the payload must be in the file before a buffer of its size is allocated (a corrupt header
    // could otherwise ask for terabytes)
    const std::streampos here = in.tellg();
    in.seekg(0, std::ios::end);
    const std::streamoff avail = in.tellg() - here;
    in.seekg(here);
    if (avail < 0 || (uint64_t)avail < (uint64_t)hdr[1] * (uint64_t)hdr[2] * (uint64_t)es) return false;
    Mat r(hdr[1], hdr[2], hdr[3]);
    in.read(reinterpret_cast<char *>(r.bytes()), (std::streamsize)r.size_bytes());
    if (!in) {  // truncated file: no Mat (a pooled buffer would expose another problem's bytes)
        m = Mat();
        return false;
    }
    m = r;
    return true;
}

bool write_binmat_file(const std::string &path, const Mat &m) {
    std::ofstream out(path, std::ios::binary);
    if (!out) return false;
    const int32_t hdr[4] = {1, m.rows, m.cols, m.type};
    out.write(reinterpret_cast<const char *>(hdr), sizeof(hdr));
    out.write(reinterpret_cast<const char *>(m.bytes()), (std::streamsize)m.size_bytes());
    return (bool)out;
}

bool MatStore::read(const std::string &path, Mat &m) {
    if (cache_) {
        std::lock_guard<std::mutex> g(mu_);
        auto it = mats_.find(path);
        if (it != mats_.end()) {
            m = it->second;
            return true;
        }
    }
    if (!read_binmat_file(path, m)) {
        std::cout << "Error opening file: \"" << path << "\"" << std::endl;
        return false;
    }
    if (cache_) {
        std::lock_guard<std::mutex> g(mu_);
        mats_.emplace(path, m);
    }
    return true;
}

bool MatStore::write(const std::string &path, const Mat &m, bool flush) {
    if (cache_) {
        std::lock_guard<std::mutex> g(mu_);
        mats_[path] = m;
    }
    if (cache_ && flush) {
        std::lock_guard<std::mutex> g(qmu_);
        if (!writer_.joinable()) writer_ = std::thread(&MatStore::writer_loop, this);
        queue_.emplace_back(path, m);
        ++inflight_;
        qcv_.notify_one();
        return true;
    }
    if (!cache_) {
        if (!write_binmat_file(path, m)) {
            std::cout << "Error opening file: \"" << path << "\"" << std::endl;
            ++failed_;
            return false;
        }
    }
    return true;
}

void MatStore::writer_loop() {
    std::unique_lock<std::mutex> l(qmu_);
    for (;;) {
        qcv_.wait(l, [&] { return stop_ || !queue_.empty(); });
        if (queue_.empty()) return;  // stop_ and drained
        auto job = std::move(queue_.front());
        queue_.pop_front();
        l.unlock();
        if (!write_binmat_file(job.first, job.second)) {
            std::cout << "Error opening file: \"" << job.first << "\"" << std::endl;
            ++failed_;
        }
        job.second = Mat();
        l.lock();
        if (--inflight_ == 0) qdone_.notify_all();
    }
}

void MatStore::drain() {
    std::unique_lock<std::mutex> l(qmu_);
    qdone_.wait(l, [&] { return inflight_ == 0; });
}

MatStore::~MatStore() {
    {
        std::lock_guard<std::mutex> g(qmu_);
        stop_ = true;
        qcv_.notify_all();
    }
    if (writer_.joinable()) writer_.join();
}

void MatStore::flush_all() {
    drain();
    std::lock_guard<std::mutex> g(mu_);
    for (auto &kv : mats_)
        if (!write_binmat_file(kv.first, kv.second)) {
            std::cout << "Error opening file: \"" << kv.first << "\"" << std::endl;
            ++failed_;
        }
    mats_.clear();
}

bool read_camera(const std::string &path, apd_camera &cam) {
    std::ifstream in(path);
    if (!in) return false;
    memset(&cam, 0, sizeof(cam));
    std::string tok;
    in >> tok;  // "extrinsic"
    for (int i = 0; i < 3; ++i) in >> cam.R[3 * i + 0] >> cam.R[3 * i + 1] >> cam.R[3 * i + 2] >> cam.t[i];
    float tmp[4];
    in >> tmp[0] >> tmp[1] >> tmp[2] >> tmp[3];
    in >> tok;  // "intrinsic"
    for (int i = 0; i < 3; ++i) in >> cam.K[3 * i + 0] >> cam.K[3 * i + 1] >> cam.K[3 * i + 2];
    for (int j = 0; j < 3; ++j)
        cam.c[j] = -(float)((double)cam.R[0 + j] * (double)cam.t[0] + (double)cam.R[3 + j] * (double)cam.t[1] +
                            (double)cam.R[6 + j] * (double)cam.t[2]);
    in >> cam.depth_min >> cam.interval;
    if (!(in >> cam.depth_num >> cam.depth_max)) {
        cam.depth_num = 192;
        cam.depth_max = cam.interval * cam.depth_num + cam.depth_min;
    }
    return true;
}

std::string format_index(int id) {
    std::ostringstream ss;
    ss << std::setw(8) << std::setfill('0') << id;
    return ss.str();
}

bool file_exists(const std::string &p) {
    struct stat st;
    return stat(p.c_str(), &st) == 0;
}

bool make_dir(const std::string &p) { return mkdir(p.c_str(), 0755) == 0 || file_exists(p); }

bool read_pair_file(const std::string &dense, std::vector<Problem> &problems, std::string &err) {
    std::ifstream file(dense + "/pair.txt");
    if (!file) { err = "cannot open " + dense + "/pair.txt"; return false; }
    static const char *exts[] = {".jpg", ".png", ".jpeg", ".JPG", ".PNG", ".JPEG"};
    std::string line;
    std::getline(file, line);
    int num_images = 0;
    std::istringstream(line) >> num_images;
    problems.clear();
    for (int i = 0; i < num_images; ++i) {
        Problem p;
        std::getline(file, line);
        std::istringstream(line) >> p.ref_image_id;
        std::getline(file, line);
        std::istringstream iss(line);
        int n = 0;
        iss >> n;
        for (int j = 0; j < n; ++j) {
            int id;
            float score;
            iss >> id >> score;
            if (score <= 0.0f) continue;
            p.src_image_ids.push_back(id);
        }
        for (const char *e : exts) {
            if (file_exists(dense + "/images/" + format_index(p.ref_image_id) + e)) {
                p.img_ext = e;
                break;
            }
        }
        if (p.img_ext.empty()) {
            err = "can not find image: " + format_index(p.ref_image_id);
            return false;
        }
        problems.push_back(p);
    }
    return true;
}

}  // namespace apdhost
