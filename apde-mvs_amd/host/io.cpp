// io.cpp — bin-mat / cam.txt / pair.txt I/O of the `apd` driver (see io.h for the reference lines).
#include "io.h"

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
    m = Mat(hdr[1], hdr[2], hdr[3]);
    in.read(reinterpret_cast<char *>(m.bytes()), (std::streamsize)m.size_bytes());
    return (bool)in;
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
    if (flush || !cache_) {
        if (!write_binmat_file(path, m)) {
            std::cout << "Error opening file: \"" << path << "\"" << std::endl;
            return false;
        }
    }
    return true;
}

void MatStore::flush_all() {
    std::lock_guard<std::mutex> g(mu_);
    for (auto &kv : mats_) write_binmat_file(kv.first, kv.second);
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
