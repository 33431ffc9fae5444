// io.h — on-disk contract of the reference's depth binary, restated without OpenCV/Boost:
// bin-mat files (APD.cpp:18-83), MVSNet cam.txt (APD.cpp:85-135), pair.txt (main.cpp:44-102),
// and the MemoryCache write-back semantics (APD.cpp:3-16, main.cpp:381-393).
#pragma once

#include <cstdint>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>
#include <condition_variable>
#include <deque>
#include <thread>
#include <atomic>

#include "../../include/apd_hip.h"

namespace apdhost {

// OpenCV type codes used by the reference's bin-mat files
enum { CV_8UC1 = 0, CV_32SC1 = 4, CV_32FC1 = 5, CV_32FC3 = 21 };
int cv_elem_size(int type);

// Pixels are reference-counted like a cv::Mat's: copying a Mat (MemoryCache reads and writes,
// priors) shares the buffer instead of copying hundreds of MB per problem. Every writer fills a
// freshly constructed Mat, so sharing never exposes a partial write. Like cv::Mat::create, the
// buffer is not zero-filled (every writer fills all of it; a 3024x2016 problem's four result Mats
// would otherwise cost ~100 MB of memset).
// Large host buffers come from a process-wide pool: a released buffer is kept (up to a byte cap)
// and handed to the next request of the same size, so the per-problem result Mats and staging
// buffers of a scan reuse resident pages instead of faulting in (and zeroing) fresh ones.
std::shared_ptr<uint8_t[]> pool_buffer(size_t bytes);
struct Mat {
    int rows = 0, cols = 0, type = CV_8UC1;
    size_t nbytes = 0;
    std::shared_ptr<uint8_t[]> buf;  // row-major, rows * cols * elem bytes
    Mat() = default;
    Mat(int r, int c, int t)
        : rows(r), cols(c), type(t), nbytes((size_t)r * c * cv_elem_size(t)), buf(pool_buffer(nbytes)) {}
    uint8_t *bytes() { return buf.get(); }
    const uint8_t *bytes() const { return buf.get(); }
    size_t size_bytes() const { return buf ? nbytes : 0; }
    template <class T> T *ptr() { return reinterpret_cast<T *>(bytes()); }
    template <class T> const T *ptr() const { return reinterpret_cast<const T *>(bytes()); }
    bool empty() const { return rows == 0 || cols == 0; }
};
Mat resize_nearest(const Mat &m, int w, int h);

// MemoryCache (APD.cpp:3-16): when enabled, bin-mat writes land in memory and reach the disk only
// when flushed; reads check the cache first. Thread-safe.
// With the cache on, a flushed write (--flush / --no_fuse) only persists a Mat that every read is
// served from memory anyway, so the file is written by a background thread (in submission order;
// drained by flush_all and the destructor) instead of on the problem's critical path. Without the
// cache, reads come from the files and writes stay synchronous.
class MatStore {
public:
    explicit MatStore(bool cache) : cache_(cache) {}
    ~MatStore();
    bool read(const std::string &path, Mat &m);                    // ReadBinMat   APD.cpp:18-56
    bool write(const std::string &path, const Mat &m, bool flush);  // WriteBinMat  APD.cpp:58-83
    void flush_all();                                              // main.cpp:381-393
    void drain();                                                  // wait for queued file writes
    bool cached() const { return cache_; }
    // result files that could not be written so far (synchronous, queued and flushed writes alike);
    // the caller waits with drain() before reading it, and main() exits non-zero when it is not 0
    size_t failed_writes() const { return failed_.load(); }

private:
    void writer_loop();
    bool cache_;
    std::mutex mu_;
    std::map<std::string, Mat> mats_;
    std::mutex qmu_;
    std::condition_variable qcv_, qdone_;
    std::deque<std::pair<std::string, Mat>> queue_;
    size_t inflight_ = 0;
    bool stop_ = false;
    std::atomic<size_t> failed_{0};
    std::thread writer_;
};

bool read_binmat_file(const std::string &path, Mat &m);
bool write_binmat_file(const std::string &path, const Mat &m);

// ReadCamera (APD.cpp:85-135): extrinsic 4x4 (last row ignored), intrinsic 3x3, depth_min interval
// [depth_num depth_max] with the depth_num = 192 fallback; centre c = -R^T t in double.
bool read_camera(const std::string &path, apd_camera &cam);

struct Problem {  // main.h:102-115
    int ref_image_id = 0;
    std::vector<int> src_image_ids;
    std::string img_ext;
};
// GenerateSampleList (main.cpp:44-102): sources with score <= 0 are dropped; the image extension
// is the first of .jpg .png .jpeg .JPG .PNG .JPEG present for the reference image.
bool read_pair_file(const std::string &dense_folder, std::vector<Problem> &problems, std::string &err);

std::string format_index(int id);  // ToFormatIndex: %08d
bool file_exists(const std::string &p);
bool make_dir(const std::string &p);

}  // namespace apdhost
