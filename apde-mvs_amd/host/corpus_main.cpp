// corpus_main.cpp — runs the host parsers over a list of (possibly corrupt) files: the gray and
// colour image decoders (image.cpp), bin-mat reads (io.cpp), cam.txt and pair.txt parsing. Built
// with AddressSanitizer + UndefinedBehaviorSanitizer by `make sanitize` (tests/test_host_sanitize.py):
// every file must be either decoded or rejected with an error, never read out of bounds.
//   corpus_main <file>...          (a directory argument is parsed as a scan folder: pair.txt)
#include <cstdio>
#include <string>

#include "image.h"
#include "io.h"

using namespace apdhost;

int main(int argc, char **argv) {
    int ok = 0, rejected = 0;
    for (int i = 1; i < argc; ++i) {
        const std::string path = argv[i];
        std::string err;
        Gray8 g;
        Bgr8 c;
        Mat m;
        apd_camera cam;
        std::vector<Problem> problems;
        const bool a = read_gray8(path, g, err);
        const bool b = read_bgr8(path, c, err);
        const bool d = read_binmat_file(path, m);
        const bool e = read_camera(path, cam);
        const bool f = read_pair_file(path, problems, err);
        // touch every decoded byte so a short buffer shows up under ASan
        unsigned sum = 0;
        for (unsigned char v : g.px) sum += v;
        for (unsigned char v : c.px) sum += v;
        for (size_t k = 0; k < m.size_bytes(); ++k) sum += m.bytes()[k];
        if (a && g.px.size() != (size_t)g.width * g.height) { std::printf("BAD gray size %s\n", argv[i]); return 2; }
        if (b && c.px.size() != (size_t)c.width * c.height * 3) { std::printf("BAD bgr size %s\n", argv[i]); return 2; }
        (a || b || d || e || f) ? ++ok : ++rejected;
        if (sum == 0xFFFFFFFFu) std::printf(".");
    }
    std::printf("corpus: %d parsed, %d rejected\n", ok, rejected);
    return 0;
}
