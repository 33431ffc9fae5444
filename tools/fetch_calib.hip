// Calibration of rocprofv3's FETCH_SIZE for the access widths and patterns of this repo's gather
// kernels (MI355X_MICROARCH.md §HBM: "other access widths are uncalibrated").
// A 1 GiB buffer (4x the 256 MiB Infinity Cache, so every line comes from HBM) is read by:
//   k_stream16      16 B per lane, coalesced, every byte once                  (the guide's reference case)
//   k_line_dword    one 4-byte load per 128-B line, every line once, lines in a permuted order (a gather)
//   k_line_dwordx2  one 8-byte load per line (the fp16 texel-pair tap of the NCC kernels)
//   k_line_2x64     two 4-byte loads per line, one in each 64-B half (sector or whole-line fills?)
//   k_line_half     one 4-byte load per line in the first 64-B half of only every line (same as
//                   k_line_dword, kept to pair with k_line_2x64 at equal line count)
// Each lane folds what it read into one dword stored per lane (vector stores; 4 B per lane written).
// FETCH_SIZE per launch / lines touched = bytes counted per line fill; with the time of each launch
// (rocprofv3 --kernel-trace --stats) that gives the factor to apply to the sweep's gather traffic.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/fetch_calib tools/fetch_calib.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CHECK(x)                                                                                  \
    do {                                                                                          \
        hipError_t e_ = (x);                                                                      \
        if (e_ != hipSuccess) {                                                                   \
            fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e_));                        \
            return 1;                                                                             \
        }                                                                                         \
    } while (0)

static constexpr size_t BYTES = (size_t)1 << 30;
static constexpr size_t LINES = BYTES / 128;        // 2^23 lines of 128 B
static constexpr uint32_t PERM = 2654435761u;       // odd: i -> i * PERM mod 2^23 is a bijection

__device__ __forceinline__ size_t line_of(size_t i) { return (size_t)((uint32_t)i * PERM) & (LINES - 1); }

__global__ void k_stream16(const uint4 *__restrict__ in, uint32_t *__restrict__ out, size_t n16) {
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x, stride = (size_t)gridDim.x * blockDim.x;
    uint32_t acc = 0;
    for (size_t i = t; i < n16; i += stride) {
        const uint4 v = in[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    out[t] = acc;
}
__global__ void k_line_dword(const uint32_t *__restrict__ in, uint32_t *__restrict__ out) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= LINES) return;
    out[i] = in[line_of(i) * 32];
}
__global__ void k_line_dwordx2(const uint2 *__restrict__ in, uint32_t *__restrict__ out) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= LINES) return;
    const uint2 v = in[line_of(i) * 16 + 3];  // 8 B inside the line (offset 24)
    out[i] = v.x ^ v.y;
}
__global__ void k_line_2x64(const uint32_t *__restrict__ in, uint32_t *__restrict__ out) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= LINES) return;
    const size_t l = line_of(i) * 32;
    out[i] = in[l + 1] ^ in[l + 17];  // offsets 4 and 68: one dword in each 64-B half
}
__global__ void k_line_half(const uint32_t *__restrict__ in, uint32_t *__restrict__ out) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= LINES) return;
    out[i] = in[line_of(i) * 32 + 1];
}
__global__ void k_fill(uint32_t *__restrict__ p, size_t n) {
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x, stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = t; i < n; i += stride) p[i] = (uint32_t)(i * 2654435761u);
}
// 512 MiB written between launches: the previous launch's lines leave the Infinity Cache
__global__ void k_evict(uint4 *__restrict__ p, size_t n16) {
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x, stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = t; i < n16; i += stride) p[i] = make_uint4((uint32_t)i, 1u, 2u, 3u);
}

int main() {
    uint32_t *buf = nullptr, *out = nullptr;
    uint4 *ev = nullptr;
    const size_t EV = (size_t)512 << 20;
    CHECK(hipMalloc(&buf, BYTES));
    CHECK(hipMalloc(&out, LINES * sizeof(uint32_t)));
    CHECK(hipMalloc(&ev, EV));
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, buf, BYTES / 4);
    CHECK(hipGetLastError());
    const dim3 g((unsigned)(LINES / 256)), b(256);
    const unsigned sg = 256 * 32;  // k_stream16: 8192 workgroups, grid-stride
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    for (int rep = 0; rep < 3; ++rep) {
        for (int k = 0; k < 5; ++k) {
            hipLaunchKernelGGL(k_evict, dim3(4096), dim3(256), 0, 0, ev, EV / 16);
            CHECK(hipEventRecord(e0, 0));
            switch (k) {
                case 0: hipLaunchKernelGGL(k_stream16, dim3(sg), b, 0, 0, (const uint4 *)buf, out, BYTES / 16); break;
                case 1: hipLaunchKernelGGL(k_line_dword, g, b, 0, 0, buf, out); break;
                case 2: hipLaunchKernelGGL(k_line_dwordx2, g, b, 0, 0, (const uint2 *)buf, out); break;
                case 3: hipLaunchKernelGGL(k_line_2x64, g, b, 0, 0, buf, out); break;
                case 4: hipLaunchKernelGGL(k_line_half, g, b, 0, 0, buf, out); break;
            }
            CHECK(hipEventRecord(e1, 0));
            CHECK(hipEventSynchronize(e1));
            CHECK(hipGetLastError());
            float ms = 0.0f;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            static const char *names[] = {"k_stream16", "k_line_dword", "k_line_dwordx2", "k_line_2x64", "k_line_half"};
            const double lines_touched = (double)LINES;
            printf("{\"kernel\": \"%s\", \"rep\": %d, \"ms\": %.4f, \"lines\": %.0f, \"bytes_in_lines\": %.0f}\n",
                   names[k], rep, ms, lines_touched, lines_touched * 128.0);
        }
    }
    CHECK(hipDeviceSynchronize());
    CHECK(hipFree(buf));
    CHECK(hipFree(out));
    CHECK(hipFree(ev));
    return 0;
}
