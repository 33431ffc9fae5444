// apd_kernels.hip — MI355X (gfx950) PatchMatch depth kernels and the C-ABI of libapd_hip.so.
//
// Work decomposition:
//   * "view-group" kernels (RandomInitialization, the Strong/Weak checkerboard sweeps, DepthToWeak,
//     LocalRefine): one 64-lane wavefront holds floor(64/N) pixels x N source views; lane = (pixel,
//     source view). Each lane evaluates the NCC of ITS view for every plane hypothesis of its pixel,
//     so the per-thread cost matrix of the reference (cost_array[8][32], APD.cu:1120, ~1 KB of
//     scratch) becomes 8 VGPRs, and the cross-view steps (view sampling CDF, weighted cost sums)
//     become in-order __shfl reductions over the N lanes of the pixel (bit-identical to the
//     reference's sequential sums).
//   * pixel kernels (anchors, RANSAC fit, filter, confidence, ...): one lane per pixel.
//   * checkerboard colours and the WEAK / non-WEAK split are compacted into pixel lists on device, so
//     no wavefront is spent on pixels another kernel owns.
// All launches go to the ctx stream; there is no host synchronisation inside the sweep loop.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <atomic>
#include <vector>

#include "../../include/apd_hip.h"
#include "apd_device.h"
#include <rocprim/device/device_scan.hpp>

using namespace apd;

#define WAVE 64
#define BLOCK 256
// profiling slots: APD_PROF_COUNTERS public counters (apd_hip.h) in slots 0..31, then the
// measurement slots of instrumented builds from APD_INSTR (-DAPD_PHASE_STAMPS: wave 0 of every
// workgroup adds the clock64() delta of each phase -- barrier to barrier -- to slot APD_INSTR + 8 +
// phase; LANE_STAT / APD_ANCHOR_STATS at APD_INSTR + their slot; read with apd_profile_counters(ctx, c, 64))
#define APD_PROF_SLOTS 64
#define APD_INSTR 32
// Each slot has APD_PROF_SPREAD copies (workgroup index modulo the spread picks one; the host sums
// them): a few million per-wave atomics on one address per launch serialise in L2 and cost the
// profiled C3 step ~10 ms.
#define APD_PROF_SPREAD 64
#define PROF_AT(ev, k) ((ev) + (k) + APD_PROF_SLOTS * (blockIdx.x & (APD_PROF_SPREAD - 1)))
#ifdef APD_PHASE_STAMPS
#define PHASE_STAMP(i)                                                                       \
    do {                                                                                     \
        if (a.evals && threadIdx.x == 0) {                                                   \
            const long long t_ = clock64();                                                  \
            atomicAdd(PROF_AT(a.evals, APD_INSTR + 8 + (i)), (unsigned long long)(t_ - t_phase_)); \
            t_phase_ = t_;                                                                   \
        }                                                                                    \
    } while (0)
#define PHASE_BEGIN long long t_phase_ = clock64()
// lane-use statistics (instrumented builds): slot += waves that issue the task, slot + 1 += active lanes
#define LANE_STAT(slot, pred)                                                                \
    do {                                                                                     \
        const unsigned long long b_ = __ballot(pred);                                        \
        if (a.evals && b_ && (threadIdx.x & 63) == 0) {                                      \
            atomicAdd(PROF_AT(a.evals, APD_INSTR + (slot)), 1ull);                            \
            atomicAdd(PROF_AT(a.evals, APD_INSTR + (slot) + 1), (unsigned long long)__builtin_popcountll(b_)); \
        }                                                                                    \
    } while (0)
#else
#define PHASE_STAMP(i) do { } while (0)
#define PHASE_BEGIN do { } while (0)
#define LANE_STAT(slot, pred) do { } while (0)
#endif
#ifndef APD_SWEEP_WAVES
#define APD_SWEEP_WAVES 2  // min waves per SIMD requested for the sweep kernels (VGPR budget 512/w)
#endif

// ---------------------------------------------------------------------------------------------
// view-group lane mapping
// ---------------------------------------------------------------------------------------------
struct Group {
    int v;        // source view index 0..N-1 of this lane (src image v+1)
    int base;     // first lane of this pixel's group
    int slot;     // pixel slot within the wave
    bool valid;   // lane owns a real pixel (writes allowed)
    int li;       // list index
    unsigned long long gmask;
};

// Dynamic LDS of the view-major kernels.
extern __shared__ float apd_dyn_lds[];
// position of the r-th (0-based) set bit of m (m has more than r set bits)
__device__ __forceinline__ int nth_set_bit(uint64_t m, int r) {
    int pos = 0;
    uint32_t x = (uint32_t)m;
    int c = __builtin_popcount(x);
    if (r >= c) { r -= c; pos = 32; x = (uint32_t)(m >> 32); }
#pragma unroll
    for (int w = 16; w >= 1; w >>= 1) {
        c = __builtin_popcount(x & ((1u << w) - 1u));
        if (r >= c) { r -= c; pos += w; x >>= w; }
    }
    return pos;
}
__device__ __forceinline__ uint32_t group_bits(bool pred, const Group &G) {
    unsigned long long m = __ballot(pred);
    return (uint32_t)((m >> G.base) & G.gmask);
}

// ---------------------------------------------------------------------------------------------
// setup kernels
// ---------------------------------------------------------------------------------------------
// Source images -> quad gather layout (one float4 = the 2x2 bilinear footprint, clamp-to-edge).
__global__ __launch_bounds__(BLOCK) void k_build_quads(const float *__restrict__ imgs, float4 *__restrict__ quad,
                                                     int W, int H, int N, size_t qstride) {
    const size_t per = (size_t)(W + 1) * (H + 1);
    const size_t total = per * N;
    for (size_t i = blockIdx.x * (size_t)BLOCK + threadIdx.x; i < total; i += (size_t)gridDim.x * BLOCK) {
        const int v = (int)(i / per);
        const size_t r = i - (size_t)v * per;
        const int iy = (int)(r / (W + 1)) - 1;
        const int ix = (int)(r % (W + 1)) - 1;
        const float *T = imgs + (size_t)(v + 1) * W * H;
        const int x0 = clampi(ix, 0, W - 1), x1 = clampi(ix + 1, 0, W - 1);
        const int y0 = clampi(iy, 0, H - 1), y1 = clampi(iy + 1, 0, H - 1);
        quad[(size_t)v * qstride + r] =
            make_float4(T[y0 * W + x0], T[y0 * W + x1], T[y1 * W + x0], T[y1 * W + x1]);
    }
}

// *flag = 0 unless every value is a quarter-integer in [0, 256) (the fp16 texel condition)
__global__ __launch_bounds__(BLOCK) void k_check_f16(const float *__restrict__ imgs, size_t n, int *flag) {
    bool ok = true;
    for (size_t i = blockIdx.x * (size_t)BLOCK + threadIdx.x; i < n; i += (size_t)gridDim.x * BLOCK) {
        const float q = imgs[i] * 4.0f;
        ok = ok && (q >= 0.0f && q < 1024.0f) && q == (float)(int)q;
    }
    if (!ok) *flag = 0;
}

// Per-problem statistics of the uploaded maps, on the device (the inputs may be device pointers, and
// at 6048x4032 three scalar host passes cost ~30 ms): out[0] += number of WEAK pixels, out[1] =
// max(out[1], the largest confidence), out[2] |= any non-zero SA label.
__global__ __launch_bounds__(BLOCK) void k_problem_stats(const uint8_t *__restrict__ weak, const uint8_t *__restrict__ conf,
                                                       const uint8_t *__restrict__ sa, size_t n, int *out) {
    int cnt = 0, mx = 0, any = 0;
    for (size_t i = blockIdx.x * (size_t)BLOCK + threadIdx.x; i < n; i += (size_t)gridDim.x * BLOCK) {
        cnt += weak[i] == APD_WEAK;
        mx = max(mx, (int)conf[i]);
        any |= sa[i] != 0;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        cnt += __shfl_xor(cnt, o);
        mx = max(mx, __shfl_xor(mx, o));
        any |= __shfl_xor(any, o);
    }
    if ((threadIdx.x & (WAVE - 1)) == 0) {
        if (cnt) atomicAdd(&out[0], cnt);
        atomicMax(&out[1], mx);
        if (any) atomicOr(&out[2], 1);
    }
}

// Source images -> fp16 vertical pairs P[(iy+1)*(W+2)+(ix+1)] = {half T(ix,iy), half T(ix,iy+1)},
// ix in [-1, W], iy in [-1, H-1], clamp-to-edge (see SrcTex in apd_device.h).
__global__ __launch_bounds__(BLOCK) void k_build_pairs(const float *__restrict__ imgs, uint32_t *__restrict__ pairs,
                                                     int W, int H, int N, size_t pstride) {
    const size_t per = (size_t)(W + 2) * (H + 1);
    const size_t total = per * N;
    for (size_t i = blockIdx.x * (size_t)BLOCK + threadIdx.x; i < total; i += (size_t)gridDim.x * BLOCK) {
        const int v = (int)(i / per);
        const size_t r = i - (size_t)v * per;
        const int iy = (int)(r / (W + 2)) - 1;
        const int ix = (int)(r % (W + 2)) - 1;
        const float *T = imgs + (size_t)(v + 1) * W * H;
        const int x0 = clampi(ix, 0, W - 1);
        const int y0 = clampi(iy, 0, H - 1), y1 = clampi(iy + 1, 0, H - 1);
        apd_h2 h;
        h.x = (_Float16)T[y0 * W + x0];
        h.y = (_Float16)T[y1 * W + x0];
        pairs[(size_t)v * pstride + r] = __builtin_bit_cast(uint32_t, h);
    }
}

// fp16 vertical pairs -> DepthToWeak's pre-differenced records D[k] = {P[k], (P[k + 1] - P[k]) / 256}
// (FastTexD in apd_device.h): padded columns 0..W read their right neighbour in the same row; the last
// padded column (never a tap's base) gets zero differences.
__global__ __launch_bounds__(BLOCK) void k_build_dpairs(const uint32_t *__restrict__ pairs, uint2 *__restrict__ dpairs,
                                                      int W, int H, int N, size_t pstride) {
    const size_t per = (size_t)(W + 2) * (H + 1);
    const size_t total = per * N;
    for (size_t i = blockIdx.x * (size_t)BLOCK + threadIdx.x; i < total; i += (size_t)gridDim.x * BLOCK) {
        const int v = (int)(i / per);
        const size_t r = i - (size_t)v * per;
        const int c = (int)(r % (W + 2));
        const size_t k = (size_t)v * pstride + r;
        const uint32_t cur = pairs[k], nxt = c < W + 1 ? pairs[k + 1] : cur;
        const apd_h2 a0 = __builtin_bit_cast(apd_h2, cur), a1 = __builtin_bit_cast(apd_h2, nxt);
        apd_h2 d;  // exact: quarter-integer texels in [0, 256) (apd_set_problem's fp16 eligibility)
        d.x = (_Float16)(((float)a1.x - (float)a0.x) * 0.00390625f);
        d.y = (_Float16)(((float)a1.y - (float)a0.y) * 0.00390625f);
        dpairs[k] = make_uint2(cur, __builtin_bit_cast(uint32_t, d));
    }
}

// Ordered compaction, one workgroup per image row.
//   mode 0: colour `colour`, weak != WEAK, y < row_limit   (Strong sweep / filter pixel set)
//   mode 1: colour `colour`, weak == WEAK, y < row_limit   (Weak sweep pixel set)
//   mode 2: every pixel with weak == WEAK -> anchors_map (the WEAK index; see apd_stage_prepare)
//   mode 3: every pixel with a WEAK index (the anchors export in the reference's row-major order)
__device__ __forceinline__ bool list_pred(const Args &a, int mode, int colour, int x, int y) {
    if (mode == 3) return a.amap[y * a.W + x] >= 0;
    const uint8_t w = a.weak[y * a.W + x];
    if (mode == 2) return w == APD_WEAK;
    if (y >= a.row_limit || (colour < 2 && ((x + y) & 1) != colour)) return false;  // colour 2: both
    return mode == 0 ? (w != APD_WEAK) : (w == APD_WEAK);
}
__global__ __launch_bounds__(BLOCK) void k_list_count(Args a, int mode, int colour, int *__restrict__ row_counts) {
    const int y = blockIdx.x;
    __shared__ int wsum[BLOCK / WAVE];
    int cnt = 0;
    for (int x = threadIdx.x; x < a.W; x += BLOCK) cnt += list_pred(a, mode, colour, x, y) ? 1 : 0;
    for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o);
    if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = cnt;
    __syncthreads();
    if (threadIdx.x == 0) row_counts[y] = wsum[0] + wsum[1] + wsum[2] + wsum[3];
}
__global__ __launch_bounds__(1024) void k_list_scan(const int *__restrict__ row_counts, int H, int *__restrict__ row_off,
                                                  int *__restrict__ total) {
    __shared__ int part[1024];
    const int per = (H + 1023) / 1024;
    const int r0 = threadIdx.x * per;
    int s = 0;
    for (int r = r0; r < min(r0 + per, H); ++r) s += row_counts[r];
    part[threadIdx.x] = s;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {
        int t = threadIdx.x >= o ? part[threadIdx.x - o] : 0;
        __syncthreads();
        part[threadIdx.x] += t;
        __syncthreads();
    }
    int off = part[threadIdx.x] - s;
    for (int r = r0; r < min(r0 + per, H); ++r) { row_off[r] = off; off += row_counts[r]; }
    if (threadIdx.x == 1023) *total = part[1023];
}
__global__ __launch_bounds__(BLOCK) void k_list_fill(Args a, int mode, int colour, const int *__restrict__ row_off,
                                                   int *__restrict__ out) {
    const int y = blockIdx.x;
    __shared__ int wcnt[BLOCK / WAVE];
    int off = row_off[y];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (int x0 = 0; x0 < a.W; x0 += BLOCK) {
        const int x = x0 + threadIdx.x;
        const bool p = x < a.W && list_pred(a, mode, colour, x, y);
        const unsigned long long m = __ballot(p);
        const int pre = __popcll(m & ((1ull << lane) - 1ull));
        if (lane == 0) wcnt[wv] = __popcll(m);
        __syncthreads();
        int wo = 0;
        for (int k = 0; k < wv; ++k) wo += wcnt[k];
        const int tot = wcnt[0] + wcnt[1] + wcnt[2] + wcnt[3];
        if (mode == 2) {
            if (x < a.W) out[y * a.W + x] = p ? off + wo + pre : -1;
        } else if (p) {
            out[off + wo + pre] = y * a.W + x;
        }
        off += tot;
        __syncthreads();
    }
}

// Tile-ordered compaction for the sweep pixel sets (modes 0/1). The order of a sweep list does not
// change any result (pixels of one colour are independent), only locality: pixels are listed by
// 16x16 tiles, and inside a tile by 4x4 micro-tiles (8 same-colour pixels = one wavefront at N=8),
// so a wavefront's and a workgroup's NCC windows overlap in the source images.
// List tiles: tw x th = 256 positions, visited in 4x4 micro-tiles (row-major inside the tile); a
// sweep workgroup's 64 list entries are then a tw x th/2 region of one colour.
#define TILE_POS 256
// Tiles are visited in super-tiles of about TILE_SUPER_PX x TILE_SUPER_PX pixels (tiles row-major
// inside, super-tiles row-major, partial ones at the right and bottom edges): the workgroups one XCD
// runs at a time then cover a compact region instead of a strip of one tile row across the image, so
// their windows in each source view stay within its L2 (XCD-aware dispatch gives each XCD a
// contiguous run of the list). TILE_SUPER_PX 0: tiles row-major.
#ifndef TILE_SUPER_PX
#define TILE_SUPER_PX 128
#endif
__device__ __forceinline__ void tile_coords(int t, int tiles_x, int tiles_y, int tw, int &tx, int &ty) {
    const int SX = TILE_SUPER_PX ? max(1, TILE_SUPER_PX / tw) : tiles_x;
    const int SY = TILE_SUPER_PX ? max(1, TILE_SUPER_PX / (TILE_POS / tw)) : 1;
    const int sy = t / (SY * tiles_x);                   // band of SY tile rows
    const int rows = min(SY, tiles_y - SY * sy);         // tile rows in this band
    const int r = t - sy * SY * tiles_x;
    const int sx = r / (rows * SX);                      // super-tile within the band
    const int cols = min(SX, tiles_x - SX * sx);
    const int r2 = r - sx * rows * SX;
    tx = SX * sx + r2 % cols;
    ty = SY * sy + r2 / cols;
}
__device__ __forceinline__ void tile_pixel(int tile, int tiles_x, int tiles_y, int tw, int k, int &x, int &y) {
    const int micro = k >> 4, inner = k & 15, mx = tw >> 2;
    const int lx = ((micro % mx) << 2) + (inner & 3);
    const int ly = ((micro / mx) << 2) + (inner >> 2);
    int tx, ty;
    tile_coords(tile, tiles_x, tiles_y, tw, tx, ty);
    x = tx * tw + lx;
    y = ty * (TILE_POS / tw) + ly;
}
__global__ __launch_bounds__(BLOCK) void k_tile_count(Args a, int mode, int colour, int tiles_x, int tw,
                                                    int *__restrict__ counts) {
    int x, y;
    tile_pixel(blockIdx.x, tiles_x, (int)gridDim.x / tiles_x, tw, threadIdx.x, x, y);
    const bool p = x < a.W && y < a.H && list_pred(a, mode, colour, x, y);
    __shared__ int wsum[BLOCK / WAVE];
    const int c = __popcll(__ballot(p));
    if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) counts[blockIdx.x] = wsum[0] + wsum[1] + wsum[2] + wsum[3];
}
__global__ __launch_bounds__(BLOCK) void k_tile_fill(Args a, int mode, int colour, int tiles_x, int tw,
                                                   const int *__restrict__ offs, int *__restrict__ out) {
    int x, y;
    tile_pixel(blockIdx.x, tiles_x, (int)gridDim.x / tiles_x, tw, threadIdx.x, x, y);
    const bool p = x < a.W && y < a.H && list_pred(a, mode, colour, x, y);
    __shared__ int wcnt[BLOCK / WAVE];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const unsigned long long m = __ballot(p);
    if (lane == 0) wcnt[wv] = __popcll(m);
    __syncthreads();
    int wo = 0;
    for (int k = 0; k < wv; ++k) wo += wcnt[k];
    const int pos = offs[blockIdx.x] + wo + __popcll(m & ((1ull << lane) - 1ull));
    if (mode == 2) {  // a map: position in tile order, -1 elsewhere
        if (x < a.W && y < a.H) out[y * a.W + x] = p ? pos : -1;
    } else if (p) {
        out[pos] = y * a.W + x;
    }
}
// The anchors export (APD.cu:2614-2626 writes them by anchors_map, the row-major WEAK index): row y's
// WEAK pixels in row order, from the row offsets of mode 3, copied from their tile-order slots.
__global__ __launch_bounds__(BLOCK) void k_anchor_export(Args a, const int *__restrict__ row_off, short2 *__restrict__ dst) {
    const int y = blockIdx.x;
    __shared__ int wcnt[BLOCK / WAVE];
    int off = row_off[y];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (int x0 = 0; x0 < a.W; x0 += BLOCK) {
        const int x = x0 + threadIdx.x;
        const int wi = x < a.W ? a.amap[y * a.W + x] : -1;
        const unsigned long long m = __ballot(wi >= 0);
        if (lane == 0) wcnt[wv] = __popcll(m);
        __syncthreads();
        int wo = 0;
        for (int k = 0; k < wv; ++k) wo += wcnt[k];
        const int tot = wcnt[0] + wcnt[1] + wcnt[2] + wcnt[3];
        if (wi >= 0) {
            const int r = off + wo + __popcll(m & ((1ull << lane) - 1ull));
#pragma unroll
            for (int k = 0; k < 9; ++k) dst[(size_t)r * 9 + k] = a.anchors[(size_t)wi * 9 + k];
        }
        off += tot;
        __syncthreads();
    }
}

// XCD-aware workgroup order (cdna_hip_programming.md §5.5 T1): workgroups are dealt round-robin to
// the 8 XCDs, so give the workgroups of one XCD (b, b+8, ...) one contiguous chunk of the pixel list;
// each XCD's L2 then serves one compact region of the source images. Bijective for any grid size.
__device__ __forceinline__ int xcd_remap(int b, int nwg) {
    const int q = nwg >> 3, r = nwg & 7, x = b & 7;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (b >> 3);
}

// ---------------------------------------------------------------------------------------------
// APD anchor kernels (pixel kernels)
// ---------------------------------------------------------------------------------------------
// FindNearestStrongPoint (APD.cu:2434-2484). Same result as the reference's 201x201 scan (min
// distance, then max confidence, then first in x-major scan order) but visits the window in rings
// of increasing distance (offsets pre-sorted by (d^2, x, y)) and stops after the first ring that
// holds a candidate.
__global__ __launch_bounds__(BLOCK) void k_find_nearest(Args a, int n_off) {
    const int c = blockIdx.x * BLOCK + threadIdx.x;
    if (c >= a.HW) return;
    const int py = c / a.W, px = c - py * a.W;
    const uint8_t w = a.weak[c];
    short2 out = make_short2(-1, -1);
    if (w == APD_WEAK || w == APD_UNKNOWN) {
        const uint8_t cc = a.conf[c];
        int best_d2 = -1, bc = -1;
        for (int k = 0; k < n_off; ++k) {
            const short2 o = a.near_offsets[k];
            const int d2 = o.x * o.x + o.y * o.y;
            if (best_d2 >= 0 && d2 > best_d2) break;
            const int tx = px + o.x, ty = py + o.y;
            if (tx < 0 || tx >= a.W || ty < 0 || ty >= a.H) continue;
            const int t = tx + ty * a.W;
            if (a.weak[t] != APD_STRONG) continue;
            const int tc = a.conf[t];
            if (tc < cc) continue;
            if (best_d2 < 0 || tc > bc) { best_d2 = d2; bc = tc; out = make_short2((short)tx, (short)ty); }
        }
    } else if (w == APD_STRONG) {
        out = make_short2((short)px, (short)py);
    }
    a.nearest[c] = out;
}

// The same result in O(r) instead of O(r^2) reads per pixel. Level L = the querying pixel's own
// confidence; the sites of level L are the STRONG pixels with confidence >= L.
//   k_near_columns: per (level, column), the vertical distance to the nearest site of that level in
//                   the column, capped at 101 (= none within the window's +-100 rows).
//   k_find_nearest_rows: D = min over |dx| <= 100 of dx^2 + g_L(x + dx, y)^2 is the smallest d^2 of a
//                   site inside the 201x201 window, i.e. the ring at which the ring search first hits;
//                   then that ring's offsets are visited in the table order with the ring search's
//                   rule (max confidence, first in order). Bit-identical to k_find_nearest.
__global__ __launch_bounds__(BLOCK) void k_near_columns(Args a, int levels, uint8_t *__restrict__ g) {
    const int t = blockIdx.x * BLOCK + threadIdx.x;
    if (t >= levels * a.W) return;
    const int L = t / a.W, x = t - L * a.W, W = a.W, H = a.H;
    uint8_t *gl = g + (size_t)L * a.HW;
    int last = -1000;
    for (int y = 0; y < H; ++y) {
        const int c = y * W + x;
        if (a.weak[c] == APD_STRONG && a.conf[c] >= L) last = y;
        gl[c] = (uint8_t)min(y - last, 101);
    }
    last = 1 << 20;
    for (int y = H - 1; y >= 0; --y) {
        const int c = y * W + x;
        if (a.weak[c] == APD_STRONG && a.conf[c] >= L) last = y;
        const int up = min(last - y, 101);
        if (up < gl[c]) gl[c] = (uint8_t)up;
    }
}
__global__ __launch_bounds__(BLOCK) void k_find_nearest_rows(Args a, const uint8_t *__restrict__ g,
                                                             const int *__restrict__ ring_start) {
    const int c = blockIdx.x * BLOCK + threadIdx.x;
    if (c >= a.HW) return;
    const int W = a.W, H = a.H;
    const int py = c / W, px = c - py * W;
    const uint8_t w = a.weak[c];
    short2 out = make_short2(-1, -1);
    if (w == APD_WEAK || w == APD_UNKNOWN) {
        const uint8_t cc = a.conf[c];
        const uint8_t *row = g + (size_t)cc * a.HW + (size_t)py * W;
        int best = 1 << 30;
        for (int dx = 0; dx <= 100 && dx * dx < best; ++dx) {
            if (px + dx < W) {
                const int gv = row[px + dx];
                if (gv <= 100) best = min(best, dx * dx + gv * gv);
            }
            if (dx > 0 && px - dx >= 0) {
                const int gv = row[px - dx];
                if (gv <= 100) best = min(best, dx * dx + gv * gv);
            }
        }
        if (best <= 20000) {
            int bc = -1;
            for (int k = ring_start[best], k1 = ring_start[best + 1]; k < k1; ++k) {
                const short2 o = a.near_offsets[k];
                const int tx = px + o.x, ty = py + o.y;
                if (tx < 0 || tx >= W || ty < 0 || ty >= H) continue;
                const int t = tx + ty * W;
                if (a.weak[t] != APD_STRONG) continue;
                const int tc = a.conf[t];
                if (tc < cc) continue;
                if (tc > bc) { bc = tc; out = make_short2((short)tx, (short)ty); }
            }
        }
    } else if (w == APD_STRONG) {
        out = make_short2((short)px, (short)py);
    }
    a.nearest[c] = out;
}

// PointinTriangle (APD.cu:122-143)
__device__ __forceinline__ bool point_in_triangle(int ax, int ay, int bx, int by, int cx, int cy, int px, int py) {
    float ABx = (float)(bx - ax), ABy = (float)(by - ay);
    float BCx = (float)(cx - bx), BCy = (float)(cy - by);
    float CAx = (float)(ax - cx), CAy = (float)(ay - cy);
    float AB = sqrtf(ABx * ABx + ABy * ABy), BC = sqrtf(BCx * BCx + BCy * BCy), CA = sqrtf(CAx * CAx + CAy * CAy);
    if (AB <= 2 || BC <= 2 || CA <= 2) return false;
    if (!(AB + BC > CA && BC + CA > AB && AB + CA > BC)) return false;
    float PAx = (float)(ax - px), PAy = (float)(ay - py);
    float PBx = (float)(bx - px), PBy = (float)(by - py);
    float PCx = (float)(cx - px), PCy = (float)(cy - py);
    float t1 = PAx * PBy - PAy * PBx;
    float t2 = PBx * PCy - PBy * PCx;
    float t3 = PCx * PAy - PCy * PAx;
    return t1 * t2 >= 0 && t1 * t3 >= 0;
}

// GenAnchors (APD.cu:1857-2082): directional search for strong anchors + RANSAC plane.
__device__ __forceinline__ bool anc_inlier(const Args &a, float d, float depth_diff) {
    return a.anc_dlim_ok ? d < a.anc_dlim : d / depth_diff < a.ransac_thr;
}
// GenAnchors' direction test (APD.cu:1936-1939): normalize2(tdx, tdy), then tdx * dx + tdy * dy > thr.
// Filtered: the same sum with 1 / sqrt from v_rsq_f32 (1 ulp) differs from the IEEE statement's by
// < 2e-6 for unit (dx, dy) (each product <= 1 in magnitude, a few roundings of 2^-24 relative each), so
// outside a 1e-4 band around thr (50x that bound) it has the same verdict; inside the band (or for a
// NaN) the IEEE statement decides. Saves the IEEE sqrt and division on the search's dependent chain.
#ifndef GA_ANGLE_FILTER
#define GA_ANGLE_FILTER 1
#endif
__device__ __forceinline__ bool ga_angle_ok(float tdx, float tdy, float dx, float dy, float thr) {
    if (GA_ANGLE_FILTER) {
        const float r = __builtin_amdgcn_rsqf(tdx * tdx + tdy * tdy);
        const float va = (tdx * r) * dx + (tdy * r) * dy;
        if (fabsf(va - thr) > 1e-4f) return va > thr;
    }
    normalize2(tdx, tdy);
    return tdx * dx + tdy * dy > thr;
}
// x % d for d in 1..32 without an integer division: with M = floor((2^64 - 1) / d) + 1, the low 64 bits
// of M * x are frac(x / d) * 2^64 (to within d * 2^-32 < 1/d), whose high part times d is x mod d
// (Lemire, Kaser, Kurz 2019 for 32-bit x and d)
struct FastMod {
    uint64_t M;
    uint32_t d;
    __device__ __forceinline__ explicit FastMod(uint32_t dd) : M(~0ull / dd + 1ull), d(dd) {}
    __device__ __forceinline__ uint32_t mod(uint32_t x) const {
        const uint64_t low = M * (uint64_t)x;
        return (uint32_t)__umul64hi(low, (uint64_t)d);
    }
};
// stage (SPLIT, one GA_STAGE_W-word row per WEAK index wi, so that k_gen_anchors_fit's wave reads its
// pixel's row in one round trip): [0] the stream position << 6 | the number of points (0: no RANSAC),
// [1] the pixel, [2 + i] point i (short2, dvalid order): k_gen_anchors_fit runs the RANSAC. (The
// points' depths gathered here instead -- one dependent load per found point in this latency-bound
// search -- made it 24 -> 30 ms at C3; the fit kernel's wave gathers them in one round trip.)
#define GA_STAGE_W 34
#ifndef GA_PHILOX_LDS
#define GA_PHILOX_LDS 1  // k_gen_anchors_fit: one Philox block per lane, shared through LDS
#endif
#ifndef GA_SEARCH_AHEAD
#define GA_SEARCH_AHEAD 0  // the shift-1 search issues the next radius's lookup before judging this one
                           // (measured slower at C3: anchors 57.1 -> 61.7 ms, profiles/r6_ab_gen_anchors.txt)
#endif
template <bool SPLIT>
__global__ __launch_bounds__(BLOCK) void k_gen_anchors(Args a, uint32_t *__restrict__ stage, int wc) {
    const int c = blockIdx.x * BLOCK + threadIdx.x;
    if (c >= a.HW) return;
    if (a.weak[c] != APD_WEAK) return;
    const int W = a.W, H = a.H;
    const int py = c / W, px = c - py * W;
    const int margin = 6;
    const float depth_diff = a.dmax - a.dmin;
    const APD_C Cam &cam = a.cams[0];
    APD_G short2 *anc = a.anchors + (size_t)a.amap[c] * 9;
    Rng g(a.seed_lo, a.seed_hi, (uint32_t)c, ORD_ANCHORS);
    if constexpr (!SPLIT) {  // (SPLIT: k_gen_anchors_fit writes the whole row, coalesced)
        for (int i = 0; i < 9; ++i) anc[i] = make_short2(-1, -1);
        anc[0] = make_short2((short)px, (short)py);
    }
    // the search finds its points in direction-slot order (di = odi * 4 + ri increases through the
    // loops), which is also the stage's dvalid order: SPLIT writes each point to its stage slot as it is
    // found instead of into a dynamically indexed private array (which lived in scratch memory)
    const size_t wi = (size_t)a.amap[c];
    uint32_t *row = SPLIT ? stage + wi * GA_STAGE_W : nullptr;
    short2 sp[SPLIT ? 1 : 32];
    uint32_t dvalid = 0;
    if constexpr (!SPLIT)
        for (int i = 0; i < 32; ++i) sp[i] = make_short2(-1, -1);
    int odi = -1, nsp = 0;
    auto found = [&](int di, short2 p) {
        if constexpr (SPLIT) row[2 + nsp] = (uint32_t)(uint16_t)p.x | ((uint32_t)(uint16_t)p.y << 16);
        else sp[di] = p;
        dvalid |= 1u << di;
        nsp++;
    };
    const int rt = a.rotate_time;
    const FastMod fshift((uint32_t)a.anc_shift);
    for (int odx = -1; odx <= 1; ++odx) {
        for (int ody = -1; ody <= 1; ++ody) {
            if (odx == 0 && ody == 0) continue;
            float dx = (float)odx, dy = (float)ody;
            normalize2(dx, dy);
            odi++;
            for (int ri = 0; ri < rt; ++ri) {
                const int di = odi * 4 + ri;
                if (a.anc_shift == 1) {
                    // rotate_time >= 3 (main.cpp's rounds 2 and 3): shift = max((int)(tan(angle / 2) * 20), 1)
                    // is 1, so every draw's offset is x % 1 = 0 and the 4 attempts of a radius sample the
                    // same point -- the same lookup and verdict. The draws only advance the stream: by 4
                    // (attempt 1 succeeds) or 16 (all fail), exactly as the general search below.
                    float ddx = dx * 20 + (float)0, ddy = dy * 20 + (float)0;
                    normalize2(ddx, ddy);
                    // (measured: lookups of four radii issued together, judged in order, made this
                    // kernel slower at C3, 24.4 -> 32.1 ms: more registers, fewer waves in flight.)
                    // One radius ahead: the next radius's lookup is issued before this one is judged,
                    // so the gather's latency overlaps the verdict's arithmetic. A radius is live when
                    // it is <= APD_MAX_SEARCH_RADIUS and its ray point is inside the image (else the
                    // search ends there, drawing nothing); its lookup only when the probe is inside
                    // the margin -- the same statements as one radius at a time.
                    auto probe = [&](int radius, bool &live, short2 &nn) {
                        const float tx = (float)px + dx * (float)radius, ty = (float)py + dy * (float)radius;
                        live = radius <= APD_MAX_SEARCH_RADIUS && !(tx < 0 || ty < 0 || tx >= (float)W || ty >= (float)H);
                        const int ax = (int16_t)(int)((float)px + ddx * (float)radius);
                        const int ay = (int16_t)(int)((float)py + ddy * (float)radius);
                        const bool in = live && !(ax < margin || ay < margin || ax >= W - margin || ay >= H - margin);
                        nn = in ? a.nearest[ax + ay * W] : make_short2(-1, -1);
                    };
#if GA_SEARCH_AHEAD
                    int radius = 2;
                    bool live;
                    short2 nn;
                    probe(radius, live, nn);
                    while (live) {
                        const int rn = min(radius * 2, radius + 25);
                        bool live_n;
                        short2 nn_n;
                        probe(rn, live_n, nn_n);
                        bool ok = !(nn.x == -1 || nn.y == -1);
                        if (ok) ok = ga_angle_ok((float)(nn.x - px), (float)(nn.y - py), dx, dy, a.anc_thr);
                        g.n += ok ? 4u : 16u;
                        if (ok) { found(di, nn); break; }
                        radius = rn; live = live_n; nn = nn_n;
                    }
#else
                    for (int radius = 2; radius <= APD_MAX_SEARCH_RADIUS; radius = min(radius * 2, radius + 25)) {
                        bool live;
                        short2 nn;
                        probe(radius, live, nn);
                        if (!live) break;
                        bool ok = !(nn.x == -1 || nn.y == -1);
                        if (ok) ok = ga_angle_ok((float)(nn.x - px), (float)(nn.y - py), dx, dy, a.anc_thr);
                        g.n += ok ? 4u : 16u;
                        if (ok) { found(di, nn); break; }
                    }
#endif
                } else
                for (int radius = 2; radius <= APD_MAX_SEARCH_RADIUS; radius = min(radius * 2, radius + 25)) {
                    float tx = (float)px + dx * (float)radius, ty = (float)py + dy * (float)radius;
                    if (tx < 0 || ty < 0 || tx >= (float)W || ty >= (float)H) break;
                    // The 4 attempts of this radius: attempt t draws 4 values, i.e. exactly Philox block
                    // n/4 + t (n stays a multiple of 4 throughout the search), so all four are generated
                    // and their nearest-STRONG lookups issued together, then judged in order; the stream
                    // resumes after the first successful attempt, as if the later ones never drew.
                    const uint32_t n0 = g.n;
                    short2 nn[4];
                    bool in[4];
#pragma unroll
                    for (int t = 0; t < 4; ++t) {
                        const uint4 b = g.block((n0 >> 2) + (uint32_t)t);
                        int rxs = (int)fshift.mod((b.x % 2u == 0) ? b.y : (0u - b.y));
                        int rys = (int)fshift.mod((b.z % 2u == 0) ? b.w : (0u - b.w));
                        float ddx = dx * 20 + (float)rxs, ddy = dy * 20 + (float)rys;
                        normalize2(ddx, ddy);
                        int ax = (int16_t)(int)((float)px + ddx * (float)radius);
                        int ay = (int16_t)(int)((float)py + ddy * (float)radius);
                        in[t] = !(ax < margin || ay < margin || ax >= W - margin || ay >= H - margin);
                        nn[t] = in[t] ? a.nearest[ax + ay * W] : make_short2(-1, -1);
                    }
                    int used = 4;
#pragma unroll
                    for (int t = 0; t < 4; ++t) {
                        if (used < 4 || !in[t] || nn[t].x == -1 || nn[t].y == -1) continue;
                        if (ga_angle_ok((float)(nn[t].x - px), (float)(nn[t].y - py), dx, dy, a.anc_thr)) { found(di, nn[t]); used = t + 1; }
                    }
#ifdef APD_ANCHOR_STATS  // measurement build: steps, the attempt that succeeded, wave-level steps
                    if (a.evals) {
                        atomicAdd(PROF_AT(a.evals, APD_INSTR + 20 + (used == 4 && !((dvalid >> di) & 1u) ? 4 : used - 1)), 1ull);
                        if ((threadIdx.x & 63) == __builtin_ctzll(__ballot(true))) atomicAdd(PROF_AT(a.evals, APD_INSTR + 25), 1ull);
                    }
#endif
                    g.n = n0 + 4u * (uint32_t)used;
                    if ((dvalid >> di) & 1u) break;
                }
                float rx = dx * a.anc_cos - dy * a.anc_sin;
                float ry = dx * a.anc_sin + dy * a.anc_cos;
                normalize2(rx, ry);
                dx = rx; dy = ry;
            }
        }
    }
    if (nsp <= 3) {
        a.reliable[c] = 0;
        if constexpr (SPLIT) { row[0] = 0u; row[1] = (uint32_t)c; }
        return;
    }
    if constexpr (SPLIT) {
        row[0] = (g.n << 6) | (uint32_t)nsp;
        row[1] = (uint32_t)c;
        return;
    } else {
        short2 vp[32];
        float v3[32][3];
        int vc = 0;
        float X[3];
        get3d(cam, (float)px, (float)py, a.plane[c].w, X);
        const float cw0 = X[0], cw1 = X[1], cw2 = X[2];
        for (int i = 0; i < 32; ++i) {
            vp[i] = make_short2(-1, -1);
            if ((dvalid >> i) & 1u) {
                vp[vc] = sp[i];
                get3d(cam, (float)sp[i].x, (float)sp[i].y, a.plane[sp[i].x + sp[i].y * W].w, X);
                v3[vc][0] = X[0]; v3[vc][1] = X[1]; v3[vc][2] = X[2];
                vc++;
            }
        }
        float4 best = make_float4(0, 0, 0, 0);
        int ua = -1, ub = -1, uc = -1;
        bool has = false;
        float min_cost = APD_FLT_MAX;
        int max_count = 3;
        const FastMod fm((uint32_t)vc);
        for (int it = 0; it < 50; ++it) {
            int ia = (int)fm.mod(g.u32());
            int ib = (int)fm.mod(g.u32());
            int ic = (int)fm.mod(g.u32());
            if (ia == ib || ib == ic || ia == ic) continue;
            if (!point_in_triangle(vp[ia].x, vp[ia].y, vp[ib].x, vp[ib].y, vp[ic].x, vp[ic].y, px, py)) continue;
            const float *A = v3[ia], *B = v3[ib], *C = v3[ic];
            float ACx = A[0] - C[0], ACy = A[1] - C[1], ACz = A[2] - C[2];
            float BCx = B[0] - C[0], BCy = B[1] - C[1], BCz = B[2] - C[2];
            float4 cr = make_float4(ACy * BCz - BCy * ACz, -(ACx * BCz - BCx * ACz), ACx * BCy - BCx * ACy, 0.0f);
            if ((cr.x == 0 && cr.y == 0 && cr.z == 0) || isnan(cr.x) || isnan(cr.y) || isnan(cr.z)) continue;
            normalize3(cr);
            cr.w = -(cr.x * A[0] + cr.y * A[1] + cr.z * A[2]);
            int tcnt = 0;
            for (int k = 0; k < vc; ++k) {
                float d = fabsf(cr.x * v3[k][0] + cr.y * v3[k][1] + cr.z * v3[k][2] + cr.w);
                if (anc_inlier(a, d, depth_diff)) tcnt++;
            }
            if (tcnt < 6) continue;
            if (tcnt > max_count) {
                max_count = tcnt;
                min_cost = fabsf(cr.x * cw0 + cr.y * cw1 + cr.z * cw2 + cr.w);
                best = cr; has = true; ua = ia; ub = ib; uc = ic;
            } else if (tcnt == max_count) {
                float cd = fabsf(cr.x * cw0 + cr.y * cw1 + cr.z * cw2 + cr.w);
                if (cd < min_cost) { min_cost = cd; best = cr; ua = ia; ub = ib; uc = ic; }
            }
        }
        if (!has) { a.reliable[c] = 0; return; }
        float wgt[32];
        for (int i = 0; i < vc; ++i) {
            float d = fabsf(best.x * v3[i][0] + best.y * v3[i][1] + best.z * v3[i][2] + best.w);
            if (!anc_inlier(a, d, depth_diff)) { vp[i] = make_short2(-1, -1); wgt[i] = APD_FLT_MAX; continue; }
            if (i == ua || i == ub || i == uc) d -= 1;
            wgt[i] = d;
        }
        for (int i = 1; i < vc; ++i) {  // sort_small_weighted, APD.cu:25-38
            short2 tp = vp[i];
            float tw = wgt[i];
            int j;
            for (j = i; j >= 1 && tw < wgt[j - 1]; j--) { vp[j] = vp[j - 1]; wgt[j] = wgt[j - 1]; }
            vp[j] = tp; wgt[j] = tw;
        }
        for (int i = 1; i < 9; ++i) anc[i] = vp[i - 1];
        a.reliable[c] = 1;
    }
}

// GenAnchors' RANSAC and anchor ordering (APD.cu:1994-2081), a wave per WEAK pixel with a pending
// RANSAC (the search's stage): lane i holds point i; lane `it` < 50 runs RANSAC iteration it (its 3
// draws are stream positions n + 3 it .. n + 3 it + 2, so a Philox block per lane stands for the
// sequential stream), counting inliers over the points broadcast lane by lane. The sequential
// selection -- a larger inlier count wins, an equal count a strictly smaller centre distance, so the
// earliest of equal candidates stays -- is replayed over the lanes in iteration order, and
// sort_small_weighted (stable insertion sort) is a rank: #{j : w_j < w_i} + #{j < i : w_j == w_i}.
// The same statements per iteration as k_gen_anchors<false> (the path taken when the stage does not
// fit): that kernel's per-lane point arrays went to scratch and to HBM (74 % waiting, L2 hit 24 %,
// profiles/r5_pmc_k_gen_anchors_c3.json), and an LDS version at one pixel per lane was as slow.
__device__ __forceinline__ uint32_t rng_draw(const Rng &g, uint32_t d) {
    const uint4 b = g.block(d >> 2);
    const uint32_t j = d & 3u;
    return j == 0 ? b.x : (j == 1 ? b.y : (j == 2 ? b.z : b.w));
}
#define GA_FIT_WAVES 4
#ifndef GA_FIT_MINW
#define GA_FIT_MINW 8  // waves per SIMD the registers are bounded for (short, issue-bound waves: occupancy hides their latency)
#endif
__global__ __launch_bounds__(GA_FIT_WAVES * WAVE, GA_FIT_MINW) void k_gen_anchors_fit(Args a, const uint32_t *__restrict__ stage, int wc) {
    const int lane = threadIdx.x & (WAVE - 1);
    const int wi = __builtin_amdgcn_readfirstlane(blockIdx.x * GA_FIT_WAVES + (int)(threadIdx.x >> 6));
    if (wi >= wc) return;
    const uint32_t *row = stage + (size_t)wi * GA_STAGE_W;
    // the row in one round trip: lanes 0 and 1 the header and pixel, lane i + 2 point i
    const uint32_t rv = (lane < GA_STAGE_W) ? row[lane] : 0u;
    const uint32_t hdr = (uint32_t)__builtin_amdgcn_readfirstlane((int)rv);
    const int vc = (int)(hdr & 63u);
    const int c = __builtin_amdgcn_readlane((int)rv, 1);
    const int W = a.W;
    const int py = c / W, px = c - py * W;
    // the pixel's anchor row (APD.cu:1890-1893: anchor 0 the pixel, the others none until the RANSAC
    // orders its inliers below), one coalesced store instead of the search kernel's nine
    APD_G short2 *anc = a.anchors + (size_t)wi * 9;
    if (lane < 9) anc[lane] = lane == 0 ? make_short2((short)px, (short)py) : make_short2(-1, -1);
    if (vc == 0) return;
    const float depth_diff = a.dmax - a.dmin;
    const APD_C Cam &cam = a.cams[0];
    // lane i: point i (X, Y, Z, packed position)
    const uint32_t qi = (uint32_t)__shfl((int)rv, lane + 2);
    float X[3] = {0.0f, 0.0f, 0.0f};
    uint32_t q = 0xFFFFFFFFu;
    if (lane < vc) {
        q = qi;
        const int qx = (int)(int16_t)(q & 0xFFFFu), qy = (int)(int16_t)(q >> 16);
        get3d(cam, (float)qx, (float)qy, a.plane[qx + qy * W].w, X);
    }
    const float X0 = X[0], X1 = X[1], X2 = X[2];
    float Cw[3];
    get3d(cam, (float)px, (float)py, a.plane[c].w, Cw);
    // lane it: RANSAC iteration it
    const Rng g(a.seed_lo, a.seed_hi, (uint32_t)c, ORD_ANCHORS);
    const FastMod fm((uint32_t)vc);
    const uint32_t d0 = (hdr >> 6) + 3u * (uint32_t)lane;
#if GA_PHILOX_LDS
    // the 50 iterations' 150 draws lie in Philox blocks n / 4 .. n / 4 + 38: lane j generates block
    // n / 4 + j once into LDS and every lane reads its three words there (instead of two blocks per lane)
    __shared__ uint4 sphil[GA_FIT_WAVES][WAVE];
    const uint32_t nb = (hdr >> 6) >> 2;
    sphil[threadIdx.x >> 6][lane] = g.block(nb + (uint32_t)lane);
    __builtin_amdgcn_wave_barrier();  // (LDS operations of one wave complete in order)
    const uint32_t *sw = reinterpret_cast<const uint32_t *>(&sphil[threadIdx.x >> 6][0]);
    auto pick = [&](uint32_t d) { return sw[d - 4u * nb]; };  // (d - 4 nb <= 3 + 3 * 63 + 2 < 256)
#else
    // the three draws d0 .. d0 + 2 lie in Philox blocks d0 / 4 and (d0 + 2) / 4: two blocks, not three
    const uint4 b0 = g.block(d0 >> 2), b1 = g.block((d0 + 2u) >> 2);
    auto pick = [&](uint32_t d) {
        const uint4 b = (d >> 2) == (d0 >> 2) ? b0 : b1;
        const uint32_t j = d & 3u;
        return j == 0 ? b.x : (j == 1 ? b.y : (j == 2 ? b.z : b.w));
    };
#endif
    const int ia = (int)fm.mod(pick(d0));
    const int ib = (int)fm.mod(pick(d0 + 1u));
    const int ic = (int)fm.mod(pick(d0 + 2u));
    bool ok = lane < 50 && !(ia == ib || ib == ic || ia == ic);
    const float Ax = __shfl(X0, ia), Ay = __shfl(X1, ia), Az = __shfl(X2, ia);
    const float Bx = __shfl(X0, ib), By = __shfl(X1, ib), Bz = __shfl(X2, ib);
    const float Cx = __shfl(X0, ic), Cy = __shfl(X1, ic), Cz = __shfl(X2, ic);
    const uint32_t qa = (uint32_t)__shfl((int)q, ia), qb = (uint32_t)__shfl((int)q, ib), qc = (uint32_t)__shfl((int)q, ic);
    ok = ok && point_in_triangle((int16_t)(qa & 0xFFFFu), (int16_t)(qa >> 16), (int16_t)(qb & 0xFFFFu), (int16_t)(qb >> 16),
                                 (int16_t)(qc & 0xFFFFu), (int16_t)(qc >> 16), px, py);
    float ACx = Ax - Cx, ACy = Ay - Cy, ACz = Az - Cz;
    float BCx = Bx - Cx, BCy = By - Cy, BCz = Bz - Cz;
    float4 cr = make_float4(ACy * BCz - BCy * ACz, -(ACx * BCz - BCx * ACz), ACx * BCy - BCx * ACy, 0.0f);
    ok = ok && !((cr.x == 0 && cr.y == 0 && cr.z == 0) || isnan(cr.x) || isnan(cr.y) || isnan(cr.z));
    if (ok) {
        normalize3(cr);
        cr.w = -(cr.x * Ax + cr.y * Ay + cr.z * Az);
    }
    // the points broadcast from LDS (one uniform-address read per point; v_readlane's SGPR results
    // stalled the loop on their read-after-write hazards)
    __shared__ float spx[GA_FIT_WAVES][WAVE], spy[GA_FIT_WAVES][WAVE], spz[GA_FIT_WAVES][WAVE];
    __shared__ float swgt[GA_FIT_WAVES][WAVE];
    const int wv = threadIdx.x >> 6;
    // (coordinates apart, two points per 8-byte read: the point pairs go straight into packed fp32
    // multiplies and adds; slots past the last point hold NaN, which is never an inlier)
    const float qnan = __builtin_nanf("");
    spx[wv][lane] = lane < vc ? X0 : qnan;
    spy[wv][lane] = lane < vc ? X1 : qnan;
    spz[wv][lane] = lane < vc ? X2 : qnan;
    __builtin_amdgcn_wave_barrier();  // (LDS operations of one wave complete in order)
    // (anc_inlier with its uniform choice taken outside the loop: inside, the compiler evaluated both
    // sides per point -- an IEEE division the common d < anc_dlim side never needs). Per point the same
    // statement, fabsf(((cr.x * x + cr.y * y) + cr.z * z) + cr.w), two points per packed operation.
    int tcnt = 0;
    const apd_f2 crx = {cr.x, cr.x}, cry = {cr.y, cr.y}, crz = {cr.z, cr.z}, crw = {cr.w, cr.w};
    auto pair_d = [&](int k) {
        const apd_f2 px2 = *reinterpret_cast<const apd_f2 *>(&spx[wv][k]);
        const apd_f2 py2 = *reinterpret_cast<const apd_f2 *>(&spy[wv][k]);
        const apd_f2 pz2 = *reinterpret_cast<const apd_f2 *>(&spz[wv][k]);
        const apd_f2 d = ((crx * px2 + cry * py2) + crz * pz2) + crw;
        return (apd_f2){fabsf(d.x), fabsf(d.y)};
    };
    if (a.anc_dlim_ok) {
        const float lim = a.anc_dlim;
#pragma unroll 4
        for (int k = 0; k < vc; k += 2) {
            const apd_f2 d = pair_d(k);
            tcnt += (d.x < lim ? 1 : 0) + (d.y < lim ? 1 : 0);
        }
    } else {
#pragma unroll 2
        for (int k = 0; k < vc; k += 2) {
            const apd_f2 d = pair_d(k);
            tcnt += (d.x / depth_diff < a.ransac_thr ? 1 : 0) + (d.y / depth_diff < a.ransac_thr ? 1 : 0);
        }
    }
    ok = ok && tcnt >= 6;
    const float cd = fabsf(cr.x * Cw[0] + cr.y * Cw[1] + cr.z * Cw[2] + cr.w);
    // The sequential selection (iteration order: a larger inlier count wins, an equal count a strictly
    // smaller centre distance) is, over the ok lanes, the largest count; among its lanes the first one,
    // unless a later one has a smaller distance (`<`: a NaN never wins, and a NaN first one is never
    // replaced) -- i.e. the earliest lane with the minimum distance, NaN taken as +inf, when the first
    // one's distance is not NaN. Computed by wave reductions instead of a replay over the lanes.
    const uint64_t okm = __ballot(ok);
    int best_it = -1;
    if (okm) {
        int mc = ok ? tcnt : -1;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) mc = max(mc, __shfl_xor(mc, o));
        const bool top = ok && tcnt == mc;
        const uint64_t topm = __ballot(top);
        const int first = __builtin_ctzll(topm);
        const float cfirst = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(cd), first));
        if (__builtin_isnan(cfirst)) {
            best_it = first;
        } else {
            float cm = top ? (__builtin_isnan(cd) ? __builtin_inff() : cd) : __builtin_inff();
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) cm = fminf(cm, __shfl_xor(cm, o));
            best_it = __builtin_ctzll(__ballot(top && !__builtin_isnan(cd) ? cd == cm : (top && cm == __builtin_inff())));
        }
    }
    if (best_it < 0) {
        if (lane == 0) a.reliable[c] = 0;
        return;
    }
    float4 best;
    best.x = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(cr.x), best_it));
    best.y = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(cr.y), best_it));
    best.z = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(cr.z), best_it));
    best.w = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(cr.w), best_it));
    const int ua = __builtin_amdgcn_readlane(ia, best_it), ub = __builtin_amdgcn_readlane(ib, best_it),
              uc = __builtin_amdgcn_readlane(ic, best_it);
    // weights, then the stable rank of each point (sort_small_weighted, APD.cu:25-38)
    float wgt = APD_FLT_MAX;
    uint32_t vq = 0xFFFFFFFFu;
    if (lane < vc) {
        float d = fabsf(best.x * X0 + best.y * X1 + best.z * X2 + best.w);
        if (anc_inlier(a, d, depth_diff)) {
            if (lane == ua || lane == ub || lane == uc) d -= 1;
            wgt = d;
            vq = q;
        }
    }
    swgt[wv][lane] = wgt;
    __builtin_amdgcn_wave_barrier();
    int rank = 0;
#pragma unroll 4
    for (int j = 0; j < vc; ++j) {
        const float wj = swgt[wv][j];
        rank += (wj < wgt || (wj == wgt && j < lane)) ? 1 : 0;
    }
    if (lane < vc && rank < 8) anc[1 + rank] = make_short2((short)(vq & 0xFFFFu), (short)(vq >> 16));
    if (lane == 0) a.reliable[c] = 1;
}

// NeigbourUpdate (APD.cu:2084-2100)
__global__ __launch_bounds__(BLOCK) void k_neighbour_update(Args a) {
    const int c = blockIdx.x * BLOCK + threadIdx.x;
    if (c >= a.HW) return;
    if (a.weak[c] == APD_WEAK && a.reliable[c] != 1) a.weak[c] = APD_UNKNOWN;
}

// RANSACToGetFitPlane (APD.cu:2486-2598). The anchor points live in LDS (one float4 per point and
// thread: X, Y, Z and the packed pixel position), so the draws' dynamically indexed reads are three
// 16-byte LDS loads instead of select chains over a register array.
__global__ __launch_bounds__(BLOCK) void k_ransac_fit(Args a, int iter) {
    __shared__ float4 pts[8][BLOCK];
    const int c = blockIdx.x * BLOCK + threadIdx.x;
    const int tid = threadIdx.x;
    if (c >= a.HW) return;
    if (a.weak[c] != APD_WEAK) { a.fit[c] = a.plane[c]; return; }
    const int W = a.W;
    const int py = c / W, px = c - py * W;
    const APD_C Cam &cam = a.cams[0];
    const APD_G short2 *anc = a.anchors + (size_t)a.amap[c] * 9;
    int cnt = 0;
    float X[3];
    for (int i = 1; i < 9; ++i) {
        short2 t = anc[i];
        if (t.x == -1 || t.y == -1) continue;
        float d = depth_from_plane(cam, a.plane[t.x + t.y * W], t.x, t.y);
        get3d(cam, (float)t.x, (float)t.y, d, X);
        pts[cnt][tid] = make_float4(X[0], X[1], X[2], __int_as_float((int)(uint16_t)t.x | ((int)t.y << 16)));
        cnt++;
    }
    if (cnt < 3) { a.fit[c] = a.plane[c]; return; }
    Rng g(a.seed_lo, a.seed_hi, (uint32_t)c, ord_fit(iter));
    float min_cost = APD_FLT_MAX;
    float4 best = make_float4(0, 0, 0, 0);
    bool has = false;
    const FastMod fm((uint32_t)cnt);  // x % cnt without a per-draw integer division (cnt <= 8)
    for (int it = 0; it < 50; ++it) {
        int ia = (int)fm.mod(g.u32());
        int ib = (int)fm.mod(g.u32());
        int ic = (int)fm.mod(g.u32());
        if (ia == ib || ib == ic || ia == ic) continue;
        const float4 A = pts[ia][tid], B = pts[ib][tid], C = pts[ic][tid];
        const int pa = __float_as_int(A.w), pb = __float_as_int(B.w), pc = __float_as_int(C.w);
        if (!point_in_triangle(pa & 0xFFFF, pa >> 16, pb & 0xFFFF, pb >> 16, pc & 0xFFFF, pc >> 16, px, py)) continue;
        float ACx = A.x - C.x, ACy = A.y - C.y, ACz = A.z - C.z;
        float BCx = B.x - C.x, BCy = B.y - C.y, BCz = B.z - C.z;
        float4 cr = make_float4(ACy * BCz - BCy * ACz, -(ACx * BCz - BCx * ACz), ACx * BCy - BCx * ACy, 0.0f);
        if ((cr.x == 0 && cr.y == 0 && cr.z == 0) || isnan(cr.x) || isnan(cr.y) || isnan(cr.z)) continue;
        normalize3(cr);
        cr.w = -(cr.x * A.x + cr.y * A.y + cr.z * A.z);
        float tc = 0.0f;
        for (int k = 0; k < cnt; ++k) {
            if (k == ia || k == ib || k == ic) continue;
            const float4 P = pts[k][tid];
            tc += fabsf(cr.x * P.x + cr.y * P.y + cr.z * P.z + cr.w);
        }
        if (tc < min_cost) { min_cost = tc; best = cr; has = true; }
        if (min_cost == 0) break;
    }
    if (has) {
        float d = depth_from_plane(cam, a.plane[c], px, py);
        float4 vd = view_dir(cam, px, py, d);
        float dot = best.x * vd.x + best.y * vd.y + best.z * vd.z;
        if (dot > 0) { best.x = -best.x; best.y = -best.y; best.z = -best.z; best.w = -best.w; }
        a.fit[c] = best;
    } else {
        a.fit[c] = make_float4(0, 0, 0, 0);
    }
}

// ---------------------------------------------------------------------------------------------
// shared pieces of the two checkerboard sweeps
// ---------------------------------------------------------------------------------------------
// Multi-hypothesis joint view selection (APD.cu:1339-1374 / 1505-1540) for the lane's view.
// Returns this lane's view weight (0..15).
__device__ __forceinline__ int view_selection(const float ca[8], float prior, int iter, Rng &g, const Group &G,
                                              int N) {
    const float thr = (float)(0.8 * (double)d_expf((float)(iter * iter) / (-90.0f)));
    float count = 0.0f, tmpw = 0.0f;
    int cf = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const float c = ca[j];
        if (c < thr) { tmpw += d_expf(c * c / (-0.18f)); count += 1.0f; }
        if (c > 1.2f) cf++;
    }
    float sp = 0.0f;
    if (count > 2 && cf < 3) sp = tmpw / count;
    else if (cf < 3) sp = d_expf(thr * thr / (-0.32f));
    sp = sp * prior;
    // TransformPDFToCDF (APD.cu:174-188): in-order sums over the pixel's N lanes
    float sum = 0.0f;
    for (int k = 0; k < N; ++k) sum += __shfl(sp, G.base + k);
    const float inv = 1.0f / sum;
    float cum = 0.0f, mycdf = 0.0f;
    for (int k = 0; k < N; ++k) {
        cum = fmaf(__shfl(sp, G.base + k), inv, cum);
        if (k == G.v) mycdf = cum;
    }
    int w = 0;
    for (int smp = 0; smp < 15; ++smp) {
        const float u = g.uniform() - APD_FLT_EPSILON;
        const uint32_t m = group_bits(mycdf > u, G);
        if (m != 0u && (__ffs(m) - 1) == G.v) w++;
    }
    return w;
}

// The same with the pixel's 15 draws precomputed (u[k * us] = the k-th uniform() of its stream).
__device__ __forceinline__ int view_selection_u(const float ca[8], float prior, int iter, const float *u, int us,
                                                const Group &G, int N) {
    const float thr = (float)(0.8 * (double)d_expf((float)(iter * iter) / (-90.0f)));
    float count = 0.0f, tmpw = 0.0f;
    int cf = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const float c = ca[j];
        if (c < thr) { tmpw += d_expf(c * c / (-0.18f)); count += 1.0f; }
        if (c > 1.2f) cf++;
    }
    float sp = 0.0f;
    if (count > 2 && cf < 3) sp = tmpw / count;
    else if (cf < 3) sp = d_expf(thr * thr / (-0.32f));
    sp = sp * prior;
    float sum = 0.0f;
    for (int k = 0; k < N; ++k) sum += __shfl(sp, G.base + k);
    const float inv = 1.0f / sum;
    float cum = 0.0f, mycdf = 0.0f;
    for (int k = 0; k < N; ++k) {
        cum = fmaf(__shfl(sp, G.base + k), inv, cum);
        if (k == G.v) mycdf = cum;
    }
    int w = 0;
    for (int smp = 0; smp < 15; ++smp) {
        const float uu = u[smp * us] - APD_FLT_EPSILON;
        const uint32_t m = group_bits(mycdf > uu, G);
        if (m != 0u && (__ffs(m) - 1) == G.v) w++;
    }
    return w;
}
#define VS_DRAWS 15  // uniform() draws of view_selection

// PlaneHypothesisRefinement{Strong,Weak} candidate generation (APD.cu:961-980 / 1054-1067)
struct Cands {
    float4 nrand, npert;
    float drand, dpert;
};
__device__ __forceinline__ Cands refine_candidates(const Args &a, int px, int py, Rng &g, float4 cur, float depth) {
    const APD_C Cam &cam = a.cams[0];
    Cands C;
    C.drand = g.uniform() * (a.dmax - a.dmin) + a.dmin;
#ifdef APD_ABLATE_RANDDEPTH  // timing-only experiment (wrong values): random-depth candidates kept local
    C.drand = depth * 1.001f;
#endif
    C.nrand = random_normal(cam, px, py, g, depth);
    float dp = depth;
    const float dminp = (1 - 0.02f) * dp;
    const float dmaxp = (1 + 0.02f) * dp;
    int guard = 0;
    do {
        dp = g.uniform() * (dmaxp - dminp) + dminp;
    } while (dp < a.dmin && dp > a.dmax && ++guard < 64);
    C.dpert = dp;
    const float pert = (float)((double)0.02f * 3.14159265358979323846);
    C.npert = perturbed_normal(cam, px, py, cur, g, pert);
    return C;
}
// candidate k of {depth_rand,cur,depth_rand,cur,perturbed} x {cur,rand,rand,perturbed,cur}
__device__ __forceinline__ float4 candidate(const Cands &C, int k, float4 cur0, float d0, float &dk) {
    dk = (k == 0 || k == 2) ? C.drand : (k == 4 ? C.dpert : d0);
    return (k == 0 || k == 4) ? cur0 : (k == 3 ? C.npert : C.nrand);
}

// ---------------------------------------------------------------------------------------------
// View-major Strong sweep (same function as k_sweep_strong, different work decomposition).
// A workgroup of VM_WAVES waves owns VM_P = 64 consecutive pixels of the (tile-ordered) list and
// runs the pixel's work in phases separated by workgroup barriers, each phase with the lane shape
// that suits it:
//   P0  lane = (pixel, direction): adaptive-checkerboard scan of one of the 8 directions; the 9
//       hypothesis planes, their validity, the 6x6 reference window and the pixel's 15 view-selection
//       draws go to LDS.
//   P1  lane = pixel, wave = (hypothesis, view) task: every gather instruction of a wave samples ONE
//       source image around 64 neighbouring pixels (compact footprint, L1 reuse across window
//       columns and across the wave's successive tasks); costs -> LDS [h][v][pixel].
//   P2a lane = (pixel, view) groups, as in k_sweep_strong: joint view selection with the in-order
//       CDF and the 15 draws -> view weights.
//   P2b lane = pixel (one wave, 64 pixels per instruction instead of 64/N): weighted hypothesis
//       costs, argmin, refinement candidates (the stream resumed after the 15 draws); candidates
//       and the running state -> LDS.
//   P3  lane = pixel, wave = (candidate, view) task: refinement NCC (+ geometric) -> LDS.
//   P4  lane = pixel: in-order weighted candidate costs, acceptance, writes.
// ---------------------------------------------------------------------------------------------
#ifndef VM_WAVES
#define VM_WAVES 4  // 4-wave workgroups: 3 per CU at <= 170 VGPRs (the sweep needs ~154 without spills)
#endif
#define VM_BLOCK (VM_WAVES * WAVE)
// Task dealing in the view-major kernels: task u goes to wave u % VM_WAVES, so the 4 waves of a
// workgroup sample the same source image around the same pixels at the same time and share the
// CU's 32 KiB L1 (contiguous per-wave chunks put up to 4 images per workgroup in flight; measured
// on the Strong sweep: 13.5 -> 8.0 L1->L2 requests per gather, 16.2 -> 13.8 ms per launch).
#define VM_P 64
#ifndef APD_VM_LDS_PAD
#define APD_VM_LDS_PAD 0  // experiments: extra LDS bytes per workgroup (fewer workgroups per CU)
#endif
// SS_LDS40 (fp16 problems): the reference taps as fp16 (exact there), the neighbour flags as bits and
// the view selection's draws regenerated per (pixel, view) lane instead of kept in LDS -- 40.8 KB at
// N = 10 (48.4 before): four workgroups per CU instead of three (the VGPRs bounded to match).
#ifndef SS_LDS40
#define SS_LDS40 1
#endif
template <class RT>
struct VmLdsT {  // static part; the cost table [9][N][64] and the weights [N][64] (uint8) follow
    RT refw[36 * VM_P];          // [k][p]
    float4 hyp[9 * VM_P];        // [h][p]: 8 propagated + current; P2 overwrites [0..4] with the
                                 // refinement candidates (VM_CAND) once the pixel's reads are done
#if SS_LDS40
    uint8_t nvq[4 * VM_P];       // [w][p]: bit r = neighbour d = w + 4r exists (P0's wave w writes its own byte)
#else
    uint8_t nval[8 * VM_P];      // [d][p]: neighbour d exists (adaptive-checkerboard scan hit)
#endif
    float4 pnow[VM_P];
    float st[4 * VM_P];          // depth_now, cost_now, cost_init, weight_norm
#if !SS_LDS40
    float vsu[VS_DRAWS * VM_P];  // [k][p]: the view selection's 15 uniform() draws of the pixel's stream
#endif
    uint32_t tsel[VM_P];         // views with a sampled weight > 0
    float rmean[VM_P], rvar[VM_P];  // reference-window moments (RefWin) of pixel slot p (P3's packed items)
    int pxy[VM_P];               // packed (x, y) of pixel slot p
};
template <bool F16>
using VmRefT = typename std::conditional<SS_LDS40 && F16, _Float16, float>::type;
template <class RT>
__device__ __forceinline__ bool vm_nval(const VmLdsT<RT> &L, int d, int p) {
#if SS_LDS40
    return (L.nvq[(d & 3) * VM_P + p] >> (d >> 2)) & 1u;
#else
    return L.nval[d * VM_P + p] != 0;
#endif
}
#ifndef SS_P3_CHUNKS
#define SS_P3_CHUNKS 3  // Strong sweep P3 batches: whole views until at least this many 64-item chunks
#endif
#define VM_CAND(L) ((L).hyp)
// per-pixel SaWin table appended to the view-major kernels' dynamic LDS when the problem has SA masks
static inline size_t sa_lds_bytes(const Args &a) { return a.sa_any ? VM_P * sizeof(SaWin) + 16 : 0; }
__device__ __forceinline__ void *sa_lds_align(void *p) { return (void *)(((uintptr_t)p + 15) & ~(uintptr_t)15); }     // [k][p], k < 5: refinement candidates (t.w = distance)
static inline size_t vm_lds_bytes(int N, bool f16) {
    return APD_VM_LDS_PAD + (f16 ? sizeof(VmLdsT<VmRefT<true>>) : sizeof(VmLdsT<VmRefT<false>>)) +
           (size_t)9 * N * VM_P * sizeof(float) + (size_t)N * VM_P;
}

// One direction of the adaptive checkerboard (APD.cu:1127-1316): d = 2*dir + far, dir in
// {up, down, left, right}, in the order of pos[]/flag[] of k_sweep_strong.
__device__ __forceinline__ int scan_direction(const APD_G float *__restrict__ cost, int d, int c, int px, int py,
                                              int W, int H) {
    const int dir = d >> 1, far = d & 1;
    // unit step toward the neighbour, and the distance to the border along it
    const int sx = dir == 2 ? -1 : (dir == 3 ? 1 : 0);
    const int sy = dir == 0 ? -1 : (dir == 1 ? 1 : 0);
    const int du = dir == 0 ? py : (dir == 1 ? H - 1 - py : (dir == 2 ? px : W - 1 - px));
    const int step = sy * W + sx;
    if (far) {
        if (!(du > 2)) return -1;
        int best = c + 3 * step;
        float cmin = cost[best];
        for (int i = 1; i < 11; ++i)
            if (du > 2 + 2 * i) {
                const int t = c + (3 + 2 * i) * step;
                const float v = cost[t];
                if (v < cmin) { cmin = v; best = t; }
            }
        return best;
    }
    if (!(du > 0)) return -1;
    // perpendicular axis: x for up/down (first -x then +x), y for left/right (first -y then +y)
    const bool vert = dir < 2;
    const int vstep = vert ? 1 : W;
    const int dneg = vert ? px : py;                       // distance to the border on the - side
    const int dpos = vert ? W - 1 - px : H - 1 - py;       // ... on the + side
    int best = c + step;
    float cmin = cost[best];
    for (int i = 0; i < 3; ++i) {
        if (du > 1 + i && dneg > i) {
            const int t = c + (i + 2) * step - (i + 1) * vstep;
            const float v = cost[t];
            if (v < cmin) { cmin = v; best = t; }
        }
        if (du > 1 + i && dpos > i) {
            const int t = c + (i + 2) * step + (i + 1) * vstep;
            const float v = cost[t];
            if (v < cmin) { cmin = v; best = t; }
        }
    }
    return best;
}

// Both directions d0 = wave, d1 = wave + 4 of a P0 lane (same near/far kind): every candidate cost is
// loaded first (out-of-range candidates read the pixel's own cost and are ignored), then the scans
// run in scan_direction's order -- one memory round trip instead of one per candidate.
__device__ __forceinline__ void scan_directions2(const APD_G float *__restrict__ cost, int d0, int c, int px, int py,
                                                 int W, int H, int q[2]) {
    const bool far = d0 & 1;
    constexpr int NC = 11;  // far: 11 strip candidates; near: the first + 3 x 2 V-shape candidates
    float v[2][NC];
    int t[2][NC];
    bool ok[2][NC];
    int du[2];
#pragma unroll
    for (int r = 0; r < 2; ++r) {
        const int dir = (d0 + 4 * r) >> 1;
        const int sx = dir == 2 ? -1 : (dir == 3 ? 1 : 0);
        const int sy = dir == 0 ? -1 : (dir == 1 ? 1 : 0);
        du[r] = dir == 0 ? py : (dir == 1 ? H - 1 - py : (dir == 2 ? px : W - 1 - px));
        const int step = sy * W + sx;
        if (far) {
#pragma unroll
            for (int i = 0; i < NC; ++i) {
                ok[r][i] = du[r] > 2 + 2 * i;
                t[r][i] = c + (3 + 2 * i) * step;
            }
        } else {
            const bool vert = dir < 2;
            const int vstep = vert ? 1 : W;
            const int dneg = vert ? px : py, dpos = vert ? W - 1 - px : H - 1 - py;
            ok[r][0] = du[r] > 0;
            t[r][0] = c + step;
#pragma unroll
            for (int i = 0; i < 3; ++i) {
                ok[r][1 + 2 * i] = du[r] > 1 + i && dneg > i;
                t[r][1 + 2 * i] = c + (i + 2) * step - (i + 1) * vstep;
                ok[r][2 + 2 * i] = du[r] > 1 + i && dpos > i;
                t[r][2 + 2 * i] = c + (i + 2) * step + (i + 1) * vstep;
            }
#pragma unroll
            for (int i = 7; i < NC; ++i) { ok[r][i] = false; t[r][i] = c; }
        }
#pragma unroll
        for (int i = 0; i < NC; ++i) v[r][i] = cost[ok[r][i] ? t[r][i] : c];
    }
#pragma unroll
    for (int r = 0; r < 2; ++r) {
        if (!ok[r][0]) { q[r] = -1; continue; }
        int best = t[r][0];
        float cmin = v[r][0];
#pragma unroll
        for (int i = 1; i < NC; ++i)
            if (ok[r][i] && v[r][i] < cmin) { cmin = v[r][i]; best = t[r][i]; }
        q[r] = best;
    }
}

template <bool F16, bool SA>
#ifndef VM_MINW
#define VM_MINW 3  // waves per SIMD -> VGPR budget 512 / VM_MINW
#endif
__global__ __launch_bounds__(VM_BLOCK, (SS_LDS40 && F16 && !SA) ? 4 : VM_MINW) void k_sweep_strong_vm(Args a, const int *__restrict__ list, int count,
                                                                  int iter) {
    const int N = a.N, W = a.W, H = a.H;
    using VmLds = VmLdsT<VmRefT<F16>>;
    VmLds &L = *reinterpret_cast<VmLds *>(apd_dyn_lds);
    float *costL = reinterpret_cast<float *>(&L + 1);                   // [9][N][64], later [5][N][64]
    uint8_t *wts = reinterpret_cast<uint8_t *>(costL + 9 * N * VM_P);    // [N][64] view weights
    SaWin *saw = reinterpret_cast<SaWin *>(wts + N * VM_P);              // [64] when a.sa_any
    const int blk = xcd_remap(blockIdx.x, gridDim.x);
    const int first = blk * VM_P;
    const int np = min(VM_P, count - first);
    const int tid = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & (WAVE - 1);
    const APD_C Cam &cam0 = a.cams[0];
    const bool geom_imp = a.geom && a.impetus;
    const float gf = a.gf;

    // ---- P0: lane = (pixel, direction)
    {
        const int p = lane;
        if (p < np) {
            const int c = list[first + p];
            const int py = c / W, px = c - py * W;
            static_assert(VM_WAVES == 4, "P0 deals the 8 directions as d = wave, wave + 4");
            int q[2];
            scan_directions2(a.cost, wave, c, px, py, W, H, q);
            // all loads first (the two picked planes, the own plane, the reference taps), then the LDS writes
            float4 hp[3];
#pragma unroll
            for (int r = 0; r < 2; ++r) hp[r] = a.plane[q[r] >= 0 ? q[r] : c];
            hp[2] = a.plane[c];
            float rv[36 / VM_WAVES];
#pragma unroll
            for (int kk = 0; kk < 36 / VM_WAVES; ++kk) {
                const int k = wave + VM_WAVES * kk, i = k / 6, j = k - 6 * (k / 6);
                rv[kk] = tex_ref(a, px - 5 + 2 * i, py - 5 + 2 * j);
            }
#pragma unroll
            for (int r = 0; r < 2; ++r) {
                const int d = wave + 4 * r;
#if !SS_LDS40
                L.nval[d * VM_P + p] = q[r] >= 0;
#endif
                if (q[r] >= 0) L.hyp[d * VM_P + p] = hp[r];
            }
#if SS_LDS40
            L.nvq[wave * VM_P + p] = (uint8_t)((q[0] >= 0 ? 1u : 0u) | (q[1] >= 0 ? 2u : 0u));
#endif
            if (wave == 0) { L.hyp[8 * VM_P + p] = hp[2]; L.pxy[p] = px | (py << 16); }
#pragma unroll
            for (int kk = 0; kk < 36 / VM_WAVES; ++kk) L.refw[(wave + VM_WAVES * kk) * VM_P + p] = (VmRefT<F16>)rv[kk];
            if (SA && wave == VM_WAVES - 1) saw[p] = sa_window(a, px, py);
#if !SS_LDS40
            if (wave == 1 % VM_WAVES) {  // the view selection's draws, once per pixel (not per view lane)
                Rng rg(a.seed_lo, a.seed_hi, (uint32_t)c, ord_strong(iter));
#pragma unroll
                for (int k = 0; k < VS_DRAWS; ++k) L.vsu[k * VM_P + p] = rg.uniform();
            }
#endif
        }
    }
    __syncthreads();

    // ---- P1: lane = pixel, wave = (hypothesis, view) tasks
    const int p1 = lane;
    const bool pv1 = p1 < np;
    int c1 = 0, px1 = 0, py1 = 0;
    if (pv1) { c1 = list[first + p1]; py1 = c1 / W; px1 = c1 - py1 * W; }
    RefWinT<VmRefT<F16>> rw = refwin_from_lds<VM_P>(&L.refw[p1]);
    if (SA) rw.sa = &saw[p1];
    if (wave == 0 && pv1) { L.rmean[p1] = rw.mean; L.rvar[p1] = rw.var; }  // (read after P1's barrier)
    // tasks whose window needs the out-of-line path are collected in `defer` (bit k = k-th task of
    // this wave) and evaluated after the loop, so the hot loop holds no call.
    uint64_t defer[2] = {0, 0};  // up to 128 tasks per wave (9 * 31 / VM_WAVES)
    uint32_t issued = 0;         // NCC-Old evaluations of this lane (profiling count, a.evals)
    // tasks in view-major order, dealt round-robin over the waves (the 4 waves of a workgroup sample
    // one source image around the same pixels at once: L1 sharing); (h, v) -> table index h * N + v.
    // (Measured and not kept: the current plane (h = 8) evaluated after the view selection for the
    // weighted views only, as the Weak sweep does: fewer evaluations, but +3 % on the texture-rich C3
    // pass -- the extra phase loses the hypotheses' shared source lines.)
    for (int u = wave, k = 0; u < 9 * N; u += VM_WAVES, ++k) {
        const int v = u / 9, h = u - 9 * v, t = h * N + v;
        float val = (h == 0 && v == 0) ? 2.0f : 0.0f;  // float cost_array[8][32] = {2.0f} (APD.cu:1120)
        const bool fh = h == 8 || vm_nval(L, h, p1);
        if (pv1 && fh) {
            const float4 pl = L.hyp[h * VM_P + p1];
            if (h == 8 && a.wcur) {  // iteration 0: RandomInitialization's NCC-Old of this plane
                val = a.wcur[(size_t)v * a.HW + c1];
            } else {
                bool slow;
                ++issued;
                val = ncc_old_fast<F16, VM_P>(a, px1, py1, v + 1, pl, rw, slow);
                if (slow) defer[k >> 6] |= 1ull << (k & 63);
            }
            if (h == 8 && geom_imp) val = fmaf(gf, geom_cost(a, px1, py1, v + 1, pl), val);
        }
        costL[t * VM_P + p1] = val;
    }
    for (int w2 = 0; w2 < 2; ++w2)
    while (defer[w2]) {
        const int k = __builtin_ctzll(defer[w2]) + 64 * w2;
        defer[w2] &= defer[w2] - 1;
        const int u = wave + k * VM_WAVES, v = u / 9, h = u - 9 * v, t = h * N + v;
        const float4 pl = L.hyp[h * VM_P + p1];
        float val = ncc_old_slow<F16, VmRefT<F16>>(a.self, px1, py1, v + 1, pl, rw.r, VM_P, rw.mean, rw.var);
        if (h == 8 && geom_imp) val = fmaf(gf, geom_cost(a, px1, py1, v + 1, pl), val);
        costL[t * VM_P + p1] = val;
    }
    __syncthreads();

    // ---- P2a: lane = (pixel, view) groups, rounds of VM_WAVES * (64/N) pixels: joint view selection
    // (the in-order CDF over the pixel's N lanes and its 15 draws) -> view weights and selection bits
    const int Gp = WAVE / N;
    const int ppr = VM_WAVES * Gp;
    for (int r0 = 0; r0 < np; r0 += ppr) {
        int g = lane / N;
        const bool lane_ok = g < Gp;
        int v = lane - g * N;
        if (!lane_ok) { g = 0; v = (lane - Gp * N) % N; }
        Group G;
        G.v = v; G.base = g * N; G.slot = g; G.li = 0;
        G.gmask = (N >= 64) ? ~0ull : ((1ull << N) - 1ull);
        const int pr = r0 + wave * Gp + g;
        G.valid = lane_ok && pr < np;
        const int p = min(pr, np - 1);
        const int c = list[first + p];
        float ca[8];
#pragma unroll
        for (int h = 0; h < 8; ++h) ca[h] = costL[(h * N + v) * VM_P + p];
        // view selection priors from the 4 direct neighbours (APD.cu:1323-1337)
        float prior = 0.0f;
        {
            const int nb[4] = {c - W, c + W, c - 1, c + 1};
#pragma unroll
            for (int i = 0; i < 4; ++i)
                if (vm_nval(L, 2 * i, p)) prior += ((a.sel[nb[i]] >> v) & 1u) ? 0.9f : 0.1f;
        }
#if SS_LDS40
        Rng rg(a.seed_lo, a.seed_hi, (uint32_t)c, ord_strong(iter));  // (the pixel's 15 draws, per lane)
        const int w = view_selection(ca, prior, iter, rg, G, N);
#else
        const int w = view_selection_u(ca, prior, iter, &L.vsu[p], VM_P, G, N);
#endif
        const uint32_t tsel = group_bits(w > 0, G);
        if (G.valid) {
            wts[v * VM_P + p] = (uint8_t)w;
            if (G.v == 0) L.tsel[p] = tsel;
        }
    }
    __syncthreads();

    // ---- P2b: lane = pixel (wave 0): weighted hypothesis costs in view order, argmin, refinement
    // candidates (the pixel's stream resumes after the view selection's 15 draws)
    if (wave == 0 && pv1) {
        const int p = p1, c = c1, px = px1, py = py1;
        float fc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        float wn = 0.0f, cost_now = 0.0f;
        for (int k = 0; k < N; ++k) {
            const int wk = wts[k * VM_P + p];
            const float fwk = (float)wk;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float ck = costL[(j * N + k) * VM_P + p];
                if (wk > 0) fc[j] = fmaf(fwk, ck, fc[j]);
            }
            if (wk > 0) wn += fwk;
            cost_now = fmaf(fwk, costL[(8 * N + k) * VM_P + p], cost_now);
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) fc[j] /= wn;
        cost_now /= wn;
        const float cost_init = cost_now;
        int mi = 0;
        {
            float m = fc[0];
#pragma unroll
            for (int j = 1; j < 8; ++j) if (fc[j] <= m) { m = fc[j]; mi = j; }
        }
        const float4 cur = L.hyp[8 * VM_P + p];
        float depth_now = depth_from_plane(cam0, cur, px, py);
        float4 pnow = cur;
        {
            float fcm = fc[0];
#pragma unroll
            for (int k = 1; k < 8; ++k) if (mi == k) fcm = fc[k];
            if (vm_nval(L, mi, p)) {
                const float4 cand = L.hyp[mi * VM_P + p];
                const float db = depth_from_plane(cam0, cand, px, py);
                if (db >= a.dmin && db <= a.dmax && fcm < cost_now) {
                    depth_now = db; pnow = cand; cost_now = fcm;
                    a.sel[c] = L.tsel[p];
                }
            }
        }
        // PlaneHypothesisRefinementStrong candidates (APD.cu:950-980)
        Rng rg(a.seed_lo, a.seed_hi, (uint32_t)c, ord_strong(iter));
        rg.n = VS_DRAWS;
        rg.refill();
        const Cands C = refine_candidates(a, px, py, rg, pnow, depth_now);
#pragma unroll 1
        for (int k = 0; k < 5; ++k) {
            float dk;
            float4 t = candidate(C, k, pnow, depth_now, dk);
            t.w = dist2origin(cam0, px, py, dk, t);
            VM_CAND(L)[k * VM_P + p] = t;
        }
        L.pnow[p] = pnow;
        L.st[0 * VM_P + p] = depth_now;
        L.st[1 * VM_P + p] = cost_now;
        L.st[2 * VM_P + p] = cost_init;
        L.st[3 * VM_P + p] = wn;
    }
    __syncthreads();

    // ---- P3: refinement evaluations (views with weight > 0) with the exact early exit of
    // k_sweep_weak_vm: a candidate is accepted only if fl(S / wn) < cost_now, cost_now never exceeds its
    // value after P2b (L.st[1]), and every view-order prefix P of the fmaf chain S (weights > 0, costs
    // >= 0) has fl(P / wn) <= fl(S / wn); so once fl(P / wn) >= L.st[1] the candidate's remaining views
    // are not evaluated and P4 skips it. As in the Weak sweep's P5, per view the (candidate, pixel) items
    // still wanted are packed into dense lanes (ballots of LDS state every wave computes alike; a wave
    // takes 64 items of ONE view), batches of whole views (>= SS_P3_CHUNKS chunks, dealt round-robin)
    // end with the fold over the batch's views. Items whose window needs the out-of-line path are
    // evaluated after the batch's item loop (the hot loop holds no call).
    // part / nxt / dead overlay hyp[5..7] (P2b was their last reader).
    float *part = reinterpret_cast<float *>(&L.hyp[5 * VM_P]);   // [5][64]
    uint8_t *nxt = reinterpret_cast<uint8_t *>(part + 5 * VM_P); // [5][64] next view to fold
    uint8_t *dead = nxt + 5 * VM_P;                              // [5][64]
    static_assert(5 * VM_P * (sizeof(float) + 2) <= 3 * VM_P * sizeof(float4), "early-exit state overlays hyp[5..7]");
    for (int i = tid; i < 5 * VM_P; i += VM_BLOCK) { part[i] = 0.0f; nxt[i] = 0; dead[i] = 0; }
    __syncthreads();
    {
        auto view_masks = [&](int v, uint64_t (&m)[5]) {
            const bool base = pv1 && wts[v * VM_P + p1] > 0;
#pragma unroll
            for (int k = 0; k < 5; ++k) m[k] = __ballot(base && !dead[k * VM_P + p1]);
        };
        // item `it` of view v's packing (masks m, prefix offsets off) -> candidate k, pixel slot p
        auto decode = [&](const uint64_t (&m)[5], const int (&off)[6], int it, int &k, int &p) {
            k = 0;
#pragma unroll
            for (int q = 1; q < 5; ++q) k += it >= off[q];
            uint64_t mk = m[0];
            int pk = 0;
#pragma unroll
            for (int q = 1; q < 5; ++q) if (k == q) { mk = m[q]; pk = off[q]; }
            p = nth_set_bit(mk, it - pk);
        };
        for (int v0 = 0; v0 < N;) {
            int v1 = v0, nch = 0;
            while (v1 < N && nch < SS_P3_CHUNKS) {
                uint64_t m[5];
                view_masks(v1, m);
                int t = 0;
#pragma unroll
                for (int k = 0; k < 5; ++k) t += __builtin_popcountll(m[k]);
                nch += (t + WAVE - 1) / WAVE;
                ++v1;
            }
            uint64_t wdef = 0, ldef = 0;  // chunks of this batch with a deferred item: in the wave / this lane's
            int g = 0;                    // chunk index within the batch
            for (int v = v0; v < v1; ++v) {
                uint64_t m[5];
                view_masks(v, m);
                int off[6];
                off[0] = 0;
#pragma unroll
                for (int k = 0; k < 5; ++k) off[k + 1] = off[k] + __builtin_popcountll(m[k]);
                const int nv_items = off[5];
                for (int j = 0; j * WAVE < nv_items; ++j, ++g) {
                    if (g % VM_WAVES != wave) continue;
                    const int it = j * WAVE + lane;
                    const bool want = it < nv_items;
                    int k = 0, p = p1;
                    if (want) decode(m, off, it, k, p);
                    const int xy = L.pxy[p];
                    const int px = xy & 0xFFFF, py = xy >> 16;
                    bool slow = false;
                    if (want) {
                        const RefWinT<VmRefT<F16>> rwq{&L.refw[p], L.rmean[p], L.rvar[p], SA ? &saw[p] : nullptr};
                        const float4 tp = VM_CAND(L)[k * VM_P + p];
                        ++issued;
                        float cv = ncc_old_fast<F16, VM_P>(a, px, py, v + 1, tp, rwq, slow);
                        if (!slow) {
                            if (geom_imp) cv = fmaf(gf, geom_cost(a, px, py, v + 1, tp), cv);
                            costL[(k * N + v) * VM_P + p] = cv;
                        }
                    }
                    if (__ballot(slow)) {
                        wdef |= 1ull << g;
                        if (slow) ldef |= 1ull << g;
                    }
                }
            }
            // this wave's deferred items: find each chunk's view and offset again (wave-uniform walk)
            while (wdef) {
                const int gd = __builtin_ctzll(wdef);
                wdef &= wdef - 1;
                int gg = 0;
                for (int v = v0; v < v1; ++v) {
                    uint64_t m[5];
                    view_masks(v, m);
                    int off[6];
                    off[0] = 0;
#pragma unroll
                    for (int k = 0; k < 5; ++k) off[k + 1] = off[k] + __builtin_popcountll(m[k]);
                    const int nc = (off[5] + WAVE - 1) / WAVE;
                    if (gd < gg + nc) {
                        if ((ldef >> gd) & 1ull) {
                            int k, p;
                            decode(m, off, (gd - gg) * WAVE + lane, k, p);
                            const int xy = L.pxy[p];
                            const int px = xy & 0xFFFF, py = xy >> 16;
                            const float4 tp = VM_CAND(L)[k * VM_P + p];
                            float cv = ncc_old_slow<F16, VmRefT<F16>>(a.self, px, py, v + 1, tp, &L.refw[p], VM_P, L.rmean[p], L.rvar[p]);
                            if (geom_imp) cv = fmaf(gf, geom_cost(a, px, py, v + 1, tp), cv);
                            costL[(k * N + v) * VM_P + p] = cv;
                        }
                        break;
                    }
                    gg += nc;
                }
            }
            __syncthreads();
            // fold views [nxt, v1) of the pixels' 5 slots (all threads: slot i / 64)
            for (int i = tid; i < 5 * VM_P; i += VM_BLOCK) {
                const int k = i / VM_P, p = i - k * VM_P;
                if (dead[i] || p >= np) continue;
                int v = nxt[i];
                float P = part[i];
                for (; v < v1; ++v) {
                    const int wk = wts[v * VM_P + p];
                    if (wk > 0) P = fmaf((float)wk, costL[(k * N + v) * VM_P + p], P);
                }
                nxt[i] = (uint8_t)v;
                part[i] = P;
                if (P / L.st[3 * VM_P + p] >= L.st[1 * VM_P + p]) dead[i] = 1;
            }
            __syncthreads();
            v0 = v1;
        }
    }

    if (a.evals) {  // profiling: one atomic per wave
        uint32_t sum = issued;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o);
        if (lane == 0) atomicAdd(PROF_AT(a.evals, 0), (unsigned long long)sum);
    }

    // ---- P4: weighted candidate costs in view order, acceptance, writes
    if (pv1) {
        const int p = p1, c = c1;
        for (int v = wave; v < N; v += VM_WAVES) a.vw[(size_t)v * a.HW + c] = (uint8_t)wts[v * VM_P + p];
        if (wave == 0) {
            float cost_now = L.st[1 * VM_P + p];
            const float cost_init = L.st[2 * VM_P + p], wn = L.st[3 * VM_P + p];
            float4 pnow = L.pnow[p];
#pragma unroll 1
            for (int k = 0; k < 5; ++k) {
                if (dead[k * VM_P + p]) continue;  // its partial cost already reached cost_now
                const float4 t = VM_CAND(L)[k * VM_P + p];
                // (P3's folds ran this slot's chain fmaf(w_v, c_v, .) over all N views in order; a weight-0
                // view adds fmaf(0, c_v, tc) == tc)
                const float tc = part[k * VM_P + p] / wn;
                const float db = depth_from_plane(cam0, t, px1, py1);
                if (db >= a.dmin && db <= a.dmax && tc < cost_now) { pnow = t; cost_now = tc; }
            }
            if (a.state == APD_REFINE_INIT) {
                if ((double)cost_now < (double)cost_init - 0.1) { a.cost[c] = cost_now; a.plane[c] = pnow; }
                else a.cost[c] = cost_init;
            } else {
                a.cost[c] = cost_now;
                a.plane[c] = pnow;
            }
        }
    }
}

// ---------------------------------------------------------------------------------------------
// View-major Weak sweep (same function as k_sweep_weak). The reference side of
// ComputeBilateralNCCNew -- the anchors' windows (6x6 centre patch, 3x3 anchor patches), their SA
// tap masks and their (sr, srr, wsum) moments -- does not depend on the view or the plane, so it is
// built once per pixel in LDS; each (plane, view) task then only projects and samples the source.
//   P0  per pixel: anchors, hypothesis planes (STRONG anchors + current), fit plane, NCC-New ref data
//   P1  (hypothesis, view) tasks, lane = pixel: NCC-New (+ geometric for the current plane)
//   P2  lane = (pixel, view): view selection, geometric hypothesis terms, argmin + acceptance
//   P3  fit-plane tasks for views with weight > 0
//   P4  lane = pixel: fit acceptance, the 5 refinement candidates (RNG continues from P2)
//   P5  (candidate, view) tasks for views with weight > 0
//   P6  lane = pixel: acceptance, writes
// ---------------------------------------------------------------------------------------------
// NCC-New reference side of a pixel slot (anchors, window taps, SA tap masks, moments): shared by the
// Weak sweep and RandomInitialization under APD
// NWIN: windows held in LDS (9: the centre window and the 8 anchor windows). (Round 4's variant with
// only the centre window in LDS and the anchor windows' reference side read from k_anchor_rec's
// image-wide records at four workgroups per CU measured equal over the whole C3 N = 10 scan --
// profiles/r5_scan_c3_n10_rec_vs_lds.txt -- and +11 % at N = 25, since its record loads scale with the
// evaluations per pixel while this layout builds each window once per pixel; it was retired in round 5.)
// SA = false (no SA masks in the problem): every tap of a window is valid, so the tap masks are
// compile-time constants and their arrays shrink to one element.
template <bool F16, int NWIN = 9, bool SA = true>
struct WvRefT {
    static constexpr int MP = SA ? VM_P : 1;  // per-pixel extent of the SA-only arrays
    uint64_t tmask0[MP];         // SA tap masks
    // per window, the reference side of ncc_finalize over its valid taps, once per pixel instead of
    // once per evaluation: sr / wsum, var_ref -- the same statements (1 / wsum: inv_lut)
    float wsrp[NWIN * VM_P], wvar[NWIN * VM_P];
    int anc[9 * VM_P];           // packed (x, y) of anchors 0..8, -1 = none
    uint32_t flags[VM_P];        // bits 0-7: hypothesis h present (anchor STRONG); 12-15: the current plane is
                                 // hypothesis (bits 12-14) when bit 15; 16-24: window k evaluated
                                 // (anchor present and SA label matches); 25-27: the best anchor
                                 // hypothesis (Weak sweep P2a); 29: the pixel has an SA label (its anchor
                                 // windows are filtered); 31: refine (fit normal != 0)
    // [tap][p]: window 0 taps 0..35 (6x6, step 2), anchor k taps 36+9(k-1).. (3x3, step 5); fp16 when
    // the images are (exactly) fp16-representable, see apd_set_problem
    typename std::conditional<F16, _Float16, float>::type rref[(36 + 9 * (NWIN - 1)) * VM_P];
    uint16_t tmask[(NWIN - 1) * MP];
    uint32_t box[2 * VM_P];      // bounding box of the anchors 0..8 (x0 | y0 << 16, x1 | y1 << 16)
    // 1 / wsum by a window's valid-tap count (wsum is that count: each valid tap adds 1.0f), 0 for an
    // empty window: wv_build_window's IEEE quotients, per workgroup (wv_init_lut) instead of per
    // (pixel, window). Without SA masks wsum is 36 or 9 and the quotient a constant.
    float inv_lut[SA ? 40 : 1];
};
template <bool F16, int NWIN, bool SA>
__device__ __forceinline__ void wv_init_lut(WvRefT<F16, NWIN, SA> &L) {
    if constexpr (SA) {
        const int t = threadIdx.x;
        if (t < 40) L.inv_lut[t] = t ? 1.0f / (float)t : 0.0f;
    }
}
// the Weak sweep's per-workgroup state: the reference side plus the hypotheses and per-pixel state
template <bool F16, int NWIN = 9, bool SA = true>
struct WvLdsT : WvRefT<F16, NWIN, SA> {
    float4 hyp[9 * VM_P];        // [h][p]: anchor planes 1..8 (if STRONG) + current; P4 overwrites [0..4]
                                 // with the refinement candidates (WV_CAND) after P2's last read
    float4 pnow[VM_P];
    float st[4 * VM_P];          // depth_now, cost_now, cost_init, weight norm
    uint32_t tsel[VM_P];         // views with weight > 0 (the selection the best anchor hypothesis brings)
    uint16_t rng_n[VM_P];
    int pxy[VM_P];               // packed (x, y) of pixel slot p (P5's packed items)
};
#define WV_CAND(L) ((L).hyp)
#ifndef WV_P5_CHUNKS
#define WV_P5_CHUNKS 3  // P5 batches: whole views until at least this many 64-item chunks
#endif
// The dynamic part after WvLdsT: the cost table (rows of 64 floats), then [N][64] view weights and
// [N][64] anchor-selection bytes (bit k-1: anchor k selected view v, P2a's priors). Rows: `direct`
// (the pair-table kernels handled every pixel, P2 reads the anchor candidates' costs from their
// buffer) N for the current / fit plane and 5 x min(WV_P5_CHUNKS, N) for one P5 batch (its views
// with items, at most one per chunk); otherwise [9][N] (P1's anchor candidates and the current plane).
__host__ __device__ __forceinline__ int wv_cost_rows(int N, bool direct) {
    const int p5 = 5 * (N < WV_P5_CHUNKS ? N : WV_P5_CHUNKS);
    const int base = direct ? N : 9 * N;
    return base > p5 ? base : p5;
}
#ifndef APD_WV_LDS_PAD
#define APD_WV_LDS_PAD 0  // experiments: extra LDS bytes per workgroup (fewer workgroups per CU)
#endif
template <bool F16, int NWIN, bool SA>
static inline size_t wv_lds_bytes(int N, bool direct = false) {
    return APD_WV_LDS_PAD + sizeof(WvLdsT<F16, NWIN, SA>) + (size_t)wv_cost_rows(N, direct) * VM_P * sizeof(float) +
           (size_t)2 * N * VM_P;
}
// Occupancy: the fp16 instantiations (direct) at N = 10 fit four workgroups per CU (160 KiB of LDS).
static_assert(sizeof(WvLdsT<true, 9, false>) + 15 * VM_P * sizeof(float) + 2 * 10 * VM_P <= 160 * 1024 / 4,
              "k_sweep_weak_vm<fp16, no SA> (direct) at N = 10 must fit four workgroups per CU");
static_assert(sizeof(WvLdsT<true, 9, true>) + 15 * VM_P * sizeof(float) + 2 * 10 * VM_P <= 160 * 1024 / 4,
              "k_sweep_weak_vm<fp16, SA> (direct) at N = 10 must fit four workgroups per CU");
__device__ __forceinline__ int sa_at_dev(const Args &a, int x, int y) {
    const long idx = (long)y * a.W + x;
    if (idx < 0 || idx >= a.HW) return -1;
    return a.sa[idx];
}
#ifndef WV_CENTRE_PIPE
#define WV_CENTRE_PIPE true  // NCC-New's centre window software-pipelined by columns (ncc_new_window PIPE)
#endif
// One NCC-New window of pixel slot p against source view s: taps (ax - 5 + inc*i, ay - 5 + inc*j),
// i outer, j inner, skipping taps outside the SA mask; the reference's moments come from WvLds.
// `fast` = window_rcp_ok for this lane (Newton reciprocal + packed taps); otherwise the IEEE
// statement. Every lane of the wave executes the same instruction stream; lanes that do not need
// this window (`live` false) run on a parked homography and discard the sums.
// Reference taps: tap tk of the window at rb[tk * rs] (WvRefT: &rref[tap0 * VM_P + p], VM_P).
// The IEEE statement of an NCC-New window's taps (lanes whose window fails window_rcp_ok).
template <bool F16, int NW, int INC, class RT>
__device__ __forceinline__ void ncc_new_window_slow(const Args &a, RT rb,
                                                    int rs, uint64_t mask, const Hom &Hm, int ax, int ay, const SrcTex<F16> &Q,
                                                    float &ss, float &sss, float &srs) {
    const float Wm1 = (float)(a.W - 1), Hm1 = (float)(a.H - 1);
    const uint32_t W1 = SrcTex<F16>::pitch(a.W);
#pragma unroll (NW <= 3 ? NW : 1)  // (3x3: rb may be a register array)
    for (int i = 0; i < NW; ++i) {
        const float x = (float)(ax - 5 + INC * i);
        const float cx = fmaf(Hm.h[0], x, Hm.h[2]);
        const float cy = fmaf(Hm.h[3], x, Hm.h[5]);
        const float cz = fmaf(Hm.h[6], x, Hm.h[8]);
#pragma unroll (NW <= 3 ? NW : 1)
        for (int j = 0; j < NW; ++j) {
            const int tk = i * NW + j;
            if (!((mask >> tk) & 1ull)) continue;
            const float y = (float)(ay - 5 + INC * j);
            const float X = fmaf(Hm.h[1], y, cx);
            const float Y = fmaf(Hm.h[4], y, cy);
            const float Z = fmaf(Hm.h[7], y, cz);
            const float iz = 1.0f / Z;
            const QuadTap t = quad_tap(Wm1, Hm1, W1, X * iz, Y * iz);
            const float v = bilerp(Q.fetch(t.idx), t.ax, t.ay);
            const float r = rb[tk * rs];
            ss += v;
            sss = fmaf(v, v, sss);
            srs = fmaf(r, v, srs);
        }
    }
}
// RT: the reference taps' type (LDS, or registers: k_gp_cost's anchor records). PIPE: the centre
// window's columns software-pipelined (more gathers in flight, ~30 more VGPRs)
template <bool F16, int NW, int INC, bool PIPE = true, class RT = const typename std::conditional<F16, _Float16, float>::type *,
          class TT = FastTex<F16, true>>
__device__ __forceinline__ void ncc_new_window(const Args &a, RT rb,
                                               int rs, uint64_t mask, const Hom &Hm, int ax, int ay, bool live,
                                               bool fast, const TT &T, const SrcTex<F16> &Q, float &ss,
                                               float &sss, float &srs) {
    const uint64_t sm = __ballot(live && !fast);
    // only the lanes whose window is evaluated issue its gathers (the gather path's cost is per
    // active lane); the others are exec-masked off instead of sampling a parked homography.
    // TT: FastTex, or FastTexD (pre-differenced fp16 texels, the same values)
    if (live && fast) {
        auto column = [&](int i, typename TT::Tap *t) {
            const float x = (float)(ax - 5 + INC * i);
            const apd_f2 cxy = {fmaf(Hm.h[0], x, Hm.h[2]), fmaf(Hm.h[3], x, Hm.h[5])};
            const float cz = fmaf(Hm.h[6], x, Hm.h[8]);
#pragma unroll
            for (int j = 0; j < NW; ++j) {
                const float y = (float)(ay - 5 + INC * j);
                const apd_f2 XY = pk_fma((apd_f2){Hm.h[1], Hm.h[4]}, (apd_f2){y, y}, cxy);
                t[j] = T.tap(XY, rcp_newton(fmaf(Hm.h[7], y, cz)));
            }
        };
        // taps in (i, j) order, skipping those outside the SA mask
        auto consume = [&](int i, const typename TT::Tap *t, const typename TT::Raw *q) {
#pragma unroll
            for (int j = 0; j < NW; ++j) {
                const int tk = i * NW + j;
                const float v = T.finish(t[j], q[j]);
                if ((mask >> tk) & 1ull) {
                    const float r = rb[tk * rs];
                    ss += v;
                    sss = fmaf(v, v, sss);
                    srs = fmaf(r, v, srs);
                }
            }
        };
        if constexpr (NW <= 3) {
            // an anchor window (3x3): all 9 gathers in flight before the first is consumed
            typename TT::Tap t[NW][NW];
            typename TT::Raw q[NW][NW];
#pragma unroll
            for (int i = 0; i < NW; ++i) column(i, t[i]);
#pragma unroll
            for (int i = 0; i < NW; ++i)
#pragma unroll
                for (int j = 0; j < NW; ++j) q[i][j] = T.load(t[i][j]);
#pragma unroll
            for (int i = 0; i < NW; ++i) consume(i, t[i], q[i]);
        } else if (!PIPE) {
            // the centre window (6x6), one column of gathers at a time (fewer registers live)
#pragma unroll
            for (int i = 0; i < NW; ++i) {
                typename TT::Tap t[NW];
                typename TT::Raw q[NW];
                column(i, t);
#pragma unroll
                for (int j = 0; j < NW; ++j) q[j] = T.load(t[j]);
                consume(i, t, q);
            }
        } else {
            // the centre window (6x6): column i+1's gathers in flight while column i is consumed
            typename TT::Tap ta[NW], tb[NW];
            typename TT::Raw qa[NW], qb[NW];
            column(0, ta);
#pragma unroll
            for (int j = 0; j < NW; ++j) qa[j] = T.load(ta[j]);
#pragma unroll
            for (int i = 0; i < NW; i += 2) {
                if (i + 1 < NW) {
                    column(i + 1, tb);
#pragma unroll
                    for (int j = 0; j < NW; ++j) qb[j] = T.load(tb[j]);
                }
                consume(i, ta, qa);
                if (i + 2 < NW) {
                    column(i + 2, ta);
#pragma unroll
                    for (int j = 0; j < NW; ++j) qa[j] = T.load(ta[j]);
                }
                if (i + 1 < NW) consume(i + 1, tb, qb);
            }
        }
    }
    if (sm && live && !fast) ncc_new_window_slow<F16, NW, INC, RT>(a, rb, rs, mask, Hm, ax, ay, Q, ss, sss, srs);
}


// NCC-New reference side of pixel slot p (APD.cu:448-575): the 9 windows' reference taps, SA tap
// masks and moments; wave w builds windows w, w + nwaves, ... (tap order = the reference's). Each
// window's taps (and SA labels) are all loaded before the in-order moment sums, so a window costs one
// memory round trip instead of one per tap.
template <bool F16, int N1, int INC, int NWIN, bool SA>
__device__ __forceinline__ void wv_build_window(const Args &a, WvRefT<F16, NWIN, SA> &L, int p1, int k, int ax, int ay,
                                                bool use_sa, int cid) {
    constexpr int NT = N1 * N1;
    const int tap0 = (k == 0) ? 0 : 36 + 9 * (k - 1);
    // branch-free loads (clamped addresses; sa_at_dev's out-of-image -1 never equals a label cid > 0)
    float r[NT];
    bool in[NT];
#pragma unroll
    for (int tk = 0; tk < NT; ++tk) {
        const int i = tk / N1, j = tk - N1 * (tk / N1);
        const int rx = ax - 5 + INC * i, ry = ay - 5 + INC * j;
        r[tk] = tex_ref(a, rx, ry);
        in[tk] = true;
    }
    if (SA && a.sa_any) {
#pragma unroll
        for (int tk = 0; tk < NT; ++tk) {
            const int i = tk / N1, j = tk - N1 * (tk / N1);
            const long idx = (long)(ay - 5 + INC * j) * a.W + (ax - 5 + INC * i);
            const bool inb = idx >= 0 && idx < a.HW;
            const int lab = a.sa[inb ? idx : 0];
            in[tk] = !use_sa || (inb && lab == cid);
        }
    }
    float sr = 0.0f, srr = 0.0f, ws = 0.0f;
    uint64_t mask = 0;
#pragma unroll
    for (int tk = 0; tk < NT; ++tk) {
        if (!in[tk]) {
            L.rref[(tap0 + tk) * VM_P + p1] = 0.0f;
            continue;
        }
        L.rref[(tap0 + tk) * VM_P + p1] = r[tk];
        mask |= 1ull << tk;
        sr += r[tk];
        srr = fmaf(r[tk], r[tk], srr);
        ws += 1.0f;
    }
    // (ncc_finalize's reference-side statements: inv = 1 / wsum, sr *= inv, srr *= inv, var_ref)
    const float inv = 1.0f / ws, srp = sr * inv, srrp = srr * inv;
    L.wsrp[k * VM_P + p1] = srp;
    L.wvar[k * VM_P + p1] = fmaf(-srp, srp, srrp);
    if constexpr (SA) {
        if (k == 0) L.tmask0[p1] = mask;
        else L.tmask[(k - 1) * VM_P + p1] = (uint16_t)mask;
    }
}
template <bool F16, int NWIN, bool SA>
__device__ __forceinline__ void wv_build_windows(const Args &a, WvRefT<F16, NWIN, SA> &L, int p, const APD_G short2 *anc, int cid,
                                                 int wave, int nwaves) {
    const bool use_sa = cid != 0;
    for (int k = wave; k < NWIN; k += nwaves) {
        const short2 ap = anc[k];
        if (ap.x == -1 || ap.y == -1) continue;
        if (k == 0) wv_build_window<F16, 6, 2, NWIN>(a, L, p, k, ap.x, ap.y, use_sa, cid);
        else wv_build_window<F16, 3, 5, NWIN>(a, L, p, k, ap.x, ap.y, use_sa, cid);
    }
}

// Anchor-window reference records: the reference side of an anchor window (k >= 1: 3x3 taps, step 5,
// APD.cu:500-575) depends only on the anchor q and on whether it is SA-filtered -- by the pixel's
// label, which for a used window is q's own (APD.cu:493-497) -- so it is built once per pixel q of
// the image, in wv_build_window's statements: record [0] unfiltered, [1] filtered by q's label.
// F16: 2 x uint4 = {taps 0..7 (fp16)}, {tap 8 | tap mask << 16, inv, srp, var}; fp32: 4 x uint4 =
// {taps 0..3}, {taps 4..7}, {tap 8, mask, inv, srp}, {var, -, -, -}.
template <bool F16> struct AncRec { static constexpr int U4 = F16 ? 2 : 4; };
__device__ __forceinline__ size_t anc_rec_index(const Args &a, int q, int filt, int u4) {
    return ((size_t)q * (a.sa_any ? 2 : 1) + (size_t)filt) * (size_t)u4;
}
template <bool F16>
__global__ __launch_bounds__(BLOCK) void k_anchor_rec(Args a, uint4 *__restrict__ out) {
    const int q = blockIdx.x * BLOCK + threadIdx.x;
    if (q >= a.HW) return;
    const int qy = q / a.W, qx = q - qy * a.W;
    float r[9];
#pragma unroll
    for (int tk = 0; tk < 9; ++tk) r[tk] = tex_ref(a, qx - 5 + 5 * (tk / 3), qy - 5 + 5 * (tk % 3));
    const int nvar = a.sa_any ? 2 : 1;
    for (int filt = 0; filt < nvar; ++filt) {
        const int cid = filt ? (int)a.sa[q] : 0;
        bool in[9];
#pragma unroll
        for (int tk = 0; tk < 9; ++tk) {
            in[tk] = true;
            if (filt) {
                const long idx = (long)(qy - 5 + 5 * (tk % 3)) * a.W + (qx - 5 + 5 * (tk / 3));
                const bool inb = idx >= 0 && idx < a.HW;
                const int lab = a.sa[inb ? idx : 0];
                in[tk] = cid == 0 || (inb && lab == cid);
            }
        }
        float sr = 0.0f, srr = 0.0f, ws = 0.0f, rv[9];
        uint32_t mask = 0;
#pragma unroll
        for (int tk = 0; tk < 9; ++tk) {
            rv[tk] = 0.0f;
            if (!in[tk]) continue;
            rv[tk] = r[tk];
            mask |= 1u << tk;
            sr += r[tk];
            srr = fmaf(r[tk], r[tk], srr);
            ws += 1.0f;
        }
        const float inv = 1.0f / ws, srp = sr * inv, srrp = srr * inv;
        const float winv = ws != 0.0f ? inv : 0.0f, wvar = fmaf(-srp, srp, srrp);
        uint4 *o = out + anc_rec_index(a, q, filt, AncRec<F16>::U4);
        if constexpr (F16) {
            uint32_t h[5];
#pragma unroll
            for (int i = 0; i < 5; ++i) {
                const _Float16 lo = (_Float16)rv[2 * i];
                const _Float16 hi = (i < 4) ? (_Float16)rv[2 * i + 1] : (_Float16)0.0f;
                h[i] = (uint32_t)__builtin_bit_cast(uint16_t, lo) | ((uint32_t)__builtin_bit_cast(uint16_t, hi) << 16);
            }
            o[0] = make_uint4(h[0], h[1], h[2], h[3]);
            o[1] = make_uint4((h[4] & 0xFFFFu) | (mask << 16), __float_as_uint(winv), __float_as_uint(srp), __float_as_uint(wvar));
        } else {
            o[0] = make_uint4(__float_as_uint(rv[0]), __float_as_uint(rv[1]), __float_as_uint(rv[2]), __float_as_uint(rv[3]));
            o[1] = make_uint4(__float_as_uint(rv[4]), __float_as_uint(rv[5]), __float_as_uint(rv[6]), __float_as_uint(rv[7]));
            o[2] = make_uint4(__float_as_uint(rv[8]), mask, __float_as_uint(winv), __float_as_uint(srp));
            o[3] = make_uint4(__float_as_uint(wvar), 0u, 0u, 0u);
        }
    }
}
// one record in registers, packed as loaded; r[tk] is tap tk (the reference-tap accessor of
// ncc_new_window: rb[tk * rs] with rs = 1)
template <bool F16>
struct AncRecV {
    uint4 u[AncRec<F16>::U4];
    __device__ __forceinline__ static uint32_t comp(const uint4 &v, int i) {
        return i == 0 ? v.x : i == 1 ? v.y : i == 2 ? v.z : v.w;
    }
    __device__ __forceinline__ float operator[](int tk) const {  // (tk a compile-time constant after unrolling)
        if constexpr (F16) {
            const uint32_t h = tk < 8 ? comp(u[0], tk >> 1) : u[1].x;
            return (float)__builtin_bit_cast(_Float16, (uint16_t)(h >> (16 * (tk & 1))));
        } else {
            return __uint_as_float(tk < 4 ? comp(u[0], tk) : tk < 8 ? comp(u[1], tk - 4) : u[2].x);
        }
    }
    __device__ __forceinline__ uint32_t mask() const { return F16 ? (u[1].x >> 16) : u[2].y; }
    __device__ __forceinline__ float inv() const { return __uint_as_float(F16 ? u[1].y : u[2].z); }
    __device__ __forceinline__ float srp() const { return __uint_as_float(F16 ? u[1].z : u[2].w); }
    __device__ __forceinline__ float var() const { return __uint_as_float(F16 ? u[1].w : u[3].x); }
};
template <bool F16>
__device__ __forceinline__ AncRecV<F16> load_anc_rec(const Args &a, int q, int filt) {
    const APD_G uint4 *src = a.arec + anc_rec_index(a, q, filt, AncRec<F16>::U4);
    AncRecV<F16> R;
#pragma unroll
    for (int i = 0; i < AncRec<F16>::U4; ++i) R.u[i] = src[i];
    return R;
}

// ComputeBilateralNCCNew + Softmax focal weighting (APD.cu:448-593, 431-446) for pixel slot p, source
// view s, plane pl, with the reference side from WvLds. Called by every lane of the wave (converged);
// `want` = the lane evaluates this task. Same operations, in the same order, as ncc_new. `seldep`
// (optional) is set when the result read an anchor's selected views (a window anchor projected out
// of the source image, APD.cu:510-520), the one input the Strong sweep changes between launches.
// SA = false: no SA masks in this problem, so every window's tap mask is full (compile-time constant:
// no per-tap mask selects). BOX: L.box holds the pixel's anchor bounding box, and one
// window_rcp_ok_box over it (taps included) stands for the per-window checks when it holds.
// PIPE: the centre window's columns software-pipelined (ncc_new_window).
template <bool F16, bool SA = true, bool BOX = false, int NWIN, bool PIPE = WV_CENTRE_PIPE>
__device__ __forceinline__ float ncc_new_vm(const Args &a, const WvRefT<F16, NWIN, SA> &L, int p, int px, int py, int s, float4 pl,
                                            bool want, bool *seldep = nullptr, uint32_t *nwc = nullptr,
                                            uint32_t *nwa = nullptr) {
    using TT = FastTex<F16, true>;  // (FastTexD measured 9 % slower in the Weak sweep: twice the texel footprint)
    const int W = a.W, H = a.H;
    const Hom Hm = homography(a, s, pl);
    float ptx, pty;
    project(Hm, (float)px, (float)py, ptx, pty);
    bool alive = want && !(ptx >= (float)W || ptx < 0.0f || pty >= (float)H || pty < 0.0f);
    const TT T(a, s);
    const SrcTex<F16> Q(a, s);
    const uint32_t awin = (L.flags[p] >> 16) & 0x1FFu;
    float sc[9];
    int ns = 0;
    float center_cost = 0.0f, strong_weight = 0.0f;
    bool dead = !alive;  // COST_MAX (centre or centre-anchor projected out of the image)
    bool box_ok = false;
    if constexpr (BOX) {
        const uint32_t b0 = L.box[p], b1 = L.box[VM_P + p];
        box_ok = alive && window_rcp_ok_box(Hm, (float)((int)(b0 & 0xFFFFu) - 5), (float)((int)(b0 >> 16) - 5),
                                            (float)((int)(b1 & 0xFFFFu) + 5), (float)((int)(b1 >> 16) + 5));
    }
#pragma unroll 1
    for (int k = 0; k < 9; ++k) {
        const int pk = L.anc[k * VM_P + p];
        const bool has = alive && pk >= 0 && ((awin >> k) & 1u);
#ifdef APD_ABLATE_ANCHOR_LOCAL  // timing-only (wrong values): anchor windows k >= 1 next to the pixel
        const int ax = has ? (k == 0 ? (pk & 0xFFFF) : min(max(px + 6 * (((k - 1) % 3) - 1), 0), W - 1)) : px;
        const int ay = has ? (k == 0 ? (pk >> 16) : min(max(py + 6 * (((k - 1) / 3) - 1), 0), H - 1)) : py;
#else
        const int ax = has ? (pk & 0xFFFF) : px, ay = has ? (pk >> 16) : py;
#endif
        bool live = has;
        if (has) {
            float asx, asy;
            if constexpr (BOX) {
                // the anchor lies in the proven box: rcp_newton(Z) is the correctly rounded 1 / Z there,
                // so X * it is project()'s value without the IEEE division (lanes outside the proof
                // take the division)
                const float X = fmaf(Hm.h[1], (float)ay, fmaf(Hm.h[0], (float)ax, Hm.h[2]));
                const float Y = fmaf(Hm.h[4], (float)ay, fmaf(Hm.h[3], (float)ax, Hm.h[5]));
                const float Z = fmaf(Hm.h[7], (float)ay, fmaf(Hm.h[6], (float)ax, Hm.h[8]));
                float iz = rcp_newton(Z);
                if (__builtin_amdgcn_ballot_w64(!box_ok)) {
                    const float q = 1.0f / Z;
                    if (!box_ok) iz = q;
                }
                asx = X * iz;
                asy = Y * iz;
            } else {
                project(Hm, (float)ax, (float)ay, asx, asy);
            }
            if (asx < 0 || asy < 0 || asx >= (float)W || asy >= (float)H) {
                live = false;
                if (k != 0) {
                    if (seldep) *seldep = true;
                    if ((a.sel[ax + ay * W] >> (s - 1)) & 1u) {
#pragma unroll
                        for (int t = 0; t < 9; ++t) if (t == ns) sc[t] = APD_COST_MAX;
                        ns++;
                        strong_weight += 1.0f;
                    }
                } else {
                    dead = true;
                    alive = false;
                }
            }
        }
        if (!__ballot(live)) continue;
        bool fast = live && box_ok;
        if (!BOX || __ballot(live && !box_ok))
            if (live && !box_ok) fast = window_rcp_ok(Hm, (float)(ax - 5), (float)(ay - 5));
        float ss = 0.0f, sss = 0.0f, srs = 0.0f;
        float inv, srp, var;
        if (k == 0) {
            uint64_t m0 = ~0ull;
            if constexpr (SA) m0 = L.tmask0[p];
            ncc_new_window<F16, 6, 2, PIPE>(a, &L.rref[p], VM_P, m0, Hm, ax, ay, live, fast, T, Q, ss, sss, srs);
            inv = 1.0f / 36.0f;  // (wv_build_window's 1 / wsum over the 36 taps)
            if constexpr (SA) inv = L.inv_lut[__builtin_popcountll(m0)];
            srp = L.wsrp[p]; var = L.wvar[p];
        } else {
            uint64_t mk = 0x1FFull;
            if constexpr (SA) mk = L.tmask[(k - 1) * VM_P + p];
            ncc_new_window<F16, 3, 5>(a, &L.rref[(36 + 9 * (k - 1)) * VM_P + p], VM_P, mk, Hm, ax, ay, live, fast, T, Q, ss, sss, srs);
            inv = 1.0f / 9.0f;
            if constexpr (SA) inv = L.inv_lut[__builtin_popcount((uint32_t)mk)];
            srp = L.wsrp[k * VM_P + p]; var = L.wvar[k * VM_P + p];
        }
        if (!live) continue;
        if (nwc) { if (k == 0) ++*nwc; else ++*nwa; }  // (profiling: windows evaluated)
        if (inv == 0.0f) continue;  // (empty window)
        const float c = ncc_finalize_pre(inv, srp, var, ss, sss, srs);
        if (k == 0) {
            center_cost = c;
        } else {
#pragma unroll
            for (int t = 0; t < 9; ++t) if (t == ns) sc[t] = c;
            ns++;
            strong_weight += 1.0f;
        }
    }
    if (dead) return APD_COST_MAX;
    if (strong_weight <= 1e-6f) return center_cost;
    float mx = -1e10f;
#pragma unroll
    for (int t = 0; t < 9; ++t) if (t < ns && sc[t] > mx) mx = sc[t];
    float e[9];
    float sum = 0.0f;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
        if (t < ns) { e[t] = d_expf(sc[t] - mx); sum += e[t]; }
    }
    float acc = 0.0f;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
        if (t < ns) { float w = e[t] / sum; acc = fmaf(w, sc[t], acc); }
    }
    acc = (acc > APD_COST_MAX) ? APD_COST_MAX : acc;
    return (float)(0.25 * (double)center_cost + 0.75 * (double)acc);
}

// Occupancy: the fp16 instantiations at four workgroups per CU -- at N = 10 38.6 KiB of LDS without
// SA masks, 39.3 KiB with them -- and 128 VGPRs, with the centre window unpipelined (the pipelined
// window needs ~30 more registers and is worth < 1 % at three per CU, profiles/r5_ab_centre_pipe.txt);
// the fp32-texel ones at three. WV_LDS_OCC overrides both (experiments).
#ifndef WV_WAVES
#define WV_WAVES 4  // waves per Weak-sweep workgroup (64 pixels)
#endif
#ifndef WV_CUR_MATCH
#define WV_CUR_MATCH 1  // P1b takes the current plane's costs from P2a when it is an anchor candidate's plane
#endif
#ifndef WV_P2_GEOM_BATCH
// P2a's 8 geometric terms with their gathers batched (1) or one at a time (0): batched was -0.7 % at
// three workgroups per CU, one at a time is -0.3 % at four (profiles/r5_ab_sa_occ4.txt, r5_ab_kept_lanes.txt)
#define WV_P2_GEOM_BATCH 0
#endif
#define WV_BLOCK (WV_WAVES * WAVE)
template <bool F16, bool SA> struct WvOcc {
#ifdef WV_LDS_OCC
    static constexpr int occ = WV_LDS_OCC;
#else
    static constexpr int occ = F16 ? 4 : 3;  // workgroups per CU the registers are bounded for
#endif
    static constexpr bool pipe = occ < 4 && WV_CENTRE_PIPE;
};
template <bool F16, bool SA>
__global__ __launch_bounds__(WV_BLOCK, (WvOcc<F16, SA>::occ)) void k_sweep_weak_vm(Args a, const int *__restrict__ list, int count,
                                                                int iter, const float *__restrict__ cand, int wc) {
    const int N = a.N, W = a.W;
    constexpr bool PIPE = WvOcc<F16, SA>::pipe;
    PHASE_BEGIN;
    // direct: the pair-table kernels evaluated every pixel's anchor candidates, so P2 reads their
    // costs from `cand`; without them (cand == nullptr: APD_NO_CAND_PAIRS=1 or a pair table that does
    // not fit) P1 evaluates the candidates here (the cost table's rows: wv_cost_rows)
    const bool direct = cand != nullptr;
    WvLdsT<F16, 9, SA> &L = *reinterpret_cast<WvLdsT<F16, 9, SA> *>(apd_dyn_lds);
    wv_init_lut(L);  // (read after P0's barrier)
    float *costL = reinterpret_cast<float *>(&L + 1);
    uint8_t *wts = reinterpret_cast<uint8_t *>(costL + wv_cost_rows(N, direct) * VM_P);  // [N][64] view weights
    uint8_t *asl = wts + N * VM_P;  // [N][64] anchor-selection bytes (bit k-1: anchor k selected view v)
    const int VB = min(WV_P5_CHUNKS, N);  // views with items per P5 batch at most
    const int blk = xcd_remap(blockIdx.x, gridDim.x);
    const int first = blk * VM_P;
    const int np = min(VM_P, count - first);
    const int tid = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & (WAVE - 1);
    const APD_C Cam &cam0 = a.cams[0];
    const bool geom = a.geom != 0;
    const float gf = a.gf;
    const int p1 = lane;
    const bool pv1 = p1 < np;
    const int c1 = list[first + min(p1, np - 1)];
    const int py1 = c1 / W, px1 = c1 - py1 * W;

    // ---- P0: anchors, planes, NCC-New reference data
    if (pv1) {
        const APD_G short2 *anc = a.anchors + (size_t)a.amap[c1] * 9;
        const int cid = a.sa_any ? a.sa[c1] : 0;
        const bool use_sa = cid != 0;
        if (wave == 0) {
            // loads in three rounds (anchors; their labels and states; the STRONG anchors' planes)
            uint32_t hflag = 0, awin = 0;
            // (branch-free: absent anchors read the pixel's own entries, which are ignored)
            short2 ap[9];
#pragma unroll
            for (int k = 0; k < 9; ++k) ap[k] = anc[k];
            int lab[9], qk[9];
            uint8_t st[9];
            uint32_t sl[9];
#pragma unroll
            for (int k = 0; k < 9; ++k) {
                const bool ok = !(ap[k].x == -1 || ap[k].y == -1);
                qk[k] = ok ? ap[k].x + ap[k].y * W : c1;  // anchors are in-image pixels
                lab[k] = a.sa_any ? (int)a.sa[qk[k]] : cid;
                st[k] = a.weak[qk[k]];
                sl[k] = a.sel[qk[k]];
            }
            for (int v = 0; v < N; ++v) {
                uint32_t b = 0;
#pragma unroll
                for (int k = 1; k < 9; ++k) b |= ((sl[k] >> v) & 1u) << (k - 1);
                asl[v * VM_P + p1] = (uint8_t)b;
            }
            float4 hp[9];
#pragma unroll
            for (int k = 1; k < 9; ++k) hp[k] = a.plane[st[k] == APD_STRONG ? qk[k] : c1];
            const float4 cur = a.plane[c1];
#pragma unroll
            for (int k = 0; k < 9; ++k) {
                const bool ok = !(ap[k].x == -1 || ap[k].y == -1);
                L.anc[k * VM_P + p1] = ok ? ((int)(uint16_t)ap[k].x | ((int)ap[k].y << 16)) : -1;
                if (ok && !(use_sa && lab[k] != cid)) awin |= 1u << k;
                if (k >= 1 && ok && st[k] == APD_STRONG) {  // (st of an absent anchor is the pixel's own: WEAK)
                    hflag |= 1u << (k - 1);
                    L.hyp[(k - 1) * VM_P + p1] = hp[k];
                }
            }
            // the current plane bitwise equal to STRONG anchor k's (a pixel keeps the anchor hypothesis
            // it took while neither plane changes): its NCC-New and geometric terms are anchor candidate
            // k - 1's, which P2a holds -- flags bit 15 + (k - 1) << 12, the first such k (WV_CUR_MATCH)
            uint32_t cmatch = 0;
#pragma unroll
            for (int k = 8; k >= 1; --k)
                if (WV_CUR_MATCH && ((hflag >> (k - 1)) & 1u) && __float_as_uint(hp[k].x) == __float_as_uint(cur.x) &&
                    __float_as_uint(hp[k].y) == __float_as_uint(cur.y) && __float_as_uint(hp[k].z) == __float_as_uint(cur.z) &&
                    __float_as_uint(hp[k].w) == __float_as_uint(cur.w))
                    cmatch = (1u << 15) | ((uint32_t)(k - 1) << 12);
            L.flags[p1] = hflag | cmatch | (awin << 16) | (use_sa ? (1u << 29) : 0u);
            LANE_STAT(0, true);         // (instrumented builds: pixels, and those whose current plane
            LANE_STAT(2, cmatch != 0);  //  is an anchor candidate's)
#ifdef APD_PHASE_STAMPS
            {  // (instrumented builds: the fit plane equal to the current plane / to an anchor candidate's)
                const float4 ft = a.fit[c1];
                auto same = [](float4 u, float4 w) {
                    return __float_as_uint(u.x) == __float_as_uint(w.x) && __float_as_uint(u.y) == __float_as_uint(w.y) &&
                           __float_as_uint(u.z) == __float_as_uint(w.z) && __float_as_uint(u.w) == __float_as_uint(w.w);
                };
                bool fc = false;
#pragma unroll
                for (int k = 1; k < 9; ++k) fc = fc || (((hflag >> (k - 1)) & 1u) && same(hp[k], ft));
                const bool has_fit = !(ft.x == 0 && ft.y == 0 && ft.z == 0);
                LANE_STAT(4, has_fit && same(ft, cur));
                LANE_STAT(6, has_fit && fc);
            }
#endif
            L.hyp[8 * VM_P + p1] = cur;
            L.pxy[p1] = px1 | (py1 << 16);
            int bx0 = px1, by0 = py1, bx1 = px1, by1 = py1;  // anchors' bounding box (+ the pixel)
#pragma unroll
            for (int k = 0; k < 9; ++k) {
                if (ap[k].x == -1 || ap[k].y == -1) continue;
                bx0 = min(bx0, (int)ap[k].x); bx1 = max(bx1, (int)ap[k].x);
                by0 = min(by0, (int)ap[k].y); by1 = max(by1, (int)ap[k].y);
            }
            L.box[p1] = (uint32_t)bx0 | ((uint32_t)by0 << 16);
            L.box[VM_P + p1] = (uint32_t)bx1 | ((uint32_t)by1 << 16);
        }
        wv_build_windows<F16>(a, L, p1, anc, cid, wave, WV_WAVES);
    }
    __syncthreads();
    PHASE_STAMP(0);

    // ---- P1 (not direct): (anchor hypothesis, view) tasks, lane = pixel. The current plane is
    // evaluated after the view selection (P1b), for the views it weights only: cost_now = sum of
    // fmaf(w_v, c_v) over all views, and a weight-0 view adds fmaf(0, c_v, .) == the sum itself (c_v
    // finite), so its value is never needed.
    uint32_t nwc = 0, nwa = 0;  // profiling: centre / anchor windows this lane evaluated
    const int ntask = direct ? 0 : 8 * N;
    for (int u = wave; u < ntask; u += WV_WAVES) {  // view-major: the waves share a source image
        const int v = u / 8, h = u - 8 * v, t = h * N + v;
        float val = (h == 0 && v == 0) ? 2.0f : 0.0f;
        const bool want = pv1 && ((L.flags[p1] >> h) & 1u);
        const float4 pl = L.hyp[h * VM_P + p1];
        const float nv = ncc_new_vm<F16, SA, true, 9, PIPE>(a, L, p1, px1, py1, v + 1, pl, want, nullptr, &nwc, &nwa);
        if (want) val = nv;
        costL[t * VM_P + p1] = val;
    }
    __syncthreads();
    PHASE_STAMP(1);

    // ---- P2a: lane = (pixel, view) groups: view selection, the anchor hypotheses' weighted costs
    // (with their geometric terms) and their argmin
    const int Gp = WAVE / N;
    const int ppr = WV_WAVES * Gp;
    for (int r0 = 0; r0 < np; r0 += ppr) {
        int g = lane / N;
        const bool lane_ok = g < Gp;
        int v = lane - g * N;
        if (!lane_ok) { g = 0; v = (lane - Gp * N) % N; }
        Group G;
        G.v = v; G.base = g * N; G.slot = g; G.li = 0;
        G.gmask = (N >= 64) ? ~0ull : ((1ull << N) - 1ull);
        const int pr = r0 + wave * Gp + g;
        G.valid = lane_ok && pr < np;
        const int p = min(pr, np - 1);
        const int c = list[first + p];
        const int py = c / W, px = c - py * W;
        const uint32_t hflag = L.flags[p] & 0x1FFu;
        float prior = 0.0f;
        const uint32_t asv = asl[v * VM_P + p];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int pk = L.anc[(i + 1) * VM_P + p];  // anchor i+1's pixel, if any
            if (pk >= 0) prior += ((asv >> i) & 1u) ? 0.9f : 0.1f;
        }
        float ca[8];
        if (direct) {  // the candidates' costs from the pair-table kernels; absent ones as P1 sets them
            const size_t wi = (size_t)a.amap[c];
#pragma unroll
            for (int h = 0; h < 8; ++h)
                ca[h] = ((hflag >> h) & 1u) ? cand[((size_t)v * 8 + h) * (size_t)wc + wi] : ((h == 0 && v == 0) ? 2.0f : 0.0f);
        } else {
#pragma unroll
            for (int h = 0; h < 8; ++h) ca[h] = costL[(h * N + v) * VM_P + p];
        }
        Rng rg(a.seed_lo, a.seed_hi, (uint32_t)c, ord_weak(iter));
        const int w = view_selection(ca, prior, iter, rg, G, N);
        const uint32_t tsel = group_bits(w > 0, G);
        float gval[8];
#ifdef APD_PHASE_STAMPS
        const long long tg0_ = clock64();
#endif
#if WV_P2_GEOM_BATCH
        // the 8 geometric terms with their source-depth gathers all in flight before the first is
        // consumed (geom_head / geom_tail: the same statements as geom_cost)
        if (geom && w > 0) {
            GeomHead gh[8];
            float sdep[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                float P[3];
                geom_point(a, px, py, L.hyp[j * VM_P + p], P);
                gh[j] = geom_head(a, v + 1, P);
            }
#pragma unroll
            for (int j = 0; j < 8; ++j) sdep[j] = ((hflag >> j) & 1u) ? a.depth[gh[j].idx] : 0.0f;
#pragma unroll
            for (int j = 0; j < 8; ++j)
                gval[j] = ((hflag >> j) & 1u) ? fmaf(gf, geom_tail(a, px, py, v + 1, gh[j], sdep[j]), ca[j]) : fmaf(gf, 3.0f, ca[j]);
        } else {
#pragma unroll
            for (int j = 0; j < 8; ++j) gval[j] = ca[j];
        }
#else
        // the candidates' world points (geom_point: depth_from_plane and world_point, view-independent)
        // once per (pixel, candidate) instead of once per (pixel, view, candidate): with N >= 8 view
        // lanes per pixel, lane v computes candidate v's and the group's lanes read it by shuffle --
        // the same statements on the same inputs, so the same bits
        const bool share_p = geom && N >= 8;
        float Pv[3] = {0.0f, 0.0f, 0.0f};
        if (share_p && v < 8) geom_point(a, px, py, L.hyp[v * VM_P + p], Pv);
#pragma unroll 1
        for (int j = 0; j < 8; ++j) {
            float cj = ca[0];
#pragma unroll
            for (int k = 1; k < 8; ++k) if (j == k) cj = ca[k];
            float vv = cj;
            float P[3];
            if (share_p) {
                P[0] = __shfl(Pv[0], G.base + j);
                P[1] = __shfl(Pv[1], G.base + j);
                P[2] = __shfl(Pv[2], G.base + j);
            }
            if (geom && w > 0) {
                if (!share_p) geom_point(a, px, py, L.hyp[j * VM_P + p], P);
                vv = ((hflag >> j) & 1u) ? fmaf(gf, geom_cost_p(a, px, py, v + 1, P), cj) : fmaf(gf, 3.0f, cj);
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) if (j == k) gval[k] = vv;
        }
#endif
#ifdef APD_PHASE_STAMPS
        if (a.evals && threadIdx.x == 0) atomicAdd(PROF_AT(a.evals, APD_INSTR + 8 + 7), (unsigned long long)(clock64() - tg0_));
#endif
        // the current plane is anchor candidate m's: P1b's cost for this view (its NCC-New + geometric
        // term, 0 for a view without weight) is gval[m], the same statements on the same inputs
        const uint32_t flp = L.flags[p];
        if (WV_CUR_MATCH && ((flp >> 15) & 1u)) {
            const int m = (int)((flp >> 12) & 7u);
            float gm = gval[0];
#pragma unroll
            for (int k = 1; k < 8; ++k) if (m == k) gm = gval[k];
            if (G.valid) costL[((direct ? 0 : 8 * N) + v) * VM_P + p] = w > 0 ? gm : 0.0f;
        }
        float fc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        float wn = 0.0f;
        for (int k = 0; k < N; ++k) {
            const int wk = __shfl(w, G.base + k);
            const float fwk = (float)wk;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float vk = __shfl(gval[j], G.base + k);
                if (wk > 0) fc[j] = fmaf(fwk, vk, fc[j]);
            }
            if (wk > 0) wn += fwk;
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) fc[j] /= wn;
        int mi = 0;
        float fcm = fc[0];
#pragma unroll
        for (int j = 1; j < 8; ++j) if (fc[j] <= fcm) { fcm = fc[j]; mi = j; }
        if (G.valid) {
            wts[v * VM_P + p] = (uint8_t)w;
            if (G.v == 0) {
                const float4 fit = a.fit[c];
                L.st[2 * VM_P + p] = fcm;  // (P1c: the argmin's weighted cost, then cost_init)
                L.st[3 * VM_P + p] = wn;
                L.tsel[p] = tsel;
                uint32_t fl = (L.flags[p] & ~(7u << 25)) | ((uint32_t)mi << 25);
                if (!(fit.x == 0 && fit.y == 0 && fit.z == 0)) fl |= 1u << 31;
                L.flags[p] = fl;
                L.rng_n[p] = (uint16_t)rg.n;  // a few dozen draws
            }
        }
    }
    __syncthreads();

    PHASE_STAMP(22);  // (instrumented builds: P2a apart from P1b + P1c)
    // ---- P1b: current-plane tasks, lane = pixel, for the views with weight > 0
    const int cur_row = direct ? 0 : 8 * N;
    const bool cur_shared = WV_CUR_MATCH && pv1 && ((L.flags[p1] >> 15) & 1u);  // (P2a wrote its row)
    for (int v = wave; v < N; v += WV_WAVES) {
        float val = 0.0f;
        const bool want = pv1 && wts[v * VM_P + p1] > 0 && !cur_shared;
        LANE_STAT(24, want);
        if (__ballot(want)) {
            const float4 pl = L.hyp[8 * VM_P + p1];
            // iteration 0: the current plane is RandomInitialization's, whose NCC-New it kept (a.wcur)
            // unless the value read a selected view (NaN); only the lanes lacking it evaluate
            const float kept = (iter == 0 && a.wcur && want) ? a.wcur[(size_t)v * a.HW + c1] : __int_as_float(0x7fc00000);
            const bool eval = want && __builtin_isnan(kept);
            float nv = kept;
            if (__ballot(eval)) {
                const float e = ncc_new_vm<F16, SA, true, 9, PIPE>(a, L, p1, px1, py1, v + 1, pl, eval, nullptr, &nwc, &nwa);
                if (eval) nv = e;
            }
            if (want) {
                val = nv;
                if (geom) val = fmaf(gf, geom_cost(a, px1, py1, v + 1, pl), val);
            }
        }
        if (!cur_shared) costL[(cur_row + v) * VM_P + p1] = val;
    }
    __syncthreads();

    // ---- P1c: lane = pixel (wave 0): the current plane's cost, acceptance of the best anchor hypothesis
    if (wave == 0 && pv1) {
        const float wn = L.st[3 * VM_P + p1];
        float cost_now = 0.0f;
        for (int k = 0; k < N; ++k) {
            const int wk = wts[k * VM_P + p1];
            if (wk > 0) cost_now = fmaf((float)wk, costL[(cur_row + k) * VM_P + p1], cost_now);
        }
        cost_now /= wn;
        const float cost_init = cost_now;
        const int mi = (int)((L.flags[p1] >> 25) & 7u);
        const float fcm = L.st[2 * VM_P + p1];
        const float4 cur = L.hyp[8 * VM_P + p1];
        float depth_now = depth_from_plane(cam0, cur, px1, py1);
        float4 pnow = cur;
        bool taken = false;
        if ((L.flags[p1] >> mi) & 1u) {
            const float4 cnd = L.hyp[mi * VM_P + p1];
            const float db = depth_from_plane(cam0, cnd, px1, py1);
            if (db >= a.dmin && db <= a.dmax && fcm < cost_now) {
                depth_now = db; pnow = cnd; cost_now = fcm;
                a.sel[c1] = L.tsel[p1];
                taken = true;
            }
        }
        LANE_STAT(16, taken);  // (instrumented builds: pixels that take the best anchor hypothesis)
        L.pnow[p1] = pnow;
        L.st[0 * VM_P + p1] = depth_now;
        L.st[1 * VM_P + p1] = cost_now;
        L.st[2 * VM_P + p1] = cost_init;
    }
    __syncthreads();
    PHASE_STAMP(2);
    const bool refine = pv1 && (L.flags[p1] >> 31) != 0u;
    const float4 fit1 = a.fit[c1];
    uint32_t issued_nn = 0, issued_g = 0;  // profiling: P3/P5 evaluations this lane issued

    // ---- early exit for the fit plane and the refinement candidates (exact). A candidate is accepted
    // only if its weighted cost tc = fl(S / wn) is below the running cost, which never exceeds the cost
    // `thr` it starts from (P3: the cost after P2; P5: after the fit plane). S accumulates
    // fmaf(w_v, c_v, .) over the weighted views in view order, with w_v > 0 and c_v >= 0, so every
    // prefix P of that chain satisfies P <= S and fl(P / wn) <= fl(S / wn): once fl(P / wn) >= thr the
    // candidate is rejected whatever its remaining views give, and they are not evaluated (P6 / P4
    // skip it). Tasks run in batches of WV_WAVES (one per wave); before each batch every (candidate,
    // pixel) folds the views completed by the previous batches into P in view order. The flags are
    // read by other waves while they are set (a stale 0 only evaluates a view that is not needed).
    // part / nxt / dead overlay hyp[5..7] (only P2 reads the anchor planes).
    float *part = reinterpret_cast<float *>(&L.hyp[5 * VM_P]);          // [6][64]: 0 fit, 1..5 candidates
    uint8_t *nxt = reinterpret_cast<uint8_t *>(part + 6 * VM_P);        // [6][64] next view to fold
    uint8_t *dead = nxt + 6 * VM_P;                                     // [6][64]
    static_assert(6 * VM_P * (sizeof(float) + 2) <= 3 * VM_P * sizeof(float4), "early-exit state overlays hyp[5..7]");
    for (int i = tid; i < 6 * VM_P; i += WV_BLOCK) { part[i] = 0.0f; nxt[i] = 0; dead[i] = 0; }
    __syncthreads();
    // fold the views of slot `s` (cost table row `row`, K tasks per view, candidate k) that the tasks
    // below `done` completed; then flag the slot when its partial cost reaches thr
    auto fold = [&](int s, int K, int k, int row, int done) {
        for (int p = tid; p < VM_P; p += WV_BLOCK) {
            const int it = s * VM_P + p;
            if (dead[it]) continue;
            int v = nxt[it];
            float P = part[it];
            const int v0 = v;
            for (; v < N && v * K + k < done; ++v) {
                const int wk = wts[v * VM_P + p];
                if (wk > 0) P = fmaf((float)wk, costL[(row + v) * VM_P + p], P);
            }
            if (v == v0) continue;
            nxt[it] = (uint8_t)v;
            part[it] = P;
            if (P / L.st[3 * VM_P + p] >= L.st[1 * VM_P + p]) dead[it] = 1;
        }
    };

    // ---- P3: fit-plane tasks (views with weight > 0), early exit against the cost after P2
    for (int v0 = 0; v0 < N; v0 += WV_WAVES) {
        if (v0 > 0) fold(0, 1, 0, 0, v0);
        const int v = v0 + wave;
        if (v < N) {
            float cv = 0.0f;
            const bool want = refine && wts[v * VM_P + p1] > 0 && !dead[p1];
            LANE_STAT(22, want);
            const float4 fit = fit1;
            const float nv = ncc_new_vm<F16, SA, true, 9, PIPE>(a, L, p1, px1, py1, v + 1, fit, want, nullptr, &nwc, &nwa);
            if (want) {
                cv = nv;
                if (geom) cv = fmaf(gf, geom_cost(a, px1, py1, v + 1, fit), cv);
                ++issued_nn;
                issued_g += geom;
            }
            costL[v * VM_P + p1] = cv;
        }
        __syncthreads();
    }
    PHASE_STAMP(3);

    // ---- P4: fit acceptance, refinement candidates (PlaneHypothesisRefinementWeak, APD.cu:1008-1067)
    if (wave == 0 && refine) {
        const float wn = L.st[3 * VM_P + p1];
        float depth_now = L.st[0 * VM_P + p1], cost_now = L.st[1 * VM_P + p1];
        float4 pnow = L.pnow[p1];
        const float4 fit = fit1;
        if (!dead[p1]) {  // (dead: the fit plane's cost reaches cost_now -- rejected)
            float tc = 0.0f;
            for (int kk = 0; kk < N; ++kk) {
                const int wk = wts[kk * VM_P + p1];
                if (wk > 0) tc = fmaf((float)wk, costL[kk * VM_P + p1], tc);
            }
            tc /= wn;
            const float db = depth_from_plane(cam0, fit, px1, py1);
            if (db >= a.dmin && db <= a.dmax && tc < cost_now) { depth_now = db; pnow = fit; cost_now = tc; }
        }
        Rng rg(a.seed_lo, a.seed_hi, (uint32_t)c1, ord_weak(iter));
        rg.n = L.rng_n[p1];
        if (rg.n & 3u) rg.refill();
        const Cands C = refine_candidates(a, px1, py1, rg, pnow, depth_now);
        for (int k = 0; k < 5; ++k) {
            float dk;
            float4 t = candidate(C, k, pnow, depth_now, dk);
            t.w = dist2origin(cam0, px1, py1, dk, t);
            WV_CAND(L)[k * VM_P + p1] = t;
        }
        L.pnow[p1] = pnow;
        L.st[0 * VM_P + p1] = depth_now;
        L.st[1 * VM_P + p1] = cost_now;
    }
    __syncthreads();
    PHASE_STAMP(4);

    // ---- P5: candidate evaluations (views with weight > 0), early exit against the cost after the fit
    // plane (slots 1..5). Per view the (candidate, pixel) items that are still wanted are packed into
    // dense lanes (a (candidate, view) task keeps only ~half of its 64 lanes: the view's weight is 0 or
    // the candidate is already rejected), in (candidate, pixel) order; a wave takes 64 items of ONE view
    // (the waves still sample one source image). Batches of whole views (at least WV_P5_CHUNKS chunks,
    // dealt round-robin over the waves) end with the fold, so a rejection found in a batch stops the
    // candidate's later views. The cost table holds [5][VB][64]: a batch's views that have items
    // (`ne`), at most one per chunk, in view order; a slot folds only views whose weight is > 0 for its
    // pixel, where it -- live until the fold -- had an item. Item masks are ballots of LDS state every
    // wave computes alike.
    {
        auto view_masks = [&](int v, uint64_t (&m)[5]) {
            const bool base = refine && wts[v * VM_P + p1] > 0;
#pragma unroll
            for (int k = 0; k < 5; ++k) m[k] = __ballot(base && !dead[(1 + k) * VM_P + p1]);
        };
        for (int v0 = 0; v0 < N;) {
            int v1 = v0, nch = 0, nne = 0;
            uint64_t ne = 0;  // bit v - v0: view v has items
            while (v1 < N && nne < VB && nch < WV_P5_CHUNKS) {
                uint64_t m[5];
                view_masks(v1, m);
                int t = 0;
#pragma unroll
                for (int k = 0; k < 5; ++k) t += __builtin_popcountll(m[k]);
                nch += (t + WAVE - 1) / WAVE;
                if (t > 0) { ne |= 1ull << (v1 - v0); ++nne; }
                ++v1;
            }
            int g = 0;  // chunk index within the batch
            for (int v = v0; v < v1; ++v) {
                uint64_t m[5];
                view_masks(v, m);
                int off[6];
                off[0] = 0;
#pragma unroll
                for (int k = 0; k < 5; ++k) off[k + 1] = off[k] + __builtin_popcountll(m[k]);
                const int nv_items = off[5];
                for (int j = 0; j * WAVE < nv_items; ++j, ++g) {
                    if (g % WV_WAVES != wave) continue;
                    const int it = j * WAVE + lane;
                    const bool want = it < nv_items;
                    int k = 0;
#pragma unroll
                    for (int q = 1; q < 5; ++q) k += it >= off[q];
                    uint64_t mk = m[0];
#pragma unroll
                    for (int q = 1; q < 5; ++q) if (k == q) mk = m[q];
                    int pk = 0;
#pragma unroll
                    for (int q = 1; q < 5; ++q) if (k == q) pk = off[q];
                    const int p = want ? nth_set_bit(mk, it - pk) : p1;
                    const int pxy = L.pxy[p];
                    const int px = pxy & 0xFFFF, py = pxy >> 16;
                    const float4 tp = WV_CAND(L)[k * VM_P + p];
                    LANE_STAT(20, want);
                    const float nv = ncc_new_vm<F16, SA, true, 9, PIPE>(a, L, p, px, py, v + 1, tp, want, nullptr, &nwc, &nwa);
                    if (want) {
                        float cv = nv;
                        if (geom) cv = fmaf(gf, geom_cost(a, px, py, v + 1, tp), cv);
                        ++issued_nn;
                        issued_g += geom;
                        costL[(k * VB + __builtin_popcountll(ne & ((1ull << (v - v0)) - 1ull))) * VM_P + p] = cv;
                    }
                }
            }
            __syncthreads();
            // fold views [nxt, v1) of the refining pixels' 5 slots (all threads: slot 1 + i / 64)
            for (int i = tid; i < 5 * VM_P; i += WV_BLOCK) {
                const int k = i / VM_P, p = i - k * VM_P, sl = (1 + k) * VM_P + p;
                if (dead[sl] || !(p < np && (L.flags[p] >> 31))) continue;
                int v = nxt[sl];
                float P = part[sl];
                for (; v < v1; ++v) {
                    const int wk = wts[v * VM_P + p];
                    if (wk > 0) P = fmaf((float)wk, costL[(k * VB + __builtin_popcountll(ne & ((1ull << (v - v0)) - 1ull))) * VM_P + p], P);
                }
                nxt[sl] = (uint8_t)v;
                part[sl] = P;
                if (P / L.st[3 * VM_P + p] >= L.st[1 * VM_P + p]) dead[sl] = 1;
            }
            __syncthreads();
            v0 = v1;
        }
    }
    PHASE_STAMP(5);

    if (a.evals && wave == 0) {
        // profiling: the NCC-New evaluations and geometric terms CheckerboardPropagationWeak issues
        // for this pixel (APD.cu:1471-1482, 1577-1589, 1026-1094) whose values are used: the valid
        // anchor candidates x N views, the current plane x N, and -- when the fit plane exists -- the
        // fit plane and the 5 refinement candidates x the views with weight > 0. Counted whether the
        // values came from the pair-table kernels, RandomInitialization's kept costs or this kernel.
        uint32_t nn = 0, ng = 0;
        if (pv1) {
            int nsel = 0;
            for (int v = 0; v < N; ++v) nsel += wts[v * VM_P + p1] > 0;
            const int nh = __builtin_popcount(L.flags[p1] & 0xFFu);
            nn = (uint32_t)(nh * N + nsel);
            ng = geom ? (uint32_t)(nh * nsel + nsel) : 0u;
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) { nn += __shfl_xor(nn, o); ng += __shfl_xor(ng, o); }
        if (lane == 0) { atomicAdd(PROF_AT(a.evals, 1), (unsigned long long)nn); atomicAdd(PROF_AT(a.evals, 2), (unsigned long long)ng); }
    }
    if (a.evals) {  // ... plus the fit-plane and refinement evaluations every wave issued (P3, P5)
        uint32_t nn = issued_nn, ng = issued_g, wc0 = nwc, wa0 = nwa;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            nn += __shfl_xor(nn, o); ng += __shfl_xor(ng, o);
            wc0 += __shfl_xor(wc0, o); wa0 += __shfl_xor(wa0, o);
        }
        if (lane == 0) {
            atomicAdd(PROF_AT(a.evals, 1), (unsigned long long)nn); atomicAdd(PROF_AT(a.evals, 2), (unsigned long long)ng);
            atomicAdd(PROF_AT(a.evals, 7), (unsigned long long)wc0); atomicAdd(PROF_AT(a.evals, 8), (unsigned long long)wa0);
        }
    }

    // ---- P6: acceptance, writes
    if (pv1) {
        for (int v = wave; v < N; v += WV_WAVES) a.vw[(size_t)v * a.HW + c1] = (uint8_t)wts[v * VM_P + p1];
        if (wave == 0) {
            float cost_now = L.st[1 * VM_P + p1];
            const float cost_init = L.st[2 * VM_P + p1], wn = L.st[3 * VM_P + p1];
            float4 pnow = L.pnow[p1];
            if (refine) {
                for (int k = 0; k < 5; ++k) {
                    if (dead[(1 + k) * VM_P + p1]) continue;  // its partial cost already reached cost_now
                    const float4 t = WV_CAND(L)[k * VM_P + p1];
                    // (P5's folds ran this slot's chain fmaf(w_v, c_v, .) over all N views in order)
                    const float tc = part[(1 + k) * VM_P + p1] / wn;
                    const float db = depth_from_plane(cam0, t, px1, py1);
                    if (db >= a.dmin && db <= a.dmax && tc < cost_now) { pnow = t; cost_now = tc; }
                }
            }
            if (a.state == APD_REFINE_INIT) {
                if ((double)cost_now < (double)cost_init - 0.1) { a.cost[c1] = cost_now; a.plane[c1] = pnow; }
                else a.cost[c1] = cost_init;
            } else {
                a.cost[c1] = cost_now;
                a.plane[c1] = pnow;
            }
        }
    }
    PHASE_STAMP(6);
}

// k_weak_cand_g's workgroups: 8 waves, wave h = anchor candidate h
#define PK_WAVES 8
#define PK_BLOCK (PK_WAVES * WAVE)
#ifndef PK_MINW
#define PK_MINW 1  // k_weak_cand_g workgroups per CU the registers are bounded for
#endif
#ifndef PK_PIPE
#define PK_PIPE true  // k_weak_cand_g's centre windows software-pipelined by columns
#endif

// ---------------------------------------------------------------------------------------------
// Image-wide anchor-window pairs (no SA masks). A WEAK pixel's anchor candidate h (the plane of its
// STRONG anchor h+1) is scored by ComputeBilateralNCCNew (APD.cu:448-593): the centre window at its
// anchor 0 and the 3x3 windows at its anchors 1..8, combined by the focal softmax. The cost of the
// window at anchor k under the plane of anchor h in view v is a function of (position of k, position
// of h, v) only -- the out-of-frame rule reads sel[k], which only the Strong sweep writes -- and the
// anchors are STRONG points on the borders of the textureless regions, shared by the region's pixels:
// at C3 (6048x4032, N = 10) 1.43 G (window, candidate) pairs per view are 102.6 M distinct pairs
// image-wide (13.9x), against 2.1x within a 64-pixel group (tools/pair_sharing.py). So:
//   per pass (apd_stage_prepare, anchors fixed): the (pixel, window slot) references are counting-
//     sorted by window anchor (k_gp_count, scan, k_gp_fill); chunks of GP_CHUNK consecutive
//     references deduplicate their (window anchor, candidate anchor) pairs in an LDS hash
//     (k_gp_dedup: pass 0 counts, a scan places the chunks, pass 1 writes the pair list and every
//     (pixel, candidate, window) slot's pair id). Pair ids are labels: their order (atomics) may
//     differ between runs, the costs never do.
//   per iteration: k_gp_cost evaluates every pair in every view (lane = pair, consecutive pairs share
//     a window anchor) into pcost[pair][view]; k_weak_cand_g evaluates the centre windows (lane =
//     pixel, wave = candidate) and the focal combination reading the pair costs, and writes the same
//     [view][candidate][WEAK index] costs the sweep reads (direct mode).
// ---------------------------------------------------------------------------------------------
#ifndef GP_CHUNK
#define GP_CHUNK 256   // references per batch of k_gp_dedup (one workgroup per window anchor)
#endif
#ifndef GP_HS
#define GP_HS 8192     // LDS hash slots
#endif
// a table closes once it holds GP_CLOSE keys after a batch; a batch adds <= 8 * GP_CHUNK: load <= 0.75
#define GP_CLOSE (GP_HS * 3 / 4 - 8 * GP_CHUNK)
static_assert(GP_CLOSE > 0 && GP_HS >= 256 && 256 % GP_CHUNK == 0, "k_gp_dedup table sizing");
// window anchors with at most GP_SMALL_N references (most of them) run in a one-wave workgroup with a
// 1 k-slot table (6 KiB of LDS instead of 48 KiB: many more workgroups per CU, the kernel is latency
// bound); their references fit one batch, so the table is the large kernel's single table
#define GP_SMALL_N 64
#define GP_SMALL_HS 1024
#define GP_MEDIUM_HS 4096  // the medium class (GP_SMALL_N < n <= GP_CHUNK: one batch, <= 8 GP_CHUNK keys)
static_assert(GP_SMALL_HS * 3 / 4 - 8 * GP_SMALL_N > 0 && 8 * GP_SMALL_N <= GP_SMALL_HS / 2, "small k_gp_dedup sizing");
#define GP_NONE 0xFFFFFFFFu

// profiling: a wave's sum of the lanes' counts, one atomic per wave
__device__ __forceinline__ void wave_count(APD_G unsigned long long *evals, int k, uint32_t n) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) n += __shfl_xor(n, o);
    if ((threadIdx.x & (WAVE - 1)) == 0 && n) atomicAdd(PROF_AT(evals, k), (unsigned long long)n);
}
// Lanes are consecutive WEAK pixels in tile order, whose anchor k is often the same STRONG point: per
// slot k the runs of equal anchors among neighbouring lanes take one atomic (run head).
__device__ __forceinline__ void gp_run(bool ok, int q, int &head_lane, int &rank, int &len) {
    const int lane = threadIdx.x & (WAVE - 1);
    const int qp = __shfl_up(q, 1);
    const bool okp = __shfl_up((int)ok, 1) != 0;
    const bool head = ok && (lane == 0 || !okp || qp != q);
    const unsigned long long hb = __ballot(head);
    // run head of this lane: the highest head at or below it
    const unsigned long long below = hb & ((lane == 63) ? ~0ull : ((2ull << lane) - 1ull));
    head_lane = below ? 63 - __builtin_clzll(below) : 0;
    rank = lane - head_lane;
    // run length (heads only): distance to the next head or to the end of the run
    const unsigned long long okb = __ballot(ok);
    const unsigned long long above = (lane == 63) ? 0ull : (hb | ~okb) & ~((2ull << lane) - 1ull);
    const int end = above ? __builtin_ctzll(above) : 64;
    len = end - lane;
}
// SA masks (APD.cu:464-465, 493-497, 526-530): with a non-zero label at the pixel, an anchor window is
// used only when the anchor carries the same label, and its taps are then filtered by that label --
// the anchor's own. With label 0 nothing is filtered. So a window's cost depends on (window anchor,
// filtered, candidate plane, view) only: the table keys windows by (anchor, filtered) and each pixel's
// used windows (wmw) replace the anchors' validity.
__device__ __forceinline__ bool gp_window_used(const Args &a, int cid, int q) { return cid == 0 || (int)a.sa[q] == cid; }
// references per window anchor (cnt), each WEAK pixel's candidate bits (cbw: anchor h+1 valid and
// STRONG) and used windows (wmw: anchor k valid and, with an SA label, carrying it; bit k - 1)
__global__ __launch_bounds__(BLOCK) void k_gp_count(Args a, const int *__restrict__ list, int count, int *__restrict__ cnt,
                                                    uint8_t *__restrict__ cbw, uint8_t *__restrict__ wmw) {
    const int i = blockIdx.x * BLOCK + threadIdx.x;
    const bool act = i < count;
    const int c = list[act ? i : count - 1];
    const int wi = a.amap[c];
    const int cid = a.sa_any ? (int)a.sa[c] : 0;
    const APD_G short2 *anc = a.anchors + (size_t)wi * 9;
    uint32_t cb = 0, wm = 0;
#pragma unroll 1
    for (int k = 1; k < 9; ++k) {
        const short2 ap = anc[k];
        const bool valid = act && !(ap.x == -1 || ap.y == -1);
        const int q = valid ? ap.x + ap.y * a.W : -1;
        if (valid && a.weak[q] == APD_STRONG) cb |= 1u << (k - 1);
        const bool ok = valid && gp_window_used(a, cid, q);
        if (ok) wm |= 1u << (k - 1);
        int hl, rk, len;
        gp_run(ok, q, hl, rk, len);
        if (ok && rk == 0) atomicAdd(&cnt[q], len);
    }
    if (act) { cbw[wi] = (uint8_t)cb; wmw[wi] = (uint8_t)wm; }
}
// k_gp_count with the references' places: the run head's atomic returns the run's first position in
// its window anchor's segment, and every reference keeps its own (loc[WEAK index * 8 + k - 1]);
// k_gp_place then writes each reference at segment offset + place -- no second pass of atomics
// (k_gp_fill, the path APD_GP_FILL=1 keeps)
#ifndef GP_LOC_BLOCK
#define GP_LOC_BLOCK 1  // k_gp_count_loc: per-workgroup aggregation of the anchors' counts in LDS
#endif
#define GP_LOC_LG 12
#define GP_LOC_HS (1 << GP_LOC_LG)  // >= 2 x the 8 * BLOCK references a workgroup can hold: load <= 0.5
static_assert(GP_LOC_HS >= 2 * 8 * BLOCK, "k_gp_count_loc LDS table sizing");
__global__ __launch_bounds__(BLOCK) void k_gp_count_loc(Args a, const int *__restrict__ list, int count, int *__restrict__ cnt,
                                                        uint8_t *__restrict__ cbw, uint8_t *__restrict__ wmw,
                                                        uint32_t *__restrict__ loc) {
    const int i = blockIdx.x * BLOCK + threadIdx.x;
    const bool act = i < count;
    const int c = list[act ? i : count - 1];
    const int wi = a.amap[c];
    const int cid = a.sa_any ? (int)a.sa[c] : 0;
    const APD_G short2 *anc = a.anchors + (size_t)wi * 9;
    // every load of the 8 windows first (anchors, their states and labels), then the 8 runs and their
    // atomics, all in flight together: the kernel is latency bound (counters: 1 % of wave time active)
    short2 ap[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) ap[k] = anc[k + 1];
    int q[8];
    bool valid[8];
    uint8_t wst[8];
    int lab[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        valid[k] = act && !(ap[k].x == -1 || ap[k].y == -1);
        q[k] = valid[k] ? ap[k].x + ap[k].y * a.W : -1;
        wst[k] = valid[k] ? a.weak[q[k]] : (uint8_t)0;
        lab[k] = (valid[k] && a.sa_any) ? (int)a.sa[q[k]] : 0;
    }
    uint32_t cb = 0, wm = 0;
    int pos[8];
    bool okk[8];
    int hl[8], rk[8];
#if GP_LOC_BLOCK
    // The workgroup's references aggregated per window anchor in LDS first (the runs' lengths added
    // into a per-anchor local count, whose returned value is the run's offset within the workgroup),
    // then one global atomic per distinct anchor of the workgroup: neighbouring tiles share their
    // anchors, and same-address global atomics from the whole GPU serialised the per-run version.
    // Positions stay unique within each anchor's segment (their order is a label, as before).
    __shared__ int hkey[GP_LOC_HS], hcnt[GP_LOC_HS];  // anchor q + 1 (0: empty); count, then global base
    for (int t = threadIdx.x; t < GP_LOC_HS; t += BLOCK) { hkey[t] = 0; hcnt[t] = 0; }
    __syncthreads();
    int slot[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        if (valid[k] && wst[k] == APD_STRONG) cb |= 1u << k;
        okk[k] = valid[k] && (cid == 0 || lab[k] == cid);  // (gp_window_used)
        if (okk[k]) wm |= 1u << k;
        int len;
        gp_run(okk[k], q[k], hl[k], rk[k], len);
        int sl = 0, lp = 0;
        if (okk[k] && rk[k] == 0) {
            const int key = q[k] + 1;
            sl = (int)(((uint32_t)key * 0x9E3779B1u) >> (32 - GP_LOC_LG));
            for (;;) {
                const int cur = hkey[sl];
                if (cur == key) break;
                if (cur == 0) {
                    const int old = atomicCAS(&hkey[sl], 0, key);
                    if (old == 0 || old == key) break;
                }
                sl = (sl + 1) & (GP_LOC_HS - 1);
            }
            lp = atomicAdd(&hcnt[sl], len);
        }
        slot[k] = __shfl(sl, hl[k]);
        pos[k] = __shfl(lp, hl[k]) + rk[k];
    }
    __syncthreads();
    for (int t = threadIdx.x; t < GP_LOC_HS; t += BLOCK)
        if (hkey[t] != 0) hcnt[t] = atomicAdd(&cnt[hkey[t] - 1], hcnt[t]);
    __syncthreads();
    uint32_t l[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) l[k] = (uint32_t)(hcnt[slot[k]] + pos[k]);  // (k_gp_place reads used windows only)
#else
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        if (valid[k] && wst[k] == APD_STRONG) cb |= 1u << k;
        okk[k] = valid[k] && (cid == 0 || lab[k] == cid);  // (gp_window_used)
        if (okk[k]) wm |= 1u << k;
        int len;
        gp_run(okk[k], q[k], hl[k], rk[k], len);
        pos[k] = 0;
        if (okk[k] && rk[k] == 0) pos[k] = atomicAdd(&cnt[q[k]], len);
    }
    uint32_t l[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) l[k] = (uint32_t)(__shfl(pos[k], hl[k]) + rk[k]);  // (k_gp_place reads used windows only)
#endif
    if (act) {
        uint4 *d = reinterpret_cast<uint4 *>(loc + (size_t)wi * 8);
        d[0] = make_uint4(l[0], l[1], l[2], l[3]);
        d[1] = make_uint4(l[4], l[5], l[6], l[7]);
        cbw[wi] = (uint8_t)cb;
        wmw[wi] = (uint8_t)wm;
    }
}
// references (WEAK index * 8 + window slot k - 1, bit 31: filtered by the SA label) into their
// window anchor's segment
#define GP_FILT 0x80000000u
__global__ __launch_bounds__(BLOCK) void k_gp_place(Args a, const int *__restrict__ list, int count, const int *__restrict__ off,
                                                    const uint8_t *__restrict__ wmw, const uint32_t *__restrict__ loc,
                                                    uint32_t *__restrict__ refs) {
    const int i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= count) return;
    const int c = list[i];
    const uint32_t wi = (uint32_t)a.amap[c];
    const uint32_t filt = (a.sa_any && a.sa[c] != 0) ? GP_FILT : 0u;
    const uint32_t wm = wmw[wi];
    const APD_G short2 *anc = a.anchors + (size_t)wi * 9;
    const uint4 l0 = *reinterpret_cast<const uint4 *>(loc + (size_t)wi * 8);
    const uint4 l1 = *reinterpret_cast<const uint4 *>(loc + (size_t)wi * 8 + 4);
    const uint32_t l[8] = {l0.x, l0.y, l0.z, l0.w, l1.x, l1.y, l1.z, l1.w};
#pragma unroll
    for (int k = 1; k < 9; ++k) {
        if (!((wm >> (k - 1)) & 1u)) continue;
        const short2 ap = anc[k];
        const int q = ap.x + ap.y * a.W;
        refs[off[q] + l[k - 1]] = (wi * 8u + (uint32_t)(k - 1)) | filt;
    }
}
__global__ __launch_bounds__(BLOCK) void k_gp_fill(Args a, const int *__restrict__ list, int count, int *__restrict__ cur,
                                                   uint32_t *__restrict__ refs) {
    const int i = blockIdx.x * BLOCK + threadIdx.x;
    const bool act = i < count;
    const int c = list[act ? i : count - 1];
    const uint32_t wi = (uint32_t)a.amap[c];
    const int cid = a.sa_any ? (int)a.sa[c] : 0;
    const uint32_t filt = cid != 0 ? GP_FILT : 0u;
    const APD_G short2 *anc = a.anchors + (size_t)wi * 9;
#pragma unroll 1
    for (int k = 1; k < 9; ++k) {
        const short2 ap = anc[k];
        const bool valid = act && !(ap.x == -1 || ap.y == -1);
        const int q = valid ? ap.x + ap.y * a.W : -1;
        const bool ok = valid && gp_window_used(a, cid, q);
        int hl, rk, len;
        gp_run(ok, q, hl, rk, len);
        int pos = 0;
        if (ok && rk == 0) pos = atomicAdd(&cur[q], len);
        pos = __shfl(pos, hl) + rk;
        if (ok) refs[pos] = (wi * 8u + (uint32_t)(k - 1)) | filt;
    }
}
// the window anchors that have references, in raster order (task list for k_gp_dedup): flags, then
// (after an exclusive scan into pos) a scatter
__global__ __launch_bounds__(BLOCK) void k_gp_flags(const int *__restrict__ off, int HW, int *__restrict__ flag) {
    const int q = blockIdx.x * BLOCK + threadIdx.x;
    if (q <= HW) flag[q] = (q < HW && off[q + 1] > off[q]) ? 1 : 0;
}
__global__ __launch_bounds__(BLOCK) void k_gp_tasks(const int *__restrict__ off, const int *__restrict__ pos, int HW,
                                                    int *__restrict__ tasks) {
    const int q = blockIdx.x * BLOCK + threadIdx.x;
    if (q < HW && off[q + 1] > off[q]) tasks[pos[q]] = q;
}
// One workgroup per window anchor q (tasks[]): its references, in batches of GP_CHUNK, insert their
// candidate anchors into an LDS hash (keys qh + 1), sized from the reference count; a table that
// reaches GP_HS / 2 keys after a batch is closed (a new run of pairs for q starts, so an anchor with
// more than ~4 k distinct candidates repeats a few pairs). Each closed table writes its pairs (plist,
// slot order) and then every (pixel, candidate, window) slot of the table's references (pidx).
// PASS 2 (the default, one pass): a closed table reserves its range of plist with one atomic on a
// global counter (acnt[0]); ranges past `pcap` entries are not written, and the host, seeing the
// counter above pcap, builds the table again with the two passes. PASS 0 counts the distinct pairs
// per anchor (acnt) and PASS 1 writes them from the scanned bases (abase): the fallback, and the
// path APD_GP_TWO_PASS=1 forces. Pair ids are labels either way: the costs never depend on them.
// (PASS 2) the tasks with NLO < n <= NHI references only: the small ones (n <= GP_SMALL_N) in a one-wave
// workgroup with a 1 k-slot table, the medium ones (n <= GP_CHUNK, one batch) in a 4 k-slot table
// (24 KiB instead of 48 KiB of LDS), the others as before.
template <int HS, int CHUNK>
struct GpLds {
    uint32_t hs[HS];
    uint16_t sid[HS];
    int scan_w[CHUNK / WAVE + 1];
    int nfresh, sbase, task;
};
// One window anchor q's references [r0, r0 + n) (see k_gp_dedup); `base` is PASS 1's first pair id.
// Returns the distinct pairs of its tables (PASS 0). Every thread of the workgroup calls it; it ends
// with a barrier, so a workgroup may run it for several anchors in turn.
template <int PASS, int HS, int CHUNK>
__device__ __forceinline__ int gp_dedup_task(const Args &a, GpLds<HS, CHUNK> &S, int q, int r0, int n, int base,
                                             const uint32_t *__restrict__ refs, const uint8_t *__restrict__ cbw,
                                             int *__restrict__ acnt, int2 *__restrict__ plist, uint32_t *__restrict__ pidx,
                                             int pcap) {
    constexpr int CLOSE = HS * 3 / 4 - 8 * CHUNK;
    static_assert(CLOSE > 0 && HS >= 256 && HS % CHUNK == 0 && 256 % CHUNK == 0, "k_gp_dedup table sizing");
    const int tid = threadIdx.x, lane = tid & (WAVE - 1), wave = tid >> 6;
    const int qx = q % a.W, qy = q / a.W;
    int cap = 256, lg = 8;
    while (cap < HS && cap < n * 16) { cap <<= 1; ++lg; }
    const uint32_t msk = (uint32_t)cap - 1u;
    auto slot_of = [&](uint32_t key) { return (key * 0x9E3779B1u) >> (32 - lg); };
    // candidates (valid, STRONG anchors 1..8) of reference r: bits + keys (candidate position + 1,
    // GP_FILT when the window is SA-filtered)
    auto cands = [&](int r, uint32_t &wi, uint32_t &k, uint32_t (&qh)[8]) {
        const uint32_t ref = refs[r];
        const uint32_t filt = ref & GP_FILT;
        wi = (ref & ~GP_FILT) >> 3;
        k = ref & 7u;
        const APD_G short2 *anc = a.anchors + (size_t)wi * 9;
        const uint32_t cb = cbw[wi];
#pragma unroll
        for (int h = 0; h < 8; ++h) {
            const short2 ap = anc[h + 1];
            qh[h] = ((uint32_t)(ap.x + ap.y * a.W) + 1u) | filt;  // (used only where cb has the bit: a valid anchor)
        }
        return cb;
    };
    for (int i = tid; i < cap; i += CHUNK) S.hs[i] = 0u;
    if (tid == 0) S.nfresh = 0;
    __syncthreads();
    int total = 0;
    int run0 = 0;  // first reference of the open table
    for (int b0 = 0; b0 < n; b0 += CHUNK) {
        const int r = b0 + tid;
        if (r < n) {
            uint32_t wi, k, qh[8];
            const uint32_t cb = cands(r0 + r, wi, k, qh);
            int fresh = 0;
#pragma unroll
            for (int h = 0; h < 8; ++h) {
                if (!((cb >> h) & 1u)) continue;
                const uint32_t key = qh[h];
                uint32_t sl = slot_of(key);
                for (;;) {
                    // most of an anchor's references share their candidates: a plain read finds the key
                    // already inserted without an LDS atomic (same-address atomics serialise)
                    const uint32_t cur = S.hs[sl];
                    if (cur == key) break;
                    if (cur == 0u) {
                        const uint32_t old = atomicCAS(&S.hs[sl], 0u, key);
                        if (old == 0u) { ++fresh; break; }
                        if (old == key) break;
                    }
                    sl = (sl + 1) & msk;
                }
            }
            if (fresh) atomicAdd(&S.nfresh, fresh);
        }
        __syncthreads();
        const int nd = S.nfresh;
        // every thread has read S.nfresh before any wave's next-batch inserts can add to it (else
        // `close` and `base` could differ between waves)
        __syncthreads();
        const bool close = nd >= CLOSE || b0 + CHUNK >= n;
        if (!close) continue;  // (uniform)
        if (PASS == 2) {
            if (tid == 0) S.sbase = atomicAdd(acnt, nd);
            __syncthreads();
            base = S.sbase;
        }
        if (PASS >= 1) {
            // plist[base + id] = (window anchor, candidate anchor)
            const int per = cap / CHUNK;  // slots per thread (cap >= CHUNK)
            const int s0 = tid * per, s1 = s0 + per;
            int c = 0;
            for (int sl = s0; sl < s1; ++sl) c += S.hs[sl] != 0u;
            int x = c;
#pragma unroll
            for (int o = 1; o < WAVE; o <<= 1) {
                const int y = __shfl_up(x, o);
                if (lane >= o) x += y;
            }
            if (lane == WAVE - 1) S.scan_w[wave] = x;
            __syncthreads();
            int next = x - c;
            for (int w = 0; w < wave; ++w) next += S.scan_w[w];
            // ids in slot order (ranking the candidates by raster position, so that a group's pixels
            // read neighbouring rows of pcost, measured: k_weak_cand_g -1 %, this pass +93 %)
            for (int sl = s0; sl < s1; ++sl) {
                const uint32_t key = S.hs[sl];
                if (!key) continue;
                // (window anchor x | SA-filtered << 15 | y << 16, candidate anchor position)
                if (PASS == 1 || base + next < pcap)
                    plist[base + next] = make_int2(qx | ((key & GP_FILT) ? 0x8000 : 0) | (qy << 16), (int)((key & ~GP_FILT) - 1u));
                S.sid[sl] = (uint16_t)next;
                ++next;
            }
            __syncthreads();
            // the table's references: pair ids of their (candidate, window) slots
            for (int rr = run0 + tid; rr < min(n, b0 + CHUNK); rr += CHUNK) {
                uint32_t wi, k, qh[8], pv[8];
                const uint32_t cb = cands(r0 + rr, wi, k, qh);
#pragma unroll
                for (int h = 0; h < 8; ++h) {
                    pv[h] = GP_NONE;
                    if (!((cb >> h) & 1u)) continue;
                    const uint32_t key = qh[h];
                    uint32_t sl = slot_of(key);
                    while (S.hs[sl] != key) sl = (sl + 1) & msk;
                    pv[h] = (uint32_t)(base + S.sid[sl]);
                }
                uint4 *dst = reinterpret_cast<uint4 *>(pidx + ((size_t)wi * 8 + k) * 8);  // [WEAK index][window k][candidate h]
                dst[0] = make_uint4(pv[0], pv[1], pv[2], pv[3]);
                dst[1] = make_uint4(pv[4], pv[5], pv[6], pv[7]);
            }
            __syncthreads();
        }
        if (PASS != 2) base += nd;
        total += nd;
        run0 = b0 + CHUNK;
        for (int i = tid; i < cap; i += CHUNK) S.hs[i] = 0u;
        __syncthreads();
        if (tid == 0) S.nfresh = 0;
        __syncthreads();
    }
    return total;
}
template <int PASS, int HS = GP_HS, int CHUNK = GP_CHUNK, int NLO = -1, int NHI = 0x7fffffff>
__global__ __launch_bounds__(CHUNK) void k_gp_dedup(Args a, const int *__restrict__ tasks, const int *__restrict__ off,
                                                    const uint32_t *__restrict__ refs, const uint8_t *__restrict__ cbw,
                                                    int *__restrict__ acnt,
                                                    const int *__restrict__ abase, int2 *__restrict__ plist,
                                                    uint32_t *__restrict__ pidx, int pcap) {
    __shared__ GpLds<HS, CHUNK> S;
    const int q = tasks[blockIdx.x];
    const int r0 = off[q], n = off[q + 1] - r0;
    if (n <= NLO || n > NHI) return;
    const int total = gp_dedup_task<PASS, HS, CHUNK>(a, S, q, r0, n, PASS == 1 ? abase[blockIdx.x] : 0, refs, cbw, acnt, plist,
                                                     pidx, pcap);
    if (PASS == 0 && threadIdx.x == 0) acnt[blockIdx.x] = total;
}
// The one-pass table without host round trips (apd_stage_prepare enqueues it whole, and
// RandomInitialization runs beside it): the window anchors with references are dealt into three
// size classes by k_gp_classes, and each class runs in a grid that fills the GPU, its workgroups
// taking the class's anchors in turn -- DYN (the large class, whose anchors differ most in size): the
// next anchor from an atomic counter; else every gridDim-th. The class's count is read from device
// memory, and every workgroup leaves the loop when it passes it.
#define GP_CLASSES 3
// A large window anchor's references are split into runs of GP_SPLIT, each deduplicated by its own
// workgroup: one workgroup per anchor left the GPU idle behind the few anchors with 10^5 references
// (counters: CUs busy 16 % of the kernel's span). A pair whose candidates meet in several runs gets
// several ids -- labels, as when a table closes -- so k_gp_cost evaluates it a few more times.
#define GP_SPLIT 4096
// lists: classes 0 and 1 as anchor positions [cap] each, then class 2 as (anchor, run) pairs [cap2]
__global__ __launch_bounds__(BLOCK) void k_gp_classes(const int *__restrict__ off, int HW, int cap, int cap2,
                                                      int *__restrict__ lists, int *__restrict__ counts) {
    const int q = blockIdx.x * BLOCK + threadIdx.x;
    const int lane = threadIdx.x & (WAVE - 1);
    const int n = q < HW ? off[q + 1] - off[q] : 0;
    const int cls = n <= GP_SMALL_N ? 0 : (n <= GP_CHUNK ? 1 : 2);
    const int runs = cls == 2 ? (n + GP_SPLIT - 1) / GP_SPLIT : 1;
    int2 *list2 = reinterpret_cast<int2 *>(lists + 2 * (size_t)cap);
#pragma unroll
    for (int c = 0; c < GP_CLASSES; ++c) {
        const bool mine = n > 0 && cls == c;
        if (!__ballot(mine)) continue;
        // the wave's entries of class c: an exclusive scan of `runs` over the lanes, one atomic
        int x = mine ? runs : 0;
        const int own = x;
#pragma unroll
        for (int o = 1; o < WAVE; o <<= 1) {
            const int y = __shfl_up(x, o);
            if (lane >= o) x += y;
        }
        int base = 0;
        if (lane == WAVE - 1) base = atomicAdd(&counts[c], x);
        base = __shfl(base, WAVE - 1) + x - own;
        if (!mine) continue;
        if (c < 2) {
            if (base < cap) lists[(size_t)c * cap + base] = q;
            else atomicOr(&counts[GP_CLASSES + 1], 1);  // (overflow: the host rebuilds synchronously)
        } else {
            for (int r = 0; r < own; ++r) {
                if (base + r < cap2) list2[base + r] = make_int2(q, r);
                else atomicOr(&counts[GP_CLASSES + 1], 1);
            }
        }
    }
}
// DYN (class 2): the list holds (anchor, run) pairs, run r covering references [r GP_SPLIT, (r + 1) GP_SPLIT)
template <int HS, int CHUNK, bool DYN>
__global__ __launch_bounds__(CHUNK) void k_gp_dedup_q(Args a, const int *__restrict__ list, const int *__restrict__ count,
                                                      int *__restrict__ next, const int *__restrict__ off,
                                                      const uint32_t *__restrict__ refs, const uint8_t *__restrict__ cbw,
                                                      int *__restrict__ acnt, int2 *__restrict__ plist, uint32_t *__restrict__ pidx,
                                                      int pcap) {
    __shared__ GpLds<HS, CHUNK> S;
    const int ntask = *count;
    for (int t = blockIdx.x;; t += gridDim.x) {
        if (DYN) {
            if (threadIdx.x == 0) S.task = atomicAdd(next, 1);
            __syncthreads();
            t = S.task;
            __syncthreads();
        }
        if (t >= ntask) break;  // (uniform)
        int q, r0, n;
        if (DYN) {
            const int2 e = reinterpret_cast<const int2 *>(list)[t];
            q = e.x;
            const int b = off[q], m = off[q + 1] - b;
            r0 = b + e.y * GP_SPLIT;
            n = min(GP_SPLIT, m - e.y * GP_SPLIT);
        } else {
            q = list[t];
            r0 = off[q];
            n = off[q + 1] - r0;
        }
        (void)gp_dedup_task<2, HS, CHUNK>(a, S, q, r0, n, 0, refs, cbw, acnt, plist, pidx, pcap);
    }
}

// every pair in every view: ComputeBilateralNCCNew's k >= 1 window (APD.cu:500-575), the same
// statements as ncc_new_vm's anchor windows; pcost[pair][v] rows padded to a multiple of 4 views
// (< 0: window absent). The block's 256 pairs are consecutive, so their rows are one contiguous
// range of pcost: the costs are staged in LDS ([pair][Np], gp_cost_lds_bytes) and written with
// coalesced 16-byte stores after the view loop (a 4-byte store per (pair, view) at the row stride
// wrote 4.2x the bytes, profiles/r3_pmc_k_gp_cost_c3b.json).
#ifndef GP_COST_STAGED
#define GP_COST_STAGED 1  // (A/B: 0 = one 4-byte store per (pair, view))
#endif
static inline size_t gp_cost_lds_bytes(int N) { return GP_COST_STAGED ? (size_t)BLOCK * ((N + 3) & ~3) * sizeof(float) : 0; }
template <bool F16, bool SA>
__global__ __launch_bounds__(BLOCK) void k_gp_cost(Args a, const int2 *__restrict__ plist, int np, float *__restrict__ pcost) {
    float *crow = apd_dyn_lds;  // [BLOCK][Np]
    const int N = a.N, W = a.W, H = a.H, Np = (N + 3) & ~3;
    const int i0 = xcd_remap(blockIdx.x, gridDim.x) * BLOCK;
    const int i = i0 + threadIdx.x;
    const bool act = i < np;
    const int2 pr = plist[act ? i : np - 1];
    const int ax = pr.x & 0x7FFF, ay = pr.x >> 16;
    const bool filt = SA && (pr.x & 0x8000) != 0;  // SA-filtered window: taps with the anchor's label only
    const float4 pl = a.plane[pr.y];
    // the window's reference side from its record (k_anchor_rec: the same statements; a filtered
    // window keeps the anchor's own tap, so its wsum >= 1 and APD.cu:543's empty window cannot occur)
    const AncRecV<F16> R = load_anc_rec<F16>(a, ax + ay * W, filt ? 1 : 0);
    const uint64_t tm = SA ? (uint64_t)R.mask() : 0x1FFull;
    const uint32_t selk = a.sel[ax + ay * W];
    uint32_t nlive = 0;
    for (int v = 0; v < N; ++v) {
        const int s = v + 1;
        const FastTex<F16, true> T(a, s);
        const SrcTex<F16> Q(a, s);
        const Hom Hm = homography(a, s, pl);
        float asx, asy;
        project(Hm, (float)ax, (float)ay, asx, asy);
        bool live = act;
        float res = -1.0f;  // absent
        if (act && (asx < 0 || asy < 0 || asx >= (float)W || asy >= (float)H)) {
            live = false;
            if ((selk >> (s - 1)) & 1u) res = APD_COST_MAX;
        }
        if (__ballot(live)) {
            const bool fast = live && window_rcp_ok(Hm, (float)(ax - 5), (float)(ay - 5));
            float ss = 0.0f, sss = 0.0f, srs = 0.0f;
            ncc_new_window<F16, 3, 5>(a, R, 1, tm, Hm, ax, ay, live, fast, T, Q, ss, sss, srs);
            if (live) res = ncc_finalize_pre(R.inv(), R.srp(), R.var(), ss, sss, srs);
        }
        nlive += live;
        if (GP_COST_STAGED) crow[threadIdx.x * Np + v] = res;
        else if (act) pcost[(size_t)i * Np + v] = res;
    }
    if (a.evals) wave_count(a.evals, 5, nlive);  // (profiling: pair windows evaluated)
    if (!GP_COST_STAGED) return;
    for (int v = N; v < Np; ++v) crow[threadIdx.x * Np + v] = -1.0f;  // (padding, never read)
    __syncthreads();
    const int nq = (min(BLOCK, np - i0) * Np) >> 2;  // float4s of the block's rows
    const float4 *src = reinterpret_cast<const float4 *>(crow);
    float4 *dst = reinterpret_cast<float4 *>(pcost + (size_t)i0 * Np);
    for (int j = threadIdx.x; j < nq; j += BLOCK) dst[j] = src[j];
}

// the focal combination (APD.cu:576-593, Softmax 431-446) of one (pixel, candidate, view): centre
// cost cc (< 0: dead -> COST_MAX) and the 8 windows' pair costs sc[k] (< 0: window absent), in anchor
// order -- ncc_new_vm's statements
__device__ __forceinline__ float gp_combine(float cc, const float (&sc)[8]) {
    if (cc < 0.0f) return APD_COST_MAX;
    const float center_cost = cc;
    uint32_t pm = 0;
    float strong_weight = 0.0f;
#pragma unroll
    for (int k = 0; k < 8; ++k)
        if (sc[k] >= 0.0f) { pm |= 1u << k; strong_weight += 1.0f; }
    if (strong_weight <= 1e-6f) return center_cost;
    float mx = -1e10f;
#pragma unroll
    for (int k = 0; k < 8; ++k) if (((pm >> k) & 1u) && sc[k] > mx) mx = sc[k];
    float e[8];
    float sum = 0.0f;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        e[k] = 0.0f;
        if ((pm >> k) & 1u) { e[k] = d_expf(sc[k] - mx); sum += e[k]; }
    }
    float acc = 0.0f;
#pragma unroll
    for (int k = 0; k < 8; ++k)
        if ((pm >> k) & 1u) { const float w = e[k] / sum; acc = fmaf(w, sc[k], acc); }
    acc = (acc > APD_COST_MAX) ? APD_COST_MAX : acc;
    return (float)(0.25 * (double)center_cost + 0.75 * (double)acc);
}

// the anchor candidates' centre windows (k_weak_cand_comb then combines them with the pair costs);
// lane = pixel, wave = candidate h. Per view (the waves take the views together: one source image,
// the CU's L1) the centre window of (pixel, h) -> out[v][h][WEAK index] (-1: dead, the pixel or its
// anchor 0 projected out of frame). With an SA label at the pixel the centre window is used only
// when anchor 0 carries the label (else center_cost stays 0, APD.cu:493-497) and its taps are
// filtered by it (APD.cu:526-530); an empty window leaves center_cost 0 (APD.cu:543).
template <bool F16, bool SA>
__global__ __launch_bounds__(PK_BLOCK, PK_MINW) void k_weak_cand_g(Args a, const int *__restrict__ list, int count,
                                                          const uint8_t *__restrict__ cbw, float *__restrict__ out, int wc) {
    using TT = FastTex<F16, true>;  // (FastTexD measured 1.4 % slower per iteration here, profiles/r5_ab_dtex_kernels.txt)
    // (fp16 reference taps when the images are: fp32 measured 6 % slower, profiles/r4_ab_cand_g_fp32_ref.txt)
    using RT = typename std::conditional<F16, _Float16, float>::type;
    __shared__ RT cref[36 * VM_P];
    __shared__ float csr[VM_P], csrr[VM_P];
    __shared__ uint64_t cmask[VM_P];
    __shared__ uint8_t cws[VM_P], cbits[VM_P];
    __shared__ int anc0[VM_P];
    const int N = a.N, W = a.W, H = a.H;
    const int blk = xcd_remap(blockIdx.x, gridDim.x);
    const int first = blk * VM_P;
    const int np = min(VM_P, count - first);
    const int tid = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & (WAVE - 1);
    const int p1 = lane;
    const bool pv1 = p1 < np;
    const int c1 = list[first + min(p1, np - 1)];
    const int py1 = c1 / W, px1 = c1 - py1 * W;
    const int wi1 = a.amap[c1];
    const int cid = a.sa_any ? (int)a.sa[c1] : 0;
    const APD_G short2 *anc1 = a.anchors + (size_t)wi1 * 9;
    if (wave == 0) {
        int a0 = -1;
        uint32_t cb = 0;
        if (pv1) {
            const short2 z = anc1[0];
            const bool ok = !(z.x == -1 || z.y == -1) && (cid == 0 || (int)a.sa[z.x + z.y * W] == cid);
            a0 = ok ? ((int)(uint16_t)z.x | ((int)z.y << 16)) : -1;  // (an unused window: as if absent)
            cb = cbw[wi1];
        }
        anc0[p1] = a0;
        cbits[p1] = (uint8_t)cb;
    }
    __syncthreads();
    if (pv1 && anc0[p1] >= 0) {  // centre window reference taps, fetched by all waves
        const int pk = anc0[p1];
        const int ax = pk & 0xFFFF, ay = pk >> 16;
        for (int t = wave; t < 36; t += PK_WAVES) {
            const int i = t / 6, j = t - 6 * i;
            cref[t * VM_P + p1] = (RT)tex_ref(a, ax - 5 + 2 * i, ay - 5 + 2 * j);
        }
    }
    __syncthreads();
    if (wave == 1) {  // tap mask and moments in wv_build_windows's tap order
        float sr = 0.0f, srr = 0.0f, ws = 0.0f;
        uint64_t m = 0;
        if (pv1 && anc0[p1] >= 0) {
            const int pk = anc0[p1];
            const int ax = pk & 0xFFFF, ay = pk >> 16;
            for (int t = 0; t < 36; ++t) {
                const int i = t / 6, j = t - 6 * i;
                if (cid != 0 && sa_at_dev(a, ax - 5 + 2 * i, ay - 5 + 2 * j) != cid) continue;
                const float r = (float)cref[t * VM_P + p1];
                m |= 1ull << t;
                sr += r;
                srr = fmaf(r, r, srr);
                ws += 1.0f;
            }
        }
        csr[p1] = sr;
        csrr[p1] = srr;
        cws[p1] = (uint8_t)ws;
        cmask[p1] = m;
    }
    __syncthreads();
    static_assert(PK_WAVES == 8, "k_weak_cand_g: wave h evaluates candidate h (8 anchor candidates)");
    const int h = wave;
    const uint32_t cb = cbits[p1];
    const bool want = pv1 && ((cb >> h) & 1u);
    float4 pl = make_float4(0.0f, 0.0f, 1.0f, 1.0f);
    if (want) {
        const short2 ap = anc1[h + 1];
        pl = a.plane[ap.x + ap.y * W];
    }
    const int pk0 = anc0[p1];
    const uint64_t tm = SA ? cmask[p1] : ~0ull;  // (no SA masks: every tap)
    uint32_t nlive = 0;
    for (int v = 0; v < N; ++v) {
        const int s = v + 1;
        const TT T(a, s);
        const SrcTex<F16> Q(a, s);
        const Hom Hm = homography(a, s, pl);
        float ptx, pty;
        project(Hm, (float)px1, (float)py1, ptx, pty);
        const bool alive = want && !(ptx >= (float)W || ptx < 0.0f || pty >= (float)H || pty < 0.0f);
        const bool has = alive && pk0 >= 0;
        const int ax = has ? (pk0 & 0xFFFF) : px1, ay = has ? (pk0 >> 16) : py1;
        bool live = has, dead = !alive;
        if (has) {
            float asx, asy;
            project(Hm, (float)ax, (float)ay, asx, asy);
            if (asx < 0 || asy < 0 || asx >= (float)W || asy >= (float)H) { live = false; dead = true; }
        }
        float center_cost = 0.0f;
        if (__ballot(live)) {
            const bool fast = live && window_rcp_ok(Hm, (float)(ax - 5), (float)(ay - 5));
            float ss = 0.0f, sss = 0.0f, srs = 0.0f;
            ncc_new_window<F16, 6, 2, PK_PIPE>(a, &cref[p1], VM_P, tm, Hm, ax, ay, live, fast, T, Q, ss, sss, srs);
            if (live) {
                const float wsum = (float)cws[p1];
                if (wsum != 0.0f) center_cost = ncc_finalize(csr[p1], csrr[p1], ss, sss, srs, wsum);
            }
        }
        nlive += live;
        // (k_weak_cand_comb reads it back and writes the candidate's cost in its place)
        if (want) out[((size_t)v * 8 + h) * (size_t)wc + wi1] = dead ? -1.0f : center_cost;
    }
    if (a.evals) wave_count(a.evals, 6, nlive);  // (profiling: centre windows evaluated)
}
// The focal combination (APD.cu:576-593, Softmax 431-446) of each (WEAK pixel, candidate) and view,
// a thread per (pixel, candidate): few registers and many waves in flight for the pair-cost gathers.
// `out` holds the centre cost (< 0: dead) and receives the candidate's cost in its place; the pixel's
// used windows (wmw) say which of its 8 pair ids exist. Block = 4 candidates x 64 pixels of one group.
// The block's pair ids ([WEAK index][window k][candidate h], 4 candidates = one 16-byte chunk per
// (pixel, k)) are staged in LDS with 16-byte loads of whole chunks first: a thread's 8 ids lie 32 B
// apart and the wave's 64 pixels 256 B apart, so loading them per thread issued 8 scattered 4-byte
// gathers touching 64 lines each.
#define COMB_STRIDE 33  // words per pixel slot in LDS (8 windows x 4 candidates, + 1 against bank conflicts)
__global__ __launch_bounds__(BLOCK) void k_weak_cand_comb(Args a, const int *__restrict__ list, int count,
                                                          const uint8_t *__restrict__ cbw, const uint8_t *__restrict__ wmw,
                                                          const uint32_t *__restrict__ pidx,
                                                          const float *__restrict__ pcost, float *__restrict__ out, int wc) {
    __shared__ uint32_t sid[VM_P * COMB_STRIDE];
    const int b = xcd_remap(blockIdx.x, gridDim.x);
    const int h0 = (b & 1) << 2, hl = threadIdx.x >> 6, h = h0 + hl;
    const int g0 = (b >> 1) * VM_P;
    const int lane = threadIdx.x & (WAVE - 1);
    for (int e = threadIdx.x; e < VM_P * 8; e += BLOCK) {
        const int slot = e >> 3, k = e & 7;
        if (g0 + slot < count) {
            const int wi2 = a.amap[list[g0 + slot]];
            const uint4 q = *reinterpret_cast<const uint4 *>(pidx + (size_t)wi2 * 64 + k * 8 + h0);
            uint32_t *d = &sid[slot * COMB_STRIDE + k * 4];
            d[0] = q.x; d[1] = q.y; d[2] = q.z; d[3] = q.w;
        }
    }
    __syncthreads();
    const int i = g0 + lane;
    if (i >= count) return;
    const int wi = a.amap[list[i]];
    if (!((cbw[wi] >> h) & 1u)) return;
    const int N = a.N, Np = (N + 3) & ~3;
    const uint32_t wm = wmw[wi];
    const float4 *pc4[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const uint32_t id = ((wm >> k) & 1u) ? sid[lane * COMB_STRIDE + k * 4 + hl] : 0u;
        pc4[k] = reinterpret_cast<const float4 *>(pcost + (size_t)id * Np);
    }
    for (int v0 = 0; v0 < N; v0 += 4) {
        float4 q[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) q[k] = ((wm >> k) & 1u) ? pc4[k][v0 >> 2] : make_float4(-1.0f, -1.0f, -1.0f, -1.0f);
#pragma unroll
        for (int dv = 0; dv < 4; ++dv) {
            const int v = v0 + dv;
            if (v >= N) break;
            float sc[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) sc[k] = dv == 0 ? q[k].x : dv == 1 ? q[k].y : dv == 2 ? q[k].z : q[k].w;
            float *o = out + ((size_t)v * 8 + h) * (size_t)wc + wi;
            *o = gp_combine(*o, sc);
        }
    }
}

// ---------------------------------------------------------------------------------------------
// post-sweep kernels
// ---------------------------------------------------------------------------------------------
// GetDepthandNormal (APD.cu:1694-1709)
__global__ __launch_bounds__(BLOCK) void k_depth_normal(Args a) {
    const int c = blockIdx.x * BLOCK + threadIdx.x;
    if (c >= a.HW) return;
    const int py = c / a.W, px = c - py * a.W;
    float4 p = a.plane[c];
    p.w = depth_from_plane(a.cams[0], p, px, py);
    a.plane[c] = to_world(a.cams[0], p);
}

// CheckerboardFilterStrong (APD.cu:1711-1821), over the Strong-sweep pixel list of one colour
__global__ __launch_bounds__(BLOCK) void k_filter(Args a, const int *__restrict__ list, int count) {
    const int li = blockIdx.x * BLOCK + threadIdx.x;
    if (li >= count) return;
    const int W = a.W, H = a.H;
    const int c = list[li];
    const int py = c / W, px = c - py * W;
    if (a.cost[c] < 0.001f) return;
    float f[21];
    int n = 0;
    f[n++] = a.plane[c].w;
    const int left = c - 1, leftleft = c - 3, up = c - W, upup = c - 3 * W;
    const int down = c + W, downdown = c + 3 * W, right = c + 1, rightright = c + 3;
    const uint8_t *wk = a.weak;
#define FADD(cond, idx) if ((cond) && wk[(idx)] == APD_STRONG) f[n++] = a.plane[(idx)].w
    FADD(py > 0, up);
    FADD(py > 2, upup);
    FADD(py > 4, upup - W * 2);
    FADD(py < H - 1, down);
    FADD(py < H - 3, downdown);
    FADD(py < H - 5, downdown + W * 2);
    FADD(px > 0, left);
    FADD(px > 2, leftleft);
    FADD(px > 4, leftleft - 2);
    FADD(px < W - 1, right);
    FADD(px < W - 3, rightright);
    FADD(px < W - 5, rightright + 2);
    FADD(py > 0 && px < W - 2, up + 2);
    FADD(py < H - 1 && px < W - 2, down + 2);
    FADD(py > 0 && px > 1, up - 2);
    FADD(py < H - 1 && px > 1, down - 2);
    FADD(px > 0 && py > 2, left - W * 2);
    FADD(px < W - 1 && py > 2, right - W * 2);
    FADD(px > 0 && py < H - 2, left + W * 2);
    FADD(px < W - 1 && py < H - 2, right + W * 2);
#undef FADD
    for (int i = 1; i < n; ++i) {
        float t = f[i];
        int j;
        for (j = i; j >= 1 && t < f[j - 1]; j--) f[j] = f[j - 1];
        f[j] = t;
    }
    const int m = n / 2;
    a.plane[c].w = (n % 2 == 0) ? (f[m - 1] + f[m]) / 2 : f[m];
}

// DepthToWeak (APD.cu:2103-2250): 61-sample disparity sweep of the selected views -> PixelState.
// The cost curve of each pixel is staged in LDS for the peak analysis.
// ---------------------------------------------------------------------------------------------
// View-major DepthToWeak (same function as k_depth_to_weak): a workgroup owns a 64-pixel row strip;
// the 61 x N (depth sample, view) NCC tasks run with lane = pixel and one source view per wave task,
// in chunks whose costs go to an LDS table; then the in-order weighted view sums per (pixel, depth)
// and the peak analysis. Waves skip every task none of their pixels selected (selected_views is
// spatially coherent), which the lanes = views layout could not.
// ---------------------------------------------------------------------------------------------
#ifndef DW_EARLY
#define DW_EARLY 1  // DepthToWeak: the inner disparity band first; pixels it decides skip the others
#endif
#ifndef DW_LDS_BUDGET
#define DW_LDS_BUDGET 53248  // bytes per workgroup: 3 per CU (8 disparities per chunk at N = 8; 2 per CU with 16 was 7 % slower)
#endif
struct DwLds {
    float refw[36 * VM_P];
    float pc[61 * VM_P];        // cost curve per pixel [d][p]
    float4 pl[VM_P];            // ref-frame plane
    float base[VM_P], disp[VM_P], wn[VM_P];
    float rmean[VM_P], rvar[VM_P];  // reference-window moments (RefWin)
    uint32_t sel[VM_P];
    uint8_t active[VM_P];
    uint8_t early[VM_P];        // decided WEAK by the inner disparity band (DW_EARLY)
    int undecided;              // some pixel of the workgroup is not (DW_EARLY)
    int pxy[VM_P];              // px | py << 16
    int vcnt[32];               // active pixels that selected view v
};
// + cost table [chunk][N][64] fp32, view weights [N][64] u8, per-view pixel slots [N][64] u8, the
// per-(disparity, pixel) plane terms of the chunk [3][chunk][64] fp32 (+ [chunk][64] plane w with
// geometric consistency) and evaluation flags [chunk][64] u8; the chunk is the largest that keeps
// the workgroup within DW_LDS_BUDGET
static inline size_t dw_per_disp(int N, bool geom) { return (size_t)N * VM_P * sizeof(float) + (size_t)VM_P * (13 + (geom ? 12 : 0)); }
static inline int dw_chunk(int N, bool geom, size_t extra) {
    const long fixed = (long)(sizeof(DwLds) + (size_t)2 * N * VM_P + extra);
    return std::max(1, std::min(61, (int)((DW_LDS_BUDGET - fixed) / (long)dw_per_disp(N, geom))));
}
static inline size_t dw_lds_bytes(int N, bool geom, int chunk) {
    return sizeof(DwLds) + (size_t)2 * N * VM_P + (size_t)chunk * dw_per_disp(N, geom);
}
template <bool F16, bool SA, bool DP = false>
__global__ __launch_bounds__(VM_BLOCK, VM_MINW) void k_depth_to_weak_vm(Args a, int chunk, int tw) {
    const int N = a.N, W = a.W, H = a.H;
    DwLds &L = *reinterpret_cast<DwLds *>(apd_dyn_lds);
    float *tcL = reinterpret_cast<float *>(&L + 1);                 // [chunk][N][64]
    uint8_t *wts = reinterpret_cast<uint8_t *>(tcL + chunk * N * VM_P);  // [N][64]
    uint8_t *vslot = wts + N * VM_P;                                 // [N][64] pixel slots per view
    const bool geom = a.geom != 0;
    float *ptm = reinterpret_cast<float *>(vslot + N * VM_P);         // [3][chunk][64] plane terms
    float *ptp = ptm + 3 * chunk * VM_P;                              // [3][chunk][64] the geometric term's world point
    uint8_t *pok = reinterpret_cast<uint8_t *>(ptp + (geom ? 3 * chunk * VM_P : 0));  // [chunk][64] evaluated
    SaWin *saw = reinterpret_cast<SaWin *>(pok + chunk * VM_P);       // [64] when a.sa_any
    const int tid = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & (WAVE - 1);
    const APD_C Cam &cam0 = a.cams[0];
    const int p = lane;
    // the workgroup's pixels: a tw x (64/tw) tile (XCD-aware tile order); pixels outside the image idle
    const int th = VM_P / tw, tiles_x = (W + tw - 1) / tw;
    const int blk = xcd_remap(blockIdx.x, gridDim.x);
    const size_t lr_slots = (size_t)gridDim.x * VM_P;  // LocalRefine hand-over: one slot per tile lane
    const int tx = blk % tiles_x, ty = blk / tiles_x;
    const int gx = tx * tw + (p % tw), gy = ty * th + (p / tw);
    const bool pv = gx < W && gy < H;
    const int px = min(gx, W - 1), py = min(gy, H - 1);
    const int c = py * W + px;
    // ---- P0: per-pixel inputs, view weights, reference window
    if (pv) {
        if (wave == 0) {
            L.pl[p] = to_ref(cam0, a.plane[c]);
            L.sel[p] = a.sel[c];
        }
        for (int v = wave; v < N; v += VM_WAVES) wts[v * VM_P + p] = a.vw[(size_t)v * a.HW + c];
        if (wave == 0) L.pxy[p] = px | (py << 16);
        for (int k = wave; k < 36; k += VM_WAVES) {
            const int i = k / 6, j = k - 6 * (k / 6);
            L.refw[k * VM_P + p] = tex_ref(a, px - 5 + 2 * i, py - 5 + 2 * j);
        }
        if (SA && wave == VM_WAVES - 1) saw[p] = sa_window(a, px, py);
    }
    __syncthreads();
    if (wave == 0 && pv) {  // baseline / weight norm over the selected views, in view order
        const uint32_t sv = L.sel[p];
        float base = 0.0f, wn = 0.0f;
        int valid = 0;
        for (int k = 0; k < N; ++k) {
            const APD_C Cam &sc = a.cams[k + 1];
            const float d0 = cam0.c[0] - sc.c[0], d1 = cam0.c[1] - sc.c[1], d2 = cam0.c[2] - sc.c[2];
            const float dk = sqrtf(d0 * d0 + d1 * d1 + d2 * d2);
            if ((sv >> k) & 1u) { wn += (float)wts[k * VM_P + p]; base += dk; valid++; }
        }
        const float od = L.pl[p].w;
        const bool border = px < 6 || py < 6 || px >= W - 6 || py >= H - 6;
        const bool active = !(border || od == 0) && valid != 0;
        if (active) base /= (float)valid;
        L.base[p] = base;
        L.wn[p] = wn;
        L.disp[p] = cam0.K[0] * base / od;
        L.active[p] = active;
    }
    __syncthreads();
    const RefWin rw = refwin_from_lds<VM_P>(&L.refw[p]);
    const bool act = pv && L.active[p] != 0;
    const float base = L.base[p], disp = L.disp[p], wn = L.wn[p];
    const uint32_t sv = L.sel[p];
    const float4 pl = L.pl[p];
    const float gf = a.gf;
    // Compacted (disparity, pixel) pairs: per view, only the active pixels that selected it (the
    // others' costs are never read), packed 64 to a wave-task, disparity-major, dealt round-robin over
    // the waves in view order -- the 4 waves sample one source image at neighbouring disparities.
    if (wave == 0) { L.rmean[p] = rw.mean; L.rvar[p] = rw.var; }
    auto build_vslot = [&](bool live) {
        for (int v = wave; v < N; v += VM_WAVES) {
            const bool on = live && ((sv >> v) & 1u);
            const uint64_t m = __ballot(on);
            if (on) vslot[v * VM_P + __popcll(m & ((1ull << lane) - 1ull))] = (uint8_t)p;
            if (lane == 0) L.vcnt[v] = __popcll(m);
        }
    };
    build_vslot(act);
    if (wave == 0) L.early[p] = 0;
    __syncthreads();
    // The peak analysis reads the costs of disparities 1..59 only (and disparity 0 when no peak is found
    // and weak_peak_radius >= 30): disparities 0 and 60 are evaluated only for the curve export.
    const bool ends = a.curve != nullptr || a.peak_radius >= 30;
    const int dlo = ends ? 0 : 1, dhi = ends ? 61 : 60;
    // Early decision (no curve export, peak radius R < 30): a pixel is STRONG only if some local
    // minimum i of its curve with |i - 30| <= R costs <= 0.5 -- otherwise the minimum peak lies
    // outside the radius, or costs > 0.5, or there is no peak, and P3 says WEAK whatever the other
    // disparities give. So the band [b0, b1) holding those i and their neighbours (and LocalRefine's
    // hand-over, disparities 25..35) runs first, and the pixels it decides skip the rest: the same
    // states, and the same curve values wherever P3 reads them.
    const bool early = DW_EARLY && !ends;
    const int b0 = early ? max(dlo, min(25, 29 - a.peak_radius)) : dlo;
    const int b1 = early ? min(dhi, max(36, 32 + a.peak_radius)) : dhi;
    bool verdicts = false;  // (workgroup-uniform)
    for (int sg = 0; sg < 3; ++sg) {
      const int s0 = sg == 0 ? b0 : (sg == 1 ? dlo : b1);
      const int s1 = sg == 0 ? b1 : (sg == 1 ? b0 : dhi);
      if (s0 >= s1) continue;
      if (sg > 0 && early && !verdicts) {
          // (once, after the band) the band's verdicts; the undecided pixels' task lists
          bool keep = false;
          if (wave == 0 && act) {
              const float *pcp = &L.pc[p];
              const int lo = max(2, 30 - a.peak_radius), hi = min(58, 30 + a.peak_radius);
              for (int i = lo; i <= hi; ++i) {
                  const float ci = pcp[i * VM_P];
                  keep = keep || (pcp[(i - 1) * VM_P] > ci && pcp[(i + 1) * VM_P] > ci && ci <= 0.5f);
              }
              L.early[p] = !keep;
          }
          if (wave == 0) {
              const bool any_keep = __ballot(keep) != 0ull;
              if (lane == 0) L.undecided = any_keep;
          }
          __syncthreads();
          if (!L.undecided) break;  // every pixel decided (or inactive)
          build_vslot(act && !L.early[p]);
          verdicts = true;
          __syncthreads();
      }
      const int nch = (s1 - s0 + chunk - 1) / chunk, cseg = (s1 - s0 + nch - 1) / nch;  // even chunks
      for (int d0 = s0; d0 < s1; d0 += cseg) {
        const int dc = min(cseg, s1 - d0);
        // t / dc for the task decode as a multiply-high: with m = ceil(2^32 / dc), umulhi(t, m) == t / dc
        // for every t < 2^32 / dc (here t < 61 * 64); dc == 1 (m = 2^32) is taken apart
        const uint32_t mdc = dc > 1 ? 0xFFFFFFFFu / (uint32_t)dc + 1u : 0u;
        // ---- P0': the view-independent terms of each (disparity, pixel) plane, once instead of once per
        // selected view: depth range test, plane w (dist2origin), homography terms n^T Kr^-1 / w
        for (int e = tid; e < dc * VM_P; e += VM_BLOCK) {
            const int q = e & (VM_P - 1), dd = e >> 6;
            const float pdepth = cam0.K[0] * L.base[q] / (L.disp[q] + (float)(d0 + dd - 30));
            const bool ok = L.active[q] != 0 && !(pdepth < a.dmin || pdepth > a.dmax);
            pok[e] = ok;
            if (ok) {
                const int xy = L.pxy[q];
                float4 tp = L.pl[q];
                tp.w = dist2origin(cam0, xy & 0xFFFF, xy >> 16, pdepth, tp);
                const float3 m = plane_terms(a, tp);
                ptm[e] = m.x; ptm[chunk * VM_P + e] = m.y; ptm[2 * chunk * VM_P + e] = m.z;
                if (geom) {  // (geom_cost's view-independent head, once per (disparity, pixel))
                    float P[3];
                    geom_point(a, xy & 0xFFFF, xy >> 16, tp, P);
                    ptp[e] = P[0]; ptp[chunk * VM_P + e] = P[1]; ptp[2 * chunk * VM_P + e] = P[2];
                }
            }
        }
        __syncthreads();
        // ---- P1: (depth, view) tasks
        uint64_t defer = 0;
        uint32_t n_ncc = 0, n_geo = 0;  // profiling: evaluations issued by this lane
        {
            // the per-view counts are read through readfirstlane: v stays wave-uniform (SGPR), so the
            // view's homography constants, cameras and texel base come through scalar loads
            int v = 0, vb = 0, nv = __builtin_amdgcn_readfirstlane(L.vcnt[0]), tv = (dc * nv + 63) >> 6;
            for (int j = wave, k = 0;; j += VM_WAVES, ++k) {
                while (v < N && j >= vb + tv) {
                    vb += tv;
                    if (++v < N) { nv = __builtin_amdgcn_readfirstlane(L.vcnt[v]); tv = (dc * nv + 63) >> 6; }
                }
                if (v >= N) break;
                const int t = (j - vb) * 64 + lane;
                const bool has = t < dc * nv;
                int dd = 0, q = 0;
                if (has) {
                    // pixel-major: a wave-task's 64 lanes are ~64/dc neighbouring pixels x their dc
                    // disparities, so one gather instruction spans a short stretch of epipolar lines
                    const int r = dc > 1 ? (int)__umulhi((uint32_t)t, mdc) : t;
                    dd = t - r * dc;
                    q = vslot[v * VM_P + r];
                }
                const int xy = L.pxy[q];
                const int qx = xy & 0xFFFF, qy = xy >> 16;
                const int e = dd * VM_P + q;
                const bool eval = has && pok[e];
                n_ncc += eval;
                n_geo += eval && geom;
                const RefWin rwq{&L.refw[q], L.rmean[q], L.rvar[q], SA ? &saw[q] : nullptr};
                float tc = 0.0f;
                bool slow = false;
                if (eval) {
                    const float3 m = make_float3(ptm[e], ptm[chunk * VM_P + e], ptm[2 * chunk * VM_P + e]);
                    tc = ncc_old_fast_h<F16, VM_P, DP>(a, qx, qy, v + 1, homography_terms(a, v + 1, m), rwq, slow);
                    if (slow) defer |= 1ull << k;
                }
                float g = 0.0f;
                if (eval && geom) {
                    const float P[3] = {ptp[e], ptp[chunk * VM_P + e], ptp[2 * chunk * VM_P + e]};
                    g = geom_cost_p(a, qx, qy, v + 1, P);
                }
                const int pd = d0 + dd - 30;
                if (a.lr_ncc && eval && !slow && pd >= -5 && pd <= 5) {
                    const size_t i = (size_t)((pd + 5) * N + v) * lr_slots + (size_t)blk * VM_P + q;
                    a.lr_ncc[i] = tc;
                    if (geom) a.lr_geo[i] = g;
                }
                if (eval && geom) tc = fmaf(gf, g, tc);
                if (has) tcL[(dd * N + v) * VM_P + q] = tc;
            }
        }
        while (defer) {
            const int k = __builtin_ctzll(defer);
            defer &= defer - 1;
            const int j = wave + k * VM_WAVES;
            int v = 0, vb = 0, nv = __builtin_amdgcn_readfirstlane(L.vcnt[0]), tv = (dc * nv + 63) >> 6;
            while (j >= vb + tv) { vb += tv; ++v; nv = __builtin_amdgcn_readfirstlane(L.vcnt[v]); tv = (dc * nv + 63) >> 6; }
            const int t = (j - vb) * 64 + lane;
            if (t < dc * nv) {
                const int r = dc > 1 ? (int)__umulhi((uint32_t)t, mdc) : t, dd = t - r * dc;
                const int q = vslot[v * VM_P + r], xy = L.pxy[q];
                const int qx = xy & 0xFFFF, qy = xy >> 16;
                const float pdepth = cam0.K[0] * L.base[q] / (L.disp[q] + (float)(d0 + dd - 30));
                float4 tp = L.pl[q];
                tp.w = dist2origin(cam0, qx, qy, pdepth, tp);  // (the same w as P0', recomputed off the hot path)
                float tc = ncc_old_slow<F16>(a.self, qx, qy, v + 1, tp, &L.refw[q], VM_P, L.rmean[q], L.rvar[q]);
                const float g = geom ? geom_cost(a, qx, qy, v + 1, tp) : 0.0f;
                const int pd = d0 + dd - 30;
                if (a.lr_ncc && pd >= -5 && pd <= 5) {
                    const size_t i = (size_t)((pd + 5) * N + v) * lr_slots + (size_t)blk * VM_P + q;
                    a.lr_ncc[i] = tc;
                    if (geom) a.lr_geo[i] = g;
                }
                if (geom) tc = fmaf(gf, g, tc);
                tcL[(dd * N + v) * VM_P + q] = tc;
            }
        }
        if (a.evals) { wave_count(a.evals, 3, n_ncc); wave_count(a.evals, 4, n_geo); }
        __syncthreads();
        // ---- P2: in-order weighted view sums per (pixel, depth)
        for (int dd = wave; dd < dc; dd += VM_WAVES) {
            const int d = d0 + dd;
            const float pdepth = cam0.K[0] * base / (disp + (float)(d - 30));
            const bool in_range = !(pdepth < a.dmin || pdepth > a.dmax);
            float pval = 0.0f;
            for (int k = 0; k < N; ++k)
                if ((sv >> k) & 1u) pval = fmaf(tcL[(dd * N + k) * VM_P + p], (float)wts[k * VM_P + p], pval);
            pval /= wn;
            const float val = in_range ? ((2.0f > pval) ? pval : 2.0f) : 2.0f;
            L.pc[d * VM_P + p] = val;
            if (a.curve && act) a.curve[(size_t)c * 61 + d] = val;
        }
        __syncthreads();
      }
    }
    // ---- P3: peak analysis (APD.cu:2200-2248)
    if (wave == 0 && pv) {
        int state = APD_UNKNOWN;
        if (act && L.early[p]) {
            state = APD_WEAK;  // (decided by the band)
        } else if (act) {
            const float *pc = &L.pc[p];
            int cnt = 0, min_peak = 0;
            float min_cost = 2.0f;
            uint64_t peaks = 0;
            for (int i = 2; i < 59; ++i) {
                const float ci = pc[i * VM_P];
                if (pc[(i - 1) * VM_P] > ci && pc[(i + 1) * VM_P] > ci) {
                    peaks |= 1ull << i;
                    cnt++;
                    if (ci < min_cost) { min_peak = i; min_cost = ci; }
                }
            }
            if (abs(min_peak - 30) > a.peak_radius || pc[min_peak * VM_P] > 0.5f) {
                state = APD_WEAK;
            } else if (cnt == 1) {
                state = (pc[min_peak * VM_P] <= 0.15f) ? APD_STRONG : APD_WEAK;
            } else {
                float var = 0.0f;
                for (int i = 2; i < 59; ++i) {
                    if (((peaks >> i) & 1ull) && i != min_peak) { float dd = pc[i * VM_P] - min_cost; var = fmaf(dd, dd, var); }
                }
                var = sqrtf(var);
                var /= (float)(cnt - 1);
                state = (var > 0.2f) ? APD_STRONG : APD_WEAK;
            }
        }
        a.weak[c] = (uint8_t)state;
    }
}

// Pixel tile of a view-major pixel kernel (RandomInit / DepthToWeak / LocalRefine): tw x 64/tw pixels
// of the image in XCD-aware tile order; lanes outside the image idle.
struct TilePix {
    int px, py, c;
    bool pv;
};
__device__ __forceinline__ TilePix tile_pix(const Args &a, int tw, int lane) {
    const int th = VM_P / tw, tiles_x = (a.W + tw - 1) / tw;
    const int blk = xcd_remap(blockIdx.x, gridDim.x);
    const int gx = (blk % tiles_x) * tw + (lane % tw), gy = (blk / tiles_x) * th + (lane / tw);
    TilePix t;
    t.pv = gx < a.W && gy < a.H;
    t.px = min(gx, a.W - 1);
    t.py = min(gy, a.H - 1);
    t.c = t.py * a.W + t.px;
    return t;
}

// ---------------------------------------------------------------------------------------------
// View-major RandomInitialization + ComputeMultiViewInitialCostandSelectedViews (same function as
// k_random_init): per-pixel plane (RNG draws in one lane), then the N per-view costs as wave tasks,
// then the stable top-k of the N costs per pixel.
// ---------------------------------------------------------------------------------------------
struct RiLds {
    float refw[36 * VM_P];
    float4 pl[VM_P];
};
// RandomInitialization when use_APD: the WEAK pixels' NCC-New through ncc_new_vm (reference side
// built once per pixel in LDS, as in the Weak sweep) instead of the per-call ncc_new
template <bool F16>
struct RiApdLds {
    WvRefT<F16> w;
    RiLds r;
};
// dynamic LDS of k_random_init_vm<F16, APD>: the layout struct, then the [N][64] cost table
template <bool F16, bool APD>
static inline size_t ri_lds_bytes(int N) {
    return (APD ? sizeof(RiApdLds<F16>) : sizeof(RiLds)) + (size_t)N * VM_P * sizeof(float);
}
template <bool F16, bool APD, bool SA>
__global__ __launch_bounds__(VM_BLOCK, VM_MINW) void k_random_init_vm(Args a, int tw) {
    const int N = a.N;
    WvRefT<F16> *W = APD ? &reinterpret_cast<RiApdLds<F16> *>(apd_dyn_lds)->w : nullptr;
    if constexpr (APD) wv_init_lut(*W);  // (read after the reference side's barrier)
    RiLds &L = APD ? reinterpret_cast<RiApdLds<F16> *>(apd_dyn_lds)->r : *reinterpret_cast<RiLds *>(apd_dyn_lds);
    float *cvL = APD ? reinterpret_cast<float *>(reinterpret_cast<RiApdLds<F16> *>(apd_dyn_lds) + 1)
                     : reinterpret_cast<float *>(&L + 1);  // [N][64]
    SaWin *saw = reinterpret_cast<SaWin *>(sa_lds_align(cvL + N * VM_P));  // [64] when a.sa_any
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & (WAVE - 1);
    const TilePix T = tile_pix(a, tw, lane);
    const int p = lane, px = T.px, py = T.py, c = T.c;
    const APD_C Cam &cam = a.cams[0];
    if (T.pv) {
        if (wave == 0) {
            float4 pl;
            if (a.state == APD_FIRST_INIT) {
                Rng g(a.seed_lo, a.seed_hi, (uint32_t)c, ORD_INIT);
                float depth = g.uniform() * (a.dmax - a.dmin) + a.dmin;
                pl = random_normal(cam, px, py, g, depth);
                pl.w = dist2origin(cam, px, py, depth, pl);
            } else {
                pl = to_ref(cam, a.plane[c]);
                float depth = pl.w;
                pl.w = dist2origin(cam, px, py, depth, pl);
            }
            L.pl[p] = pl;
        }
        for (int k = wave; k < 36; k += VM_WAVES) {
            const int i = k / 6, j = k - 6 * (k / 6);
            L.refw[k * VM_P + p] = tex_ref(a, px - 5 + 2 * i, py - 5 + 2 * j);
        }
        if (SA && wave == VM_WAVES - 1) saw[p] = sa_window(a, px, py);
        if constexpr (APD) {
            if (a.weak[c] == APD_WEAK) {  // the NCC-New reference side (anchors, windows, SA masks)
                const APD_G short2 *anc = a.anchors + (size_t)a.amap[c] * 9;
                const int cid = a.sa_any ? a.sa[c] : 0;
                if (wave == 0) {
                    uint32_t awin = 0;
                    for (int k = 0; k < 9; ++k) {
                        const short2 ap = anc[k];
                        const bool ok = !(ap.x == -1 || ap.y == -1);
                        W->anc[k * VM_P + p] = ok ? ((int)(uint16_t)ap.x | ((int)ap.y << 16)) : -1;
                        if (ok && !(cid != 0 && sa_at_dev(a, ap.x, ap.y) != cid)) awin |= 1u << k;
                    }
                    W->flags[p] = awin << 16;
                }
                wv_build_windows<F16>(a, *W, p, anc, cid, wave, VM_WAVES);
            }
        }
    }
    __syncthreads();
    RefWin rw = refwin_from_lds<VM_P>(&L.refw[p]);
    if (SA) rw.sa = &saw[p];
    const bool use_new = a.use_apd && a.weak[c] == APD_WEAK;
    const float4 pl = L.pl[p];
    uint64_t defer = 0;
    for (int v = wave, k = 0; v < N; v += VM_WAVES, ++k) {
        float cv = 0.0f;
        float nv = 0.0f;
        if constexpr (APD) {
            bool seldep = false;
            nv = ncc_new_vm<F16>(a, *W, p, px, py, v + 1, pl, T.pv && use_new, &seldep);  // all lanes
            if (a.wcur && T.pv && use_new) a.wcur[(size_t)v * a.HW + c] = seldep ? __int_as_float(0x7fc00000) : nv;
        }
        if (T.pv) {
            if (use_new) {  // (APD instantiations only: use_new needs a.use_apd)
                cv = nv;
            } else {
                bool slow;
                cv = ncc_old_fast<F16, VM_P>(a, px, py, v + 1, pl, rw, slow);
                if (slow) defer |= 1ull << k;
            }
        }
        cvL[v * VM_P + p] = cv;
    }
    while (defer) {
        const int k = __builtin_ctzll(defer);
        defer &= defer - 1;
        const int v = wave + k * VM_WAVES;
        cvL[v * VM_P + p] = ncc_old_slow<F16>(a.self, px, py, v + 1, pl, rw.r, VM_P, rw.mean, rw.var);
    }
    __syncthreads();
    if (wave == 0 && T.pv) {
        // stable top-k of the N costs (insertion sort, APD.cu:3-12, 754-769)
        const int topk_max = 4;
        float t0 = 0, t1 = 0, t2 = 0, t3 = 0;
        int nt = 0, nvalid = 0;
        for (int k = 0; k < N; ++k) {
            const float x = cvL[k * VM_P + p];
            if (x < APD_COST_MAX) nvalid++;
            int q = (nt > 0 && t0 <= x) + (nt > 1 && t1 <= x) + (nt > 2 && t2 <= x) + (nt > 3 && t3 <= x);
            if (q < topk_max) {
                if (q <= 2) t3 = t2;
                if (q <= 1) t2 = t1;
                if (q <= 0) t1 = t0;
                if (q == 0) t0 = x;
                else if (q == 1) t1 = x;
                else if (q == 2) t2 = x;
                else t3 = x;
                if (nt < topk_max) nt++;
            }
        }
        const int top_k = min(nvalid, a.top_k);
        const float thr = top_k <= 1 ? t0 : (top_k == 2 ? t1 : (top_k == 3 ? t2 : t3));
        float cost_out = APD_COST_MAX;
        uint32_t sv = 0;
        if (top_k > 0) {
            float sum = 0.0f;
            sum += t0;
            if (top_k > 1) sum += t1;
            if (top_k > 2) sum += t2;
            if (top_k > 3) sum += t3;
            cost_out = sum / (float)top_k;
            for (int k = 0; k < N; ++k) if (cvL[k * VM_P + p] <= thr) sv |= 1u << k;
        }
        a.plane[c] = pl;
        a.cost[c] = cost_out;
        if (a.wcur && !use_new)  // the Strong sweep's first launches re-evaluate exactly these
            for (int k = 0; k < N; ++k) a.wcur[(size_t)k * a.HW + c] = cvL[k * VM_P + p];
        a.sel_next[c] = sv;  // launch-start snapshot semantics (oracle k_random_init)
    }
}

// ---------------------------------------------------------------------------------------------
// View-major LocalRefine (same function as k_local_refine, APD.cu:2346-2432): the current-depth costs
// as N wave tasks, then the +-5 disparity candidates as (candidate, view) tasks in LDS chunks, with
// the in-order weighted sums (NCC and geometric terms weighted separately, as the reference adds them).
// ---------------------------------------------------------------------------------------------
struct LrLds {
    float refw[36 * VM_P];
    float4 pl[VM_P];
    float base[VM_P], disp[VM_P], wn[VM_P], cost_now[VM_P];
    uint32_t sel[VM_P];
    int run[VM_P];
};
static inline int lr_chunk(int N) { return std::max(1, std::min(11, 32768 / (2 * N * VM_P * (int)sizeof(float)))); }
static inline size_t lr_lds_bytes(int N) {
    return sizeof(LrLds) + (size_t)(2 * lr_chunk(N) + 1) * N * VM_P * sizeof(float) + (size_t)N * VM_P * sizeof(int);
}
template <bool F16, bool SA>
__global__ __launch_bounds__(VM_BLOCK, VM_MINW) void k_local_refine_vm(Args a, int chunk, int tw) {
    const int N = a.N;
    LrLds &L = *reinterpret_cast<LrLds *>(apd_dyn_lds);
    float *t0L = reinterpret_cast<float *>(&L + 1);   // [N][64] current-depth costs
    float *nvL = t0L + N * VM_P;                      // [chunk][N][64] NCC
    float *gvL = nvL + chunk * N * VM_P;              // [chunk][N][64] gf * geometric
    int *wts = reinterpret_cast<int *>(gvL + chunk * N * VM_P);
    SaWin *saw = reinterpret_cast<SaWin *>(wts + N * VM_P);           // [64] when a.sa_any
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & (WAVE - 1);
    const TilePix T = tile_pix(a, tw, lane);
    const int p = lane, px = T.px, py = T.py, c = T.c;
    const APD_C Cam &cam0 = a.cams[0];
    const bool geom = a.geom != 0;
    const float gf = a.gf;
    if (T.pv) {
        if (wave == 0) {
            L.pl[p] = to_ref(cam0, a.plane[c]);
            L.sel[p] = a.sel[c];
        }
        for (int v = wave; v < N; v += VM_WAVES) wts[v * VM_P + p] = a.vw[(size_t)v * a.HW + c];
        for (int k = wave; k < 36; k += VM_WAVES) {
            const int i = k / 6, j = k - 6 * (k / 6);
            L.refw[k * VM_P + p] = tex_ref(a, px - 5 + 2 * i, py - 5 + 2 * j);
        }
        if (SA && wave == VM_WAVES - 1) saw[p] = sa_window(a, px, py);
    }
    __syncthreads();
    RefWin rw = refwin_from_lds<VM_P>(&L.refw[p]);
    if (SA) rw.sa = &saw[p];
    const float4 pl = L.pl[p];
    const float od = pl.w;
    const uint32_t sv = L.sel[p];
    const bool live = T.pv && od != 0;
    // ---- current-depth costs, one task per view
    {
        uint64_t defer = 0;
        for (int v = wave, k = 0; v < N; v += VM_WAVES, ++k) {
            float tc0 = 0.0f;
            if (live && ((sv >> v) & 1u)) {
                float4 t = pl;
                t.w = dist2origin(cam0, px, py, od, t);
                bool slow;
                tc0 = ncc_old_fast<F16, VM_P>(a, px, py, v + 1, t, rw, slow);
                if (slow) defer |= 1ull << k;
                if (geom) tc0 = fmaf(gf, geom_cost(a, px, py, v + 1, t), tc0);
            }
            t0L[v * VM_P + p] = tc0;
        }
        while (defer) {
            const int k = __builtin_ctzll(defer);
            defer &= defer - 1;
            const int v = wave + k * VM_WAVES;
            float4 t = pl;
            t.w = dist2origin(cam0, px, py, od, t);
            float tc0 = ncc_old_slow<F16>(a.self, px, py, v + 1, t, rw.r, VM_P, rw.mean, rw.var);
            if (geom) tc0 = fmaf(gf, geom_cost(a, px, py, v + 1, t), tc0);
            t0L[v * VM_P + p] = tc0;
        }
    }
    __syncthreads();
    if (wave == 0 && T.pv) {
        float cost_now = 0.0f, base = 0.0f, wn = 0.0f;
        int valid = 0;
        for (int k = 0; k < N; ++k) {
            const APD_C Cam &sc = a.cams[k + 1];
            const float d0 = cam0.c[0] - sc.c[0], d1 = cam0.c[1] - sc.c[1], d2 = cam0.c[2] - sc.c[2];
            const float dk = sqrtf(d0 * d0 + d1 * d1 + d2 * d2);
            if ((sv >> k) & 1u) {
                const float wk = (float)wts[k * VM_P + p];
                cost_now = fmaf(t0L[k * VM_P + p], wk, cost_now);
                wn += wk;
                base += dk;
                valid++;
            }
        }
        const bool run = live && !(wn == 0 || valid == 0);
        if (run) { cost_now /= wn; base /= (float)valid; }
        L.cost_now[p] = cost_now;
        L.base[p] = base;
        L.wn[p] = wn;
        L.disp[p] = cam0.K[0] * base / od;
        L.run[p] = run;
    }
    __syncthreads();
    const bool run = T.pv && L.run[p] != 0;
    const float base = L.base[p], disp = L.disp[p], wn = L.wn[p];
    // DepthToWeak evaluated this pixel's samples (same plane, views, base line and depths: active
    // there = not within 6 px of the border, od != 0, a selected view; run implies the last two)
    const bool dwc = a.lr_ncc != nullptr &&
                     !(px < 6 || py < 6 || px >= a.W - 6 || py >= a.H - 6);
    const size_t lr_slots = (size_t)gridDim.x * VM_P, lr_px = (size_t)xcd_remap(blockIdx.x, gridDim.x) * VM_P + p;
    float min_cost = 2.0f, best = od;  // tracked by wave 0's lane of the pixel
    for (int d0 = 0; d0 < 11; d0 += chunk) {
        const int dc = min(chunk, 11 - d0);
        uint64_t defer = 0;
        for (int u = wave, k = 0; u < dc * N; u += VM_WAVES, ++k) {
            const int v = u / dc, dd = u - dc * v, t = dd * N + v;
            const int d = d0 + dd - 5;
            const float pdepth = cam0.K[0] * base / (disp + (float)d);
            const bool in_range = !(pdepth < a.dmin || pdepth > a.dmax);
            float nv = 0.0f, gv = 0.0f;
            if (run && in_range && ((sv >> v) & 1u)) {
                if (dwc) {
                    const size_t i = (size_t)((d + 5) * N + v) * lr_slots + lr_px;
                    nv = a.lr_ncc[i];
                    if (geom) gv = gf * a.lr_geo[i];
                } else {
                    float4 tp = pl;
                    tp.w = dist2origin(cam0, px, py, pdepth, tp);
                    bool slow;
                    nv = ncc_old_fast<F16, VM_P>(a, px, py, v + 1, tp, rw, slow);
                    if (slow) defer |= 1ull << k;
                    if (geom) gv = gf * geom_cost(a, px, py, v + 1, tp);
                }
            }
            nvL[t * VM_P + p] = nv;
            gvL[t * VM_P + p] = gv;
        }
        while (defer) {
            const int k = __builtin_ctzll(defer);
            defer &= defer - 1;
            const int u = wave + k * VM_WAVES, v = u / dc, dd = u - dc * v, t = dd * N + v;
            const float pdepth = cam0.K[0] * base / (disp + (float)(d0 + dd - 5));
            float4 tp = pl;
            tp.w = dist2origin(cam0, px, py, pdepth, tp);
            nvL[t * VM_P + p] = ncc_old_slow<F16>(a.self, px, py, v + 1, tp, rw.r, VM_P, rw.mean, rw.var);
        }
        __syncthreads();
        if (wave == 0 && T.pv) {
            for (int dd = 0; dd < dc; ++dd) {
                const float pdepth = cam0.K[0] * base / (disp + (float)(d0 + dd - 5));
                const bool in_range = !(pdepth < a.dmin || pdepth > a.dmax);
                float tc = 0.0f;
                for (int k = 0; k < N; ++k) {
                    if ((sv >> k) & 1u) {
                        const float wk = (float)wts[k * VM_P + p];
                        tc = fmaf(nvL[(dd * N + k) * VM_P + p], wk, tc);
                        if (geom) tc = fmaf(gvL[(dd * N + k) * VM_P + p], wk, tc);
                    }
                }
                tc /= wn;
                if (run && in_range && tc < min_cost) { min_cost = tc; best = pdepth; }
            }
        }
        __syncthreads();
    }
    if (wave == 0 && run && (double)(L.cost_now[p] - min_cost) > 0.1) a.plane[c].w = best;
}

// ConfidenceCompute (APD.cu:2282-2344)
__global__ __launch_bounds__(BLOCK) void k_confidence(Args a) {
    const int c = blockIdx.x * BLOCK + threadIdx.x;
    if (c >= a.HW) return;
    const int W = a.W;
    const int py = c / W, px = c - py * W;
    a.conf[c] = 0;
    const APD_C Cam &rc = a.cams[0];
    const uint32_t sv = a.sel[c];
    const float rd = a.plane[c].w;
    if (rd <= 0.0f) { a.weak[c] = APD_UNKNOWN; return; }
    float P[3];
    world_point(rc, (float)px, (float)py, rd, P);
    int nc = 1;
    for (int i = 0; i < a.N; ++i) {
        if (!((sv >> i) & 1u)) continue;
        const int s = i + 1;
        const APD_C Cam &sc = a.cams[s];
        float sx, sy, sd;
        project_cam(P, sc, sx, sy, sd);
        const float src_depth = a.depth[(size_t)s * a.HW + trunc_clamp(sy, a.H) * W + trunc_clamp(sx, W)];
        if (src_depth <= 0.0f) continue;
        nc += 1;
        float Q[3];
        world_point(sc, sx, sy, src_depth, Q);
        float bx, by, refd;
        project_cam(Q, rc, bx, by, refd);
        const float dx = (float)px - bx, dy = (float)py - by;
        if (sqrtf(dx * dx + dy * dy) <= 2.0f) nc += 2;
        if (fabsf(rd - refd) / rd <= 0.02f) nc += 2;
    }
    if (nc > 255) nc = 255;
    a.conf[c] = (uint8_t)nc;
}

// cv::resize INTER_NEAREST between device buffers with the host library's index arithmetic
// (host/image.cpp resize_nearest: floor(x * (1 / (dw / sw))) in double, clamped to the source)
__global__ __launch_bounds__(BLOCK) void k_resize_nearest(const uint8_t *__restrict__ src, int sw, int sh,
                                                        uint8_t *__restrict__ dst, int dw, int dh, int elem) {
    const double ifx = 1.0 / ((double)dw / sw), ify = 1.0 / ((double)dh / sh);
    const size_t n = (size_t)dw * dh;
    for (size_t i = blockIdx.x * (size_t)BLOCK + threadIdx.x; i < n; i += (size_t)gridDim.x * BLOCK) {
        const int y = (int)(i / dw), x = (int)(i - (size_t)y * dw);
        const int sx = min((int)floor(x * ifx), sw - 1), sy = min((int)floor(y * ify), sh - 1);
        const uint8_t *s = src + ((size_t)sy * sw + sx) * elem;
        uint8_t *d = dst + i * elem;
        if (elem == 4) {
            *reinterpret_cast<uint32_t *>(d) = *reinterpret_cast<const uint32_t *>(s);
        } else if (elem == 16) {
            *reinterpret_cast<uint4 *>(d) = *reinterpret_cast<const uint4 *>(s);
        } else {
            for (int b = 0; b < elem; ++b) d[b] = s[b];
        }
    }
}

// ProcessProblem's epilogue (main.cpp:168-178) on the device: depth = plane.w, 0 outside
// [depth_min, depth_max] (NaN kept, as apd_epilogue); planes_out = (normal, that depth)
__global__ __launch_bounds__(BLOCK) void k_result_epilogue(const float4 *__restrict__ planes, size_t n, float dmin,
                                                         float dmax, float *__restrict__ depth_out,
                                                         float4 *__restrict__ planes_out) {
    for (size_t i = blockIdx.x * (size_t)BLOCK + threadIdx.x; i < n; i += (size_t)gridDim.x * BLOCK) {
        float4 p = planes[i];
        if (p.w < dmin || p.w > dmax) p.w = 0.0f;
        if (depth_out) depth_out[i] = p.w;
        if (planes_out) planes_out[i] = p;
    }
}

// =============================================================================================
// host side: context, buffers, C ABI
// =============================================================================================
namespace {

struct DevBuf {
    void *p = nullptr;
    size_t bytes = 0;
};

const char *g_global_err = "";
std::string g_global_err_store;

void set_global_err(const std::string &s) {
    g_global_err_store = s;
    g_global_err = g_global_err_store.c_str();
}

}  // namespace

struct apd_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    // side streams of the loop body: RANSACToGetFitPlane and k_gp_cost run beside the anchor
    // candidates' centre windows (none of them reads what another writes); the ctx stream joins them
    // before the kernels that read their outputs. ev_fork / ev_side: ordering only (no timing).
    hipStream_t side[2] = {nullptr, nullptr};
    hipEvent_t ev_fork = nullptr, ev_side[2] = {nullptr, nullptr};
    bool overlap = true;           // APD_NO_OVERLAP=1: the loop body on the ctx stream alone
    std::string err;
    // buffers
    DevBuf imgs, quad, depth, views, cams, plane, cost, sel, sel2, vw, weak, conf, sa, amap, anchors, reliable, nearest,
        fit, curve, lists, rowcnt, rowoff, totals, near_off, dargs, evals, near_ring, near_g, wcand, lrs, wcur, arec, ga_stage,
        wlist, gp_cb, gp_cnt, gp_cur, gp_refs, gp_ccnt, gp_cbase, gp_plist, gp_pidx, gp_pcost, gp_tmp, dpairs, gp_cls;
    int n_near = 0;
    int host_stat[4] = {0, 0, 0, 0};  // apd_set_problem's read-back (see there)
    int near_levels = 0;  // confidence levels of k_near_columns (max confidence + 1), 0 = ring search
    Args args{};
    bool loaded = false, prepared = false;
    int optional_fallbacks = 0;    // optional buffers try_ensure could not allocate
    bool prep_timed = false;       // the prepare events (ev[0..3], ev[14], ev[15]) of the last apd_stage_prepare
    int dw_tile_w = 8;             // DepthToWeak pixel tile width (64 / tile height); APD_DW_TILE_W
    int tile_w = 16;               // sweep list tile width (tile = tile_w x 256/tile_w positions); APD_TILE_W
                                   // (16 x 16: -1 % per C3 iteration against 8 x 32, profiles/r4_ab_tile_shape.txt)
    bool cand_pairs = true;        // Weak sweep candidates through the image-wide pair table; APD_NO_CAND_PAIRS=1
                                   // leaves them to the sweep
    bool gp_on = false;            // the pair table of the prepared problem is built (apd_stage_prepare)
    bool ga_split = true;          // GenAnchors' RANSAC in k_gen_anchors_fit; APD_NO_GA_SPLIT=1: in k_gen_anchors
    bool rec_on = false;           // the anchor-window records of the prepared problem are built (k_anchor_rec)
    bool dtex = true;              // DepthToWeak over pre-differenced fp16 texels (FastTexD); APD_NO_DTEX=1 disables
    int gp_np = 0;                 // its distinct pairs
    bool gp_one_pass = true;       // k_gp_dedup in one pass (atomic plist ranges); APD_GP_TWO_PASS=1: count + write
    bool gp_async = true;          // the one-pass table enqueued without host round trips; APD_GP_SYNC=1: build_global_pairs
    bool gp_pending = false;       // an async table is in flight (finish_global_pairs completes it)
    size_t gp_pcap = 0;            // its pair-list capacity
    int ncu = 256;                 // compute units of the device (persistent grids)
    bool gp_place = true;          // k_gp_count_loc + k_gp_place; APD_GP_FILL=1: k_gp_count + k_gp_fill (atomics twice)
    bool gp_small = true;          // one-pass small / medium anchors in smaller-table workgroups; APD_GP_NO_SMALL=1: all in the 48 KiB one
    int gp_cap_factor = 2;         // one-pass plist capacity in pairs per reference (8 after an overflow)
    bool lr_handover = true;       // LocalRefine reads DepthToWeak's samples; APD_NO_LR_HANDOVER=1 disables
    bool wcur_on = true;           // RandomInit keeps WEAK current-plane costs for iteration 0; APD_NO_WCUR=1 disables
    bool wcur_fresh = false;       // they belong to the current planes (set by prepare, cleared by iteration)
    int weak_count = 0;
    size_t lrs_need = 0;           // bytes of the LocalRefine hand-over this problem uses (0: none)
    int cnt[4] = {0, 0, 0, 0};     // strong black, strong red, weak black, weak red
    size_t list_cap = 0;
    bool want_curve = false;
    apd_params params{};
    // timing
    hipEvent_t ev[16] = {};
    apd_timing timing{};
    // profiling of the loop-body kernels (HIP events around each launch on the ctx stream)
    struct ProfEv {
        hipEvent_t e0, e1;
        int kind;    // APD_PROF_STRONG_SWEEP, APD_PROF_RANSAC_FIT, APD_PROF_WEAK_CAND, APD_PROF_WEAK_SWEEP
        int64_t px;  // pixels the launch covered
    };
    bool prof = false;
    std::vector<ProfEv> prof_ev;
    std::vector<hipEvent_t> prof_pool;  // recycled events (created once; no system-scope fence)
};

#define HIP_OK(ctx, call)                                                                          \
    do {                                                                                           \
        hipError_t e_ = (call);                                                                    \
        if (e_ != hipSuccess) {                                                                    \
            (ctx)->err = std::string(#call) + ": " + hipGetErrorString(e_);                        \
            return APD_EDEVICE;                                                                    \
        }                                                                                          \
    } while (0)

static int ensure(apd_ctx *ctx, DevBuf &b, size_t bytes) {
    if (bytes == 0) bytes = 16;
    if (b.bytes >= bytes) return APD_OK;
    if (b.p) (void)hipFree(b.p);
    b.p = nullptr;
    b.bytes = 0;
    if (hipMalloc(&b.p, bytes) != hipSuccess) {
        ctx->err = "hipMalloc(" + std::to_string(bytes) + ") failed";
        return APD_ENOMEM;
    }
    b.bytes = bytes;
    return APD_OK;
}

static int check_launch(apd_ctx *ctx, const char *what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        ctx->err = std::string("launch ") + what + ": " + hipGetErrorString(e);
        return APD_EDEVICE;
    }
    return APD_OK;
}

// Per-source precompute of the homography pieces, in double (same formulas as the oracle).
static void precompute_views(const apd_camera *cams, int ni, SrcView *views, Args &a) {
    const apd_camera &r = cams[0];
    const double kr0 = r.K[0], kr2 = r.K[2], kr4 = r.K[4], kr5 = r.K[5];
    const double Kri[9] = {1.0 / kr0, 0.0, -kr2 / kr0, 0.0, 1.0 / kr4, -kr5 / kr4, 0.0, 0.0, 1.0};
    a.ikx = (float)(1.0 / kr0);
    a.iky = (float)(1.0 / kr4);
    a.cxk = (float)(kr2 / kr0);
    a.cyk = (float)(kr5 / kr4);
    double rC[3];
    for (int j = 0; j < 3; ++j)
        rC[j] = -((double)r.R[j] * r.t[0] + (double)r.R[3 + j] * r.t[1] + (double)r.R[6 + j] * r.t[2]);
    for (int s = 0; s < ni; ++s) {
        const apd_camera &c = cams[s];
        double sC[3], Crel[3], trel[3], Rrel[9];
        for (int j = 0; j < 3; ++j)
            sC[j] = -((double)c.R[j] * c.t[0] + (double)c.R[3 + j] * c.t[1] + (double)c.R[6 + j] * c.t[2]);
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j)
                Rrel[3 * i + j] = (double)c.R[3 * i] * r.R[3 * j] + (double)c.R[3 * i + 1] * r.R[3 * j + 1] +
                                  (double)c.R[3 * i + 2] * r.R[3 * j + 2];
        for (int j = 0; j < 3; ++j) Crel[j] = rC[j] - sC[j];
        for (int i = 0; i < 3; ++i)
            trel[i] = (double)c.R[3 * i] * Crel[0] + (double)c.R[3 * i + 1] * Crel[1] + (double)c.R[3 * i + 2] * Crel[2];
        const double Ks[9] = {c.K[0], 0.0, c.K[2], 0.0, c.K[4], c.K[5], 0.0, 0.0, c.K[8]};
        double KR[9], A[9];
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j)
                KR[3 * i + j] = Ks[3 * i] * Rrel[j] + Ks[3 * i + 1] * Rrel[3 + j] + Ks[3 * i + 2] * Rrel[6 + j];
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j)
                A[3 * i + j] = KR[3 * i] * Kri[j] + KR[3 * i + 1] * Kri[3 + j] + KR[3 * i + 2] * Kri[6 + j];
        for (int k = 0; k < 9; ++k) views[s].A[k] = (float)A[k];
        for (int i = 0; i < 3; ++i)
            views[s].b[i] = (float)(Ks[3 * i] * trel[0] + Ks[3 * i + 1] * trel[1] + Ks[3 * i + 2] * trel[2]);
    }
}

static int build_near_offsets(apd_ctx *ctx) {
    if (ctx->n_near) return APD_OK;
    std::vector<short2> off;
    off.reserve(201 * 201);
    for (int x = -100; x <= 100; ++x)
        for (int y = -100; y <= 100; ++y) off.push_back(make_short2((short)x, (short)y));
    std::stable_sort(off.begin(), off.end(), [](const short2 &p, const short2 &q) {
        return p.x * p.x + p.y * p.y < q.x * q.x + q.y * q.y;  // stable: keeps x-major, y-minor order
    });
    int st = ensure(ctx, ctx->near_off, off.size() * sizeof(short2));
    if (st) return st;
    HIP_OK(ctx, hipMemcpy(ctx->near_off.p, off.data(), off.size() * sizeof(short2), hipMemcpyHostToDevice));
    // ring_start[D] = first table index with d^2 >= D, D = 0 .. 20001
    std::vector<int> ring(20002, (int)off.size());
    for (int k = (int)off.size() - 1; k >= 0; --k) ring[off[k].x * off[k].x + off[k].y * off[k].y] = k;
    for (int D = 20000; D >= 0; --D) ring[D] = std::min(ring[D], ring[D + 1]);
    if ((st = ensure(ctx, ctx->near_ring, ring.size() * sizeof(int)))) return st;
    HIP_OK(ctx, hipMemcpy(ctx->near_ring.p, ring.data(), ring.size() * sizeof(int), hipMemcpyHostToDevice));
    ctx->n_near = (int)off.size();
    return APD_OK;
}

// host -> device pointer of any address space (the Args members are address_space(1) on device)
template <class T>
static inline T devptr(const void *p) { return reinterpret_cast<T>(reinterpret_cast<uintptr_t>(p)); }

// launch the fp16-pair or the fp32-quad instantiation of a sampling kernel
#define LAUNCH_TEX(kern, grid, block, lds, stream, ...)                                            \
    do {                                                                                         \
        if (ctx->args.tex_f16) hipLaunchKernelGGL((kern<true>), grid, block, lds, stream, __VA_ARGS__); \
        else hipLaunchKernelGGL((kern<false>), grid, block, lds, stream, __VA_ARGS__);            \
    } while (0)

// ... and of its SA-masked (SA quadrant windows on the fast taps) or unmasked form
// (the same with a third template argument)
#define LAUNCH_TEX_SA(kern, grid, block, lds, stream, ...)                                          \
    do {                                                                                         \
        const bool sa_ = ctx->args.sa_any != 0;                                                  \
        if (ctx->args.tex_f16) {                                                                 \
            if (sa_) hipLaunchKernelGGL((kern<true, true>), grid, block, lds, stream, __VA_ARGS__); \
            else hipLaunchKernelGGL((kern<true, false>), grid, block, lds, stream, __VA_ARGS__);  \
        } else {                                                                                 \
            if (sa_) hipLaunchKernelGGL((kern<false, true>), grid, block, lds, stream, __VA_ARGS__); \
            else hipLaunchKernelGGL((kern<false, false>), grid, block, lds, stream, __VA_ARGS__); \
        }                                                                                        \
    } while (0)

// The smallest non-negative float d with fl(d / D) >= t (IEEE single division, monotone in d for
// D > 0), so that fl(d / D) < t <=> d < limit for every d >= 0 (NaN: false both ways). False when D
// or t rules the search out; GenAnchors then divides.
static bool inlier_limit(float D, float t, float *limit) {
    if (!(D > 0.0f) || !std::isfinite(D) || !std::isfinite(t)) return false;
    auto reach = [&](uint32_t bits) {
        float d;
        std::memcpy(&d, &bits, 4);
        volatile float q = d / D;
        return q >= t;
    };
    uint32_t lo = 0u, hi = 0x7f800000u;  // [+0, +inf]
    if (!reach(hi)) return false;
    while (lo < hi) {
        const uint32_t mid = lo + (hi - lo) / 2u;
        if (reach(mid)) hi = mid;
        else lo = mid + 1u;
    }
    std::memcpy(limit, &lo, 4);
    return true;
}

// Wait for everything the ctx launched, on its stream and on both side streams. A stage that returns
// early between a fork (RandomInitialization, RANSAC, k_gp_cost on side streams) and its join leaves
// that work running; every entry point that reuses or frees ctx buffers drains first.
static void drain(apd_ctx *ctx) {
    (void)hipStreamSynchronize(ctx->stream);
    for (auto &ss : ctx->side)
        if (ss) (void)hipStreamSynchronize(ss);
}

static inline unsigned blocks_for(size_t n, int per_block) { return (unsigned)((n + per_block - 1) / per_block); }

extern "C" {

int32_t apd_abi_version(void) { return APD_ABI_VERSION; }

int32_t apd_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

apd_ctx *apd_create(int32_t device) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) {
        set_global_err("no HIP device visible");
        return nullptr;
    }
    if (device < 0 || device >= n) {
        set_global_err("device index out of range");
        return nullptr;
    }
    if (hipSetDevice(device) != hipSuccess) {
        set_global_err("hipSetDevice failed");
        return nullptr;
    }
    apd_ctx *ctx = new apd_ctx();
    ctx->device = device;
    if (hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess) {
        set_global_err("hipStreamCreate failed");
        delete ctx;
        return nullptr;
    }
    for (auto &e : ctx->ev) (void)hipEventCreateWithFlags(&e, hipEventDisableSystemFence);  // timing only
    // side stream 0 (RandomInitialization beside the lists and the pair table; RANSAC beside the
    // candidate kernels) at the lowest priority: its work fills what the ctx stream's kernels leave
    // free instead of sharing the CUs with them evenly (APD_SIDE_PRIORITY=0: every stream at the default)
    // (priorities: a lower value is a higher priority; when the default is already the least, the ctx
    // stream and side stream 1 are raised instead)
    int prio_least = 0, prio_greatest = 0;
    (void)hipDeviceGetStreamPriorityRange(&prio_least, &prio_greatest);
    const bool low_side = !(getenv("APD_SIDE_PRIORITY") && atoi(getenv("APD_SIDE_PRIORITY")) == 0);
    if (low_side && prio_least <= 0 && prio_greatest < 0) {
        hipStream_t hi = nullptr;
        if (hipStreamCreateWithPriority(&hi, hipStreamNonBlocking, prio_greatest) == hipSuccess) {
            (void)hipStreamDestroy(ctx->stream);
            ctx->stream = hi;
        }
    }
    if (getenv("APD_DEBUG_PRIO")) fprintf(stderr, "apd: stream priorities least %d greatest %d\n", prio_least, prio_greatest);
    for (auto &ss : ctx->side) {
        int prio = 0;
        if (low_side && prio_least > 0 && &ss == &ctx->side[0]) prio = prio_least;
        if (low_side && prio_least <= 0 && prio_greatest < 0 && &ss == &ctx->side[1]) prio = prio_greatest;
        if (hipStreamCreateWithPriority(&ss, hipStreamNonBlocking, prio) != hipSuccess) {
            set_global_err("hipStreamCreate failed");
            for (auto &t : ctx->side) if (t) (void)hipStreamDestroy(t);
            (void)hipStreamDestroy(ctx->stream);
            delete ctx;
            return nullptr;
        }
    }
    (void)hipEventCreateWithFlags(&ctx->ev_fork, hipEventDisableTiming);
    for (auto &e : ctx->ev_side) (void)hipEventCreateWithFlags(&e, hipEventDisableTiming);
    ctx->overlap = getenv("APD_NO_OVERLAP") == nullptr;
    ctx->cand_pairs = getenv("APD_NO_CAND_PAIRS") == nullptr;
    ctx->ga_split = getenv("APD_NO_GA_SPLIT") == nullptr;
    ctx->lr_handover = getenv("APD_NO_LR_HANDOVER") == nullptr;
    ctx->wcur_on = getenv("APD_NO_WCUR") == nullptr;
    ctx->dtex = getenv("APD_NO_DTEX") == nullptr;
    ctx->gp_one_pass = getenv("APD_GP_TWO_PASS") == nullptr;
    ctx->gp_small = getenv("APD_GP_NO_SMALL") == nullptr;
    ctx->gp_place = getenv("APD_GP_FILL") == nullptr;
    ctx->gp_async = getenv("APD_GP_SYNC") == nullptr && ctx->gp_one_pass && ctx->gp_small && ctx->gp_place;
    {
        int n = 0;
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && n > 0) ctx->ncu = n;
    }
    if (const char *e = getenv("APD_GP_CAP_FACTOR")) ctx->gp_cap_factor = std::max(0, std::min(8, atoi(e)));  // test hook

    // tile_pix needs the tile width to divide the 64-pixel tile (otherwise two workgroups share pixels)
    if (const char *e = getenv("APD_DW_TILE_W")) {
        const int t = atoi(e);
        if (t == 1 || t == 2 || t == 4 || t == 8 || t == 16 || t == 32 || t == 64) ctx->dw_tile_w = t;
    }
    if (const char *e = getenv("APD_TILE_W")) {
        const int t = atoi(e);
        if (t == 4 || t == 8 || t == 16 || t == 32 || t == 64) ctx->tile_w = t;
    }
    // the view-major sweep's LDS grows with N (> 64 KiB from N = 15 on); gfx950 has 160 KiB per CU
    const void *vm_kernels[] = {
        (const void *)k_sweep_strong_vm<true, false>, (const void *)k_sweep_strong_vm<false, false>,
        (const void *)k_sweep_strong_vm<true, true>, (const void *)k_sweep_strong_vm<false, true>,
        (const void *)k_sweep_weak_vm<true, false>, (const void *)k_sweep_weak_vm<false, false>,
        (const void *)k_sweep_weak_vm<true, true>, (const void *)k_sweep_weak_vm<false, true>,
        (const void *)k_depth_to_weak_vm<true, false>, (const void *)k_depth_to_weak_vm<false, false>,
        (const void *)k_depth_to_weak_vm<true, true>, (const void *)k_depth_to_weak_vm<false, true>,
        (const void *)k_depth_to_weak_vm<true, false, true>, (const void *)k_depth_to_weak_vm<true, true, true>,
        (const void *)k_local_refine_vm<true, false>, (const void *)k_local_refine_vm<false, false>,
        (const void *)k_local_refine_vm<true, true>, (const void *)k_local_refine_vm<false, true>,
        (const void *)k_random_init_vm<true, false, false>, (const void *)k_random_init_vm<false, false, false>,
        (const void *)k_random_init_vm<true, true, false>, (const void *)k_random_init_vm<false, true, false>,
        (const void *)k_random_init_vm<true, false, true>, (const void *)k_random_init_vm<false, false, true>,
        (const void *)k_random_init_vm<true, true, true>, (const void *)k_random_init_vm<false, true, true>};
    for (const void *k : vm_kernels) (void)hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    return ctx;
}

void apd_destroy(apd_ctx *ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    drain(ctx);
    DevBuf *bufs[] = {&ctx->imgs, &ctx->quad, &ctx->depth, &ctx->views, &ctx->cams, &ctx->plane, &ctx->cost,
                      &ctx->sel, &ctx->sel2, &ctx->vw, &ctx->weak, &ctx->conf, &ctx->sa, &ctx->amap, &ctx->anchors,
                      &ctx->reliable, &ctx->nearest, &ctx->fit, &ctx->curve, &ctx->lists, &ctx->rowcnt,
                      &ctx->rowoff, &ctx->totals, &ctx->near_off, &ctx->dargs, &ctx->evals, &ctx->near_ring, &ctx->near_g, &ctx->wcand, &ctx->arec, &ctx->ga_stage,
                      &ctx->lrs, &ctx->wcur, &ctx->wlist, &ctx->gp_cb, &ctx->gp_cnt, &ctx->gp_cur, &ctx->gp_refs, &ctx->gp_ccnt,
                      &ctx->gp_cbase, &ctx->gp_plist, &ctx->gp_pidx, &ctx->gp_pcost, &ctx->gp_tmp, &ctx->dpairs, &ctx->gp_cls};
    for (DevBuf *b : bufs)
        if (b->p) (void)hipFree(b->p);
    for (auto &e : ctx->ev) (void)hipEventDestroy(e);
    for (auto &pe : ctx->prof_ev) { (void)hipEventDestroy(pe.e0); (void)hipEventDestroy(pe.e1); }
    for (hipEvent_t e : ctx->prof_pool) (void)hipEventDestroy(e);
    for (auto &ss : ctx->side) if (ss) { (void)hipStreamSynchronize(ss); (void)hipStreamDestroy(ss); }
    if (ctx->ev_fork) (void)hipEventDestroy(ctx->ev_fork);
    for (auto &e : ctx->ev_side) if (e) (void)hipEventDestroy(e);
    (void)hipStreamDestroy(ctx->stream);
    delete ctx;
}

const char *apd_last_error(const apd_ctx *ctx) { return ctx ? ctx->err.c_str() : g_global_err; }

// ensure() for optional buffers: a failed allocation leaves no error behind (the caller falls back to
// a slower exact path); the first few are reported on stderr, since a device store sized too greedily
// by the caller shows up here first
static bool try_ensure(apd_ctx *ctx, DevBuf &b, size_t bytes) {
    if (ensure(ctx, b, bytes) == APD_OK) return true;
    (void)hipGetLastError();
    ctx->err.clear();
    if (ctx->optional_fallbacks++ < 8)
        fprintf(stderr, "apd: optional device buffer of %zu bytes not allocated on device %d: its exact fallback path runs\n",
                bytes, ctx->device);
    return false;
}

int32_t apd_set_problem(apd_ctx *ctx, const apd_problem *pb) {
    if (!ctx || !pb) return APD_EINVAL;
    (void)hipSetDevice(ctx->device);
    drain(ctx);  // (a previous stage that failed between a fork and its join: its side work reads these buffers)
    ctx->loaded = ctx->prepared = ctx->prep_timed = false;
    const int W = pb->width, H = pb->height, NI = pb->num_images;
    if (NI > APD_MAX_IMAGES) { ctx->err = "num_images > 32"; return APD_ETOOMANYVIEWS; }
    if (W < 1 || H < 1 || NI < 2 || !pb->images || !pb->cameras) { ctx->err = "bad problem dimensions"; return APD_EINVAL; }
    if (W > 32767 || H > 32767 || (size_t)W * H > (size_t)1 << 30) { ctx->err = "image too large"; return APD_EINVAL; }
    const apd_params &P = pb->params;
    if (P.strong_radius != 5 || P.strong_increment != 2 || P.weak_radius != 5 || P.weak_increment != 5) {
        ctx->err = "kernels are specialised for strong 5/2 and weak 5/5 windows (main.h:88-91)";
        return APD_EINVAL;
    }
    if (P.top_k < 1 || P.top_k > 4) { ctx->err = "top_k must be 1..4"; return APD_EINVAL; }
    if (P.max_iterations < 0) { ctx->err = "max_iterations < 0"; return APD_EINVAL; }
    if (P.use_APD && (P.rotate_time < 1 || P.rotate_time > 4)) { ctx->err = "rotate_time must be 1..4"; return APD_EINVAL; }
    if ((P.geom_consistency || P.use_APD) && !pb->depths) { ctx->err = "depth maps required (geom/APD)"; return APD_EINVAL; }
    const int N = NI - 1;
    const size_t HW = (size_t)W * H;
    int st;
    hipStream_t s = ctx->stream;
    // Every input may be a host or a device pointer (hipMemcpyDefault): a caller that keeps a scan's
    // images and depth maps resident in HBM (scan_runner.py) hands device pointers over and nothing
    // crosses PCIe here.
    if ((st = ensure(ctx, ctx->imgs, HW * NI * sizeof(float)))) return st;
    if ((st = ensure(ctx, ctx->totals, 16 * sizeof(int)))) return st;
    if ((st = ensure(ctx, ctx->plane, HW * sizeof(float4)))) return st;
    if ((st = ensure(ctx, ctx->cost, HW * sizeof(float)))) return st;
    if ((st = ensure(ctx, ctx->sel, HW * sizeof(uint32_t)))) return st;
    if ((st = ensure(ctx, ctx->sel2, HW * sizeof(uint32_t)))) return st;
    if ((st = ensure(ctx, ctx->vw, HW * N))) return st;
    if ((st = ensure(ctx, ctx->weak, HW))) return st;
    if ((st = ensure(ctx, ctx->conf, HW))) return st;
    if ((st = ensure(ctx, ctx->sa, HW))) return st;
    if ((st = ensure(ctx, ctx->lists, (HW + 8) * sizeof(int)))) return st;
    if ((st = ensure(ctx, ctx->views, NI * sizeof(SrcView)))) return st;
    if ((st = ensure(ctx, ctx->cams, NI * sizeof(Cam)))) return st;
    const size_t units = std::max<size_t>((size_t)H, (size_t)(W + 3) / 4 * ((H + 3) / 4));  // any tile shape
    if ((st = ensure(ctx, ctx->rowcnt, units * sizeof(int)))) return st;
    if ((st = ensure(ctx, ctx->rowoff, units * sizeof(int)))) return st;
    const bool need_depth = P.geom_consistency || P.use_APD;
    if (need_depth && (st = ensure(ctx, ctx->depth, HW * NI * sizeof(float)))) return st;
    for (int i = 0; i < NI; ++i) {
        if (!pb->images[i]) { ctx->err = "null image pointer"; return APD_EINVAL; }
        HIP_OK(ctx, hipMemcpyAsync((float *)ctx->imgs.p + HW * i, pb->images[i], HW * sizeof(float), hipMemcpyDefault, s));
    }
    if (need_depth) {
        for (int i = 0; i < NI; ++i) {
            if (!pb->depths[i]) { ctx->err = "null depth pointer"; return APD_EINVAL; }
            HIP_OK(ctx, hipMemcpyAsync((float *)ctx->depth.p + HW * i, pb->depths[i], HW * sizeof(float), hipMemcpyDefault, s));
        }
    }
    // priors (APD.cpp:612-683)
    if (P.state != APD_FIRST_INIT && pb->init_planes)
        HIP_OK(ctx, hipMemcpyAsync(ctx->plane.p, pb->init_planes, HW * sizeof(float4), hipMemcpyDefault, s));
    else
        HIP_OK(ctx, hipMemsetAsync(ctx->plane.p, 0, HW * sizeof(float4), s));
    if (P.use_APD && pb->weak_info) HIP_OK(ctx, hipMemcpyAsync(ctx->weak.p, pb->weak_info, HW, hipMemcpyDefault, s));
    else HIP_OK(ctx, hipMemsetAsync(ctx->weak.p, APD_STRONG, HW, s));
    if (P.use_APD && pb->confidence) HIP_OK(ctx, hipMemcpyAsync(ctx->conf.p, pb->confidence, HW, hipMemcpyDefault, s));
    else HIP_OK(ctx, hipMemsetAsync(ctx->conf.p, 1, HW, s));
    if (pb->sa_mask) HIP_OK(ctx, hipMemcpyAsync(ctx->sa.p, pb->sa_mask, HW, hipMemcpyDefault, s));
    else HIP_OK(ctx, hipMemsetAsync(ctx->sa.p, 0, HW, s));
    // one read-back for everything the host needs to size the rest: the fp16-texel eligibility of the
    // source images (a quarter-integer in [0, 256) -- 8-bit images and their INTER_LINEAR 2^-k
    // downscales -- is exact in fp16 together with its horizontal differences, which FastTex::sample
    // relies on; else fp32 quads), the WEAK count, the largest confidence and whether any SA label is set
    bool tex_f16 = getenv("APD_TEX_F32") == nullptr;
    {
        int *stat = (int *)ctx->totals.p + 8;  // [8] f16 ok, [9] WEAK count, [10] max confidence, [11] SA any
        const int init[4] = {1, 0, 0, 0};
        HIP_OK(ctx, hipMemcpyAsync(stat, init, sizeof(init), hipMemcpyHostToDevice, s));
        if (tex_f16) {
            const size_t n = HW * NI;
            hipLaunchKernelGGL(k_check_f16, dim3((unsigned)std::min<size_t>(blocks_for(n, BLOCK), 8192)), dim3(BLOCK), 0, s,
                               (const float *)ctx->imgs.p, n, stat);
        }
        hipLaunchKernelGGL(k_problem_stats, dim3((unsigned)std::min<size_t>(blocks_for(HW, BLOCK), 4096)), dim3(BLOCK), 0, s,
                           (const uint8_t *)ctx->weak.p, (const uint8_t *)ctx->conf.p, (const uint8_t *)ctx->sa.p, HW,
                           stat + 1);
        if ((st = check_launch(ctx, "problem statistics"))) return st;
        HIP_OK(ctx, hipMemcpyAsync(ctx->host_stat, stat, 4 * sizeof(int), hipMemcpyDeviceToHost, s));
        HIP_OK(ctx, hipStreamSynchronize(s));
        tex_f16 = tex_f16 && ctx->host_stat[0] != 0;
    }
    const int weak_count = P.use_APD ? ctx->host_stat[1] : 0;
    const int max_conf = ctx->host_stat[2];
    const int sa_any = ctx->host_stat[3];
    const size_t qstride = tex_f16 ? (size_t)(W + 2) * (H + 1) : (size_t)(W + 1) * (H + 1);
    if ((st = ensure(ctx, ctx->quad, qstride * N * (tex_f16 ? sizeof(uint32_t) : sizeof(float4))))) return st;
    std::vector<Cam> cams(NI);
    std::vector<SrcView> views(NI);
    for (int i = 0; i < NI; ++i) {
        memcpy(cams[i].K, pb->cameras[i].K, 9 * sizeof(float));
        memcpy(cams[i].R, pb->cameras[i].R, 9 * sizeof(float));
        memcpy(cams[i].t, pb->cameras[i].t, 3 * sizeof(float));
        memcpy(cams[i].c, pb->cameras[i].c, 3 * sizeof(float));
    }
    Args &a = ctx->args;
    a = Args{};
    precompute_views(pb->cameras, NI, views.data(), a);
    HIP_OK(ctx, hipMemcpyAsync(ctx->cams.p, cams.data(), NI * sizeof(Cam), hipMemcpyHostToDevice, s));
    HIP_OK(ctx, hipMemcpyAsync(ctx->views.p, views.data(), NI * sizeof(SrcView), hipMemcpyHostToDevice, s));
    HIP_OK(ctx, hipMemsetAsync(ctx->vw.p, 0, HW * N, s));
    HIP_OK(ctx, hipMemsetAsync(ctx->cost.p, 0, HW * sizeof(float), s));
    HIP_OK(ctx, hipMemsetAsync(ctx->sel.p, 0, HW * sizeof(uint32_t), s));
    ctx->weak_count = weak_count;
    if (P.use_APD) {
        if ((st = ensure(ctx, ctx->amap, HW * sizeof(int)))) return st;
        if ((st = ensure(ctx, ctx->anchors, (size_t)std::max(weak_count, 1) * 9 * sizeof(short2)))) return st;
        if ((st = ensure(ctx, ctx->reliable, HW))) return st;
        if ((st = ensure(ctx, ctx->nearest, HW * sizeof(short2)))) return st;
        if ((st = ensure(ctx, ctx->fit, HW * sizeof(float4)))) return st;
        HIP_OK(ctx, hipMemsetAsync(ctx->reliable.p, 0, HW, s));
        HIP_OK(ctx, hipMemsetAsync(ctx->fit.p, 0, HW * sizeof(float4), s));
        if ((st = build_near_offsets(ctx))) return st;
        // per-level column distances for k_find_nearest_rows (confidence is an input here)
        ctx->near_levels = std::max(max_conf, 1) + 1;
        if (getenv("APD_NEAREST_RING") || (size_t)ctx->near_levels * HW > ((size_t)4 << 30)) ctx->near_levels = 0;
        if (ctx->near_levels && (st = ensure(ctx, ctx->near_g, (size_t)ctx->near_levels * HW))) return st;
    }
    // kernel arguments
    a.W = W; a.H = H; a.HW = (int)HW; a.N = N;
    {
        const int hh = H / 2;
        const int rl = 32 * ((hh + 15) / 16);  // half-grid coverage of BLOCK_H=16 blocks (APD.cu:2676-2683)
        a.row_limit = rl < H ? rl : H;
    }
    a.state = P.state;
    a.dmin = P.depth_min; a.dmax = P.depth_max; a.gf = P.geom_factor; a.ransac_thr = P.ransac_threshold;
    a.geom = P.geom_consistency != 0; a.impetus = P.use_impetus != 0; a.use_apd = P.use_APD != 0;
    a.peak_radius = P.weak_peak_radius; a.rotate_time = P.rotate_time; a.sa_any = sa_any; a.top_k = P.top_k;
    a.seed_lo = (uint32_t)pb->seed; a.seed_hi = (uint32_t)(pb->seed >> 32);
    if (P.use_APD) {  // GenAnchors per-launch constants in double, as the reference (APD.cu:1897-1901)
        const float angle = 45.0f / (float)P.rotate_time;
        a.anc_cos = (float)cos((double)angle * 3.14159265358979323846 / 180.0f);
        a.anc_sin = (float)sin((double)angle * 3.14159265358979323846 / 180.0f);
        a.anc_thr = (float)cos((double)(angle / 2.0f) * 3.14159265358979323846 / 180.0f);
        const int sr = (int)(tan((double)(angle / 2.0f) * 3.14159265358979323846 / 180.0f) * 20);
        a.anc_shift = sr < 1 ? 1 : sr;
        a.anc_dlim_ok = inlier_limit(a.dmax - a.dmin, a.ransac_thr, &a.anc_dlim) ? 1 : 0;
    }
    a.qstride = qstride;
    a.ref = devptr<decltype(a.ref)>(ctx->imgs.p);
    a.quad = devptr<decltype(a.quad)>(ctx->quad.p);
    a.pairs = devptr<decltype(a.pairs)>(ctx->quad.p);
    a.tex_f16 = tex_f16 ? 1 : 0;
    a.force_slow = getenv("APD_FORCE_SLOW_NCC") != nullptr;  // test hook (tests/test_gpu_parity.py)
    a.depth = devptr<decltype(a.depth)>(need_depth ? ctx->depth.p : nullptr);
    a.views = devptr<decltype(a.views)>(ctx->views.p);
    a.cams = devptr<decltype(a.cams)>(ctx->cams.p);
    a.plane = devptr<decltype(a.plane)>(ctx->plane.p);
    a.cost = devptr<decltype(a.cost)>(ctx->cost.p);
    a.sel = devptr<decltype(a.sel)>(ctx->sel.p);
    a.sel_next = devptr<decltype(a.sel_next)>(ctx->sel2.p);
    a.vw = devptr<decltype(a.vw)>(ctx->vw.p);
    a.weak = devptr<decltype(a.weak)>(ctx->weak.p);
    a.conf = devptr<decltype(a.conf)>(ctx->conf.p);
    a.sa = devptr<decltype(a.sa)>(ctx->sa.p);
    a.amap = devptr<decltype(a.amap)>(P.use_APD ? ctx->amap.p : nullptr);
    a.anchors = devptr<decltype(a.anchors)>(P.use_APD ? ctx->anchors.p : nullptr);
    a.reliable = devptr<decltype(a.reliable)>(P.use_APD ? ctx->reliable.p : nullptr);
    a.nearest = devptr<decltype(a.nearest)>(P.use_APD ? ctx->nearest.p : nullptr);
    a.fit = devptr<decltype(a.fit)>(P.use_APD ? ctx->fit.p : nullptr);
    a.near_offsets = devptr<decltype(a.near_offsets)>(P.use_APD ? ctx->near_off.p : nullptr);
    a.arec = nullptr;  // (apd_stage_prepare, when a kernel reads the records)
    a.curve = nullptr;
    a.lr_ncc = nullptr;
    a.lr_geo = nullptr;
    a.wcur = nullptr;
    if (ctx->wcur_on) {  // the initial planes' costs per view (NCC-New for WEAK pixels), [N][H*W]
        if ((st = ensure(ctx, ctx->wcur, HW * N * sizeof(float)))) return st;
        a.wcur = devptr<decltype(a.wcur)>(ctx->wcur.p);
    }
    if ((st = ensure(ctx, ctx->dargs, sizeof(Args)))) return st;
    a.self = devptr<decltype(a.self)>(ctx->dargs.p);
    HIP_OK(ctx, hipMemcpyAsync(ctx->dargs.p, &a, sizeof(Args), hipMemcpyHostToDevice, s));
    // source images -> quad gather layout
    {
        const size_t total = qstride * N;
        unsigned g = (unsigned)std::min<size_t>(blocks_for(total, BLOCK), 65535u * 8u);
        if (tex_f16)
            hipLaunchKernelGGL(k_build_pairs, dim3(g), dim3(BLOCK), 0, s, (const float *)ctx->imgs.p,
                               (uint32_t *)ctx->quad.p, W, H, N, qstride);
        else
            hipLaunchKernelGGL(k_build_quads, dim3(g), dim3(BLOCK), 0, s, (const float *)ctx->imgs.p,
                               (float4 *)ctx->quad.p, W, H, N, qstride);
        if ((st = check_launch(ctx, "k_build_quads"))) return st;
    }
    // fp16 problems: the pre-differenced texel records (FastTexD) DepthToWeak samples, 8 B per padded
    // texel position and view (2 GB at C3); optional
    a.dpairs = nullptr;
    if (tex_f16 && ctx->dtex && try_ensure(ctx, ctx->dpairs, qstride * (size_t)N * sizeof(uint2))) {
        const size_t dpn = qstride * (size_t)N;
        hipLaunchKernelGGL(k_build_dpairs, dim3((unsigned)std::min<size_t>(blocks_for(dpn, BLOCK), 65535u * 8u)), dim3(BLOCK), 0, s,
                           (const uint32_t *)ctx->quad.p, (uint2 *)ctx->dpairs.p, W, H, N, qstride);
        if ((st = check_launch(ctx, "k_build_dpairs"))) return st;
        a.dpairs = devptr<decltype(a.dpairs)>(ctx->dpairs.p);
    }
    ctx->want_curve = pb->export_reliable_curve != 0;
    if (ctx->want_curve) {  // DepthToWeak cost curves (APD.cu:2188-2198, 2713-2724)
        if ((st = ensure(ctx, ctx->curve, HW * 61 * sizeof(float)))) return st;
        HIP_OK(ctx, hipMemsetAsync(ctx->curve.p, 0, HW * 61 * sizeof(float), s));
    }
    // DepthToWeak -> LocalRefine hand-over ([11][N][tile slots] fp32 NCC-Old, and as much again for
    // the geometric terms: 21.5 GB at 6048x4032, N = 10, with geometry). Sized here, after every
    // buffer the path needs, so that no allocation sits inside the timed stages: held at exactly this
    // problem's size (a larger buffer from an earlier problem is released, so a scan's geometric
    // pass does not keep it through the next round's init pass), and only when it fits in the
    // device's free memory with 4 GiB to spare -- else LocalRefine evaluates the samples itself.
    ctx->lrs_need = 0;
    if (ctx->lr_handover) {
        const int tw = ctx->dw_tile_w, th = VM_P / tw;
        const size_t slots = (size_t)(((W + tw - 1) / tw) * ((H + th - 1) / th)) * VM_P;
        const size_t need = (size_t)11 * N * slots * sizeof(float) * (P.geom_consistency ? 2 : 1);
        if (ctx->lrs.p && ctx->lrs.bytes != need) {
            (void)hipFree(ctx->lrs.p);
            ctx->lrs.p = nullptr;
            ctx->lrs.bytes = 0;
        }
        size_t free_b = 0, total_b = 0;
        const size_t spare = (size_t)4 << 30;
        if (!ctx->lrs.p && hipMemGetInfo(&free_b, &total_b) == hipSuccess && free_b > spare && need <= free_b - spare) {
            if (ensure(ctx, ctx->lrs, need) != APD_OK) {  // not fatal: clear the allocation error
                (void)hipGetLastError();
                ctx->err.clear();
            }
        }
        if (ctx->lrs.p) ctx->lrs_need = need;
    }
    ctx->params = P;
    ctx->loaded = true;
    return APD_OK;
}

// device-side ordered compaction of one pixel set
// Sweep lists (modes 0/1) in tile order: count per tile, scan, fill.
static void tile_count_scan(apd_ctx *ctx, int mode, int colour, int *total_dev) {
    Args &a = ctx->args;
    const int tw = ctx->tile_w, th = TILE_POS / tw;
    const int tx = (a.W + tw - 1) / tw, ty = (a.H + th - 1) / th;
    hipLaunchKernelGGL(k_tile_count, dim3(tx * ty), dim3(BLOCK), 0, ctx->stream, a, mode, colour, tx, tw,
                       (int *)ctx->rowcnt.p);
    hipLaunchKernelGGL(k_list_scan, dim3(1), dim3(1024), 0, ctx->stream, (const int *)ctx->rowcnt.p, tx * ty,
                       (int *)ctx->rowoff.p, total_dev);
}
static int build_tile_list(apd_ctx *ctx, int mode, int colour, int *out, int *total_dev) {
    Args &a = ctx->args;
    const int tw = ctx->tile_w, th = TILE_POS / tw;
    const int tx = (a.W + tw - 1) / tw, ty = (a.H + th - 1) / th;
    tile_count_scan(ctx, mode, colour, total_dev);
    hipLaunchKernelGGL(k_tile_fill, dim3(tx * ty), dim3(BLOCK), 0, ctx->stream, a, mode, colour, tx, tw,
                       (const int *)ctx->rowoff.p, out);
    return check_launch(ctx, "tile list build");
}
// anchors_map (mode 2) in row-major order (APD.cpp:627-640)
static int build_list(apd_ctx *ctx, int mode, int colour, int *out, int *total_dev) {
    Args &a = ctx->args;
    hipStream_t s = ctx->stream;
    hipLaunchKernelGGL(k_list_count, dim3(a.H), dim3(BLOCK), 0, s, a, mode, colour, (int *)ctx->rowcnt.p);
    hipLaunchKernelGGL(k_list_scan, dim3(1), dim3(1024), 0, s, (const int *)ctx->rowcnt.p, a.H, (int *)ctx->rowoff.p,
                       total_dev);
    hipLaunchKernelGGL(k_list_fill, dim3(a.H), dim3(BLOCK), 0, s, a, mode, colour, (const int *)ctx->rowoff.p, out);
    return check_launch(ctx, "list build");
}

static int *list_ptr(apd_ctx *ctx, int which) {
    // 4 lists share one HW-sized buffer: [strong black][strong red][weak black][weak red] are disjoint
    // subsets of the pixels, so their concatenation never exceeds H*W entries.
    int *base = (int *)ctx->lists.p;
    size_t off = 0;
    for (int i = 0; i < which; ++i) off += (size_t)ctx->cnt[i];
    return base + off;
}


// exclusive prefix sum of n ints (rocPRIM) on the ctx stream
// test hook (tests/test_gpu_cli.py): APD_TEST_LIB_ENOMEM_AT=k makes the k-th APD apd_stage_prepare of the
// process fail as if its candidate-cost buffer did not fit -- after RandomInitialization was started on
// a side stream, the early return the callers' release-and-retry must survive (drain())
static bool test_enomem_hook(apd_ctx *ctx) {
    static std::atomic<int> n{0};
    const char *e = getenv("APD_TEST_LIB_ENOMEM_AT");
    if (!e || ++n != atoi(e)) return false;
    ctx->err = "hipMalloc failed (APD_TEST_LIB_ENOMEM_AT)";
    return true;
}

static int exclusive_scan_int(apd_ctx *ctx, const int *in, int *out, size_t n) {
    size_t tb = 0;
    HIP_OK(ctx, rocprim::exclusive_scan(nullptr, tb, in, out, 0, n, rocprim::plus<int>(), ctx->stream));
    if (!try_ensure(ctx, ctx->gp_tmp, tb)) return APD_ENOMEM;
    HIP_OK(ctx, rocprim::exclusive_scan(ctx->gp_tmp.p, tb, in, out, 0, n, rocprim::plus<int>(), ctx->stream));
    return APD_OK;
}

// The image-wide (window anchor, candidate anchor) pair table of the prepared problem (see
// k_gp_dedup); ctx->gp_on stays false (k_weak_cand_vm's per-group pairs) when a buffer does not fit.
static int build_global_pairs(apd_ctx *ctx, int nw) {
    Args &a = ctx->args;
    hipStream_t s = ctx->stream;
    const size_t HW = (size_t)a.HW, wc = (size_t)std::max(ctx->weak_count, 1);
    ctx->gp_on = false;
    ctx->gp_np = 0;
    if (!try_ensure(ctx, ctx->gp_cnt, (HW + 1) * sizeof(int)) || !try_ensure(ctx, ctx->gp_cur, (HW + 1) * sizeof(int)) ||
        !try_ensure(ctx, ctx->gp_refs, (size_t)nw * 8 * sizeof(uint32_t)) ||
        !try_ensure(ctx, ctx->gp_pidx, wc * 64 * sizeof(uint32_t)) || !try_ensure(ctx, ctx->gp_cb, 2 * wc))
        return APD_OK;
    int *cnt = (int *)ctx->gp_cnt.p, *cur = (int *)ctx->gp_cur.p;
    HIP_OK(ctx, hipMemsetAsync(cnt, 0, (HW + 1) * sizeof(int), s));
    // gp_cb: candidate bits [wc], then used windows [wc]
    // (the references' places live in gp_pidx until k_gp_dedup writes the pair ids there)
    uint32_t *loc = (uint32_t *)ctx->gp_pidx.p;
    if (ctx->gp_place)
        hipLaunchKernelGGL(k_gp_count_loc, dim3(blocks_for((size_t)nw, BLOCK)), dim3(BLOCK), 0, s, a, (const int *)ctx->wlist.p, nw,
                           cnt, (uint8_t *)ctx->gp_cb.p, (uint8_t *)ctx->gp_cb.p + wc, loc);
    else
        hipLaunchKernelGGL(k_gp_count, dim3(blocks_for((size_t)nw, BLOCK)), dim3(BLOCK), 0, s, a, (const int *)ctx->wlist.p, nw, cnt,
                           (uint8_t *)ctx->gp_cb.p, (uint8_t *)ctx->gp_cb.p + wc);
    int st;
    if ((st = exclusive_scan_int(ctx, cnt, cur, HW + 1))) return st == APD_ENOMEM ? APD_OK : st;
    int nrefs = 0;
    HIP_OK(ctx, hipMemcpyAsync(&nrefs, cur + HW, sizeof(int), hipMemcpyDeviceToHost, s));
    if (ctx->gp_place) {
        hipLaunchKernelGGL(k_gp_place, dim3(blocks_for((size_t)nw, BLOCK)), dim3(BLOCK), 0, s, a, (const int *)ctx->wlist.p, nw,
                           (const int *)cur, (const uint8_t *)ctx->gp_cb.p + wc, (const uint32_t *)loc, (uint32_t *)ctx->gp_refs.p);
    } else {
        HIP_OK(ctx, hipMemcpyAsync(cnt, cur, HW * sizeof(int), hipMemcpyDeviceToDevice, s));  // fill cursors
        hipLaunchKernelGGL(k_gp_fill, dim3(blocks_for((size_t)nw, BLOCK)), dim3(BLOCK), 0, s, a, (const int *)ctx->wlist.p, nw, cnt,
                           (uint32_t *)ctx->gp_refs.p);
    }
    HIP_OK(ctx, hipStreamSynchronize(s));
    if (nrefs <= 0) { ctx->gp_on = true; return check_launch(ctx, "pair table"); }
    // window anchors with references -> one dedup workgroup each
    if (!try_ensure(ctx, ctx->gp_ccnt, (HW + 1) * sizeof(int)) || !try_ensure(ctx, ctx->gp_cbase, 2 * (HW + 1) * sizeof(int)))
        return APD_OK;
    int *tpos = (int *)ctx->gp_ccnt.p, *tasks = cnt;  // (the fill cursors are done with)
    hipLaunchKernelGGL(k_gp_flags, dim3(blocks_for(HW + 1, BLOCK)), dim3(BLOCK), 0, s, (const int *)cur, (int)HW, cnt);
    if ((st = exclusive_scan_int(ctx, cnt, tpos, HW + 1))) return st == APD_ENOMEM ? APD_OK : st;
    hipLaunchKernelGGL(k_gp_tasks, dim3(blocks_for(HW, BLOCK)), dim3(BLOCK), 0, s, (const int *)cur, (const int *)tpos, (int)HW, tasks);
    int ntask = 0;
    HIP_OK(ctx, hipMemcpyAsync(&ntask, tpos + HW, sizeof(int), hipMemcpyDeviceToHost, s));
    HIP_OK(ctx, hipStreamSynchronize(s));
    int *acnt = (int *)ctx->gp_cbase.p, *abase = acnt + (HW + 1);
    int npairs = 0;
    bool one_pass = false;
    if (ctx->gp_one_pass && ntask > 0) {
        // one pass: the closed tables reserve their plist ranges with an atomic. Capacity: gp_cap_factor
        // pairs per reference (a reference has <= 8 candidates; at C3 116 M distinct pairs for 183 M
        // references); a table past it is detected and the two passes below run instead
        const size_t pcap = std::min<size_t>((size_t)nrefs * ctx->gp_cap_factor, (size_t)INT32_MAX);
        if (try_ensure(ctx, ctx->gp_plist, pcap * sizeof(int2))) {
            HIP_OK(ctx, hipMemsetAsync(acnt, 0, sizeof(int), s));
            if (ctx->gp_small) {
#define GP_DEDUP_ARGS                                                                                                        \
    s, a, (const int *)tasks, (const int *)cur, (const uint32_t *)ctx->gp_refs.p, (const uint8_t *)ctx->gp_cb.p, acnt,      \
        (const int *)nullptr, (int2 *)ctx->gp_plist.p, (uint32_t *)ctx->gp_pidx.p, (int)pcap
                hipLaunchKernelGGL((k_gp_dedup<2, GP_SMALL_HS, WAVE, -1, GP_SMALL_N>), dim3(ntask), dim3(WAVE), 0, GP_DEDUP_ARGS);
                hipLaunchKernelGGL((k_gp_dedup<2, GP_MEDIUM_HS, GP_CHUNK, GP_SMALL_N, GP_CHUNK>), dim3(ntask), dim3(GP_CHUNK), 0,
                                   GP_DEDUP_ARGS);
                hipLaunchKernelGGL((k_gp_dedup<2, GP_HS, GP_CHUNK, GP_CHUNK>), dim3(ntask), dim3(GP_CHUNK), 0, GP_DEDUP_ARGS);
#undef GP_DEDUP_ARGS
            } else {
                hipLaunchKernelGGL((k_gp_dedup<2>), dim3(ntask), dim3(GP_CHUNK), 0, s, a, (const int *)tasks, (const int *)cur,
                                   (const uint32_t *)ctx->gp_refs.p, (const uint8_t *)ctx->gp_cb.p, acnt, (const int *)nullptr,
                                   (int2 *)ctx->gp_plist.p, (uint32_t *)ctx->gp_pidx.p, (int)pcap);
            }
            HIP_OK(ctx, hipMemcpyAsync(&npairs, acnt, sizeof(int), hipMemcpyDeviceToHost, s));
            HIP_OK(ctx, hipStreamSynchronize(s));
            if ((st = check_launch(ctx, "pair table"))) return st;
            one_pass = npairs >= 0 && (size_t)npairs <= pcap;
            if (!one_pass) ctx->gp_cap_factor = 8;  // (the exact bound from now on)
        }
    }
    if (!one_pass) {
        HIP_OK(ctx, hipMemsetAsync(acnt + ntask, 0, sizeof(int), s));
        if (ntask > 0)
            hipLaunchKernelGGL((k_gp_dedup<0>), dim3(ntask), dim3(GP_CHUNK), 0, s, a, (const int *)tasks, (const int *)cur,
                               (const uint32_t *)ctx->gp_refs.p, (const uint8_t *)ctx->gp_cb.p, acnt, (const int *)nullptr,
                               (int2 *)nullptr, (uint32_t *)nullptr, 0);
        if ((st = exclusive_scan_int(ctx, acnt, abase, (size_t)ntask + 1))) return st == APD_ENOMEM ? APD_OK : st;
        HIP_OK(ctx, hipMemcpyAsync(&npairs, abase + ntask, sizeof(int), hipMemcpyDeviceToHost, s));
        HIP_OK(ctx, hipStreamSynchronize(s));
        if (npairs > 0 && !try_ensure(ctx, ctx->gp_plist, (size_t)npairs * sizeof(int2))) return APD_OK;
        if (npairs > 0)
            hipLaunchKernelGGL((k_gp_dedup<1>), dim3(ntask), dim3(GP_CHUNK), 0, s, a, (const int *)tasks, (const int *)cur,
                               (const uint32_t *)ctx->gp_refs.p, (const uint8_t *)ctx->gp_cb.p, (int *)nullptr, (const int *)abase,
                               (int2 *)ctx->gp_plist.p, (uint32_t *)ctx->gp_pidx.p, 0);
    }
    if (npairs > 0 && !try_ensure(ctx, ctx->gp_pcost, (size_t)npairs * ((a.N + 3) & ~3) * sizeof(float))) return APD_OK;
    if ((st = check_launch(ctx, "pair table"))) return st;
    ctx->gp_np = npairs;
    ctx->gp_on = true;
    return APD_OK;
}

// The same pair table without a host round trip (the default): everything is enqueued at once and
// RandomInitialization, on the low-priority side stream, fills what the pair-table kernels leave free.
// The window anchors are dealt into size classes on the device (k_gp_classes; at most HW - WEAK
// anchors, all STRONG) and k_gp_dedup_q runs each class in a grid that fills the GPU; the pair list's
// capacity is an upper bound from the WEAK count. apd_stage_prepare's end (finish_global_pairs) reads
// the pair count back once, allocates the costs, and rebuilds the table with the synchronous path
// above if a bound was exceeded.
static int build_global_pairs_async(apd_ctx *ctx, int nw) {
    Args &a = ctx->args;
    hipStream_t s = ctx->stream;
    const size_t HW = (size_t)a.HW, wc = (size_t)std::max(ctx->weak_count, 1);
    ctx->gp_on = false;
    ctx->gp_np = 0;
    ctx->gp_pending = false;
    const size_t U = HW > (size_t)ctx->weak_count ? HW - (size_t)ctx->weak_count : 1;  // anchors: STRONG pixels
    const size_t cap2 = U + 1 + (size_t)nw * 8 / GP_SPLIT + 1;  // class-2 runs: <= anchors + references / GP_SPLIT
    const size_t pcap = std::min<size_t>((size_t)nw * 4 * (size_t)ctx->gp_cap_factor, (size_t)INT32_MAX);
    if (!try_ensure(ctx, ctx->gp_cnt, (HW + 1) * sizeof(int)) || !try_ensure(ctx, ctx->gp_cur, (HW + 1) * sizeof(int)) ||
        !try_ensure(ctx, ctx->gp_refs, (size_t)nw * 8 * sizeof(uint32_t)) ||
        !try_ensure(ctx, ctx->gp_pidx, wc * 64 * sizeof(uint32_t)) || !try_ensure(ctx, ctx->gp_cb, 2 * wc) ||
        !try_ensure(ctx, ctx->gp_cls, (2 * (U + 1) + 2 * cap2 + 8) * sizeof(int)) ||
        !try_ensure(ctx, ctx->gp_plist, std::max<size_t>(pcap, 1) * sizeof(int2)))
        return APD_OK;
    int *cnt = (int *)ctx->gp_cnt.p, *cur = (int *)ctx->gp_cur.p;
    int *lists = (int *)ctx->gp_cls.p, *ctr = lists + 2 * (U + 1) + 2 * cap2;  // ctr: [3] class counts, [3] next, [4] overflow, [5] pairs
    uint32_t *loc = (uint32_t *)ctx->gp_pidx.p;
    HIP_OK(ctx, hipMemsetAsync(cnt, 0, (HW + 1) * sizeof(int), s));
    HIP_OK(ctx, hipMemsetAsync(ctr, 0, 8 * sizeof(int), s));
    hipLaunchKernelGGL(k_gp_count_loc, dim3(blocks_for((size_t)nw, BLOCK)), dim3(BLOCK), 0, s, a, (const int *)ctx->wlist.p, nw,
                       cnt, (uint8_t *)ctx->gp_cb.p, (uint8_t *)ctx->gp_cb.p + wc, loc);
    int st;
    if ((st = exclusive_scan_int(ctx, cnt, cur, HW + 1))) return st == APD_ENOMEM ? APD_OK : st;
    hipLaunchKernelGGL(k_gp_place, dim3(blocks_for((size_t)nw, BLOCK)), dim3(BLOCK), 0, s, a, (const int *)ctx->wlist.p, nw,
                       (const int *)cur, (const uint8_t *)ctx->gp_cb.p + wc, (const uint32_t *)loc, (uint32_t *)ctx->gp_refs.p);
    hipLaunchKernelGGL(k_gp_classes, dim3(blocks_for(HW, BLOCK)), dim3(BLOCK), 0, s, (const int *)cur, (int)HW, (int)(U + 1),
                       (int)cap2, lists, ctr);
    const int ncu = ctx->ncu;
#define GP_Q_ARGS(c)                                                                                                         \
    s, a, (const int *)(lists + (size_t)(c) * (U + 1)), (const int *)(ctr + (c)), ctr + 3, (const int *)cur,                \
        (const uint32_t *)ctx->gp_refs.p, (const uint8_t *)ctx->gp_cb.p, ctr + 5, (int2 *)ctx->gp_plist.p,                  \
        (uint32_t *)ctx->gp_pidx.p, (int)pcap
    hipLaunchKernelGGL((k_gp_dedup_q<GP_SMALL_HS, WAVE, false>), dim3(ncu * 32), dim3(WAVE), 0, GP_Q_ARGS(0));
    hipLaunchKernelGGL((k_gp_dedup_q<GP_MEDIUM_HS, GP_CHUNK, false>), dim3(ncu * 6), dim3(GP_CHUNK), 0, GP_Q_ARGS(1));
    hipLaunchKernelGGL((k_gp_dedup_q<GP_HS, GP_CHUNK, true>), dim3(ncu * 3), dim3(GP_CHUNK), 0, GP_Q_ARGS(2));
#undef GP_Q_ARGS
    if ((st = check_launch(ctx, "pair table"))) return st;
    ctx->gp_pending = true;
    ctx->gp_on = true;
    ctx->gp_pcap = pcap;
    return APD_OK;
}

// the async table's pair count (one read-back, after the prepare phase's kernels), its cost buffer,
// and the synchronous rebuild when a bound was exceeded
static int finish_global_pairs(apd_ctx *ctx, int nw) {
    if (!ctx->gp_pending) return APD_OK;
    ctx->gp_pending = false;
    const size_t HW = (size_t)ctx->args.HW;
    const size_t U = HW > (size_t)ctx->weak_count ? HW - (size_t)ctx->weak_count : 1;
    const size_t cap2 = U + 1 + (size_t)nw * 8 / GP_SPLIT + 1;
    const int *ctr = (const int *)ctx->gp_cls.p + 2 * (U + 1) + 2 * cap2;
    int h[8] = {};
    HIP_OK(ctx, hipMemcpyAsync(h, ctr, 8 * sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
    HIP_OK(ctx, hipStreamSynchronize(ctx->stream));
    const int npairs = h[5];
    if (h[4] != 0 || npairs < 0 || (size_t)npairs > ctx->gp_pcap) {
        if (npairs < 0 || (size_t)npairs > ctx->gp_pcap) ctx->gp_cap_factor = 8;
        const bool rec = ctx->rec_on;
        int st = build_global_pairs(ctx, nw);
        if (st) return st;
        if (!rec) ctx->gp_on = false;  // (the anchor-window records were not built)
        return check_launch(ctx, "pair table");
    }
    if (npairs > 0 && !try_ensure(ctx, ctx->gp_pcost, (size_t)npairs * ((ctx->args.N + 3) & ~3) * sizeof(float))) {
        ctx->gp_on = false;
        return APD_OK;
    }
    ctx->gp_np = npairs;
    return APD_OK;
}

int32_t apd_stage_prepare(apd_ctx *ctx) {
    if (!ctx || !ctx->loaded) return APD_ESTATE;
    (void)hipSetDevice(ctx->device);
    Args &a = ctx->args;
    hipStream_t s = ctx->stream;
    const unsigned gpx = blocks_for((size_t)a.HW, BLOCK);
    int st;
    ctx->gp_on = false;
    (void)hipEventRecord(ctx->ev[0], s);
    if (a.use_apd) {
        // anchors_map from the input WEAK mask (APD.cpp:627-640). The reference numbers the WEAK pixels
        // row-major; here they are numbered in the sweep lists' tile order, so the per-WEAK-pixel
        // arrays (anchors, the candidates' bits, pair ids and costs) are read and written in runs by
        // the tile-ordered kernels (row-major, a 64-pixel list chunk scattered its 4-byte writes over
        // 4 rows: k_weak_cand_comb wrote 2.2x its bytes). Only the anchors export sees the numbering,
        // and apd_result restores the row-major order.
        if ((st = build_tile_list(ctx, 2, 0, (int *)ctx->amap.p, (int *)ctx->totals.p + 4))) return st;
        if (ctx->near_levels) {
            hipLaunchKernelGGL(k_near_columns, dim3(blocks_for((size_t)ctx->near_levels * a.W, BLOCK)), dim3(BLOCK), 0, s, a,
                               ctx->near_levels, (uint8_t *)ctx->near_g.p);
            hipLaunchKernelGGL(k_find_nearest_rows, dim3(gpx), dim3(BLOCK), 0, s, a, (const uint8_t *)ctx->near_g.p,
                               (const int *)ctx->near_ring.p);
        } else {
            hipLaunchKernelGGL(k_find_nearest, dim3(gpx), dim3(BLOCK), 0, s, a, ctx->n_near);
        }
        {
            Args ag = a;  // (profiling counters: instrumented builds of k_gen_anchors only)
            ag.evals = (ctx->prof && ctx->evals.p) ? (APD_G unsigned long long *)ctx->evals.p : nullptr;
            // the RANSAC in its own kernel when the stage fits (GA_STAGE_W words per WEAK pixel); else in k_gen_anchors
            const size_t wc = (size_t)std::max(ctx->weak_count, 1);
            uint32_t *stage = (ctx->ga_split && ctx->weak_count > 0 &&
                               try_ensure(ctx, ctx->ga_stage, (size_t)GA_STAGE_W * wc * sizeof(uint32_t)))
                                  ? (uint32_t *)ctx->ga_stage.p : nullptr;
            if (stage) {
                hipLaunchKernelGGL(k_gen_anchors<true>, dim3(gpx), dim3(BLOCK), 0, s, ag, stage, (int)wc);
                hipLaunchKernelGGL(k_gen_anchors_fit, dim3(blocks_for(wc, GA_FIT_WAVES)), dim3(GA_FIT_WAVES * WAVE), 0, s, a,
                                   (const uint32_t *)stage, (int)wc);
            } else {
                hipLaunchKernelGGL(k_gen_anchors<false>, dim3(gpx), dim3(BLOCK), 0, s, ag, stage, (int)wc);
            }
        }
        hipLaunchKernelGGL(k_neighbour_update, dim3(gpx), dim3(BLOCK), 0, s, a);
        if ((st = check_launch(ctx, "anchors"))) return st;
    }
    (void)hipEventRecord(ctx->ev[1], s);
    // RandomInitialization needs the anchors and the input state only: with overlap it runs on side
    // stream 0 beside the lists and the pair table (which read neither what it writes -- planes,
    // costs, the next selections, view weights, kept costs -- nor write what it reads)
    hipStream_t sri = s;
    if (ctx->overlap) {
        HIP_OK(ctx, hipEventRecord(ctx->ev_fork, s));
        HIP_OK(ctx, hipStreamWaitEvent(ctx->side[0], ctx->ev_fork, 0));
        sri = ctx->side[0];
    }
    {
        const int tw = ctx->dw_tile_w, th = VM_P / tw;
        const unsigned nb = (unsigned)(((a.W + tw - 1) / tw) * ((a.H + th - 1) / th));
        if (a.use_apd) {
            if (a.sa_any) {
                if (a.tex_f16) hipLaunchKernelGGL((k_random_init_vm<true, true, true>), dim3(nb), dim3(VM_BLOCK), (ri_lds_bytes<true, true>(a.N) + sa_lds_bytes(a)), sri, a, tw);
                else hipLaunchKernelGGL((k_random_init_vm<false, true, true>), dim3(nb), dim3(VM_BLOCK), (ri_lds_bytes<false, true>(a.N) + sa_lds_bytes(a)), sri, a, tw);
            } else {
                if (a.tex_f16) hipLaunchKernelGGL((k_random_init_vm<true, true, false>), dim3(nb), dim3(VM_BLOCK), (ri_lds_bytes<true, true>(a.N)), sri, a, tw);
                else hipLaunchKernelGGL((k_random_init_vm<false, true, false>), dim3(nb), dim3(VM_BLOCK), (ri_lds_bytes<false, true>(a.N)), sri, a, tw);
            }
        } else {
            if (a.sa_any) {
                if (a.tex_f16) hipLaunchKernelGGL((k_random_init_vm<true, false, true>), dim3(nb), dim3(VM_BLOCK), (ri_lds_bytes<true, false>(a.N) + sa_lds_bytes(a)), sri, a, tw);
                else hipLaunchKernelGGL((k_random_init_vm<false, false, true>), dim3(nb), dim3(VM_BLOCK), (ri_lds_bytes<false, false>(a.N) + sa_lds_bytes(a)), sri, a, tw);
            } else {
                if (a.tex_f16) hipLaunchKernelGGL((k_random_init_vm<true, false, false>), dim3(nb), dim3(VM_BLOCK), (ri_lds_bytes<true, false>(a.N)), sri, a, tw);
                else hipLaunchKernelGGL((k_random_init_vm<false, false, false>), dim3(nb), dim3(VM_BLOCK), (ri_lds_bytes<false, false>(a.N)), sri, a, tw);
            }
        }
        if ((st = check_launch(ctx, "k_random_init"))) return st;
        (void)hipEventRecord(ctx->ev[15], sri);  // (apd_timing.init_ms = ev[1] -> ev[15])
        if (ctx->overlap) HIP_OK(ctx, hipEventRecord(ctx->ev_side[0], sri));
    }
    // pixel lists for the sweeps (after NeigbourUpdate)
    {
        int *tot = (int *)ctx->totals.p;
        // the four lists are packed back to back: counts first (one small read-back), then fill
        const int modes[4][2] = {{0, 0}, {0, 1}, {1, 0}, {1, 1}};
        for (int i = 0; i < 4; ++i) tile_count_scan(ctx, modes[i][0], modes[i][1], tot + i);
        int host_tot[4];
        HIP_OK(ctx, hipMemcpyAsync(host_tot, tot, 4 * sizeof(int), hipMemcpyDeviceToHost, s));
        HIP_OK(ctx, hipStreamSynchronize(s));
        for (int i = 0; i < 4; ++i) ctx->cnt[i] = host_tot[i];
        for (int i = 0; i < 4; ++i) {
            if ((st = build_tile_list(ctx, modes[i][0], modes[i][1], list_ptr(ctx, i), tot + i))) return st;
        }
        if (a.use_apd && ctx->cand_pairs && ctx->cnt[2] + ctx->cnt[3] > 0) {
            // the anchor candidates' kernels run once per iteration over the WEAK pixels of both
            // colours (tile order): between the two Weak launches no anchor plane or selection
            // changes. Costs are kept by WEAK index.
            const size_t wc = (size_t)std::max(ctx->weak_count, 1);
            if (test_enomem_hook(ctx)) return APD_ENOMEM;  // (RandomInitialization is in flight on side stream 0)
            if ((st = ensure(ctx, ctx->wcand, (size_t)a.N * 8 * wc * sizeof(float)))) return st;
            if ((st = ensure(ctx, ctx->wlist, (size_t)(ctx->cnt[2] + ctx->cnt[3]) * sizeof(int)))) return st;
            if ((st = build_tile_list(ctx, 1, 2, (int *)ctx->wlist.p, tot + 5))) return st;
            (void)hipEventRecord(ctx->ev[14], s);
            // (the table's keys hold a pixel index below 2^25 and x below 2^15; else the sweep
            // evaluates the candidates itself)
            // (a pair packs x | filtered << 15 | y << 16 into an int: H < 32768 is also apd_set_problem's limit)
            if ((size_t)a.HW < (1u << 25) && a.W < 32768 && a.H < 32768 &&
                (st = ctx->gp_async ? build_global_pairs_async(ctx, ctx->cnt[2] + ctx->cnt[3])
                                    : build_global_pairs(ctx, ctx->cnt[2] + ctx->cnt[3])))
                return st;
        } else {
            (void)hipEventRecord(ctx->ev[14], s);
        }
        // the anchor windows' reference side (k_anchor_rec: taps, tap mask, finalisation terms; 32 B
        // with fp16 taps, else 64 B, per pixel and SA variant), built only when k_gp_cost reads it.
        // Optional: without room the pair table is dropped (the sweep evaluates the candidates itself).
        ctx->rec_on = false;
        a.arec = nullptr;
        if (a.use_apd && ctx->gp_on && (ctx->gp_np > 0 || ctx->gp_pending)) {
            const size_t rb = (size_t)a.HW * (a.sa_any ? 2 : 1) * (a.tex_f16 ? 2 : 4) * sizeof(uint4);
            if (try_ensure(ctx, ctx->arec, rb)) {
                a.arec = devptr<decltype(a.arec)>(ctx->arec.p);
                const unsigned g = blocks_for((size_t)a.HW, BLOCK);
                if (a.tex_f16) hipLaunchKernelGGL(k_anchor_rec<true>, dim3(g), dim3(BLOCK), 0, s, a, (uint4 *)ctx->arec.p);
                else hipLaunchKernelGGL(k_anchor_rec<false>, dim3(g), dim3(BLOCK), 0, s, a, (uint4 *)ctx->arec.p);
                if ((st = check_launch(ctx, "k_anchor_rec"))) return st;
                ctx->rec_on = true;
            } else {
                ctx->gp_on = false;
            }
        }
    }
    (void)hipEventRecord(ctx->ev[2], s);
    if (ctx->overlap) HIP_OK(ctx, hipStreamWaitEvent(s, ctx->ev_side[0], 0));  // join RandomInitialization
    HIP_OK(ctx, hipMemcpyAsync(ctx->sel.p, ctx->sel2.p, (size_t)a.HW * sizeof(uint32_t), hipMemcpyDeviceToDevice, s));
    (void)hipEventRecord(ctx->ev[3], s);
    if ((st = finish_global_pairs(ctx, ctx->cnt[2] + ctx->cnt[3]))) return st;
    ctx->prep_timed = true;
    ctx->wcur_fresh = a.wcur != nullptr;
    ctx->prepared = true;
    return APD_OK;
}

// profiling brackets around one launch (no-ops unless apd_profile_reset(ctx, 1)). The events are
// timing-only: without the system-scope release fence a record does not write back and invalidate
// the caches between the bracketed kernels (with the default fence the brackets cost the C3 step
// ~15 ms), and they are recycled instead of created per launch.
static hipEvent_t prof_event(apd_ctx *ctx) {
    hipEvent_t e = nullptr;
    if (!ctx->prof_pool.empty()) {
        e = ctx->prof_pool.back();
        ctx->prof_pool.pop_back();
    } else {
        (void)hipEventCreateWithFlags(&e, hipEventDisableSystemFence);
    }
    return e;
}
static hipEvent_t prof_begin(apd_ctx *ctx, hipStream_t st = nullptr) {
    hipEvent_t e0 = nullptr;
    if (ctx->prof) {
        e0 = prof_event(ctx);
        (void)hipEventRecord(e0, st ? st : ctx->stream);
    }
    return e0;
}
static void prof_end(apd_ctx *ctx, hipEvent_t e0, int kind, int64_t px, hipStream_t st = nullptr) {
    if (!ctx->prof) return;
    hipEvent_t e1 = prof_event(ctx);
    (void)hipEventRecord(e1, st ? st : ctx->stream);
    ctx->prof_ev.push_back({e0, e1, kind, px});
}

int32_t apd_stage_iteration(apd_ctx *ctx, int32_t iter) {
    if (!ctx || !ctx->prepared) return APD_ESTATE;
    (void)hipSetDevice(ctx->device);
    Args &a = ctx->args;
    hipStream_t s = ctx->stream;
    int st;
    APD_G unsigned long long *evals = (ctx->prof && ctx->evals.p) ? (APD_G unsigned long long *)ctx->evals.p : nullptr;
    for (int colour = 0; colour < 2; ++colour) {
        const int n = ctx->cnt[colour];
        if (n <= 0) continue;
        hipEvent_t e0 = prof_begin(ctx);
        Args ak = a;
        ak.evals = evals;
        if (!(ctx->wcur_fresh && iter == 0)) ak.wcur = nullptr;  // RandomInitialization's costs: iteration 0 only
        LAUNCH_TEX_SA(k_sweep_strong_vm, dim3(blocks_for((size_t)n, VM_P)), dim3(VM_BLOCK), vm_lds_bytes(a.N, ctx->args.tex_f16 != 0) + sa_lds_bytes(a), s,
                      ak, (const int *)list_ptr(ctx, colour), n, iter);
        prof_end(ctx, e0, APD_PROF_STRONG_SWEEP, n);
        if ((st = check_launch(ctx, "k_sweep_strong"))) return st;
    }
    if (a.use_apd) {
        // the Weak path's wall time (RANSAC beside the candidate kernels, then the Weak sweeps)
        hipEvent_t ewp = prof_begin(ctx);
        // fork: RANSAC (side stream 0) and k_gp_cost (side stream 1) beside k_weak_cand_g (ctx stream)
        hipStream_t sr = s, sg = s;
        if (ctx->overlap) {
            HIP_OK(ctx, hipEventRecord(ctx->ev_fork, s));
            HIP_OK(ctx, hipStreamWaitEvent(ctx->side[0], ctx->ev_fork, 0));
            HIP_OK(ctx, hipStreamWaitEvent(ctx->side[1], ctx->ev_fork, 0));
            sr = ctx->side[0];
            sg = ctx->side[1];
        }
        hipEvent_t e0 = prof_begin(ctx, sr);
        hipLaunchKernelGGL(k_ransac_fit, dim3(blocks_for((size_t)a.HW, BLOCK)), dim3(BLOCK), 0, sr, a, iter);
        prof_end(ctx, e0, APD_PROF_RANSAC_FIT, a.HW, sr);
        if (ctx->overlap) HIP_OK(ctx, hipEventRecord(ctx->ev_side[0], sr));
        const int nw = ctx->cnt[2] + ctx->cnt[3];
        const int wc = std::max(ctx->weak_count, 1);
        const float *cand = nullptr;
        if (ctx->cand_pairs && nw > 0 && ctx->gp_on) {
            if (ctx->wcand.bytes < (size_t)a.N * 8 * (size_t)wc * sizeof(float) || ctx->wlist.bytes < (size_t)nw * sizeof(int)) {
                ctx->err = "candidate cost buffers not sized by apd_stage_prepare";
                return APD_ESTATE;
            }
            Args ac = a;
            ac.evals = evals;
            {
                hipEvent_t e1 = prof_begin(ctx, sg);
                if (ctx->gp_np > 0)
                    LAUNCH_TEX_SA(k_gp_cost, dim3(blocks_for((size_t)ctx->gp_np, BLOCK)), dim3(BLOCK), gp_cost_lds_bytes(a.N), sg, ac,
                               (const int2 *)ctx->gp_plist.p, ctx->gp_np, (float *)ctx->gp_pcost.p);
                prof_end(ctx, e1, APD_PROF_GP_COST, ctx->gp_np, sg);
                if (ctx->overlap) HIP_OK(ctx, hipEventRecord(ctx->ev_side[1], sg));
                e1 = prof_begin(ctx);
                LAUNCH_TEX_SA(k_weak_cand_g, dim3(blocks_for((size_t)nw, VM_P)), dim3(PK_BLOCK), 0, s, ac, (const int *)ctx->wlist.p, nw,
                              (const uint8_t *)ctx->gp_cb.p, (float *)ctx->wcand.p, wc);
                prof_end(ctx, e1, APD_PROF_WEAK_CAND_G, nw);
                if (ctx->overlap) HIP_OK(ctx, hipStreamWaitEvent(s, ctx->ev_side[1], 0));  // join k_gp_cost
                e1 = prof_begin(ctx);
                hipLaunchKernelGGL(k_weak_cand_comb, dim3(2 * blocks_for((size_t)nw, VM_P)), dim3(BLOCK), 0, s, ac,
                                   (const int *)ctx->wlist.p, nw, (const uint8_t *)ctx->gp_cb.p, (const uint8_t *)ctx->gp_cb.p + wc,
                                   (const uint32_t *)ctx->gp_pidx.p, (const float *)ctx->gp_pcost.p, (float *)ctx->wcand.p, wc);
                prof_end(ctx, e1, APD_PROF_WEAK_CAND_COMB, nw);
            }
            cand = (const float *)ctx->wcand.p;
        }
        if (ctx->overlap) HIP_OK(ctx, hipStreamWaitEvent(s, ctx->ev_side[0], 0));  // join RANSAC (the sweep reads a.fit)
        for (int colour = 0; colour < 2; ++colour) {
            const int n = ctx->cnt[2 + colour];
            if (n <= 0) continue;
            // RandomInitialization's kept costs are valid for the first iteration after it only
            Args aw = a;
            aw.evals = evals;
            if (!(ctx->wcur_fresh && iter == 0)) aw.wcur = nullptr;
            e0 = prof_begin(ctx);
            // k_sweep_weak_vm's small cost table when every pixel's candidates are in `cand`
            const bool direct = cand != nullptr;
            LAUNCH_TEX_SA(k_sweep_weak_vm, dim3(blocks_for((size_t)n, VM_P)), dim3(WV_BLOCK),
                          (ctx->args.tex_f16 ? (ctx->args.sa_any ? wv_lds_bytes<true, 9, true>(a.N, direct) : wv_lds_bytes<true, 9, false>(a.N, direct))
                                             : (ctx->args.sa_any ? wv_lds_bytes<false, 9, true>(a.N, direct) : wv_lds_bytes<false, 9, false>(a.N, direct))),
                          s,
                          aw, (const int *)list_ptr(ctx, 2 + colour), n, iter, cand, wc);
            prof_end(ctx, e0, APD_PROF_WEAK_SWEEP, n);
        }
        prof_end(ctx, ewp, APD_PROF_WEAK_PATH, ctx->cnt[2] + ctx->cnt[3]);
        if ((st = check_launch(ctx, "weak sweep"))) return st;
    }
    ctx->wcur_fresh = false;
    return APD_OK;
}

int32_t apd_stage_finish(apd_ctx *ctx) {
    if (!ctx || !ctx->prepared) return APD_ESTATE;
    (void)hipSetDevice(ctx->device);
    Args a = ctx->args;
    hipStream_t s = ctx->stream;
    int st;
    const unsigned gpx = blocks_for((size_t)a.HW, BLOCK);
    hipLaunchKernelGGL(k_depth_normal, dim3(gpx), dim3(BLOCK), 0, s, a);
    for (int colour = 0; colour < 2; ++colour) {
        const int n = ctx->cnt[colour];
        if (n > 0)
            hipLaunchKernelGGL(k_filter, dim3(blocks_for((size_t)n, BLOCK)), dim3(BLOCK), 0, s, a,
                               (const int *)list_ptr(ctx, colour), n);
    }
    if (ctx->want_curve && ctx->curve.p) a.curve = devptr<decltype(a.curve)>(ctx->curve.p);
    a.lr_ncc = nullptr;
    a.lr_geo = nullptr;
    if (ctx->lr_handover && ctx->lrs_need > 0 && ctx->lrs.p && ctx->lrs.bytes >= ctx->lrs_need) {
        // DepthToWeak hands LocalRefine the NCC-Old / geometric terms of the 11 samples they share
        // (buffer sized by apd_set_problem; without it LocalRefine evaluates them itself)
        const size_t plane = ctx->lrs_need / (sizeof(float) * (a.geom ? 2 : 1));
        a.lr_ncc = devptr<decltype(a.lr_ncc)>(ctx->lrs.p);
        a.lr_geo = a.geom ? devptr<decltype(a.lr_geo)>((float *)ctx->lrs.p + plane) : nullptr;
    }
    {
        const int tw = ctx->dw_tile_w, th = VM_P / tw;
        const unsigned nb = (unsigned)(((a.W + tw - 1) / tw) * ((a.H + th - 1) / th));
        const int dwc = dw_chunk(a.N, a.geom != 0, sa_lds_bytes(a));
        Args ad = a;
        ad.evals = (ctx->prof && ctx->evals.p) ? (APD_G unsigned long long *)ctx->evals.p : nullptr;
        // fp16 problems: DepthToWeak's taps over the pre-differenced texels (FastTexD, apd_set_problem)
        const bool dp = a.dpairs != nullptr;
        hipEvent_t e0 = prof_begin(ctx);
        if (dp) {
            const size_t lds = dw_lds_bytes(a.N, a.geom != 0, dwc) + sa_lds_bytes(a);
            if (a.sa_any) hipLaunchKernelGGL((k_depth_to_weak_vm<true, true, true>), dim3(nb), dim3(VM_BLOCK), lds, s, ad, dwc, tw);
            else hipLaunchKernelGGL((k_depth_to_weak_vm<true, false, true>), dim3(nb), dim3(VM_BLOCK), lds, s, ad, dwc, tw);
        } else {
            LAUNCH_TEX_SA(k_depth_to_weak_vm, dim3(nb), dim3(VM_BLOCK), dw_lds_bytes(a.N, a.geom != 0, dwc) + sa_lds_bytes(a), s, ad, dwc, tw);
        }
        prof_end(ctx, e0, APD_PROF_DEPTH_TO_WEAK, a.HW);
    }
    if (a.geom || a.use_apd) hipLaunchKernelGGL(k_confidence, dim3(gpx), dim3(BLOCK), 0, s, a);
    {
        const int tw = ctx->dw_tile_w, th = VM_P / tw;
        const unsigned nb = (unsigned)(((a.W + tw - 1) / tw) * ((a.H + th - 1) / th));
        LAUNCH_TEX_SA(k_local_refine_vm, dim3(nb), dim3(VM_BLOCK), lr_lds_bytes(a.N) + sa_lds_bytes(a), s, a, lr_chunk(a.N), tw);
    }
    if ((st = check_launch(ctx, "finish"))) return st;
    return APD_OK;
}

// the prepare phase's fields of apd_timing from its events (the ctx stream has passed ev[3]).
// RandomInitialization runs first after the anchors, beside the lists and the pair table when the
// ctx overlaps (side stream 0): init_ms is its own duration, lists_ms + pairs_ms the ctx stream's,
// join_ms the ctx stream's wait for it, and anchors + lists + pairs + join == prepare.
static void prepare_timing(apd_ctx *ctx, apd_timing &t) {
    memset(&t, 0, sizeof(t));
    if (!ctx->prep_timed) return;
    (void)hipEventElapsedTime(&t.anchors_ms, ctx->ev[0], ctx->ev[1]);
    (void)hipEventElapsedTime(&t.lists_ms, ctx->ev[1], ctx->ev[14]);
    (void)hipEventElapsedTime(&t.pairs_ms, ctx->ev[14], ctx->ev[2]);
    (void)hipEventElapsedTime(&t.join_ms, ctx->ev[2], ctx->ev[3]);
    (void)hipEventElapsedTime(&t.prepare_ms, ctx->ev[0], ctx->ev[3]);
    (void)hipEventElapsedTime(&t.init_ms, ctx->ev[1], ctx->ev[15]);
}

int32_t apd_get_prepare_timing(apd_ctx *ctx, apd_timing *timing) {
    if (!ctx || !timing) return APD_EINVAL;
    if (!ctx->prepared) return APD_ESTATE;
    (void)hipSetDevice(ctx->device);
    HIP_OK(ctx, hipStreamSynchronize(ctx->stream));
    prepare_timing(ctx, *timing);
    return APD_OK;
}

int32_t apd_run_patchmatch(apd_ctx *ctx) {
    if (!ctx || !ctx->loaded) return APD_ESTATE;
    (void)hipSetDevice(ctx->device);
    int st;
    hipStream_t s = ctx->stream;
    if ((st = apd_stage_prepare(ctx))) return st;
    const int iters = ctx->params.max_iterations;
    for (int i = 0; i < iters; ++i) {
        if (i < 8) (void)hipEventRecord(ctx->ev[4 + i], s);
        if ((st = apd_stage_iteration(ctx, i))) return st;
    }
    (void)hipEventRecord(ctx->ev[12], s);
    if ((st = apd_stage_finish(ctx))) return st;
    (void)hipEventRecord(ctx->ev[13], s);
    HIP_OK(ctx, hipStreamSynchronize(s));
    apd_timing &t = ctx->timing;
    prepare_timing(ctx, t);
    (void)hipEventElapsedTime(&t.total_ms, ctx->ev[0], ctx->ev[13]);
    (void)hipEventElapsedTime(&t.sweep_ms, ctx->ev[3], ctx->ev[12]);
    (void)hipEventElapsedTime(&t.post_ms, ctx->ev[12], ctx->ev[13]);
    const int ni = std::min(iters, 8);
    for (int i = 0; i < ni; ++i)
        (void)hipEventElapsedTime(&t.iter_ms[i], ctx->ev[4 + i], (i + 1 < ni) ? ctx->ev[5 + i] : ctx->ev[12]);
    t.iterations = iters;
    return APD_OK;
}

int32_t apd_synchronize(apd_ctx *ctx) {
    if (!ctx) return APD_EINVAL;
    (void)hipSetDevice(ctx->device);
    HIP_OK(ctx, hipStreamSynchronize(ctx->stream));
    return APD_OK;
}

int32_t apd_get_results(apd_ctx *ctx, const apd_outputs *out) {
    if (!ctx || !out) return APD_EINVAL;
    if (!ctx->loaded) return APD_ESTATE;
    (void)hipSetDevice(ctx->device);
    hipStream_t s = ctx->stream;
    const Args &a = ctx->args;
    const size_t HW = (size_t)a.HW;
    // outputs may be host or device buffers (hipMemcpyDefault): scan_runner.py keeps them in HBM
    if (out->planes) HIP_OK(ctx, hipMemcpyAsync(out->planes, ctx->plane.p, HW * sizeof(float4), hipMemcpyDefault, s));
    if (out->weak_info) HIP_OK(ctx, hipMemcpyAsync(out->weak_info, ctx->weak.p, HW, hipMemcpyDefault, s));
    if (out->confidence) HIP_OK(ctx, hipMemcpyAsync(out->confidence, ctx->conf.p, HW, hipMemcpyDefault, s));
    if (out->costs) HIP_OK(ctx, hipMemcpyAsync(out->costs, ctx->cost.p, HW * sizeof(float), hipMemcpyDefault, s));
    if (out->selected_views)
        HIP_OK(ctx, hipMemcpyAsync(out->selected_views, ctx->sel.p, HW * sizeof(uint32_t), hipMemcpyDefault, s));
    if (out->view_weights) HIP_OK(ctx, hipMemcpyAsync(out->view_weights, ctx->vw.p, HW * a.N, hipMemcpyDefault, s));
    if (out->anchors && a.use_apd && ctx->weak_count > 0) {
        // the device keeps them by tile-order WEAK index: back to the row-major order of the export
        const size_t nb = (size_t)ctx->weak_count * 9 * sizeof(short2);
        void *tmp = nullptr;
        if (hipMalloc(&tmp, nb) != hipSuccess) {
            ctx->err = "hipMalloc(" + std::to_string(nb) + ") failed (anchors export)";
            return APD_ENOMEM;
        }
        hipLaunchKernelGGL(k_list_count, dim3(a.H), dim3(BLOCK), 0, s, a, 3, 0, (int *)ctx->rowcnt.p);
        hipLaunchKernelGGL(k_list_scan, dim3(1), dim3(1024), 0, s, (const int *)ctx->rowcnt.p, a.H, (int *)ctx->rowoff.p,
                           (int *)ctx->totals.p + 6);
        hipLaunchKernelGGL(k_anchor_export, dim3(a.H), dim3(BLOCK), 0, s, a, (const int *)ctx->rowoff.p, (short2 *)tmp);
        hipError_t e = hipGetLastError();
        if (e == hipSuccess) e = hipMemcpyAsync(out->anchors, tmp, nb, hipMemcpyDefault, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        (void)hipFree(tmp);
        if (e != hipSuccess) {
            ctx->err = std::string("anchors export: ") + hipGetErrorString(e);
            return APD_EDEVICE;
        }
    }
    if (out->reliable_curve && ctx->want_curve)
        HIP_OK(ctx, hipMemcpyAsync(out->reliable_curve, ctx->curve.p, HW * 61 * sizeof(float), hipMemcpyDefault, s));
    if (out->weak_count) *out->weak_count = ctx->weak_count;
    HIP_OK(ctx, hipStreamSynchronize(s));
    return APD_OK;
}

int32_t apd_get_timing(apd_ctx *ctx, apd_timing *timing) {
    if (!ctx || !timing) return APD_EINVAL;
    *timing = ctx->timing;
    return APD_OK;
}

int32_t apd_profile_reset(apd_ctx *ctx, int32_t enable) {
    if (!ctx) return APD_EINVAL;
    (void)hipSetDevice(ctx->device);
    (void)hipStreamSynchronize(ctx->stream);
    for (auto &pe : ctx->prof_ev) { ctx->prof_pool.push_back(pe.e0); ctx->prof_pool.push_back(pe.e1); }
    ctx->prof_ev.clear();
    ctx->prof = enable != 0;
    if (ctx->prof) {
        const size_t bytes = (size_t)APD_PROF_SLOTS * APD_PROF_SPREAD * sizeof(unsigned long long);
        int st = ensure(ctx, ctx->evals, bytes);
        if (st) return st;
        HIP_OK(ctx, hipMemsetAsync(ctx->evals.p, 0, bytes, ctx->stream));
    }
    return APD_OK;
}

int32_t apd_profile_counters(apd_ctx *ctx, int64_t *counts, int32_t n) {
    if (!ctx || !counts || n < 0) return APD_EINVAL;
    (void)hipSetDevice(ctx->device);
    HIP_OK(ctx, hipStreamSynchronize(ctx->stream));
    std::vector<unsigned long long> c((size_t)APD_PROF_SLOTS * APD_PROF_SPREAD, 0ull);
    if (ctx->evals.p) HIP_OK(ctx, hipMemcpy(c.data(), ctx->evals.p, c.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    for (int i = 0; i < n; ++i) {
        int64_t t = 0;
        if (i < APD_PROF_SLOTS)
            for (int r = 0; r < APD_PROF_SPREAD; ++r) t += (int64_t)c[(size_t)r * APD_PROF_SLOTS + i];
        counts[i] = t;
    }
    return APD_OK;
}

int32_t apd_profile_evaluations(apd_ctx *ctx, int64_t *ncc_evaluations) {
    if (!ncc_evaluations) return APD_EINVAL;
    return apd_profile_counters(ctx, ncc_evaluations, 1);
}

int32_t apd_profile_kernel(apd_ctx *ctx, int32_t kind, double *ms_total, int64_t *launches, int64_t *pixels) {
    if (!ctx) return APD_EINVAL;
    (void)hipSetDevice(ctx->device);
    HIP_OK(ctx, hipStreamSynchronize(ctx->stream));
    double tot = 0.0;
    int64_t nl = 0, px = 0;
    for (auto &pe : ctx->prof_ev) {
        // APD_PROF_WEAK_CAND: the three candidate kernels together (one launch = one k_weak_cand_g)
        const bool sub = kind == APD_PROF_WEAK_CAND &&
                         (pe.kind == APD_PROF_GP_COST || pe.kind == APD_PROF_WEAK_CAND_G || pe.kind == APD_PROF_WEAK_CAND_COMB);
        if (pe.kind != kind && !sub) continue;
        float ms = 0.0f;
        (void)hipEventElapsedTime(&ms, pe.e0, pe.e1);
        tot += ms;
        if (!sub || pe.kind == APD_PROF_WEAK_CAND_G) {
            ++nl;
            px += pe.px;
        }
    }
    if (ms_total) *ms_total = tot;
    if (launches) *launches = nl;
    if (pixels) *pixels = px;
    return APD_OK;
}

int32_t apd_profile_query(apd_ctx *ctx, double *sweep_ms_total, int64_t *sweep_launches, int64_t *sweep_pixels) {
    return apd_profile_kernel(ctx, APD_PROF_STRONG_SWEEP, sweep_ms_total, sweep_launches, sweep_pixels);
}

int32_t apd_device_alloc(apd_ctx *ctx, size_t bytes, void **ptr) {
    if (!ctx || !ptr) return APD_EINVAL;
    (void)hipSetDevice(ctx->device);
    *ptr = nullptr;
    if (hipMalloc(ptr, bytes ? bytes : 16) != hipSuccess) {
        (void)hipGetLastError();
        *ptr = nullptr;
        ctx->err = "hipMalloc(" + std::to_string(bytes) + ") failed";
        return APD_ENOMEM;
    }
    return APD_OK;
}

int32_t apd_device_free(apd_ctx *ctx, void *ptr) {
    if (!ctx) return APD_EINVAL;
    (void)hipSetDevice(ctx->device);
    if (ptr) {
        drain(ctx);
        HIP_OK(ctx, hipFree(ptr));
    }
    return APD_OK;
}

int32_t apd_device_copy(apd_ctx *ctx, void *dst, const void *src, size_t bytes) {
    if (!ctx || (!dst && bytes) || (!src && bytes)) return APD_EINVAL;
    (void)hipSetDevice(ctx->device);
    HIP_OK(ctx, hipMemcpyAsync(dst, src, bytes, hipMemcpyDefault, ctx->stream));
    HIP_OK(ctx, hipStreamSynchronize(ctx->stream));
    return APD_OK;
}

int32_t apd_device_copy_peer(apd_ctx *dst_ctx, void *dst, apd_ctx *src_ctx, const void *src, size_t bytes) {
    if (!dst_ctx || !src_ctx || (!dst && bytes) || (!src && bytes)) return APD_EINVAL;
    if (!bytes) return APD_OK;
    (void)hipSetDevice(dst_ctx->device);
    if (dst_ctx->device == src_ctx->device) {
        HIP_OK(dst_ctx, hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, dst_ctx->stream));
    } else {
        // direct over xGMI when the devices can map each other (enabled once per device pair; an
        // already-enabled pair reports hipErrorPeerAccessAlreadyEnabled), else staged by the runtime
        int can = 0;
        if (hipDeviceCanAccessPeer(&can, dst_ctx->device, src_ctx->device) == hipSuccess && can) {
            const hipError_t e = hipDeviceEnablePeerAccess(src_ctx->device, 0);
            if (e != hipSuccess) (void)hipGetLastError();
        }
        HIP_OK(dst_ctx, hipMemcpyPeerAsync(dst, dst_ctx->device, src, src_ctx->device, bytes, dst_ctx->stream));
    }
    HIP_OK(dst_ctx, hipStreamSynchronize(dst_ctx->stream));
    return APD_OK;
}

int32_t apd_device_bytes(apd_ctx *ctx, size_t *bytes) {
    if (!ctx || !bytes) return APD_EINVAL;
    const DevBuf *bufs[] = {&ctx->imgs, &ctx->quad, &ctx->depth, &ctx->views, &ctx->cams, &ctx->plane, &ctx->cost,
                            &ctx->sel, &ctx->sel2, &ctx->vw, &ctx->weak, &ctx->conf, &ctx->sa, &ctx->amap, &ctx->anchors,
                            &ctx->reliable, &ctx->nearest, &ctx->fit, &ctx->curve, &ctx->lists, &ctx->rowcnt,
                            &ctx->rowoff, &ctx->totals, &ctx->near_off, &ctx->dargs, &ctx->evals, &ctx->near_ring, &ctx->near_g,
                            &ctx->wcand, &ctx->arec, &ctx->ga_stage, &ctx->lrs, &ctx->wcur, &ctx->wlist, &ctx->gp_cb, &ctx->gp_cnt,
                            &ctx->gp_cur, &ctx->gp_refs, &ctx->gp_ccnt, &ctx->gp_cbase, &ctx->gp_plist, &ctx->gp_pidx,
                            &ctx->gp_pcost, &ctx->gp_tmp, &ctx->dpairs, &ctx->gp_cls};
    size_t t = 0;
    for (const DevBuf *b : bufs) t += b->bytes;
    *bytes = t;
    return APD_OK;
}

int32_t apd_device_mem_info(apd_ctx *ctx, size_t *free_bytes, size_t *total_bytes) {
    if (!ctx || !free_bytes || !total_bytes) return APD_EINVAL;
    (void)hipSetDevice(ctx->device);
    HIP_OK(ctx, hipMemGetInfo(free_bytes, total_bytes));
    return APD_OK;
}

int32_t apd_device_resize_nearest(apd_ctx *ctx, const void *src, int32_t sw, int32_t sh, void *dst, int32_t dw,
                                  int32_t dh, int32_t elem_bytes) {
    if (!ctx || !src || !dst || sw < 1 || sh < 1 || dw < 1 || dh < 1 || elem_bytes < 1) return APD_EINVAL;
    (void)hipSetDevice(ctx->device);
    const size_t n = (size_t)dw * dh;
    hipLaunchKernelGGL(k_resize_nearest, dim3((unsigned)std::min<size_t>(blocks_for(n, BLOCK), 65535)), dim3(BLOCK), 0,
                       ctx->stream, (const uint8_t *)src, sw, sh, (uint8_t *)dst, dw, dh, elem_bytes);
    int st = check_launch(ctx, "k_resize_nearest");
    if (st) return st;
    HIP_OK(ctx, hipStreamSynchronize(ctx->stream));
    return APD_OK;
}

int32_t apd_result_device(apd_ctx *ctx, float *depth_dev, float *planes_dev) {
    if (!ctx) return APD_EINVAL;
    if (!ctx->loaded) return APD_ESTATE;
    (void)hipSetDevice(ctx->device);
    const Args &a = ctx->args;
    const size_t n = (size_t)a.HW;
    hipLaunchKernelGGL(k_result_epilogue, dim3((unsigned)std::min<size_t>(blocks_for(n, BLOCK), 65535)), dim3(BLOCK), 0,
                       ctx->stream, (const float4 *)ctx->plane.p, n, ctx->params.depth_min, ctx->params.depth_max,
                       depth_dev, (float4 *)planes_dev);
    int st = check_launch(ctx, "k_result_epilogue");
    if (st) return st;
    HIP_OK(ctx, hipStreamSynchronize(ctx->stream));
    return APD_OK;
}

int32_t apd_epilogue(int32_t width, int32_t height, const float *planes, float depth_min, float depth_max,
                     float *depth_out, float *normal_out, uint8_t *weak_inout) {
    if (!planes || width < 1 || height < 1) return APD_EINVAL;
    const size_t HW = (size_t)width * height;
    for (size_t i = 0; i < HW; ++i) {
        float d = planes[4 * i + 3];
        if (d < depth_min || d > depth_max) {
            d = 0;
            if (weak_inout) weak_inout[i] = APD_UNKNOWN;
        }
        if (depth_out) depth_out[i] = d;
        if (normal_out) {
            normal_out[3 * i] = planes[4 * i];
            normal_out[3 * i + 1] = planes[4 * i + 1];
            normal_out[3 * i + 2] = planes[4 * i + 2];
        }
    }
    return APD_OK;
}

}  // extern "C"
