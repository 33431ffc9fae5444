// Exhaustive check (every fp32 significand, a spread of exponents, both signs): is
//   r = v_rcp_f32(z); e = fma(-z, r, 1); r' = fma(e, r, r)
// the correctly rounded 1/z that the IEEE division sequence produces? Build:
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o /tmp/rcp tools/rcp_exhaustive.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
__global__ void k(int exp_lo, int exp_hi, unsigned long long *bad, unsigned *first) {
    const uint32_t m = blockIdx.x * blockDim.x + threadIdx.x;
    if (m >= (1u << 23)) return;
    for (int e = exp_lo; e <= exp_hi; ++e) {
        for (int sgn = 0; sgn < 2; ++sgn) {
            const uint32_t bits = ((uint32_t)sgn << 31) | ((uint32_t)(e + 127) << 23) | m;
            const float z = __uint_as_float(bits);
            volatile float one = 1.0f;
            const float ref = one / z;
            const float r = __builtin_amdgcn_rcpf(z);
            const float er = __builtin_fmaf(-z, r, 1.0f);
            const float f = __builtin_fmaf(er, r, r);
            if (__float_as_uint(f) != __float_as_uint(ref)) {
                unsigned long long n = atomicAdd(bad, 1ull);
                if (n < 16) first[n] = bits;
            }
        }
    }
}
int main() {
    unsigned long long *bad; unsigned *first;
    (void)hipMalloc(&bad, 8); (void)hipMalloc(&first, 64);
    (void)hipMemset(bad, 0, 8); (void)hipMemset(first, 0, 64);
    const int ranges[][2] = {{-126, -101}, {-100, -1}, {0, 99}, {100, 127}};
    for (auto &r : ranges) {
        (void)hipMemset(bad, 0, 8);
        hipLaunchKernelGGL(k, dim3((1u << 23) / 256), dim3(256), 0, 0, r[0], r[1], bad, first);
        unsigned long long h = 0; unsigned f[16];
        (void)hipMemcpy(&h, bad, 8, hipMemcpyDeviceToHost);
        (void)hipMemcpy(f, first, 64, hipMemcpyDeviceToHost);
        printf("exponents [%d,%d]: %llu mismatches", r[0], r[1], h);
        for (unsigned i = 0; i < (h < 4 ? h : 4); ++i) printf(" 0x%08x", f[i]);
        printf("\n");
    }
    return 0;
}
