// Exhaustive check of reciprocal sequences against IEEE 1.0f/s on the GPU,
// for every float s = m * 2^e with m in [1,2) (all 2^23 significands) and
// e in [-90, 119] -- the fast-path range of hc_lu.hpp's rcp_rn.
//   A: rcp + 2 fma (one Newton step)        B: A + 2 fma        C: B + 2 fma (= hipcc's div core)
// Output: one JSON line with mismatch counts.  Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k(int e0, unsigned long long *bad) {
    const unsigned m = blockIdx.x * blockDim.x + threadIdx.x;   // 23-bit significand
    const int e = e0 + (int)blockIdx.y;
    if (m >= (1u << 23)) return;
    const float s = __uint_as_float(((unsigned)(e + 127) << 23) | m);
    volatile float one = 1.0f;
    const float ref = one / s;                                   // IEEE (div_scale / div_fmas / div_fixup)
    const float r0 = __builtin_amdgcn_rcpf(s);
    const float e0v = __builtin_fmaf(-s, r0, 1.0f);
    const float a = __builtin_fmaf(e0v, r0, r0);
    const float e1 = __builtin_fmaf(-s, a, 1.0f);
    const float b = __builtin_fmaf(e1, a, a);
    const float e2 = __builtin_fmaf(-s, b, 1.0f);
    const float c = __builtin_fmaf(e2, a, b);
    unsigned long long fa = __float_as_uint(a) != __float_as_uint(ref);
    unsigned long long fb = __float_as_uint(b) != __float_as_uint(ref);
    unsigned long long fc = __float_as_uint(c) != __float_as_uint(ref);
    if (fa) atomicAdd(&bad[0], 1ull);
    if (fb) atomicAdd(&bad[1], 1ull);
    if (fc) atomicAdd(&bad[2], 1ull);
    if (fa && e == 0) atomicAdd(&bad[3], 1ull);
}

int main() {
    unsigned long long *d, h[4] = {0, 0, 0, 0};
    if (hipMalloc(&d, sizeof(h)) != hipSuccess) return 1;
    hipMemset(d, 0, sizeof(h));
    const int lo = -90, hi = 119;
    dim3 grid((1u << 23) / 256, hi - lo + 1);
    hipLaunchKernelGGL(k, grid, dim3(256), 0, 0, lo, d);
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    printf("{\"tested\": %llu, \"exp_range\": [%d, %d], \"bad_rcp_1newton\": %llu, \"bad_rcp_2newton\": %llu, "
           "\"bad_full_core\": %llu, \"bad_rcp_1newton_in_[1,2)\": %llu}\n",
           (unsigned long long)(hi - lo + 1) << 23, lo, hi, h[0], h[1], h[2], h[3]);
    return 0;
}
