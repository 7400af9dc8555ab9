// mfma_probe.hip -- v_mfma_f32_4x4x1_16b_f32 on gfx950: operand/result lane
// layout, bitwise equality with an fmaf per element, and issue cost beside VALU.
// Build: hipcc --offload-arch=gfx950 -O3 -o scripts/mfma_probe scripts/mfma_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <cmath>
#include <random>
typedef float f4v __attribute__((ext_vector_type(4)));

__global__ void k_layout(const float *a, const float *b, const float *c, float *d) {
    const int l = threadIdx.x;
    f4v acc = {c[l * 4], c[l * 4 + 1], c[l * 4 + 2], c[l * 4 + 3]};
    acc = __builtin_amdgcn_mfma_f32_4x4x1f32(a[l], b[l], acc, 0, 0, 0);
    for (int i = 0; i < 4; i++) d[l * 4 + i] = acc[i];
}

// N iterations of: M MFMAs on independent accumulators + V independent v_pk_fma_f32
template <int M, int V>
__global__ void k_time(float *o, long long *cyc, int n) {
    const int l = threadIdx.x;
    f4v acc[4] = {};
    typedef float f2v __attribute__((ext_vector_type(2)));
    f2v p[8];
    for (int i = 0; i < 8; i++) p[i] = f2v{(float)l, (float)i};
    float a = 1.0f + l * 1e-3f, b = 0.5f;
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < n; it++) {
#pragma unroll
        for (int m = 0; m < M; m++) acc[m & 3] = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, acc[m & 3], 0, 0, 0);
#pragma unroll
        for (int v = 0; v < V; v++)
            asm volatile("v_pk_fma_f32 %0, %0, %1, %0" : "+v"(p[v & 7]) : "v"(p[(v + 3) & 7]));
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    float s = 0;
    for (int i = 0; i < 4; i++) s += acc[i][0] + acc[i][3];
    for (int i = 0; i < 8; i++) s += p[i][0];
    o[blockIdx.x * blockDim.x + l] = s;
    if (l == 0) cyc[blockIdx.x] = t1 - t0;
}

static uint32_t bits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }

template <int M, int V>
static void timeit(int waves_per_simd) {
    float *o; long long *cyc;
    const int blocks = 256 * 4 * waves_per_simd;   // one-wave blocks
    hipMalloc(&o, blocks * 64 * 4); hipMalloc(&cyc, blocks * 8);
    const int n = 2000;
    hipLaunchKernelGGL((k_time<M, V>), dim3(blocks), dim3(64), 0, 0, o, cyc, n);
    hipDeviceSynchronize();
    long long *h = new long long[blocks];
    hipMemcpy(h, cyc, blocks * 8, hipMemcpyDeviceToHost);
    double s = 0; for (int i = 0; i < blocks; i++) s += h[i];
    // s_memtime counts the shader clock
    printf("{\"mfma\": %d, \"pk_fma\": %d, \"waves_per_simd\": %d, \"cycles_per_iter\": %.2f}\n", M, V, waves_per_simd, s / blocks / n);
    delete[] h; hipFree(o); hipFree(cyc);
}

int main() {
    float ha[64], hb[64], hc[256], hd[256];
    // layout: a = lane, b = 1000 + lane (products unique), c = 0
    for (int l = 0; l < 64; l++) { ha[l] = (float)l; hb[l] = 1000.0f + l; }
    memset(hc, 0, sizeof(hc));
    float *da, *db, *dc, *dd;
    hipMalloc(&da, 256); hipMalloc(&db, 256); hipMalloc(&dc, 1024); hipMalloc(&dd, 1024);
    hipMemcpy(da, ha, 256, hipMemcpyHostToDevice); hipMemcpy(db, hb, 256, hipMemcpyHostToDevice);
    hipMemcpy(dc, hc, 1024, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_layout, dim3(1), dim3(64), 0, 0, da, db, dc, dd);
    hipMemcpy(hd, dd, 1024, hipMemcpyDeviceToHost);
    int amap[256], bmap[256];
    bool layout_ok = true;
    for (int l = 0; l < 64; l++)
        for (int i = 0; i < 4; i++) {
            float v = hd[l * 4 + i];
            int found = 0;
            for (int x = 0; x < 64; x++) for (int y = 0; y < 64; y++)
                if ((float)x * (1000.0f + y) == v) { amap[l * 4 + i] = x; bmap[l * 4 + i] = y; found++; }
            if (found != 1) layout_ok = false;
        }
    printf("{\"layout_unique\": %s, \"lane0\": [[%d,%d],[%d,%d],[%d,%d],[%d,%d]], \"lane5\": [[%d,%d],[%d,%d],[%d,%d],[%d,%d]], \"lane37\": [[%d,%d],[%d,%d],[%d,%d],[%d,%d]]}\n",
           layout_ok ? "true" : "false",
           amap[0], bmap[0], amap[1], bmap[1], amap[2], bmap[2], amap[3], bmap[3],
           amap[20], bmap[20], amap[21], bmap[21], amap[22], bmap[22], amap[23], bmap[23],
           amap[148], bmap[148], amap[149], bmap[149], amap[150], bmap[150], amap[151], bmap[151]);
    // hypothesis: lane l, VGPR i holds A[4*(l/4) + i] * B[l]
    bool hyp = layout_ok;
    for (int l = 0; l < 64 && hyp; l++)
        for (int i = 0; i < 4; i++)
            if (amap[l * 4 + i] != 4 * (l / 4) + i || bmap[l * 4 + i] != l) hyp = false;
    printf("{\"layout_A_quad_row_B_own_lane\": %s}\n", hyp ? "true" : "false");
    // bitwise fmaf: random operands incl. subnormals, zeros of both signs, inf, NaN, huge
    std::mt19937 g(7);
    long long mism = 0, total = 0;
    for (int trial = 0; trial < 4000; trial++) {
        for (int l = 0; l < 64; l++) {
            uint32_t u[3];
            for (int k = 0; k < 3; k++) {
                uint32_t r = g();
                switch (r % 11) {
                    case 0: u[k] = r & 0x807FFFFFu; break;               // subnormal / zero
                    case 1: u[k] = (r & 0x80000000u); break;             // +-0
                    case 2: u[k] = (r & 0x80000000u) | 0x7F800000u; break; // inf
                    case 3: u[k] = (r & 0x80000000u) | 0x7F000000u | (r & 0x7FFFFF); break; // huge
                    default: u[k] = (r & 0x80000000u) | ((0x30 + (r >> 8) % 0x20) << 23) | (g() & 0x7FFFFF); break;
                }
            }
            memcpy(&ha[l], &u[0], 4); memcpy(&hb[l], &u[1], 4);
            for (int i = 0; i < 4; i++) { uint32_t w = (i == 0) ? u[2] : (g() & 0x80000000u) | ((0x30 + g() % 0x20) << 23) | (g() & 0x7FFFFF); if (trial % 3 == 0 && i == 1) w = g() & 0x807FFFFFu; memcpy(&hc[l * 4 + i], &w, 4); }
        }
        hipMemcpy(da, ha, 256, hipMemcpyHostToDevice); hipMemcpy(db, hb, 256, hipMemcpyHostToDevice);
        hipMemcpy(dc, hc, 1024, hipMemcpyHostToDevice);
        hipLaunchKernelGGL(k_layout, dim3(1), dim3(64), 0, 0, da, db, dc, dd);
        hipMemcpy(hd, dd, 1024, hipMemcpyDeviceToHost);
        for (int l = 0; l < 64; l++)
            for (int i = 0; i < 4; i++) {
                const float ref = fmaf(ha[4 * (l / 4) + i], hb[l], hc[l * 4 + i]);
                const float got = hd[l * 4 + i];
                total++;
                if (!(bits(ref) == bits(got) || (std::isnan(ref) && std::isnan(got)))) {
                    if (mism < 5) printf("{\"mismatch\": [\"%08x\", \"%08x\", \"%08x\", \"%08x\", \"%08x\"]}\n", bits(ha[4*(l/4)+i]), bits(hb[l]), bits(hc[l*4+i]), bits(ref), bits(got));
                    mism++;
                }
            }
    }
    printf("{\"fmaf_bitwise_mismatches\": %lld, \"elements\": %lld}\n", mism, total);
    for (int w : {1, 5}) {
        timeit<8, 0>(w); timeit<0, 16>(w); timeit<8, 16>(w); timeit<4, 16>(w); timeit<16, 0>(w); timeit<16, 16>(w);
    }
    return 0;
}
