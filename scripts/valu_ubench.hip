// valu_ubench.hip -- VALU issue micro-benchmark (development tool, GPU only):
// cycles per wave64 instruction on one SIMD for plain FP32 FMA, packed FP32
// FMA, DPP max and v_rcp_f32, at 1..8 waves per SIMD, with independent
// chains (throughput) and one dependent chain (latency).  Calibrates what the
// tracker's SQ_ACTIVE_INST_VALU / SQ_INSTS_VALU counters mean on gfx950.
//   hipcc -O3 --offload-arch=gfx950 scripts/valu_ubench.hip -o /tmp/valu_ubench
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float pf2 __attribute__((ext_vector_type(2)));
constexpr int ITERS = 4096;

template <int KIND, int CHAINS>
__global__ void __launch_bounds__(64) kern(float *out, unsigned long long *cyc) {
    float a[8], b = 1.0001f, c = 0.999f;
    pf2 p[8], pb = {1.0001f, 0.9999f};
    int k[8];
    for (int i = 0; i < 8; i++) { a[i] = threadIdx.x * 0.001f + i; p[i] = pf2{a[i], a[i] + 1.0f}; k[i] = threadIdx.x + i; }
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < ITERS; it++) {
#pragma unroll
        for (int q = 0; q < CHAINS; q++) {
            if constexpr (KIND == 0) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a[q]) : "v"(b), "v"(c));
            if constexpr (KIND == 1) asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(p[q]) : "v"(pb));
            if constexpr (KIND == 2) asm volatile("s_nop 1\n v_max_i32_dpp %0, %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "+v"(k[q]));
            if constexpr (KIND == 3) asm volatile("v_rcp_f32 %0, %0" : "+v"(a[q]));
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    float s = 0.0f;
    for (int i = 0; i < 8; i++) s += a[i] + p[i].x + p[i].y + (float)k[i];
    out[blockIdx.x * 64 + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int KIND, int CHAINS>
void run(const char *name, int waves_per_simd, float *d_out, unsigned long long *d_cyc) {
    const int cus = 256, blocks = cus * 4 * waves_per_simd;   // 64-thread blocks spread over the SIMDs
    hipLaunchKernelGGL((kern<KIND, CHAINS>), dim3(blocks), dim3(64), 0, 0, d_out, d_cyc);
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL((kern<KIND, CHAINS>), dim3(blocks), dim3(64), 0, 0, d_out, d_cyc);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0; hipEventElapsedTime(&ms, e0, e1);
    static unsigned long long h[8192];
    hipMemcpy(h, d_cyc, sizeof(unsigned long long) * blocks, hipMemcpyDeviceToHost);
    double avg = 0; for (int i = 0; i < blocks; i++) avg += (double)h[i]; avg /= blocks;
    const double insts = (double)ITERS * CHAINS;
    printf("{\"op\": \"%s\", \"chains\": %d, \"waves_per_simd\": %d, \"cycles_per_inst_per_wave\": %.3f, "
           "\"simd_cycles_per_inst\": %.3f, \"ms\": %.4f}\n",
           name, CHAINS, waves_per_simd, avg / insts, avg / insts / waves_per_simd, ms);
}

int main() {
    float *d_out; unsigned long long *d_cyc;
    hipMalloc(&d_out, 8192 * 64 * sizeof(float));
    hipMalloc(&d_cyc, 8192 * sizeof(unsigned long long));
    for (int w : {1, 2, 4, 8}) {
        run<0, 8>("v_fma_f32", w, d_out, d_cyc);
        run<0, 1>("v_fma_f32", w, d_out, d_cyc);
        run<1, 8>("v_pk_fma_f32", w, d_out, d_cyc);
        run<1, 1>("v_pk_fma_f32", w, d_out, d_cyc);
        run<2, 8>("s_nop1+v_max_i32_dpp", w, d_out, d_cyc);
        run<3, 8>("v_rcp_f32", w, d_out, d_cyc);
    }
    return 0;
}
