// LU lab (development tool, not part of the product): latency and throughput
// of LU variants on tracker-like systems (scripts/data/lu_cases.bin, made by
// make_lu_cases.py).  lat: one wave per CU, each solving REPS systems in a
// row -- the per-solve latency a lone wave sees; thr: 16 waves per CU.  Every
// variant is checked bitwise against variant 0 (the product's lu_solve3s).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-fast-math \
//        -I../include lu_lab.hip -o lu_lab
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../trifocal_pose_estimation_using_improved_gpuhc_amd/csrc/hc_lu3s.hpp"
#ifdef LU_LAB_EXTRA
#include LU_LAB_EXTRA
#endif

using namespace hc;

template <int V>
__device__ __forceinline__ cf lab_solve(cf (&rA)[NV], cf rB, int lane, uint32_t pat, LUBuf &L) {
    if constexpr (V == 0) return lu_solve3s(rA, rB, lane, pat, L);
#ifdef LU_LAB_EXTRA
    else return lab_variant<V>(rA, rB, lane, pat, L);
#else
    else return rB;
#endif
}

template <int V, int WAVES>
__global__ void __launch_bounds__(64 * WAVES) k_lab(int nc, const cf *__restrict__ A, const cf *__restrict__ B,
                                                   const uint32_t *__restrict__ P, cf *__restrict__ X, int reps) {
    __shared__ LUBuf s_lu[2 * WAVES];
    const int lane = __lane_id();
    const int r = lane & 31;
    const int wid = threadIdx.x / 64;
    const int gw = blockIdx.x * WAVES + wid;
    const bool ok = r < NV;
    const uint32_t pat = ok ? P[r] : 0u;
    cf acc = cmk(0.0f, 0.0f);
    for (int it = 0; it < reps; it++) {
        const int sys = (gw * 2 + (lane >> 5) + it * 2) % nc;
        int lv = lane;
        asm volatile("" : "+v"(lv));
        cf rA[NV];
#pragma unroll
        for (int c = 0; c < NV; c++) rA[c] = ok ? A[((size_t)sys * NV + r) * NV + c] : cmk(0.0f, 0.0f);
        const cf rB = ok ? B[(size_t)sys * NV + r] : cmk(0.0f, 0.0f);
        const cf x = lab_solve<V>(rA, rB, lv, pat, s_lu[wid * 2 + (lane >> 5)]);
        if (it == 0 && gw * 2 < nc && ok) X[(size_t)sys * NV + r] = x;
        acc.x += x.x;
        acc.y += x.y;
    }
    if (acc.x == 1234.5f && acc.y == 0.0f) X[0] = acc;
}

struct Dev { const cf *A, *B; const uint32_t *P; cf *X; int nc, cus; };

template <int V, int WAVES>
static float timed(const Dev &d, int reps) {
    const int grid = WAVES == 1 ? d.cus : d.cus * 4;
    hipLaunchKernelGGL((k_lab<V, WAVES>), dim3(grid), dim3(64 * WAVES), 0, 0, d.nc, d.A, d.B, d.P, d.X, 2);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipEventRecord(a);
    hipLaunchKernelGGL((k_lab<V, WAVES>), dim3(grid), dim3(64 * WAVES), 0, 0, d.nc, d.A, d.B, d.P, d.X, reps);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    return ms;
}

template <int V>
static void run(const Dev &d, int reps, const std::vector<cf> *ref, std::vector<cf> &out) {
    // every case solved once, for the bitwise check
    hipMemset(d.X, 0, sizeof(cf) * d.nc * NV);
    const int grid1 = (d.nc / 2 + 3) / 4;
    hipLaunchKernelGGL((k_lab<V, 4>), dim3(grid1), dim3(256), 0, 0, d.nc, d.A, d.B, d.P, d.X, 1);
    out.resize((size_t)d.nc * NV);
    hipMemcpy(out.data(), d.X, out.size() * sizeof(cf), hipMemcpyDeviceToHost);
    const float lat = timed<V, 1>(d, reps);
    const float thr = timed<V, 4>(d, reps);
    const double lat_ns = lat * 1e6 / reps;                                  // per solve, one wave per CU
    const double thr_ns = thr * 1e6 / ((double)d.cus * 16 * 2 * reps);        // per solve, chip-wide
    bool eq = true;
    if (ref)
        for (size_t i = 0; i < out.size(); i++) {
            const cf a = out[i], b = (*ref)[i];
            const bool same = (a.x == b.x || (a.x != a.x && b.x != b.x)) && (a.y == b.y || (a.y != a.y && b.y != b.y));
            eq = eq && same;
        }
    printf("{\"variant\": %d, \"lat_ns_per_solve\": %.1f, \"thr_ns_per_solve\": %.4f, \"equal_v0\": %s}\n", V, lat_ns,
           thr_ns, eq ? "true" : "false");
}

int main(int argc, char **argv) {
    const char *path = argc > 1 ? argv[1] : "scripts/data/lu_cases.bin";
    const int reps = argc > 2 ? atoi(argv[2]) : 2000;
    FILE *f = fopen(path, "rb");
    if (!f) { fprintf(stderr, "no %s\n", path); return 1; }
    int nc = 0;
    if (fread(&nc, 4, 1, f) != 1) return 1;
    std::vector<cf> hA((size_t)nc * NV * NV), hB((size_t)nc * NV);
    for (int i = 0; i < nc; i++) {
        if (fread(&hA[(size_t)i * NV * NV], sizeof(cf), NV * NV, f) != NV * NV) return 1;
        if (fread(&hB[(size_t)i * NV], sizeof(cf), NV, f) != NV) return 1;
    }
    std::vector<uint32_t> hP(32, 0u);
    if (fread(hP.data(), 4, NV, f) != NV) return 1;
    fclose(f);
    Dev d;
    d.nc = nc;
    hipDeviceGetAttribute(&d.cus, hipDeviceAttributeMultiprocessorCount, 0);
    cf *dA, *dB, *dX;
    uint32_t *dP;
    if (hipMalloc(&dA, hA.size() * sizeof(cf)) != hipSuccess || hipMalloc(&dB, hB.size() * sizeof(cf)) != hipSuccess ||
        hipMalloc(&dX, hB.size() * sizeof(cf)) != hipSuccess || hipMalloc(&dP, 32 * 4) != hipSuccess)
        return 1;
    hipMemcpy(dA, hA.data(), hA.size() * sizeof(cf), hipMemcpyHostToDevice);
    hipMemcpy(dB, hB.data(), hB.size() * sizeof(cf), hipMemcpyHostToDevice);
    hipMemcpy(dP, hP.data(), 32 * 4, hipMemcpyHostToDevice);
    d.A = dA; d.B = dB; d.P = dP; d.X = dX;
    std::vector<cf> ref, o;
    run<0>(d, reps, nullptr, ref);
#ifdef LU_LAB_EXTRA
    LU_LAB_RUNS
#endif
    return hipDeviceSynchronize() == hipSuccess ? 0 : 2;
}
