// hc_device.hpp -- CDNA4 (gfx950) device building blocks of the GPU-HC tracker.
//
// Complex values are float2 (cf).  Arithmetic follows the spec in DESIGN.md §4
// ("Arithmetic specification") op for op; the CPU oracle (oracle/hc_oracle.c)
// implements the same spec.  Compile with -ffp-contract=off: the only FMAs are
// the explicit __builtin_fmaf calls and the packed FMAs of hc_eval.hpp.
//
// Cross-lane traffic is in registers (DPP, v_permlane16_swap, v_readlane) or a
// per-path LDS buffer; nothing here touches HBM except the scoring loads.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace hc {

constexpr int NV = 30;        // unknowns / equations            (gpuhc_settings.yaml:17)
constexpr int NPP = 34;       // parameters incl. homogenising 1 (gpuhc_settings.yaml:18 + 1)
constexpr int NTRK = 312;     // tracks per RANSAC sample        (gpuhc_settings.yaml:19)
constexpr int WAVE = 64;
constexpr int HX_TERMS = 8, HX_PARTS = 5, HT_TERMS = 16, HT_PARTS = 6;   // ..._TrunPaths.cu:311-320
constexpr int HX_SIZE = NV * NV * HX_TERMS * HX_PARTS;  // 36000
constexpr int HT_SIZE = NV * HT_TERMS * HT_PARTS;       // 2880

struct cf { float x, y; };

__device__ __forceinline__ cf cmk(float x, float y) { cf r; r.x = x; r.y = y; return r; }
__device__ __forceinline__ cf cadd(cf a, cf b) { return cmk(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ cf csub(cf a, cf b) { return cmk(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ cf cscale(cf a, float s) { return cmk(a.x * s, a.y * s); }
__device__ __forceinline__ cf cdivs(cf a, float s) { return cmk(a.x / s, a.y / s); }
// The complex products of the spec.  The kernels use the packed
// forms of hc_eval.hpp (pcmul / pcmadd / pcmsub), which compute each component
// with exactly these fma chains.
// a*b: re = fma(a.x,b.x,-(a.y*b.y)), im = fma(a.x,b.y,a.y*b.x)
__device__ __forceinline__ cf cmul(cf a, cf b) {
    return cmk(__builtin_fmaf(a.x, b.x, -(a.y * b.y)), __builtin_fmaf(a.x, b.y, a.y * b.x));
}
// acc + a*b
__device__ __forceinline__ cf cmadd(cf acc, cf a, cf b) {
    return cmk(__builtin_fmaf(-a.y, b.y, __builtin_fmaf(a.x, b.x, acc.x)),
               __builtin_fmaf(a.y, b.x, __builtin_fmaf(a.x, b.y, acc.y)));
}
// acc - a*b
__device__ __forceinline__ cf cmsub(cf acc, cf a, cf b) {
    return cmk(__builtin_fmaf(a.y, b.y, __builtin_fmaf(-a.x, b.x, acc.x)),
               __builtin_fmaf(-a.y, b.x, __builtin_fmaf(-a.x, b.y, acc.y)));
}

// Division factors of cuCdivf (MAGMA_C_DIV) for divisor y; the quotient
// x / y is then cdiv_apply(x, f).  Literal ops, IEEE-correct division.
struct divf { float o1, brs, bis, o2; };
__device__ __forceinline__ divf cdiv_factors(cf y) {
    divf f;
    const float s = __builtin_fabsf(y.x) + __builtin_fabsf(y.y);
    f.o1 = 1.0f / s;
    f.brs = y.x * f.o1;
    f.bis = y.y * f.o1;
    const float s2 = (f.brs * f.brs) + (f.bis * f.bis);
    f.o2 = 1.0f / s2;
    return f;
}
__device__ __forceinline__ cf cdiv_apply(cf x, const divf &f) {
    const float ars = x.x * f.o1, ais = x.y * f.o1;
    return cmk(((ars * f.brs) + (ais * f.bis)) * f.o2, ((ais * f.brs) - (ars * f.bis)) * f.o2);
}

// Phase markers of the HC_DIAG_ISA build (scripts/isa_phases.py): assembly
// comments that split the tracker's ISA into the phases of a stage.  Empty in
// every other build.
#ifdef HC_DIAG_ISA
#define HC_ISA_MARK(name) asm volatile(";HCPH " name)
#define HC_ISA_MARK_I(name, i) asm volatile(";HCPH " name " %0" ::"i"(i))
#else
#define HC_ISA_MARK(name) do { } while (0)
#define HC_ISA_MARK_I(name, i) do { } while (0)
#endif

// ------------------------------------------------------------------ lanes
__device__ __forceinline__ int lane_id() { return __lane_id(); }
// The lane id computed where it is used (v_mbcnt on an opaque all-ones mask):
// LICM cannot hoist it out of the tracker's path loop, where the register
// allocator would spill it and reload it from scratch every stage.
__device__ __forceinline__ int lane_fresh() {
    unsigned m = ~0u;
    asm volatile("" : "+s"(m));
    return (int)__builtin_amdgcn_mbcnt_hi(m, __builtin_amdgcn_mbcnt_lo(m, 0u));
}

template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
template <int CTRL>
__device__ __forceinline__ int dpp_i(int v) {
    return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, false);
}
// ds_swizzle bit-mode, xor 16 inside each 32-lane half
__device__ __forceinline__ float swz_xor16_f(float v) {
    return __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(v), 0x401F));
}
__device__ __forceinline__ int swz_xor16_i(int v) { return __builtin_amdgcn_ds_swizzle(v, 0x401F); }

constexpr int DPP_QP_1032 = 0xB1;   // quad_perm [1,0,3,2]
constexpr int DPP_QP_2301 = 0x4E;   // quad_perm [2,3,0,1]
constexpr int DPP_ROW_MIRROR = 0x140;
constexpr int DPP_ROW_HALF_MIRROR = 0x141;
constexpr int DPP_ROW_SHL1 = 0x101, DPP_ROW_SHL2 = 0x102, DPP_ROW_SHL4 = 0x104, DPP_ROW_SHL8 = 0x108;

__device__ __forceinline__ int half_min_i(int v) {
    v = min(v, dpp_i<DPP_QP_1032>(v));
    v = min(v, dpp_i<DPP_QP_2301>(v));
    v = min(v, dpp_i<DPP_ROW_HALF_MIRROR>(v));
    v = min(v, dpp_i<DPP_ROW_MIRROR>(v));
    v = min(v, swz_xor16_i(v));
    return v;
}
// sum over each 32-lane half, result in every lane of the half
__device__ __forceinline__ int half_sum_i(int v) {
    v += dpp_i<DPP_QP_1032>(v);
    v += dpp_i<DPP_QP_2301>(v);
    v += dpp_i<DPP_ROW_HALF_MIRROR>(v);
    v += dpp_i<DPP_ROW_MIRROR>(v);
    v += swz_xor16_i(v);
    return v;
}
__device__ __forceinline__ int wave_sum_i(int v) {
    v += __shfl_xor(v, 32);
    v += __shfl_xor(v, 16);
    v += __shfl_xor(v, 8);
    v += __shfl_xor(v, 4);
    v += __shfl_xor(v, 2);
    v += __shfl_xor(v, 1);
    return __builtin_amdgcn_readfirstlane(v);
}
__device__ __forceinline__ int bperm_i(int v, int src_lane) { return __builtin_amdgcn_ds_bpermute(src_lane << 2, v); }
// lane 0 of each 32-lane half to the whole half (address from lane_fresh)
__device__ __forceinline__ int bcast_half0(int v) { return __builtin_amdgcn_ds_bpermute((lane_fresh() & 32) << 2, v); }
// broadcast relative lane L (compile-time) of each 32-lane half to the whole half
template <int L>
__device__ __forceinline__ float hbcast_f(float v) {
    return __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(v), (L & 31) << 5));
}
// per-half version of the reference's 32-slot __shfl_down_sync tree
// (..._TrunPaths.cu:235-238, offsets 16, 8, 4, 2, 1; lanes r >= 30 hold 0):
// lane 0's value ((((a0+a8)+(a4+a12))+((a2+a10)+(a6+a14)))+...), a_l = v_l + v_{l+16},
// broadcast to the half
__device__ __forceinline__ float tree_sum_half(float v) {
    float a = v + swz_xor16_f(v);
    float b = a + dpp_f<DPP_ROW_SHL8>(a);
    float c = b + dpp_f<DPP_ROW_SHL4>(b);
    float d = c + dpp_f<DPP_ROW_SHL2>(c);
    float e = d + dpp_f<DPP_ROW_SHL1>(d);
    return hbcast_f<0>(e);
}

// Compiler barrier + wave-scope ordering for LDS written by one lane and read
// by another lane of the SAME wave (LDS ops of one wave execute in order).
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// ------------------------------------------------------------------ scoring
// magmaHC/dev-trifocal_2op1p-eval.cuh:28-250.  rnorm3df -> 1/sqrtf(a*a+b*b+c*c),
// hypotf -> sqrtf(x*x+y*y), fdividef -> IEEE division: documented spec choices
// (DESIGN.md §4).
struct Hyp { float R[18]; float T[6]; };

__device__ __forceinline__ float rnorm3(float a, float b, float c) { return 1.0f / __builtin_sqrtf(a * a + b * b + c * c); }

// R21 / R31 from the Cayley parameters x[24..26] / x[27..29] with columns
// scaled by rnorm3df, T21 = x[18..20], T31 = x[21..23] (eval.cuh:55-120)
__device__ __forceinline__ void make_hypothesis(const cf *s_x, Hyp &h) {
#pragma unroll
    for (int m = 0; m < 2; m++) {
        const float a = s_x[m * 3 + 24].x, b = s_x[m * 3 + 25].x, c = s_x[m * 3 + 26].x;
        float *r = h.R + m * 9;
        r[0] = 1.0f + a * a - (b * b + c * c);
        r[1] = 2.0f * (a * b - c);
        r[2] = 2.0f * (a * c + b);
        r[3] = 2.0f * (a * b + c);
        r[4] = 1.0f + b * b - (a * a + c * c);
        r[5] = 2.0f * (b * c - a);
        r[6] = 2.0f * (a * c - b);
        r[7] = 2.0f * (b * c + a);
        r[8] = 1.0f + c * c - (a * a + b * b);
        const float n0 = rnorm3(r[0], r[3], r[6]);
        const float n1 = rnorm3(r[1], r[4], r[7]);
        const float n2 = rnorm3(r[2], r[5], r[8]);
        r[0] *= n0; r[1] *= n0; r[2] *= n0;
        r[3] *= n1; r[4] *= n1; r[5] *= n1;
        r[6] *= n2; r[7] *= n2; r[8] *= n2;
    }
#pragma unroll
    for (int i = 0; i < 6; i++) h.T[i] = s_x[18 + i].x;
}

}  // namespace hc
