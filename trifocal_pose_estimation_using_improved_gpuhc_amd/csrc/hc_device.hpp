// hc_device.hpp -- CDNA4 (gfx950) device building blocks of the GPU-HC tracker.
//
// One wavefront (64 lanes) owns one homotopy path.  Lane r < 30 owns row r of
// the 30x30 complex Jacobian, the RHS entry r and the unknown x_r.  All
// cross-lane traffic is in registers: DPP / ds_swizzle for the pivot search and
// the norm reductions, v_readlane (SGPR broadcast) for the pivot row, and
// v_writelane for the permutation / per-pivot division factors.  The only LDS
// use is the gather source for the polynomial evaluation (x, p(t), d) and the
// compacted index tables.
//
// Arithmetic follows the spec in DESIGN.md ("Arithmetic specification") op for
// op; the CPU oracle (oracle/hc_oracle.c) implements the same spec.  Compile
// with -ffp-contract=off: the only FMAs are the explicit __builtin_fmaf calls.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace hc {

constexpr int NV = 30;        // unknowns / equations
constexpr int NPP = 34;       // parameters incl. homogenising 1
constexpr int NTRK = 312;     // tracks per RANSAC sample
constexpr int WAVE = 64;
constexpr int HX_TERMS = 8, HX_PARTS = 5, HT_TERMS = 16, HT_PARTS = 6;
constexpr int HX_SIZE = NV * NV * HX_TERMS * HX_PARTS;  // 36000
constexpr int HT_SIZE = NV * HT_TERMS * HT_PARTS;       // 2880
constexpr int HX_SLOT_CAP = 128;  // compacted dH/dx slots (this problem: 78)

struct cf { float x, y; };

__device__ __forceinline__ cf cmk(float x, float y) { cf r; r.x = x; r.y = y; return r; }
__device__ __forceinline__ cf cadd(cf a, cf b) { return cmk(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ cf csub(cf a, cf b) { return cmk(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ cf cscale(cf a, float s) { return cmk(a.x * s, a.y * s); }
__device__ __forceinline__ cf cdivs(cf a, float s) { return cmk(a.x / s, a.y / s); }
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

// ------------------------------------------------------------------ lanes
__device__ __forceinline__ int lane_id() { return __lane_id(); }

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

// max over lanes 0..31 (and independently 32..63), result in every lane
__device__ __forceinline__ float half_max(float v) {
    v = __builtin_fmaxf(v, dpp_f<DPP_QP_1032>(v));
    v = __builtin_fmaxf(v, dpp_f<DPP_QP_2301>(v));
    v = __builtin_fmaxf(v, dpp_f<DPP_ROW_HALF_MIRROR>(v));
    v = __builtin_fmaxf(v, dpp_f<DPP_ROW_MIRROR>(v));
    v = __builtin_fmaxf(v, swz_xor16_f(v));
    return v;
}
__device__ __forceinline__ int half_min_i(int v) {
    v = min(v, dpp_i<DPP_QP_1032>(v));
    v = min(v, dpp_i<DPP_QP_2301>(v));
    v = min(v, dpp_i<DPP_ROW_HALF_MIRROR>(v));
    v = min(v, dpp_i<DPP_ROW_MIRROR>(v));
    v = min(v, swz_xor16_i(v));
    return v;
}
// The reference's 32-slot __shfl_down_sync tree (kernel ..._TrunPaths.cu:235-238)
// evaluated for lane 0: ((((a0+a8)+(a4+a12))+((a2+a10)+(a6+a14))) + ...), a_l = v_l + v_{l+16};
// lanes >= 30 must hold 0.  Returns lane 0's value broadcast.
__device__ __forceinline__ float tree_sum32(float v) {
    float a = v + swz_xor16_f(v);
    float b = a + dpp_f<DPP_ROW_SHL8>(a);
    float c = b + dpp_f<DPP_ROW_SHL4>(b);
    float d = c + dpp_f<DPP_ROW_SHL2>(c);
    float e = d + dpp_f<DPP_ROW_SHL1>(d);
    return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(e)));
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
__device__ __forceinline__ float rdl(float v, int l) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
__device__ __forceinline__ int rdl_i(int v, int l) { return __builtin_amdgcn_readlane(v, l); }
// v_writelane equivalent (this toolchain has no __builtin_amdgcn_writelane): lane l takes val
__device__ __forceinline__ float wrl(float val, int l, float old) { return (__lane_id() == l) ? val : old; }
__device__ __forceinline__ int wrl_i(int val, int l, int old) { return (__lane_id() == l) ? val : old; }
__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ float uni_f(float v) { return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v))); }

// Compiler barrier + wave-scope ordering for LDS written by one lane and read
// by another lane of the SAME wave (LDS ops of one wave execute in order).
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// ------------------------------------------------------------------ tables
// Compacted dH/dx table: for column c, nslot[c] slots, slot k holds (per row r)
// the k-th non-padding term of entry (r, c) packed as
//   coef(4b signed) | a<<4 (6b) | b<<10 (6b) | u<<16 (5b) | v<<21 (5b)   (coef 0: no term)
// dH/dt table: 16 slots, per row the k-th non-padding term packed as
//   coef | a<<4 | b<<10 | u<<16 | v<<21 | w<<26
struct TableWS {
    // control block, zeroed by the launcher every call (first 64 bytes)
    unsigned queue;
    unsigned status;
    unsigned found;          // device-side "good hypothesis found" flag
    unsigned pad0;
    unsigned long long t_start;
    unsigned long long t_found;
    unsigned pad1[8];
    // written by the table-prep kernel
    int nslot[32];           // per column; [30] = total slots
    int slot_base[32];
    uint32_t hx[HX_SLOT_CAP * 32];
    uint32_t ht[HT_TERMS * 32];
};

__device__ __forceinline__ int sext4(uint32_t w) { return ((int)(w << 28)) >> 28; }

// ------------------------------------------------------------------ evals
// gpu-idx-evals/dev-eval-indxing-trifocal_2op1p_30x30_LimUnroll_L2Cache.cuh:57-88
// rA[c] = sum_k c*p[a]*p[b]*x[u]*x[v] over the non-padding terms of (row, c).
__device__ __forceinline__ void eval_hx(cf (&rA)[NV], const uint32_t *s_hx, const int *__restrict__ g_nslot,
                                        const int *__restrict__ g_base, const cf *s_x, const cf *s_p, int l32) {
#pragma unroll
    for (int c = 0; c < NV; c++) {
        cf acc = cmk(0.0f, 0.0f);
        const int n = g_nslot[c];
        const uint32_t *tab = s_hx + g_base[c] * 32 + l32;
        for (int k = 0; k < n; k++) {
            const uint32_t w = tab[k * 32];
            const int co = sext4(w);
            const cf pa = s_p[(w >> 4) & 63], pb = s_p[(w >> 10) & 63];
            const cf xu = s_x[(w >> 16) & 31], xv = s_x[(w >> 21) & 31];
            const cf P = cmul(cmul(cscale(pa, (float)co), pb), xu);
            const cf nv = cmadd(acc, P, xv);
            acc.x = co ? nv.x : acc.x;
            acc.y = co ? nv.y : acc.y;
        }
        rA[c] = acc;
    }
}
// :91-119  b = -sum_k c*(d[a]*p[b] + d[b]*p[a])*x[u]*x[v]*x[w]
__device__ __forceinline__ cf eval_ht(const uint32_t *s_ht, const cf *s_x, const cf *s_p, const cf *s_d, int l32) {
    cf acc = cmk(0.0f, 0.0f);
#pragma unroll 4
    for (int j = 0; j < HT_TERMS; j++) {
        const uint32_t w = s_ht[j * 32 + l32];
        const int co = sext4(w);
        const int a = (w >> 4) & 63, b = (w >> 10) & 63;
        cf s = cmadd(cmul(s_d[a], s_p[b]), s_d[b], s_p[a]);
        s = cscale(s, (float)co);
        const cf P = cmul(cmul(s, s_x[(w >> 16) & 31]), s_x[(w >> 21) & 31]);
        const cf nv = cmsub(acc, P, s_x[(w >> 26) & 31]);
        acc.x = co ? nv.x : acc.x;
        acc.y = co ? nv.y : acc.y;
    }
    return acc;
}
// :122-148  b = sum_k c*p[a]*p[b]*x[u]*x[v]*x[w]
__device__ __forceinline__ cf eval_h(const uint32_t *s_ht, const cf *s_x, const cf *s_p, int l32) {
    cf acc = cmk(0.0f, 0.0f);
#pragma unroll 4
    for (int j = 0; j < HT_TERMS; j++) {
        const uint32_t w = s_ht[j * 32 + l32];
        const int co = sext4(w);
        const cf P = cmul(cmul(cmul(cscale(s_p[(w >> 4) & 63], (float)co), s_p[(w >> 10) & 63]), s_x[(w >> 16) & 31]),
                          s_x[(w >> 21) & 31]);
        const cf nv = cmadd(acc, P, s_x[(w >> 26) & 31]);
        acc.x = co ? nv.x : acc.x;
        acc.y = co ? nv.y : acc.y;
    }
    return acc;
}

// ------------------------------------------------------------------ LU solve
// magmaHC/dev-cgesv-batched-small.cuh:38-107, wave64 form.
// Lane r (< 30) holds original row r in rA and its RHS in rB; rowid is the
// row's logical position (pivoting relabels positions, rows never move).
// Pivot search = (|re|+|im| desc, position asc) argmax via a DPP max + ballot;
// pivot row broadcast by v_readlane into SGPRs; the cuCdivf factors of each
// pivot are parked in lane i of four VGPRs (v_writelane) and reused by the
// back substitution.  Returns x_r in lane r.
__device__ __forceinline__ cf lu_solve(cf (&rA)[NV], cf rB, int lane) {
    int rowid = lane;   // lanes >= 30 keep rowid >= 30: never eligible, never pivot
    int perm = lane;    // lane p: the lane holding position p
    float fo1 = 0.0f, fbr = 0.0f, fbi = 0.0f, fo2 = 0.0f;
    const bool row_lane = lane < NV;
#pragma unroll
    for (int i = 0; i < NV; i++) {
        const float v = __builtin_fabsf(rA[i].x) + __builtin_fabsf(rA[i].y);  // :55
        const bool elig = row_lane && rowid >= i;
        const bool isn = v != v;
        const float key = (elig && !isn) ? v : -1.0f;
        const float mx = half_max(key);
        int pl;  // pivot lane (uniform)
        float piv_abs;
        const unsigned long long nanm = __ballot(elig && isn && rowid == i);
        if (nanm != 0ull) {                     // dsx[i] is NaN: nothing beats it (:57-64)
            pl = __builtin_ctzll(nanm);
            piv_abs = __builtin_nanf("");
        } else {
            const unsigned long long m = __ballot(elig && key == mx) & 0x3FFFFFFFull;
            if (__builtin_popcountll(m) == 1) {
                pl = __builtin_ctzll(m);
            } else {                            // exact ties: first position wins
                const int cand = ((m >> lane) & 1ull) ? rowid : 1 << 20;
                const int mn = uni(half_min_i(cand));
                pl = __builtin_ctzll(__ballot(row_lane && rowid == mn));
            }
            piv_abs = uni_f(mx);
        }
        pl = uni(pl);
        const int piv_pos = rdl_i(rowid, pl);
        const int qlane = rdl_i(perm, i);       // lane currently at position i
        const bool zero = (piv_abs == 0.0f);    // :66
        // pivot row (positions i..29).  The reference scales it by update =
        // zero ? 0 : 1 (:68-76); when zero fires every eligible entry of column i
        // is an exact zero, so the scaling can only change the sign of exact
        // zeros -- it is not materialised here (it would force the
        // pivot row out of SGPRs).
        cf sx[NV];
#pragma unroll
        for (int j = i; j < NV; j++) sx[j] = cmk(rdl(rA[j].x, pl), rdl(rA[j].y, pl));
        const cf sB0 = cmk(rdl(rB.x, pl), rdl(rB.y, pl));   // :77
        // relabel (:70-82): pivot lane -> position i, lane at i -> old pivot position
        if (lane == pl) rowid = i;
        else if (rowid == i) rowid = piv_pos;
        perm = wrl_i(pl, i, perm);
        perm = wrl_i(qlane, piv_pos, perm);
        // reciprocal of the pivot (:84); factors parked for the back substitution
        const divf f = cdiv_factors(sx[i]);
        fo1 = wrl(f.o1, i, fo1);
        fbr = wrl(f.brs, i, fbr);
        fbi = wrl(f.bis, i, fbi);
        fo2 = wrl(f.o2, i, fo2);
        // opaque per-step state: stops the compiler from carrying per-step
        // copies of rowid / perm / factors (it otherwise folds their later
        // readlanes and keeps ~4 VGPRs per pivot step live)
        asm volatile("" : "+v"(rowid), "+v"(perm), "+v"(fo1), "+v"(fbr), "+v"(fbi), "+v"(fo2));
        const cf reg = zero ? cmk(1.0f, 0.0f) : cdiv_apply(cmk(1.0f, 0.0f), f);
        // scal + ger on the rows below (:86-93)
        if (rowid > i) {
            const cf l = cmul(rA[i], reg);
            rA[i] = l;
#pragma unroll
            for (int j = i + 1; j < NV; j++) rA[j] = cmsub(rA[j], l, sx[j]);
            rB = cmsub(rB, l, sB0);
        }
    }
    // back substitution (:97-106): position p's RHS lives in lane perm[p].
    // The empty asm makes the lane-parked factors opaque: otherwise the
    // compiler folds readlane(select(lane==i, f_i, .), i) -> f_i and keeps all
    // 4x30 factors live in VGPRs across the elimination.
    asm volatile("" : "+v"(fo1), "+v"(fbr), "+v"(fbi), "+v"(fo2), "+v"(perm));
    cf xs = cmk(0.0f, 0.0f);
#pragma unroll
    for (int i = NV - 1; i >= 0; i--) {
        const int li = rdl_i(perm, i);
        const cf bi = cmk(rdl(rB.x, li), rdl(rB.y, li));
        divf f;
        f.o1 = rdl(fo1, i); f.brs = rdl(fbr, i); f.bis = rdl(fbi, i); f.o2 = rdl(fo2, i);
        const cf xi = cdiv_apply(bi, f);
        if (rowid < i) rB = cmsub(rB, xi, rA[i]);
        xs.x = wrl(xi.x, i, xs.x);
        xs.y = wrl(xi.y, i, xs.y);
    }
    return xs;
}

// ------------------------------------------------------------------ scoring
// magmaHC/dev-trifocal_2op1p-eval.cuh:28-250 over all 64 lanes (the reference
// uses 30).  rnorm3df -> 1/sqrtf(a*a+b*b+c*c), hypotf -> sqrtf(x*x+y*y),
// fdividef -> IEEE division: documented spec choices.
struct Hyp { float R[18]; float T[6]; };

__device__ __forceinline__ float rnorm3(float a, float b, float c) { return 1.0f / __builtin_sqrtf(a * a + b * b + c * c); }

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

// returns (inliers21, inliers31) summed over the wave
__device__ __forceinline__ int2 score_hypothesis(const Hyp &h, const float *__restrict__ loc, int E,
                                                 float fx, float fy, float cx, float cy, int lane) {
    const float *R = h.R;
    const float d18 = h.T[0], d19 = h.T[1], d20 = h.T[2], d21 = h.T[3], d22 = h.T[4], d23 = h.T[5];
    int c21 = 0, c31 = 0;
    for (int e = lane; e < E; e += WAVE) {
        const float2 g01 = *reinterpret_cast<const float2 *>(loc + (size_t)e * 6);
        const float2 g23 = *reinterpret_cast<const float2 *>(loc + (size_t)e * 6 + 2);
        const float2 g45 = *reinterpret_cast<const float2 *>(loc + (size_t)e * 6 + 4);
        const float g0 = g01.x, g1 = g01.y, g2 = g23.x, g3 = g23.y, g4 = g45.x, g5 = g45.y;
        float num, den, v0, v1, v2, ex, ey;
        num = d20 * (R[2] * g2 + R[5] * g3 + R[8]) - (R[2] * d18 + R[5] * d19 + R[8] * d20);
        den = 1.0f - (R[6] * g0 + R[7] * g1 + R[8]) * (R[2] * g2 + R[5] * g3 + R[8]);
        v2 = num * (R[6] * g0 + R[7] * g1 + R[8]) + den * d20;
        v0 = (num * (R[0] * g0 + R[1] * g1 + R[2]) + den * d18) / v2;
        v1 = (num * (R[3] * g0 + R[4] * g1 + R[5]) + den * d19) / v2;
        ex = (v0 * fx + cx) - (g2 * fx + cx);
        ey = (v1 * fy + cy) - (g3 * fy + cy);
        c21 += (__builtin_sqrtf(ex * ex + ey * ey) < 2.0f) ? 1 : 0;
        num = d23 * (R[11] * g4 + R[14] * g5 + R[17]) - (R[11] * d21 + R[14] * d22 + R[17] * d23);
        den = 1.0f - (R[15] * g0 + R[16] * g1 + R[17]) * (R[11] * g4 + R[14] * g5 + R[17]);
        v2 = num * (R[15] * g0 + R[16] * g1 + R[17]) + den * d23;
        v0 = (num * (R[9] * g0 + R[10] * g1 + R[11]) + den * d21) / v2;
        v1 = (num * (R[12] * g0 + R[13] * g1 + R[14]) + den * d22) / v2;
        ex = (v0 * fx + cx) - (g4 * fx + cx);
        ey = (v1 * fy + cy) - (g5 * fy + cy);
        c31 += (__builtin_sqrtf(ex * ex + ey * ey) < 2.0f) ? 1 : 0;
    }
    return make_int2(wave_sum_i(c21), wave_sum_i(c31));
}

}  // namespace hc
