// hc_lu3s.hpp -- v8 LU: v3 (hc_lu3.hpp) that skips the structurally zero
// parts of the pivot rows.
//
// The trifocal Jacobian is sparse (170 of 900 entries carry terms, DESIGN.md
// §3) and partial-pivot elimination fills it in only partly: on tracker
// Jacobians 64 % of the pivot-row entries an elimination step broadcasts are
// exact zeros, and for 53 % of the aligned entry pairs both paths of a wave
// have a zero pair (26 % of the 6-column chunks the update works in).  Each
// lane keeps the structural pattern of its row (bit c:
// column c may be non-zero) -- initially the columns with index terms (the
// compacted tables' column->slot map), then OR-ed with the pivot row's pattern
// whenever the row takes a multiple of it (fill-in).  The pivot patterns of
// the wave's two paths are read with v_readlane; a chunk of columns that is
// zero in both is neither written to LDS by the pivot lanes nor read and used
// in the rank-1 update (a wave-uniform branch per chunk).
//
// Exactness.  A structurally zero entry holds an exact zero as long as no
// product in the elimination is infinite or NaN (0 * inf = NaN in the
// reference), and then a - l*0 == a up to the sign of an exact zero (the
// equivalence class DESIGN.md §4 already uses; cuCdivf by a zero of either
// sign is NaN and |.|-based pivoting ignores signs).  Guarantees:
//  * the solve runs sparse only if every entry is finite with |re|, |im| <
//    2^88 (wave-uniform check; else every step is dense).  Pivoting on
//    |re|+|im| bounds every multiplier by sqrt(2) and the element growth by
//    (1+sqrt(2))^29 < 2^37, so no intermediate can overflow;
//  * a step whose 1/pivot leaves the fast range (|pivot| < 2^-90: 1/pivot may
//    overflow; zero or NaN pivot) is executed densely and makes the pattern
//    of every row below it dense.
#pragma once

#include "hc_lu3.hpp"

namespace hc {

#ifndef HC_LU3S_CHUNK
#define HC_LU3S_CHUNK 4
#endif
constexpr int LU3S_CHUNK = HC_LU3S_CHUNK;   // columns per skippable group (even)

// structural pattern of row r from its column->entry-slot map (slot 6 = zero)
__device__ __forceinline__ uint32_t row_pattern(const uint32_t (&map)[3]) {
    uint32_t m = 0;
#pragma unroll
    for (int c = 0; c < NV; c++)
        if (((map[c / 10] >> (3 * (c % 10))) & 7u) != 6u) m |= 1u << c;
    return m;
}

// pivot lane: row elements J.. in the groups lu3s_update uses (a leading odd
// column alone, then chunks of LU3S_CHUNK columns), each group only if it is
// non-zero in some pivot row of the wave
template <int J0>
__device__ __forceinline__ void lu3s_put_row(const cf (&rA)[NV], uint32_t pmw, LUBuf &L) {
    if constexpr (J0 < NV) {
        if constexpr ((J0 & 1) || J0 + 1 >= NV) {
            if (pmw & (1u << J0)) L.row[J0] = rA[J0];
            lu3s_put_row<J0 + 1>(rA, pmw, L);
        } else {
            constexpr int N0 = (NV - J0) < LU3S_CHUNK ? (NV - J0) : LU3S_CHUNK;
            constexpr int N = N0 & ~1;
            constexpr uint32_t CH = ((1u << N) - 1u) << J0;
            if (pmw & CH) {
#pragma unroll
                for (int q = 0; q < N; q += 2) st4(&L.row[J0 + q], rA[J0 + q], rA[J0 + q + 1]);
            }
            lu3s_put_row<J0 + N>(rA, pmw, L);
        }
    }
}

// a_j -= l * u_j on the rows below for the groups that are non-zero somewhere
template <int J0>
__device__ __forceinline__ void lu3s_update(cf (&rA)[NV], const cf &l, bool below, uint32_t pmw, const LUBuf &L) {
    if constexpr (J0 < NV) {
        if constexpr ((J0 & 1) || J0 + 1 >= NV) {
            if (pmw & (1u << J0)) {
                const cf u = L.row[J0];
                if (below) rA[J0] = cmsub(rA[J0], l, u);
            }
            lu3s_update<J0 + 1>(rA, l, below, pmw, L);
        } else {
            constexpr int N0 = (NV - J0) < LU3S_CHUNK ? (NV - J0) : LU3S_CHUNK;
            constexpr int N = N0 & ~1;
            constexpr uint32_t CH = ((1u << N) - 1u) << J0;
            if (pmw & CH) {
                cf u[N];
#pragma unroll
                for (int q = 0; q < N; q += 2) ld4(&L.row[J0 + q], u[q], u[q + 1]);
                if (below) {
#pragma unroll
                    for (int q = 0; q < N; q++) rA[J0 + q] = cmsub(rA[J0 + q], l, u[q]);
                }
            }
            __builtin_amdgcn_sched_barrier(0);
            lu3s_update<J0 + N>(rA, l, below, pmw, L);
        }
    }
}

// reciprocals (o1, o2) of the cuCdivf factors of the pivot a lane owns, kept
// from the forward step that chose it (brs, bis = pivot * o1 are recomputed
// from the pivot element, which stays in the owner's rA)
struct PivF { pf2 oo; };

// s in the fast reciprocal range [2^-90, 2^120), on the bit pattern of a
// non-negative float (NaN and the -1 "no candidate" key fall outside)
__device__ __forceinline__ bool rcp_fast_bits(int bits) {
    return (uint32_t)(bits - 0x12800000) < (uint32_t)(0x7B800000 - 0x12800000);
}

// diagnostic builds (HC_DIAG_LU): shader cycles of the forward step's parts,
// summed into lg[0..3]; lg[7] holds the last timestamp
#ifdef HC_DIAG_LU
#define LU_MARK(k) do { if (lg) { const uint64_t n_ = __builtin_amdgcn_s_memtime(); lg[k] += n_ - lg[7]; lg[7] = n_; } } while (0)
#else
#define LU_MARK(k) do { } while (0)
#endif

template <int I>
__device__ __forceinline__ void lu3s_forward(cf (&rA)[NV], cf &rB, int &rowid, uint32_t &pat, bool all_dense,
                                             int lane, int r, int hb, bool row_lane, PivF &my, LUBuf &L,
                                             uint64_t *lg) {
    if constexpr (I < NV) {
        const float v = __builtin_fabsf(rA[I].x) + __builtin_fabsf(rA[I].y);          // :55
        const bool elig = rowid >= I && row_lane;
        const bool isn = v != v;
        const int key = (elig && !isn) ? __float_as_int(v) : -1;
        const int mx = half_max_int_p16(key);
        const bool cand = key == mx;
        const unsigned long long m = __builtin_amdgcn_ballot_w64(cand);
        const unsigned long long nanm = __builtin_amdgcn_ballot_w64(isn) & __builtin_amdgcn_ballot_w64(rowid == I);
        const unsigned mlo = (unsigned)m, mhi = (unsigned)(m >> 32);
        bool is_piv;
        float piv_abs;
        int pl0, pl1;   // pivot lanes of the two halves
        if (__builtin_expect(nanm != 0ull || __builtin_popcount(mlo) > 1 || __builtin_popcount(mhi) > 1, 0)) {
            const unsigned nlo = (unsigned)nanm, nhi = (unsigned)(nanm >> 32);
            const unsigned mine_m = hb ? mhi : mlo, mine_n = hb ? nhi : nlo;
            const int c2 = ((mine_m >> r) & 1u) ? rowid : (1 << 20);
            const int mn = half_min_i(c2);
            const unsigned long long w = __builtin_amdgcn_ballot_w64(row_lane && rowid == mn);
            const unsigned wm = hb ? (unsigned)(w >> 32) : (unsigned)w;
            const int pl = mine_n ? hb + __builtin_ctz(mine_n) : hb + (wm ? __builtin_ctz(wm) : 0);
            is_piv = lane == pl;
            piv_abs = mine_n ? __builtin_nanf("") : __int_as_float(mx);
            const unsigned long long pm = __builtin_amdgcn_ballot_w64(is_piv);
            pl0 = __builtin_ctz((unsigned)pm | 0x80000000u);
            pl1 = 32 + __builtin_ctz((unsigned)(pm >> 32) | 0x80000000u);
        } else {
            is_piv = cand;
            piv_abs = __int_as_float(mx);
            pl0 = __builtin_ctz(mlo | 0x80000000u);
            pl1 = 32 + __builtin_ctz(mhi | 0x80000000u);
        }
        // structural patterns of the two pivot rows (wave-uniform) and of this half's
        const uint32_t pp0 = (uint32_t)__builtin_amdgcn_readlane((int)pat, pl0);
        const uint32_t pp1 = (uint32_t)__builtin_amdgcn_readlane((int)pat, pl1);
        constexpr uint32_t FULL = 0xFFFFFFFFu << (I + 1);
        // a pivot outside the fast reciprocal range (tiny, zero, NaN) makes the step dense
        const bool dense = all_dense || __builtin_amdgcn_ballot_w64(!rcp_fast_bits(__float_as_int(piv_abs))) != 0ull;
        const uint32_t pmw = dense ? FULL : ((pp0 | pp1) & FULL);
        LU_MARK(0);
        if (is_piv) {                                          // pivot row -> buffer
            L.row[I] = rA[I];
            lu3s_put_row<I + 1>(rA, pmw, L);
            L.row[30] = rB;
            L.row[31].x = __int_as_float(rowid);
        }
        wave_lds_sync();
        const cf sxi = L.row[I];
        cf sB0, pr;
        ld4(&L.row[30], sB0, pr);
        const int piv_pos = __float_as_int(pr.x);
        LU_MARK(1);
        if (is_piv) rowid = I;                                 // :70-82
        else if (rowid == I) rowid = piv_pos;
        // 1 / pivot as cuCdivf(1, pivot) (:84); the pivot lane keeps the factors
        // for its position of the back substitution (same inputs, same ops as
        // recomputing them there from its rA[I], which no later step changes)
        cf reg;
        divf f;
        if (__builtin_expect(!dense, 1)) {
            f = cdiv_factors_fast(sxi, piv_abs);               // piv_abs == |sxi.re| + |sxi.im|, in range
            reg = cmk((f.o1 * f.brs) * f.o2, (-(f.o1 * f.bis)) * f.o2);
        } else {
            f = cdiv_factors(sxi);
            reg = (piv_abs == 0.0f) ? cmk(1.0f, 0.0f) : cdiv_apply(cmk(1.0f, 0.0f), f);   // :66
        }
        if (is_piv) my.oo = pf2{f.o1, f.o2};
        // opaque: the select chain must be resolved here, not carried as 30
        // per-step factor pairs into the back substitution
        asm volatile("" : "+v"(my.oo));
        const bool below = rowid > I;                          // :86-93
        cf l = cmk(0.0f, 0.0f);
        if (below) {
            const pf2 lp = pcmul(pf2{rA[I].x, rA[I].y}, pf2{reg.x, reg.y});
            const pf2 bp = pcmsub(pf2{rB.x, rB.y}, lp, pf2{sB0.x, sB0.y});
            l = cmk(lp.x, lp.y);
            rB = cmk(bp.x, bp.y);
        }
        // fill-in: a row below whose column I may be non-zero takes the pivot
        // patterns (both halves': a superset of its own pivot row's, one VALU op);
        // after a dense step (l may be non-finite) nothing is known zero
        if (below && (dense || ((pat >> I) & 1u))) pat |= dense ? 0xFFFFFFFFu : pmw;
        LU_MARK(2);
        lu3s_update<I + 1>(rA, l, below, pmw, L);
        LU_MARK(3);
        lu3s_forward<I + 1>(rA, rB, rowid, pat, all_dense, lane, r, hb, row_lane, my, L, lg);
    }
}

// cdiv_apply(b, f) = cuCdivf(b, pivot) in packed FP32, op for op:
// (brs, bis) = pivot*o1; (ars, ais) = b*o1; re = (ars*brs + ais*bis)*o2; im = (ais*brs - ars*bis)*o2
__device__ __forceinline__ pf2 pcdiv_apply(pf2 b, pf2 piv, const PivF &f) {
    pf2 bb, a, t1, t2, s, q;
    asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[1,0]" : "=v"(bb) : "v"(piv), "v"(f.oo));
    asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[1,0]" : "=v"(a) : "v"(b), "v"(f.oo));
    asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[1,0]" : "=v"(t1) : "v"(a), "v"(bb));
    asm("v_pk_mul_f32 %0, %1, %2 op_sel:[1,1] op_sel_hi:[0,1]" : "=v"(t2) : "v"(a), "v"(bb));
    asm("v_pk_add_f32 %0, %1, %2 neg_hi:[0,1]" : "=v"(s) : "v"(t1), "v"(t2));
    asm("v_pk_mul_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,1]" : "=v"(q) : "v"(s), "v"(f.oo));
    return q;
}

// back substitution (:97-106): the lane with final rowid == I owns position I
// and divides its right-hand side by its pivot with the factors kept in the
// forward pass; x_I is published through the buffer
template <int I>
__device__ __forceinline__ void lu3s_backward(const cf (&rA)[NV], cf &rB, int rowid, const PivF &my, LUBuf &L) {
    if constexpr (I >= 0) {
        if (rowid == I) {
            const pf2 q = pcdiv_apply(pf2{rB.x, rB.y}, pf2{rA[I].x, rA[I].y}, my);
            L.row[I] = cmk(q.x, q.y);
        }
        wave_lds_sync();
        const cf xi = L.row[I];
        if (rowid < I) {
            const pf2 v = pcmsub(pf2{rB.x, rB.y}, pf2{xi.x, xi.y}, pf2{rA[I].x, rA[I].y});
            rB = cmk(v.x, v.y);
        }
        lu3s_backward<I - 1>(rA, rB, rowid, my, L);
    }
}

__device__ __forceinline__ cf lu_solve3s(cf (&rA)[NV], cf rB, int lane, uint32_t pattern, LUBuf &L,
                                        uint64_t *t_mid = nullptr, uint64_t *lg = nullptr) {
    // every entry finite and below 2^88 in magnitude (NaN fails the compare)
    bool ok = true;
#pragma unroll
    for (int c = 0; c < NV; c++)
        ok = ok && __builtin_fabsf(rA[c].x) < 0x1p88f && __builtin_fabsf(rA[c].y) < 0x1p88f;
    const bool all_dense = __builtin_amdgcn_ballot_w64(!ok) != 0ull;   // then every step is dense
    const int r = lane & 31, hb = lane & 32;
    const bool row_lane = r < NV;
    int rowid = row_lane ? r : 99;   // padding lanes never pivot
    uint32_t pat = row_lane ? pattern : 0u;
    PivF my{pf2{0.0f, 0.0f}};
#ifdef HC_DIAG_LU
    if (lg) lg[7] = __builtin_amdgcn_s_memtime();
#endif
    lu3s_forward<0>(rA, rB, rowid, pat, all_dense, lane, r, hb, row_lane, my, L, lg);
    if (t_mid) *t_mid = __builtin_amdgcn_s_memtime();   // diagnostic builds only
    lu3s_backward<NV - 1>(rA, rB, rowid, my, L);
    wave_lds_sync();
    return L.row[row_lane ? r : 0];
}

}  // namespace hc
