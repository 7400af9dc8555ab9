// hc_lu3.hpp -- v3 LU of the two-paths-per-wave tracker.
//
// Same semantics as lu_solve() / lu_solve2() (dev-cgesv-batched-small.cuh:38-107:
// partial pivot on |re|+|im|, first-max ties, rowid relabelling, zero pivot ->
// recip 1, cuCdivf back substitution), restructured for the CDNA4 issue limits
// measured on v2 (profiles/r1_v2_pmc_summary.json: VALU issue ~70 % busy, LDS
// issue stalls 23 % of wave time):
//
//  * pivot-row broadcast through LDS: the pivot lane of each half writes its
//    row (+ rhs + rowid) into a per-half buffer with ds_write_b128 and every
//    lane reads it back with broadcast ds_read_b128 -- K/2 + K/2 LDS
//    instructions per step instead of 2K ds_bpermute;
//  * the lane with final rowid i owns position i and still holds pivot i in
//    rA[i]: the back substitution recomputes its cuCdivf factors there (no
//    factor storage, no permutation array);
//  * the half-wave max of the pivot search ends with v_permlane16_swap (VALU)
//    instead of an LDS swizzle;
//  * 1/s and 1/s2 use v_rcp_f32 + one Newton step when s is in [2^-90, 2^120)
//    (exhaustively verified correctly rounded there), the IEEE '/' otherwise;
//  * cuCdivf(1, y) is evaluated as ((o1*brs)*o2, -(o1*bis)*o2), which equals
//    the literal formula except for the sign of exact zeros.
//
// The buffer aliases the per-path dH/dx entry block (SlotLDS::ent), which is
// dead between the gather of the Jacobian into registers and the next eval.
#pragma once

#include "hc_eval3.hpp"

namespace hc {

typedef float f4v __attribute__((ext_vector_type(4)));
typedef float f2v __attribute__((ext_vector_type(2)));

struct alignas(16) LUBuf {
    cf row[32];    // current pivot row: [0..29] A, [30] rhs, [31].x = rowid (int bits); reused for x in the back sub
};
static_assert(sizeof(divf) == 16, "divf layout");
static_assert(sizeof(LUBuf) <= sizeof(cf) * NV * 7, "LUBuf must fit in SlotLDS::ent");
static_assert(offsetof(SlotLDS, ent) % 16 == 0, "SlotLDS::ent must be 16-B aligned");

constexpr int LU3_CHUNK = 6;   // update columns per LDS batch (even)

// Correctly rounded 1/s for s in [2^-90, 2^120): v_rcp_f32 plus one Newton
// step.  Verified bit-identical to the IEEE division (hipcc's div_scale /
// div_fmas / div_fixup sequence) for every float in that range -- all 2^23
// significands x 210 binades, scripts/rcp_check.hip, profiles/r1_rcp_check.json.
__device__ __forceinline__ float rcp_rn(float s) {
    const float r0 = __builtin_amdgcn_rcpf(s);
    const float e0 = __builtin_fmaf(-s, r0, 1.0f);
    return __builtin_fmaf(e0, r0, r0);
}
__device__ __forceinline__ bool rcp_fast_ok(float s) { return s >= 0x1p-90f && s < 0x1p+120f; }
// cuCdivf factors of y with s = |y.re| + |y.im| in the fast range (== cdiv_factors(y))
__device__ __forceinline__ divf cdiv_factors_fast(cf y, float s) {
    divf f;
    f.o1 = rcp_rn(s);
    f.brs = y.x * f.o1;
    f.bis = y.y * f.o1;
    f.o2 = rcp_rn((f.brs * f.brs) + (f.bis * f.bis));   // argument in [0.5, 1]
    return f;
}

__device__ __forceinline__ void st4(cf *p, cf a, cf b) {
    f4v v = {a.x, a.y, b.x, b.y};
    *reinterpret_cast<f4v *>(p) = v;
}
__device__ __forceinline__ void ld4(const cf *p, cf &a, cf &b) {
    const f4v v = *reinterpret_cast<const f4v *>(p);
    a = cmk(v.x, v.y);
    b = cmk(v.z, v.w);
}

// max over each 32-lane half: DPP inside 16-lane rows, then v_permlane16_swap
// across the row pair (VALU; no LDS round trip unlike ds_swizzle)
__device__ __forceinline__ int half_max_int_p16(int v) {
    v = max(v, dpp_i<DPP_QP_1032>(v));
    v = max(v, dpp_i<DPP_QP_2301>(v));
    v = max(v, dpp_i<DPP_ROW_HALF_MIRROR>(v));
    v = max(v, dpp_i<DPP_ROW_MIRROR>(v));
    const auto sw = __builtin_amdgcn_permlane16_swap((unsigned)v, (unsigned)v, false, false);
    return max((int)sw[0], (int)sw[1]);
}

// pivot lane: row elements J.. of the register row into the buffer
template <int J>
__device__ __forceinline__ void lu3_put_row(const cf (&rA)[NV], LUBuf &L) {
    if constexpr (J < NV) {
        if constexpr (J & 1) {
            L.row[J] = rA[J];
            lu3_put_row<J + 1>(rA, L);
        } else {
            st4(&L.row[J], rA[J], rA[J + 1]);
            lu3_put_row<J + 2>(rA, L);
        }
    }
}

// a_j -= l * u_j for j in [J0, JE), u from the broadcast buffer
template <int J0, int JE = NV>
__device__ __forceinline__ void lu3_update(cf (&rA)[NV], const cf &l, bool below, const LUBuf &L) {
    if constexpr (J0 < JE) {
        if constexpr ((J0 & 1) || J0 + 1 >= JE) {
            const cf u = L.row[J0];
            if (below) rA[J0] = cmsub(rA[J0], l, u);
            lu3_update<J0 + 1, JE>(rA, l, below, L);
        } else {
            constexpr int N0 = (JE - J0) < LU3_CHUNK ? (JE - J0) : LU3_CHUNK;
            constexpr int N = N0 & ~1;
            cf u[N];
#pragma unroll
            for (int q = 0; q < N; q += 2) ld4(&L.row[J0 + q], u[q], u[q + 1]);
            if (below) {
#pragma unroll
                for (int q = 0; q < N; q++) rA[J0 + q] = cmsub(rA[J0 + q], l, u[q]);
            }
            __builtin_amdgcn_sched_barrier(0);
            lu3_update<J0 + N, JE>(rA, l, below, L);
        }
    }
}

template <int I>
__device__ __forceinline__ void lu3_forward(cf (&rA)[NV], cf &rB, int &rowid, int lane, int r, int hb,
                                            bool row_lane, LUBuf &L) {
    if constexpr (I < NV) {
        const float v = __builtin_fabsf(rA[I].x) + __builtin_fabsf(rA[I].y);          // :55
        const bool elig = rowid >= I && row_lane;
        const bool isn = v != v;
        const int key = (elig && !isn) ? __float_as_int(v) : -1;   // |.|+|.| >= +0: bits order like ints
        const int mx = half_max_int_p16(key);
        // key == mx alone marks the candidates: mx >= 0 unless every eligible entry is
        // NaN, and then position I is NaN too (rare path).  Single compares ballot
        // straight into SGPRs (an && chain would be materialised first).
        const bool cand = key == mx;
        const unsigned long long m = __builtin_amdgcn_ballot_w64(cand);
        const unsigned long long nanm = __builtin_amdgcn_ballot_w64(isn) & __builtin_amdgcn_ballot_w64(rowid == I);
        const unsigned mlo = (unsigned)m, mhi = (unsigned)(m >> 32);
        bool is_piv;      // this lane holds the pivot row of its half
        float piv_abs;
        if (__builtin_expect(nanm != 0ull || __builtin_popcount(mlo) > 1 || __builtin_popcount(mhi) > 1, 0)) {
            // rare: NaN at position I wins (:57-64); exact ties: first position wins
            const unsigned nlo = (unsigned)nanm, nhi = (unsigned)(nanm >> 32);
            const unsigned mine_m = hb ? mhi : mlo, mine_n = hb ? nhi : nlo;
            const int c2 = ((mine_m >> r) & 1u) ? rowid : (1 << 20);
            const int mn = half_min_i(c2);
            const unsigned long long w = __builtin_amdgcn_ballot_w64(row_lane && rowid == mn);
            const unsigned wm = hb ? (unsigned)(w >> 32) : (unsigned)w;
            const int pl = mine_n ? hb + __builtin_ctz(mine_n) : hb + (wm ? __builtin_ctz(wm) : 0);
            is_piv = lane == pl;
            piv_abs = mine_n ? __builtin_nanf("") : __int_as_float(mx);
        } else {
            is_piv = cand;   // exactly one candidate per half
            piv_abs = __int_as_float(mx);
        }
        if (is_piv) {                                          // pivot row -> buffer
            lu3_put_row<I>(rA, L);
            L.row[30] = rB;
            L.row[31].x = __int_as_float(rowid);
        }
        wave_lds_sync();                                       // cross-lane: pivot lane -> all lanes
        const cf sxi = L.row[I];
        cf sB0, pr;
        ld4(&L.row[30], sB0, pr);
        const int piv_pos = __float_as_int(pr.x);
        if (is_piv) rowid = I;                                 // :70-82
        else if (rowid == I) rowid = piv_pos;
        // 1 / pivot as cuCdivf(1, pivot) (:84); the back substitution recomputes the
        // same factors from the pivot element its owner lane still holds
        cf reg;
        const float s = __builtin_fabsf(sxi.x) + __builtin_fabsf(sxi.y);   // == piv_abs
        if (__builtin_expect(__builtin_amdgcn_ballot_w64(!rcp_fast_ok(s)) == 0ull, 1)) {
            const divf f = cdiv_factors_fast(sxi, s);          // s in [2^-90, 2^120): non-zero, finite
            reg = cmk((f.o1 * f.brs) * f.o2, (-(f.o1 * f.bis)) * f.o2);
        } else {
            const divf f = cdiv_factors(sxi);
            reg = (piv_abs == 0.0f) ? cmk(1.0f, 0.0f) : cdiv_apply(cmk(1.0f, 0.0f), f);   // :66
        }
        const bool below = rowid > I;                          // :86-93
        cf l = cmk(0.0f, 0.0f);
        if (below) {
            const pf2 lp = pcmul(pf2{rA[I].x, rA[I].y}, pf2{reg.x, reg.y});
            const pf2 bp = pcmsub(pf2{rB.x, rB.y}, lp, pf2{sB0.x, sB0.y});
            l = cmk(lp.x, lp.y);
            rA[I] = l;
            rB = cmk(bp.x, bp.y);
        }
        lu3_update<I + 1>(rA, l, below, L);
        lu3_forward<I + 1>(rA, rB, rowid, lane, r, hb, row_lane, L);
    }
}

// back substitution (:97-106): the lane with final rowid == I owns position I;
// its rA[I] is still the pivot element of step I, so it recomputes that pivot's
// cuCdivf factors (same inputs, same ops as the forward step), computes x_I and
// publishes it in row[I]
template <int I>
__device__ __forceinline__ void lu3_backward(const cf (&rA)[NV], cf &rB, int rowid, LUBuf &L) {
    if constexpr (I >= 0) {
        const cf piv = rA[I];
        const float s = __builtin_fabsf(piv.x) + __builtin_fabsf(piv.y);
        const bool own = rowid == I;
        divf f;
        if (__builtin_expect((__builtin_amdgcn_ballot_w64(!rcp_fast_ok(s)) & __builtin_amdgcn_ballot_w64(own)) == 0ull, 1))
            f = cdiv_factors_fast(piv, s);
        else
            f = cdiv_factors(piv);
        const cf cand = cdiv_apply(rB, f);
        if (own) L.row[I] = cand;
        wave_lds_sync();
        const cf xi = L.row[I];
        if (rowid < I) rB = cmsub(rB, xi, rA[I]);
        lu3_backward<I - 1>(rA, rB, rowid, L);
    }
}

// Solves the system of each half; L is this half's buffer (16-B aligned).
__device__ __forceinline__ cf lu_solve3(cf (&rA)[NV], cf rB, int lane, LUBuf &L) {
    const int r = lane & 31, hb = lane & 32;
    const bool row_lane = r < NV;
    int rowid = row_lane ? r : 99;   // padding lanes never pivot
    lu3_forward<0>(rA, rB, rowid, lane, r, hb, row_lane, L);
    lu3_backward<NV - 1>(rA, rB, rowid, L);
    wave_lds_sync();
    return L.row[row_lane ? r : 0];
}

}  // namespace hc
