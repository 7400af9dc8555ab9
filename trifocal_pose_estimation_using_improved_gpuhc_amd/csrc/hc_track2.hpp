// hc_track2.hpp -- v2 tracker: two homotopy paths per wavefront.
//
// The 64 lanes of a wave are two independent "path slots" (half-waves): lane
// l belongs to slot h = l >> 5 and owns equation row r = l & 31 (r < 30) of
// that slot's path.  Both slots execute the same instruction stream -- one
// predictor / corrector stage per iteration: p(t) + dH/dx + dH/dt|H + LU --
// while each slot runs its own stage machine (its own t, step size, stage,
// path id).  Everything uniform per path lives in VGPRs (uniform per half).
//
//  * LU: lane-per-row partial-pivot elimination as in v1, but the per-pivot
//    work (pivot search, cuCdivf factors, relabel, bookkeeping) is shared by
//    the two paths; the pivot row is broadcast inside each half with
//    ds_bpermute, static-lane broadcasts use ds_swizzle (and=0, or=lane).
//  * dH/dx: per-lane term lists (row r walks only its own 11..23 non-padding
//    terms), finished entries go to a per-path compact LDS block (7 slots per
//    row, slot 6 = 0) and are gathered back into the register row through a
//    per-lane column->slot map kept in 3 VGPRs.
//  * dH/dt and H: per-lane 16-slot lists as in v1.
//
// Arithmetic is identical, op for op, to v1 / the oracle.
#pragma once

#include "hc_device.hpp"

namespace hc {

constexpr int HX2_SLOT_CAP = 48;   // per-lane dH/dx term list length (this problem: 23)

// v2 tables, built by the prep kernel next to the v1 tables
struct TableWS2 {
    int hx_len;                    // max terms per row (uniform loop count)
    int status;
    int pad[2];
    uint32_t map[3][32];           // per row: 10 columns x 3-bit slot code per word (6 = structural zero)
    uint32_t hx[HX2_SLOT_CAP * 32];
    // word: coef(4, signed) | a<<4 (6) | b<<10 (6) | u<<16 (5) | v<<21 (5) | slot<<26 (3) | last<<29 (1)
};

// uniform state of a path slot, parked in LDS while a stage runs
struct SlotState {
    float t0, t_step, dt, h2, scale;
    int s, stepidx, coef, succ, nsteps, ncorr, b, smp, ph, flags;
    int pad;
};
// per path-slot LDS block
struct alignas(16) SlotLDS {
    cf x[32];        // current track (x[30] = 1)
    cf xl[32];       // last successful track
    cf sols[32];     // RK accumulator
    cf p[NPP];       // p(t)
    cf tgt[NPP];     // target params
    cf dif[NPP];     // diff params
    cf ent[NV * 7];  // dH/dx entries of row r at [r*7 + slot], slot 6 = 0
    SlotState st;
    char bank_pad[16];   // slot stride = 16 mod 256 B: the slots of one wave (same offsets,
                         // different bases) land on different LDS banks
};
static_assert(sizeof(SlotLDS) % 256 == 16, "SlotLDS stride must shift the LDS banks by 4 per slot");

__device__ __forceinline__ float bperm_f(float v, int src_lane) {
    return __int_as_float(__builtin_amdgcn_ds_bpermute(src_lane << 2, __float_as_int(v)));
}
__device__ __forceinline__ int bperm_i(int v, int src_lane) { return __builtin_amdgcn_ds_bpermute(src_lane << 2, v); }
// broadcast relative lane L (compile-time) of each 32-lane half to the whole half
template <int L>
__device__ __forceinline__ int hbcast_i(int v) { return __builtin_amdgcn_ds_swizzle(v, (L & 31) << 5); }
template <int L>
__device__ __forceinline__ float hbcast_f(float v) { return __int_as_float(hbcast_i<L>(__float_as_int(v))); }
__device__ __forceinline__ int half_max_int(int v) {
    v = max(v, dpp_i<DPP_QP_1032>(v));
    v = max(v, dpp_i<DPP_QP_2301>(v));
    v = max(v, dpp_i<DPP_ROW_HALF_MIRROR>(v));
    v = max(v, dpp_i<DPP_ROW_MIRROR>(v));
    v = max(v, swz_xor16_i(v));
    return v;
}
// per-half version of the reference's shfl_down tree (lanes r >= 30 hold 0):
// the value of relative lane 0 of each half, broadcast to the half
__device__ __forceinline__ float tree_sum_half(float v) {
    float a = v + swz_xor16_f(v);
    float b = a + dpp_f<DPP_ROW_SHL8>(a);
    float c = b + dpp_f<DPP_ROW_SHL4>(b);
    float d = c + dpp_f<DPP_ROW_SHL2>(c);
    float e = d + dpp_f<DPP_ROW_SHL1>(d);
    return hbcast_f<0>(e);
}

// ---------------------------------------------------------------- LU (2 systems / wave)
// Same semantics as lu_solve() (dev-cgesv-batched-small.cuh:38-107) for the
// system of each half.  r = lane & 31, hb = lane & 32.  Written with template
// recursion so every register index is a compile-time constant.
struct LU2State {
    int rowid, perm;
    float fo1, fbr, fbi, fo2;
};
constexpr int LU_CHUNK = 6;

// a_j -= l * u_j for j in [J0, NV): u_j fetched from the pivot lane in chunks of
// LU_CHUNK (ds_bpermute needs every lane active, the update is exec-masked)
template <int J0>
__device__ __forceinline__ void lu2_update(cf (&rA)[NV], const cf &l, bool below, int pl) {
    if constexpr (J0 < NV) {
        constexpr int N = (NV - J0) < LU_CHUNK ? (NV - J0) : LU_CHUNK;
        cf u[N];
#pragma unroll
        for (int q = 0; q < N; q++) u[q] = cmk(bperm_f(rA[J0 + q].x, pl), bperm_f(rA[J0 + q].y, pl));
        if (below) {
#pragma unroll
            for (int q = 0; q < N; q++) rA[J0 + q] = cmsub(rA[J0 + q], l, u[q]);
        }
        __builtin_amdgcn_sched_barrier(0);
        lu2_update<J0 + N>(rA, l, below, pl);
    }
}

template <int I>
__device__ __forceinline__ void lu2_forward(cf (&rA)[NV], cf &rB, LU2State &st, int lane, int r, int hb,
                                            bool row_lane) {
    if constexpr (I < NV) {
        const float v = __builtin_fabsf(rA[I].x) + __builtin_fabsf(rA[I].y);          // :55
        const bool elig = st.rowid >= I && row_lane;
        const bool isn = v != v;
        const int key = (elig && !isn) ? __float_as_int(v) : -1;   // |.|+|.| >= +0: bits order like ints
        const int mx = half_max_int(key);
        const unsigned long long m = __ballot(elig && key == mx);
        const unsigned long long nanm = __ballot(elig && isn && st.rowid == I);
        const unsigned mlo = (unsigned)m & 0x3FFFFFFFu, mhi = (unsigned)(m >> 32) & 0x3FFFFFFFu;
        int pl;   // absolute pivot lane of this lane's half
        float piv_abs;
        if (__builtin_expect(nanm != 0ull || __builtin_popcount(mlo) > 1 || __builtin_popcount(mhi) > 1, 0)) {
            // rare: NaN at position I wins (:57-64); exact ties: first position wins
            const unsigned nlo = (unsigned)nanm, nhi = (unsigned)(nanm >> 32);
            const unsigned mine_m = hb ? mhi : mlo, mine_n = hb ? nhi : nlo;
            const int cand = ((mine_m >> r) & 1u) ? st.rowid : (1 << 20);
            const int mn = half_min_i(cand);
            const unsigned long long w = __ballot(row_lane && st.rowid == mn);
            const unsigned wm = hb ? (unsigned)(w >> 32) : (unsigned)w;
            pl = mine_n ? hb + __builtin_ctz(mine_n) : hb + (wm ? __builtin_ctz(wm) : 0);
            piv_abs = mine_n ? __builtin_nanf("") : __int_as_float(mx);
        } else {
            pl = hb ? (32 + (mhi ? __builtin_ctz(mhi) : 0)) : (mlo ? __builtin_ctz(mlo) : 0);
            piv_abs = __int_as_float(mx);
        }
        const int piv_pos = bperm_i(st.rowid, pl);
        const int qlane = bperm_i(st.perm, hb + I);            // lane at position I of this half
        const bool zero = (piv_abs == 0.0f);                   // :66
        const cf sxi = cmk(bperm_f(rA[I].x, pl), bperm_f(rA[I].y, pl));
        const cf sB0 = cmk(bperm_f(rB.x, pl), bperm_f(rB.y, pl));
        if (lane == pl) st.rowid = I;                          // :70-82
        else if (st.rowid == I) st.rowid = piv_pos;
        st.perm = (r == I) ? pl : st.perm;
        st.perm = (r == piv_pos) ? qlane : st.perm;
        const divf f = cdiv_factors(sxi);                      // :84, parked for the back substitution
        st.fo1 = (r == I) ? f.o1 : st.fo1;
        st.fbr = (r == I) ? f.brs : st.fbr;
        st.fbi = (r == I) ? f.bis : st.fbi;
        st.fo2 = (r == I) ? f.o2 : st.fo2;
        asm volatile("" : "+v"(st.rowid), "+v"(st.perm), "+v"(st.fo1), "+v"(st.fbr), "+v"(st.fbi), "+v"(st.fo2));
        const cf reg = zero ? cmk(1.0f, 0.0f) : cdiv_apply(cmk(1.0f, 0.0f), f);
        const bool below = st.rowid > I;                       // :86-93
        cf l = cmk(0.0f, 0.0f);
        if (below) {
            l = cmul(rA[I], reg);
            rA[I] = l;
            rB = cmsub(rB, l, sB0);
        }
        lu2_update<I + 1>(rA, l, below, pl);
        lu2_forward<I + 1>(rA, rB, st, lane, r, hb, row_lane);
    }
}

template <int I>
__device__ __forceinline__ void lu2_backward(cf (&rA)[NV], cf &rB, const LU2State &st, cf &xs, int r, int hb) {
    if constexpr (I >= 0) {                                    // :97-106
        const int li = bperm_i(st.perm, hb + I);
        const cf bi = cmk(bperm_f(rB.x, li), bperm_f(rB.y, li));
        divf f;
        f.o1 = bperm_f(st.fo1, hb + I);
        f.brs = bperm_f(st.fbr, hb + I);
        f.bis = bperm_f(st.fbi, hb + I);
        f.o2 = bperm_f(st.fo2, hb + I);
        const cf xi = cdiv_apply(bi, f);
        if (st.rowid < I) rB = cmsub(rB, xi, rA[I]);
        xs.x = (r == I) ? xi.x : xs.x;
        xs.y = (r == I) ? xi.y : xs.y;
        lu2_backward<I - 1>(rA, rB, st, xs, r, hb);
    }
}

__device__ __forceinline__ cf lu_solve2(cf (&rA)[NV], cf rB, int lane) {
    const int r = lane & 31, hb = lane & 32;
    const bool row_lane = r < NV;
    LU2State st;
    st.rowid = row_lane ? r : 99;   // padding lanes never pivot
    st.perm = lane;                 // lane hb+p: absolute lane holding position p
    st.fo1 = st.fbr = st.fbi = st.fo2 = 0.0f;
    lu2_forward<0>(rA, rB, st, lane, r, hb, row_lane);
    asm volatile("" : "+v"(st.perm), "+v"(st.fo1), "+v"(st.fbr), "+v"(st.fbi), "+v"(st.fo2));
    cf xs = cmk(0.0f, 0.0f);
    lu2_backward<NV - 1>(rA, rB, st, xs, r, hb);
    return xs;
}

// ---------------------------------------------------------------- evals (per half)
// dH/dx (gpu-idx-evals/..._LimUnroll_L2Cache.cuh:57-88) via per-lane term lists
__device__ __forceinline__ void eval_hx2(cf (&rA)[NV], const uint32_t *s_hx2, int hx_len, const uint32_t (&map)[3],
                                         SlotLDS &S, int r) {
    cf acc = cmk(0.0f, 0.0f);
    cf *ent_row = S.ent + (r < NV ? r : 0) * 7;
    if (r < NV) ent_row[6] = cmk(0.0f, 0.0f);   // structural zero (the v3 LU reuses this block)
    for (int k = 0; k < hx_len; k++) {
        const uint32_t w = s_hx2[k * 32 + r];
        const int co = sext4(w);
        const cf pa = S.p[(w >> 4) & 63], pb = S.p[(w >> 10) & 63];
        const cf xu = S.x[(w >> 16) & 31], xv = S.x[(w >> 21) & 31];
        const cf P = cmul(cmul(cscale(pa, (float)co), pb), xu);
        const cf nv = cmadd(acc, P, xv);
        acc.x = co ? nv.x : acc.x;
        acc.y = co ? nv.y : acc.y;
        if ((w >> 29) & 1u) {           // last term of an entry (never set on padding words)
            ent_row[(w >> 26) & 7] = acc;
            acc = cmk(0.0f, 0.0f);
        }
    }
    wave_lds_sync();
#pragma unroll
    for (int c = 0; c < NV; c++) {
        const uint32_t code = (map[c / 10] >> (3 * (c % 10))) & 7u;
        rA[c] = ent_row[code];
    }
}
__device__ __forceinline__ cf eval_ht2(const uint32_t *s_ht, const SlotLDS &S, int r) {
    return eval_ht(s_ht, S.x, S.p, S.dif, r);
}
__device__ __forceinline__ cf eval_h2(const uint32_t *s_ht, const SlotLDS &S, int r) {
    return eval_h(s_ht, S.x, S.p, r);
}

}  // namespace hc
