// hc_lu9.hpp -- latency-oriented restructuring of the v8 LU (hc_lu3s.hpp).
//
// Same arithmetic, op for op, as lu_solve3s (and so as lu_solve3 / the
// reference's dev-cgesv-batched-small.cuh:38-107 up to the sign of exact
// zeros).  What changes is how long one wave waits: the lane
// counters (profiles/r1*_phases.json) show a lone wave parked on s_waitcnt for
// ~46 % of its time, most of it on the LDS round trips of the LU.  Feature bits
// of F (each bit-identical on its own; scripts/lu_lab.hip measures them):
//
//  LU9_SPEC  every lane computes cuCdivf(1, rA[I]) for its own candidate while
//            the pivot is being searched; the pivot lane publishes 1/pivot in
//            place of the pivot, so the reciprocal chain leaves the critical
//            path after the broadcast;
//  LU9_NOMASK steps that run sparse (every entry finite) update
//            every lane without an exec mask: rows not below the pivot take
//            l = 0, and a - 0*u == a for finite u up to the sign of an exact
//            zero;
//  LU9_PF    the update reads the next column chunk of the pivot row before
//            it applies the current one (two chunk buffers in flight);
//  LU9_BRL   the back substitution broadcasts x_I with v_readlane from its
//            owner lane (one per half) instead of an LDS round trip.
#pragma once

#include "hc_lu3s.hpp"

namespace hc {

enum : int { LU9_SPEC = 1, LU9_NOMASK = 2, LU9_PF = 4, LU9_BRL = 8, LU9_LEAN = 16, LU9_BOUT = 32, LU9_ONEB = 1024, LU9_RCPA = 2048, LU9_BSPLIT = 4096, LU9_EARLY = 8192,
             // timing-only ablations for scripts/lu_lab.hip (results wrong)
             LU9_X_NOUPD = 64, LU9_X_NOBACK = 128, LU9_X_NOSEARCH = 256, LU9_X_NOBCAST = 512 };
// the tracker's configuration (scripts/lu_lab.hip: fastest bit-identical combination)
#ifndef HC_LU9_EXTRA
#define HC_LU9_EXTRA 0
#endif
#ifndef HC_LU9_DROP
#define HC_LU9_DROP 0
#endif
constexpr int LU9_PROD = ((LU9_BRL | LU9_LEAN | LU9_ONEB | LU9_RCPA) & ~HC_LU9_DROP) | HC_LU9_EXTRA;


// cuCdivf(1, y) for s = |y.re| + |y.im| in the fast range, in packed FP32 with
// the spec's ops (cdiv_factors_fast + the quotient of DESIGN.md §4):
// o1 = 1/s, (brs, bis) = y*o1, o2 = 1/(brs*brs + bis*bis),
// 1/y = ((o1*brs)*o2, (-(o1*bis))*o2); -(o1*bis) is computed as o1*(-bis)
// (IEEE: the same value).  oo returns (o1, o2).
__device__ __forceinline__ pf2 recip_fast(pf2 y, float s, pf2 &oo) {
    oo.x = rcp_rn(s);
    pf2 bb, sq, q, r;
    asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[1,0]" : "=v"(bb) : "v"(y), "v"(oo));
    asm("v_pk_mul_f32 %0, %1, %1" : "=v"(sq) : "v"(bb));
    oo.y = rcp_rn(sq.x + sq.y);
    asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1] neg_hi:[0,1]" : "=v"(q) : "v"(oo), "v"(bb));
    asm("v_pk_mul_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,1]" : "=v"(r) : "v"(q), "v"(oo));
    return r;
}

// column chunks of the update of step I: a leading single column when I+1 is
// odd, then groups of CH (even) columns
template <int CH>
struct Lu9Chunks {
    static constexpr int single(int I) { return ((I + 1) & 1) && (I + 1 < NV) ? 1 : 0; }
    static constexpr int start(int I, int k) { return k < single(I) ? I + 1 : I + 1 + single(I) + (k - single(I)) * CH; }
    static constexpr int len(int I, int k) {
        return k < single(I) ? 1 : ((NV - start(I, k)) < CH ? (NV - start(I, k)) : CH);
    }
    static constexpr int count(int I) { return single(I) + (NV - (I + 1 + single(I)) + CH - 1) / CH; }
    static constexpr uint32_t mask(int I, int k) { return ((1u << len(I, k)) - 1u) << start(I, k); }
};

template <int CH>
struct Lu9Buf { cf u[2][CH]; };

template <int CH, int I, int K>
__device__ __forceinline__ void lu9_load(Lu9Buf<CH> &B, const LUBuf &L) {
    using C = Lu9Chunks<CH>;
    constexpr int J = C::start(I, K), N = C::len(I, K);
    if constexpr (N == 1) {
        B.u[K & 1][0] = L.row[J];
    } else {
#pragma unroll
        for (int q = 0; q < N; q += 2) ld4(&L.row[J + q], B.u[K & 1][q], B.u[K & 1][q + 1]);
    }
}
template <int CH, int I, int K>
__device__ __forceinline__ void lu9_fma(cf (&rA)[NV], const cf &l, const Lu9Buf<CH> &B) {
    using C = Lu9Chunks<CH>;
    constexpr int J = C::start(I, K), N = C::len(I, K);
#pragma unroll
    for (int q = 0; q < N; q++) {
        const pf2 v = pcmsub(pf2{rA[J + q].x, rA[J + q].y}, pf2{l.x, l.y}, pf2{B.u[K & 1][q].x, B.u[K & 1][q].y});
        rA[J + q] = cmk(v.x, v.y);
    }
}

// chunks K.. of step I; MASK: exec-mask the FMAs to the rows below
template <int F, int CH, int I, int K, bool MASK>
__device__ __forceinline__ void lu9_update(cf (&rA)[NV], const cf &l, bool below, uint32_t pmw, const LUBuf &L,
                                           Lu9Buf<CH> &B) {
    using C = Lu9Chunks<CH>;
    if constexpr (K < C::count(I)) {
        if constexpr (F & LU9_PF) {
            // chunk K was loaded by the caller / previous chunk; read K+1 now
            if constexpr (K + 1 < C::count(I)) {
                if (pmw & C::mask(I, K + 1)) lu9_load<CH, I, K + 1>(B, L);
            }
        } else if constexpr (!((F & LU9_EARLY) && K == 0)) {
            if (pmw & C::mask(I, K)) lu9_load<CH, I, K>(B, L);
        }
        if (pmw & C::mask(I, K)) {
            if constexpr (MASK) {
                if (below) lu9_fma<CH, I, K>(rA, l, B);
            } else {
                lu9_fma<CH, I, K>(rA, l, B);
            }
        }
        if constexpr (!(F & LU9_PF)) __builtin_amdgcn_sched_barrier(0);
        lu9_update<F, CH, I, K + 1, MASK>(rA, l, below, pmw, L, B);
    }
}

template <int F, int CH, int I>
__device__ __forceinline__ void lu9_forward(cf (&rA)[NV], cf &rB, int &rowid, uint32_t &pat, bool all_dense,
                                            int lane, int r, int hb, bool row_lane, PivF &my, LUBuf &L) {
    if constexpr (I < NV) {
        const float v = __builtin_fabsf(rA[I].x) + __builtin_fabsf(rA[I].y);          // :55
        const bool elig = rowid >= I && row_lane;
        bool is_piv;
        float piv_abs;
        int pl0, pl1;   // pivot lanes of the two halves
        bool dense;
        divf f;
        cf rg;
        if constexpr (F & LU9_LEAN) {
            // NaN keys take part (positive NaN bits order above every finite
            // value): a maximum outside the fast reciprocal range (NaN, inf,
            // zero, tiny, huge) or a tie sends the step to the exact rare path
            const int key = elig ? __float_as_int(v) : -1;
            const int mx = half_max_int_p16(key);
            if constexpr (F & LU9_SPEC) {
                f = cdiv_factors_fast(rA[I], v);
                rg = cmk((f.o1 * f.brs) * f.o2, (-(f.o1 * f.bis)) * f.o2);
            }
            const unsigned long long m = __builtin_amdgcn_ballot_w64(key == mx);
            const unsigned long long bad = __builtin_amdgcn_ballot_w64(!rcp_fast_bits(mx));
            const unsigned mlo = (unsigned)m, mhi = (unsigned)(m >> 32);
            if (__builtin_expect(((mlo & (mlo - 1u)) | (mhi & (mhi - 1u))) != 0u || bad != 0ull || all_dense, 0)) {
                const bool isn = v != v;
                const int key2 = (elig && !isn) ? __float_as_int(v) : -1;
                const int mx2 = half_max_int_p16(key2);
                const unsigned long long m2 = __builtin_amdgcn_ballot_w64(key2 == mx2);
                const unsigned long long nanm = __builtin_amdgcn_ballot_w64(isn) & __builtin_amdgcn_ballot_w64(rowid == I);
                const unsigned nlo = (unsigned)nanm, nhi = (unsigned)(nanm >> 32);
                const unsigned mine_m = hb ? (unsigned)(m2 >> 32) : (unsigned)m2, mine_n = hb ? nhi : nlo;
                const int c2 = ((mine_m >> r) & 1u) ? rowid : (1 << 20);
                const int mn = half_min_i(c2);
                const unsigned long long w = __builtin_amdgcn_ballot_w64(row_lane && rowid == mn);
                const unsigned wm = hb ? (unsigned)(w >> 32) : (unsigned)w;
                const int pl = mine_n ? hb + __builtin_ctz(mine_n) : hb + (wm ? __builtin_ctz(wm) : 0);
                is_piv = lane == pl;
                piv_abs = mine_n ? __builtin_nanf("") : __int_as_float(mx2);
                const unsigned long long pm = __builtin_amdgcn_ballot_w64(is_piv);
                pl0 = __builtin_ctz((unsigned)pm | 0x80000000u);
                pl1 = 32 + __builtin_ctz((unsigned)(pm >> 32) | 0x80000000u);
                dense = all_dense || __builtin_amdgcn_ballot_w64(!rcp_fast_bits(__float_as_int(piv_abs))) != 0ull;
            } else {
                is_piv = key == mx;
                piv_abs = __int_as_float(mx);
                pl0 = __builtin_ctz(mlo | 0x80000000u);
                pl1 = 32 + __builtin_ctz(mhi | 0x80000000u);
                dense = false;
            }
        } else {
        const bool isn = v != v;
        const int key = (elig && !isn) ? __float_as_int(v) : -1;
        const int mx = (F & LU9_X_NOSEARCH) ? (rowid == I ? key : -2) : half_max_int_p16(key);
        if constexpr (F & LU9_SPEC) {
            // cuCdivf(1, rA[I]) of every lane's own candidate; only the pivot lane's is used
            f = cdiv_factors_fast(rA[I], v);
            rg = cmk((f.o1 * f.brs) * f.o2, (-(f.o1 * f.bis)) * f.o2);
        }
        const bool cand = key == mx;
        const unsigned long long m = __builtin_amdgcn_ballot_w64(cand);
        const unsigned long long nanm = __builtin_amdgcn_ballot_w64(isn) & __builtin_amdgcn_ballot_w64(rowid == I);
        const unsigned mlo = (unsigned)m, mhi = (unsigned)(m >> 32);
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
        dense = all_dense || __builtin_amdgcn_ballot_w64(!rcp_fast_bits(__float_as_int(piv_abs))) != 0ull;
        }
        const uint32_t pp0 = (uint32_t)__builtin_amdgcn_readlane((int)pat, pl0);
        const uint32_t pp1 = (uint32_t)__builtin_amdgcn_readlane((int)pat, pl1);
        constexpr uint32_t FULL = 0xFFFFFFFFu << (I + 1);
        const uint32_t pmw = dense ? FULL : ((pp0 | pp1) & FULL);
        if constexpr (F & LU9_SPEC) {
            if (__builtin_expect(dense, 0)) {
                f = cdiv_factors(rA[I]);
                rg = (piv_abs == 0.0f) ? cmk(1.0f, 0.0f) : cdiv_apply(cmk(1.0f, 0.0f), f);   // :66
            }
        }
        if (!(F & LU9_X_NOBCAST) && is_piv) {                  // pivot row -> buffer
            if constexpr (F & LU9_SPEC) {
                L.row[I] = rg;
                my.oo = pf2{f.o1, f.o2};
            } else {
                L.row[I] = rA[I];
            }
            lu3s_put_row<I + 1>(rA, pmw, L);
            L.row[30] = rB;
            L.row[31].x = __int_as_float(rowid);
        }
        if constexpr (F & LU9_SPEC) asm volatile("" : "+v"(my.oo));
        wave_lds_sync();
        Lu9Buf<LU3S_CHUNK> B;
        if constexpr ((F & (LU9_PF | LU9_EARLY)) && Lu9Chunks<LU3S_CHUNK>::count(I) > 0) {
            if (pmw & Lu9Chunks<LU3S_CHUNK>::mask(I, 0)) lu9_load<LU3S_CHUNK, I, 0>(B, L);
        }
        const cf sxi = L.row[I];
        cf sB0, pr;
        ld4(&L.row[30], sB0, pr);
        const int piv_pos = __float_as_int(pr.x);
        if (is_piv) rowid = I;                                 // :70-82
        else if (rowid == I) rowid = piv_pos;
        cf reg;
        if constexpr (F & LU9_SPEC) {
            reg = sxi;
        } else {
            if (__builtin_expect(!dense, 1)) {
                if constexpr (F & LU9_RCPA) {
                    pf2 oo;
                    const pf2 rg = recip_fast(pf2{sxi.x, sxi.y}, piv_abs, oo);
                    reg = cmk(rg.x, rg.y);
                    f.o1 = oo.x;
                    f.o2 = oo.y;
                } else {
                    f = cdiv_factors_fast(sxi, piv_abs);
                    reg = cmk((f.o1 * f.brs) * f.o2, (-(f.o1 * f.bis)) * f.o2);
                }
            } else {
                f = cdiv_factors(sxi);
                reg = (piv_abs == 0.0f) ? cmk(1.0f, 0.0f) : cdiv_apply(cmk(1.0f, 0.0f), f);   // :66
            }
            if (is_piv) my.oo = pf2{f.o1, f.o2};
            asm volatile("" : "+v"(my.oo));
        }
        const bool below = rowid > I;                          // :86-93
        if constexpr (F & LU9_ONEB) {
            // one exec-masked region per step: multiplier, right-hand side,
            // fill-in pattern (branch-free) and the rank-1 update
            const uint32_t pmwd = dense ? 0xFFFFFFFFu : pmw;
            if (below) {
                const pf2 lp = pcmul(pf2{rA[I].x, rA[I].y}, pf2{reg.x, reg.y});
                const pf2 bp = pcmsub(pf2{rB.x, rB.y}, lp, pf2{sB0.x, sB0.y});
                rB = cmk(bp.x, bp.y);
                pat |= (((pat >> I) & 1u) != 0u || dense) ? pmwd : 0u;
                lu9_update<F, LU3S_CHUNK, I, 0, false>(rA, cmk(lp.x, lp.y), below, pmw, L, B);
            }
            lu9_forward<F, CH, I + 1>(rA, rB, rowid, pat, all_dense, lane, r, hb, row_lane, my, L);
            return;
        }
        cf l = cmk(0.0f, 0.0f);
        if (below) {
            const pf2 lp = pcmul(pf2{rA[I].x, rA[I].y}, pf2{reg.x, reg.y});
            const pf2 bp = pcmsub(pf2{rB.x, rB.y}, lp, pf2{sB0.x, sB0.y});
            l = cmk(lp.x, lp.y);
            rB = cmk(bp.x, bp.y);
        }
        if (below && (dense || ((pat >> I) & 1u))) pat |= dense ? 0xFFFFFFFFu : pmw;
        if constexpr (F & LU9_X_NOUPD) {
        } else if constexpr (F & LU9_NOMASK) {
            if (__builtin_expect(!dense, 1)) lu9_update<F, LU3S_CHUNK, I, 0, false>(rA, l, below, pmw, L, B);
            else lu9_update<F, LU3S_CHUNK, I, 0, true>(rA, l, below, pmw, L, B);
        } else if constexpr (F & LU9_BOUT) {
            if (below) lu9_update<F, LU3S_CHUNK, I, 0, false>(rA, l, below, pmw, L, B);
        } else {
            lu9_update<F, LU3S_CHUNK, I, 0, true>(rA, l, below, pmw, L, B);
        }
        lu9_forward<F, CH, I + 1>(rA, rB, rowid, pat, all_dense, lane, r, hb, row_lane, my, L);
    }
}

// back substitution, x_I broadcast with v_readlane from the owner lane of each
// half (found by a ballot on the final row ids)
template <int I, bool SPLIT>
__device__ __forceinline__ void lu9_backward_rl(const cf (&rA)[NV], cf &rB, int rowid, const PivF &my, int hb) {
    if constexpr (I >= 0) {
        const unsigned long long own = __builtin_amdgcn_ballot_w64(rowid == I);
        const int o0 = __builtin_ctz((unsigned)own | 0x80000000u);
        const int o1 = 32 + __builtin_ctz((unsigned)(own >> 32) | 0x80000000u);
        const pf2 q = pcdiv_apply(pf2{rB.x, rB.y}, pf2{rA[I].x, rA[I].y}, my);
        const float x0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(q.x), o0));
        const float y0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(q.y), o0));
        const float x1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(q.x), o1));
        const float y1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(q.y), o1));
        if constexpr (SPLIT) {
            // each half subtracts its own owner's x_I, an SGPR pair operand
            const bool own_lane = rowid == I;
            if (rowid < I) {
                const pf2 a = pf2{rA[I].x, rA[I].y};
                pf2 v = pf2{rB.x, rB.y}, t;
                if (hb == 0) {
                    const pf2 xs = pf2{x0, y0};
                    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[0,1,1] neg_lo:[1,0,0] neg_hi:[1,0,0]" : "=v"(t) : "s"(xs), "v"(a), "v"(v));
                    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_hi:[1,0,0]" : "=v"(v) : "s"(xs), "v"(a), "v"(t));
                } else {
                    const pf2 xs = pf2{x1, y1};
                    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[0,1,1] neg_lo:[1,0,0] neg_hi:[1,0,0]" : "=v"(t) : "s"(xs), "v"(a), "v"(v));
                    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_hi:[1,0,0]" : "=v"(v) : "s"(xs), "v"(a), "v"(t));
                }
                rB = cmk(v.x, v.y);
            }
            if (own_lane) rB = cmk(q.x, q.y);   // the owner keeps its x_I (returned below)
        } else {
        const cf xi = hb ? cmk(x1, y1) : cmk(x0, y0);
        if (rowid < I) {
            const pf2 v = pcmsub(pf2{rB.x, rB.y}, pf2{xi.x, xi.y}, pf2{rA[I].x, rA[I].y});
            rB = cmk(v.x, v.y);
        }
        if (rowid == I) rB = xi;   // the owner keeps its x_I (returned below)
        }
        lu9_backward_rl<I - 1, SPLIT>(rA, rB, rowid, my, hb);
    }
}

template <int F>
__device__ __forceinline__ cf lu_solve9(cf (&rA)[NV], cf rB, int lane, uint32_t pattern, LUBuf &L) {
    bool ok = true;
#pragma unroll
    for (int c = 0; c < NV; c++)
        ok = ok && __builtin_fabsf(rA[c].x) < 0x1p88f && __builtin_fabsf(rA[c].y) < 0x1p88f;
    const bool all_dense = __builtin_amdgcn_ballot_w64(!ok) != 0ull;
    const int r = lane & 31, hb = lane & 32;
    const bool row_lane = r < NV;
    int rowid = row_lane ? r : 99;
    uint32_t pat = row_lane ? pattern : 0u;
    PivF my{pf2{0.0f, 0.0f}};
    lu9_forward<F, LU3S_CHUNK, 0>(rA, rB, rowid, pat, all_dense, lane, r, hb, row_lane, my, L);
    if constexpr (F & LU9_X_NOBACK) {
        wave_lds_sync();
        return L.row[row_lane ? r : 0];
    } else if constexpr (F & LU9_BRL) {
        lu9_backward_rl<NV - 1, (F & LU9_BSPLIT) != 0>(rA, rB, rowid, my, hb);
        // lane r returns x_r: the owner of position r holds it in rB
        const unsigned long long dummy = 0;
        (void)dummy;
        wave_lds_sync();
        if (row_lane) L.row[rowid] = rB;
        wave_lds_sync();
        return L.row[row_lane ? r : 0];
    } else {
        lu3s_backward<NV - 1>(rA, rB, rowid, my, L);
        wave_lds_sync();
        return L.row[row_lane ? r : 0];
    }
}

}  // namespace hc
