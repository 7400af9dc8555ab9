// hc_track4.hpp -- v4 building blocks: FOUR homotopy paths per wavefront.
//
// A path slot is one 16-lane DPP row (a quarter wave).  Lane r (0..15) of a
// slot owns equation rows r ("slot 0") and r + 16 ("slot 1", real for r < 14)
// of that path's Jacobian, their right-hand sides, and the unknowns x_r and
// x_{r+16}.  Every cross-lane step of a path is a DPP op inside its own row
// (pivot max, ties, the corrector's norm tree); LDS carries the pivot row.
//
// Why (profiles/r1c_pmc_summary.json): the v3 LU spends its
// time in the LDS pipe, and an LDS write instruction costs the same whatever
// its exec mask -- the pivot lane of each path writes its row with
// ds_write_b128.  With two rows per lane one write instruction carries the
// pivot rows of four paths instead of two, and the per-step pivot search,
// division factors and bookkeeping are shared by four paths.
//
// Semantics and arithmetic are exactly v3's / the oracle's
// (dev-cgesv-batched-small.cuh:38-107 for the LU, the index evals of
// gpu-idx-evals/..._LimUnroll_L2Cache.cuh:57-148): only the data layout
// changes, so every result is bit-identical.
#pragma once

#include "hc_lu3.hpp"

namespace hc {

constexpr int QL = 16;   // lanes per path slot

// Per-path-slot LDS block of v4: only what the evaluations read (x, p(t), d)
// and the dH/dx entry block (reused as the LU broadcast buffer).  The RK
// state, t, step sizes and the target parameters stay in VGPRs.  The v3 term
// words address p / d relative to SlotLDS; v4 rebases them once when it copies
// the tables to LDS (rebase_p_offsets).
struct alignas(16) SlotLDS4 {
    cf x[32];        // current track (x[30] = 1)
    cf p[NPP];       // p(t)
    cf dif[NPP];     // diff params of the current sample
    cf ent[NV * 7];  // dH/dx entries of row r at [r*7 + slot], slot 6 = 0
    char bank_pad[96];   // stride = 16 mod 256 B: the four slots of a wave use different LDS banks
};
static_assert(sizeof(SlotLDS4) % 256 == 16, "SlotLDS4 stride must shift the LDS banks by 4 per slot");
static_assert(offsetof(SlotLDS4, x) == SLOT_OFF_X, "x offsets are shared with the v3 tables");
static_assert(offsetof(SlotLDS4, ent) % 16 == 0, "SlotLDS4::ent must be 16-B aligned");
constexpr uint32_t SLOT4_P_REBASE = (uint32_t)(SLOT_OFF_P - (int)offsetof(SlotLDS4, p));
constexpr int SLOT4_DIF_DELTA = (int)offsetof(SlotLDS4, dif) - (int)offsetof(SlotLDS4, p);
__device__ __forceinline__ uint2 rebase_p_offsets(uint2 w) {
    return make_uint2(((w.x & 0xFFFFu) - SLOT4_P_REBASE) | (((w.x >> 16) - SLOT4_P_REBASE) << 16), w.y);
}

// ---------------------------------------------------------------- row (16-lane) reductions
__device__ __forceinline__ int row_max_i(int v) {
    v = max(v, dpp_i<DPP_QP_1032>(v));
    v = max(v, dpp_i<DPP_QP_2301>(v));
    v = max(v, dpp_i<DPP_ROW_HALF_MIRROR>(v));
    v = max(v, dpp_i<DPP_ROW_MIRROR>(v));
    return v;
}
__device__ __forceinline__ int row_min_i(int v) {
    v = min(v, dpp_i<DPP_QP_1032>(v));
    v = min(v, dpp_i<DPP_QP_2301>(v));
    v = min(v, dpp_i<DPP_ROW_HALF_MIRROR>(v));
    v = min(v, dpp_i<DPP_ROW_MIRROR>(v));
    return v;
}
__device__ __forceinline__ int row_sum_i(int v) {
    v += dpp_i<DPP_QP_1032>(v);
    v += dpp_i<DPP_QP_2301>(v);
    v += dpp_i<DPP_ROW_HALF_MIRROR>(v);
    v += dpp_i<DPP_ROW_MIRROR>(v);
    return v;
}
// lane 0 of each 16-lane row, broadcast to the row (ds_swizzle bit mode:
// src = lane & 0x10 inside each 32-lane group)
__device__ __forceinline__ int qbcast0_i(int v) { return __builtin_amdgcn_ds_swizzle(v, 0x10); }
__device__ __forceinline__ float qbcast0_f(float v) { return __int_as_float(qbcast0_i(__float_as_int(v))); }
// The reference's shfl_down tree (..._TrunPaths.cu:235-238) for one path:
// a = v_r + v_{r+16} (lanes r holding rows r, r+16), then offsets 8, 4, 2, 1
// inside the row; lane 0's value broadcast.  Same additions in the same order
// as tree_sum_half / the oracle.
__device__ __forceinline__ float tree_sum_q(float a) {
    const float b = a + dpp_f<DPP_ROW_SHL8>(a);
    const float c = b + dpp_f<DPP_ROW_SHL4>(b);
    const float d = c + dpp_f<DPP_ROW_SHL2>(c);
    const float e = d + dpp_f<DPP_ROW_SHL1>(d);
    return qbcast0_f(e);
}

// ---------------------------------------------------------------- evals (2 rows per lane)
// dH/dx (:57-88): rows r and r+16 of the slot's Jacobian into A0 / A1.  The
// term lists are v3's (TableWS3, one list per row, p offsets rebased to
// SlotLDS4); finished entries go to the
// slot's entry block and are gathered back through the per-row column->slot
// maps.  Rows 30 / 31 (slot 1 of lanes 14, 15) only hold padding terms (coef
// 0, never "last"), so they write nothing and gather the structural zero.
__device__ __forceinline__ void eval_hx4(cf (&A0)[NV], cf (&A1)[NV], const uint2 *s_hx3, int hx_len,
                                         const uint32_t (&map0)[3], const uint32_t (&map1)[3], SlotLDS4 &S, int r) {
    const char *sb = reinterpret_cast<const char *>(&S);
    const int r1 = r + QL;
    cf *ent0 = S.ent + r * 7;
    cf *ent1 = S.ent + (r1 < NV ? r1 : r) * 7;
    char *eb0 = reinterpret_cast<char *>(ent0);
    char *eb1 = reinterpret_cast<char *>(ent1);
    ent0[6] = cmk(0.0f, 0.0f);   // structural zero (the LU reuses this block)
    if (r1 < NV) ent1[6] = cmk(0.0f, 0.0f);
    pf2 acc0 = {0.0f, 0.0f}, acc1 = {0.0f, 0.0f};
    for (int k = 0; k < hx_len; k++) {
        const uint2 w0 = s_hx3[k * 32 + r];
        const uint2 w1 = s_hx3[k * 32 + r1];
        const pf2 pa0 = ldp(sb, w0.x & 0xFFFFu), pb0 = ldp(sb, w0.x >> 16);
        const pf2 pa1 = ldp(sb, w1.x & 0xFFFFu), pb1 = ldp(sb, w1.x >> 16);
        const pf2 xu0 = ldp(sb, w0.y & 0xFFu), xv0 = ldp(sb, (w0.y >> 8) & 0xFFu);
        const pf2 xu1 = ldp(sb, w1.y & 0xFFu), xv1 = ldp(sb, (w1.y >> 8) & 0xFFu);
        const float co0 = (float)(int)(int8_t)(uint8_t)(w0.y >> 16);
        const float co1 = (float)(int)(int8_t)(uint8_t)(w1.y >> 16);
        pf2 P0 = pa0 * pf2{co0, co0};
        pf2 P1 = pa1 * pf2{co1, co1};
        P0 = pcmul(P0, pb0);
        P1 = pcmul(P1, pb1);
        P0 = pcmul(P0, xu0);
        P1 = pcmul(P1, xu1);
        acc0 = pcmadd(acc0, P0, xv0);
        acc1 = pcmadd(acc1, P1, xv1);
        if ((int)w0.y < 0) {
            *reinterpret_cast<pf2 *>(eb0 + ((w0.y >> 24) & 0x7Fu)) = acc0;
            acc0 = pf2{0.0f, 0.0f};
        }
        if ((int)w1.y < 0) {
            *reinterpret_cast<pf2 *>(eb1 + ((w1.y >> 24) & 0x7Fu)) = acc1;
            acc1 = pf2{0.0f, 0.0f};
        }
    }
    wave_lds_sync();
#pragma unroll
    for (int c = 0; c < NV; c++) {
        const uint32_t c0 = (map0[c / 10] >> (3 * (c % 10))) & 7u;
        const uint32_t c1 = (map1[c / 10] >> (3 * (c % 10))) & 7u;
        A0[c] = ent0[c0];
        A1[c] = ent1[c1];
    }
}

// dH/dt (:91-119) for rows r, r+16
__device__ __forceinline__ void eval_ht4(const uint2 *s_ht3, const SlotLDS4 &S, int r, cf &b0, cf &b1) {
    const char *sb = reinterpret_cast<const char *>(&S);
    pf2 acc0 = {0.0f, 0.0f}, acc1 = {0.0f, 0.0f};
#pragma unroll 2
    for (int j = 0; j < HT_TERMS; j++) {
        const uint2 w0 = s_ht3[j * 32 + r];
        const uint2 w1 = s_ht3[j * 32 + r + QL];
        const uint32_t oa0 = w0.x & 0xFFFFu, ob0 = w0.x >> 16, oa1 = w1.x & 0xFFFFu, ob1 = w1.x >> 16;
        const pf2 pa0 = ldp(sb, oa0), pb0 = ldp(sb, ob0), pa1 = ldp(sb, oa1), pb1 = ldp(sb, ob1);
        const pf2 da0 = ldp(sb + SLOT4_DIF_DELTA, oa0), db0 = ldp(sb + SLOT4_DIF_DELTA, ob0);
        const pf2 da1 = ldp(sb + SLOT4_DIF_DELTA, oa1), db1 = ldp(sb + SLOT4_DIF_DELTA, ob1);
        const pf2 xu0 = ldp(sb, w0.y & 0xFFu), xv0 = ldp(sb, (w0.y >> 8) & 0xFFu), xw0 = ldp(sb, (w0.y >> 16) & 0xFFu);
        const pf2 xu1 = ldp(sb, w1.y & 0xFFu), xv1 = ldp(sb, (w1.y >> 8) & 0xFFu), xw1 = ldp(sb, (w1.y >> 16) & 0xFFu);
        const float co0 = (float)((int)w0.y >> 24), co1 = (float)((int)w1.y >> 24);
        pf2 s0 = pcmadd(pcmul(da0, pb0), db0, pa0);
        pf2 s1 = pcmadd(pcmul(da1, pb1), db1, pa1);
        s0 = s0 * pf2{co0, co0};
        s1 = s1 * pf2{co1, co1};
        const pf2 P0 = pcmul(pcmul(s0, xu0), xv0);
        const pf2 P1 = pcmul(pcmul(s1, xu1), xv1);
        acc0 = pcmsub(acc0, P0, xw0);
        acc1 = pcmsub(acc1, P1, xw1);
    }
    b0 = cmk(acc0.x, acc0.y);
    b1 = cmk(acc1.x, acc1.y);
}

// H (:122-148) for rows r, r+16
__device__ __forceinline__ void eval_h4(const uint2 *s_ht3, const SlotLDS4 &S, int r, cf &b0, cf &b1) {
    const char *sb = reinterpret_cast<const char *>(&S);
    pf2 acc0 = {0.0f, 0.0f}, acc1 = {0.0f, 0.0f};
#pragma unroll 2
    for (int j = 0; j < HT_TERMS; j++) {
        const uint2 w0 = s_ht3[j * 32 + r];
        const uint2 w1 = s_ht3[j * 32 + r + QL];
        const pf2 pa0 = ldp(sb, w0.x & 0xFFFFu), pb0 = ldp(sb, w0.x >> 16);
        const pf2 pa1 = ldp(sb, w1.x & 0xFFFFu), pb1 = ldp(sb, w1.x >> 16);
        const pf2 xu0 = ldp(sb, w0.y & 0xFFu), xv0 = ldp(sb, (w0.y >> 8) & 0xFFu), xw0 = ldp(sb, (w0.y >> 16) & 0xFFu);
        const pf2 xu1 = ldp(sb, w1.y & 0xFFu), xv1 = ldp(sb, (w1.y >> 8) & 0xFFu), xw1 = ldp(sb, (w1.y >> 16) & 0xFFu);
        const float co0 = (float)((int)w0.y >> 24), co1 = (float)((int)w1.y >> 24);
        pf2 P0 = pa0 * pf2{co0, co0};
        pf2 P1 = pa1 * pf2{co1, co1};
        P0 = pcmul(pcmul(pcmul(P0, pb0), xu0), xv0);
        P1 = pcmul(pcmul(pcmul(P1, pb1), xu1), xv1);
        acc0 = pcmadd(acc0, P0, xw0);
        acc1 = pcmadd(acc1, P1, xw1);
    }
    b0 = cmk(acc0.x, acc0.y);
    b1 = cmk(acc1.x, acc1.y);
}

// ---------------------------------------------------------------- LU (4 systems / wave)
// Pivot row of slot q of the pivot lane: rows J.. into the buffer.  One
// v_cndmask per float selects the slot (the pivot lane is the only writer of
// its path; the instruction count is what costs, not the lanes).
template <int J>
__device__ __forceinline__ void lu4_put_row(const cf (&A0)[NV], const cf (&A1)[NV], bool s1, LUBuf &L) {
    if constexpr (J < NV) {
        if constexpr (J & 1) {
            L.row[J] = s1 ? A1[J] : A0[J];
            lu4_put_row<J + 1>(A0, A1, s1, L);
        } else {
            st4(&L.row[J], s1 ? A1[J] : A0[J], s1 ? A1[J + 1] : A0[J + 1]);
            lu4_put_row<J + 2>(A0, A1, s1, L);
        }
    }
}

// a_j -= l * u_j for j in [J0, NV) on the rows below, u from the buffer
template <int J0>
__device__ __forceinline__ void lu4_update(cf (&A0)[NV], cf (&A1)[NV], const pf2 &l0, const pf2 &l1, bool below0,
                                           bool below1, const LUBuf &L) {
    if constexpr (J0 < NV) {
        if constexpr ((J0 & 1) || J0 + 1 >= NV) {
            const cf u = L.row[J0];
            if (below0) { const pf2 t = pcmsub(pf2{A0[J0].x, A0[J0].y}, l0, pf2{u.x, u.y}); A0[J0] = cmk(t.x, t.y); }
            if (below1) { const pf2 t = pcmsub(pf2{A1[J0].x, A1[J0].y}, l1, pf2{u.x, u.y}); A1[J0] = cmk(t.x, t.y); }
            lu4_update<J0 + 1>(A0, A1, l0, l1, below0, below1, L);
        } else {
            constexpr int N0 = (NV - J0) < LU3_CHUNK ? (NV - J0) : LU3_CHUNK;
            constexpr int N = N0 & ~1;
            cf u[N];
#pragma unroll
            for (int q = 0; q < N; q += 2) ld4(&L.row[J0 + q], u[q], u[q + 1]);
            if (below0) {
#pragma unroll
                for (int q = 0; q < N; q++) {
                    const pf2 t = pcmsub(pf2{A0[J0 + q].x, A0[J0 + q].y}, l0, pf2{u[q].x, u[q].y});
                    A0[J0 + q] = cmk(t.x, t.y);
                }
            }
            if (below1) {
#pragma unroll
                for (int q = 0; q < N; q++) {
                    const pf2 t = pcmsub(pf2{A1[J0 + q].x, A1[J0 + q].y}, l1, pf2{u[q].x, u[q].y});
                    A1[J0 + q] = cmk(t.x, t.y);
                }
            }
            __builtin_amdgcn_sched_barrier(0);
            lu4_update<J0 + N>(A0, A1, l0, l1, below0, below1, L);
        }
    }
}

// one elimination step (:51-94) for the path of each 16-lane row
template <int I>
__device__ __forceinline__ void lu4_forward(cf (&A0)[NV], cf (&A1)[NV], cf &b0, cf &b1, int &rid0, int &rid1,
                                            int qb, LUBuf &L) {
    if constexpr (I < NV) {
        const float v0 = __builtin_fabsf(A0[I].x) + __builtin_fabsf(A0[I].y);   // :55
        const float v1 = __builtin_fabsf(A1[I].x) + __builtin_fabsf(A1[I].y);
        const bool n0 = v0 != v0, n1 = v1 != v1;
        const int k0 = (rid0 >= I && !n0) ? __float_as_int(v0) : -1;          // rid0 <= 29 always
        const int k1 = (rid1 >= I && rid1 < NV && !n1) ? __float_as_int(v1) : -1;
        const int mx = row_max_i(max(k0, k1));
        const bool c0 = k0 == mx, c1 = k1 == mx;
        const unsigned long long m0 = __builtin_amdgcn_ballot_w64(c0);
        const unsigned long long m1 = __builtin_amdgcn_ballot_w64(c1);
        const unsigned long long nanm = (__builtin_amdgcn_ballot_w64(n0) & __builtin_amdgcn_ballot_w64(rid0 == I)) |
                                        (__builtin_amdgcn_ballot_w64(n1) & __builtin_amdgcn_ballot_w64(rid1 == I));
        bool p0, p1;   // this lane holds the pivot row of its path in slot 0 / 1
        // mx >= 0 in every row leaves at least one candidate per row: exactly 4
        // candidates <=> one per path
        if (__builtin_expect(nanm != 0ull || __builtin_popcountll(m0) + __builtin_popcountll(m1) != 4, 0)) {
            // rare: NaN at position I wins (:57-64); exact ties: first position wins
            const bool mine_n = ((nanm >> qb) & 0xFFFFull) != 0ull;
            const int cr = min(c0 ? rid0 : (1 << 20), c1 ? rid1 : (1 << 20));
            const int mn = row_min_i(cr);
            const int want = mine_n ? I : mn;
            p0 = rid0 == want;
            p1 = rid1 == want;
        } else {
            p0 = c0;
            p1 = c1;
        }
        if (p0 || p1) {                                        // pivot row -> buffer
            lu4_put_row<I>(A0, A1, p1, L);
            st4(&L.row[30], p1 ? b1 : b0, cmk(__int_as_float(p1 ? rid1 : rid0), 0.0f));
        }
        wave_lds_sync();                                       // pivot lane -> its row
        const cf sxi = L.row[I];
        cf sB0, pr;
        ld4(&L.row[30], sB0, pr);
        const int piv_pos = __float_as_int(pr.x);
        if (p0) rid0 = I;                                      // :70-82
        else if (rid0 == I) rid0 = piv_pos;
        if (p1) rid1 = I;
        else if (rid1 == I) rid1 = piv_pos;
        cf reg;                                                // cuCdivf(1, pivot) (:84)
        const float s = __builtin_fabsf(sxi.x) + __builtin_fabsf(sxi.y);
        if (__builtin_expect(__builtin_amdgcn_ballot_w64(!rcp_fast_ok(s)) == 0ull, 1)) {
            const divf f = cdiv_factors_fast(sxi, s);
            reg = cmk((f.o1 * f.brs) * f.o2, (-(f.o1 * f.bis)) * f.o2);
        } else {
            const divf f = cdiv_factors(sxi);
            reg = (s == 0.0f) ? cmk(1.0f, 0.0f) : cdiv_apply(cmk(1.0f, 0.0f), f);   // :66
        }
        const bool below0 = rid0 > I, below1 = rid1 > I;      // :86-93
        pf2 l0 = {0.0f, 0.0f}, l1 = {0.0f, 0.0f};
        if (below0) {
            l0 = pcmul(pf2{A0[I].x, A0[I].y}, pf2{reg.x, reg.y});
            const pf2 t = pcmsub(pf2{b0.x, b0.y}, l0, pf2{sB0.x, sB0.y});
            b0 = cmk(t.x, t.y);
        }
        if (below1) {
            l1 = pcmul(pf2{A1[I].x, A1[I].y}, pf2{reg.x, reg.y});
            const pf2 t = pcmsub(pf2{b1.x, b1.y}, l1, pf2{sB0.x, sB0.y});
            b1 = cmk(t.x, t.y);
        }
        lu4_update<I + 1>(A0, A1, l0, l1, below0, below1, L);
        lu4_forward<I + 1>(A0, A1, b0, b1, rid0, rid1, qb, L);
    }
}

// back substitution (:97-106): the (lane, slot) with rowid == I owns position
// I and still holds pivot I in A[I]; it recomputes that pivot's factors
template <int I>
__device__ __forceinline__ void lu4_backward(const cf (&A0)[NV], const cf (&A1)[NV], cf &b0, cf &b1, int rid0,
                                             int rid1, LUBuf &L) {
    if constexpr (I >= 0) {
        const bool o0 = rid0 == I, o1 = rid1 == I;
        const cf piv = o1 ? A1[I] : A0[I];
        const cf bq = o1 ? b1 : b0;
        const float s = __builtin_fabsf(piv.x) + __builtin_fabsf(piv.y);
        divf f;
        if (__builtin_expect((__builtin_amdgcn_ballot_w64(!rcp_fast_ok(s)) & __builtin_amdgcn_ballot_w64(o0 || o1)) == 0ull,
                             1))
            f = cdiv_factors_fast(piv, s);
        else
            f = cdiv_factors(piv);
        const cf cand = cdiv_apply(bq, f);
        if (o0 || o1) L.row[I] = cand;
        wave_lds_sync();
        const cf xi = L.row[I];
        if (rid0 < I) b0 = cmsub(b0, xi, A0[I]);
        if (rid1 < I) b1 = cmsub(b1, xi, A1[I]);
        lu4_backward<I - 1>(A0, A1, b0, b1, rid0, rid1, L);
    }
}

// Solves the system of each 16-lane row; L is that row's buffer (16-B aligned).
// Returns x_r in x0 and x_{r+16} in x1 (r = lane & 15).
__device__ __forceinline__ void lu_solve4(cf (&A0)[NV], cf (&A1)[NV], cf b0, cf b1, int lane, LUBuf &L, cf &x0,
                                          cf &x1) {
    const int r = lane & 15, qb = lane & 48;
    int rid0 = r;
    int rid1 = r + QL < NV ? r + QL : 99;   // rows 30, 31: never eligible, never own a position
    lu4_forward<0>(A0, A1, b0, b1, rid0, rid1, qb, L);
    lu4_backward<NV - 1>(A0, A1, b0, b1, rid0, rid1, L);
    wave_lds_sync();
    x0 = L.row[r];
    x1 = L.row[r + QL < NV ? r + QL : r];
}

}  // namespace hc
