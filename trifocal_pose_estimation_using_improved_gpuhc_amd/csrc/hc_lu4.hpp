// hc_lu4.hpp -- the batched 30x30 complex LU solve with FOUR systems per
// wavefront: lane l serves system g = l >> 4 (a 16-lane DPP row) and holds
// rows q = l & 15 (slot 0) and q + 16 (slot 1, rows 16..29; lanes 14, 15 pad).
//
// Same semantics and the same per-element operations as hc_lu.hpp (the
// reference's dev-cgesv-batched-small.cuh:38-107): partial
// pivoting on cabs1 with first-maximum ties and NaN-at-position-I, rows
// relabelled through rowid, cuCdivf back substitution, structurally sparse
// column groups.  What changes is what one instruction serves:
//  * a pivot step's fixed work -- search, 1/pivot, row-id and pattern
//    bookkeeping, the branch on the column groups -- is issued once for four
//    systems instead of two;
//  * one ds_write_b128 carries the pivot rows of four systems (the pivot lane
//    of each group first selects its pivot slot's columns with v_cndmask);
//    the LDS store costs the same whatever its EXEC mask (MI355X_MICROARCH.md
//    §LDS), so the store count per system halves;
//  * one broadcast ds_read_b128 serves both rows a lane holds;
//  * the group reductions are four DPP steps inside a 16-lane row (no
//    v_permlane16_swap), and the reference's 32-slot norm tree starts with
//    the lane-local a_q + a_{q+16}.
// Registers: two rows (120 VGPRs) per lane.
#pragma once

#include "hc_lu.hpp"

namespace hc {

struct alignas(16) LUBuf4 {
    cf row[32];     // pivot row: [0..29] columns, [30] pivot, [31] rhs
    cf x[32];       // back substitution: x_I at [I]
    int pos;        // the pivot row's position (rowid) before the swap
    int pad[3];
};
static_assert(sizeof(LUBuf4) % 256 == 16, "LUBuf4 stride shifts the LDS banks by 4 dwords per group");

// max / min over each 16-lane DPP row (one system)
__device__ __forceinline__ int grp_max16(int v) {
    v = max(v, dpp_i<DPP_QP_1032>(v));
    v = max(v, dpp_i<DPP_QP_2301>(v));
    v = max(v, dpp_i<DPP_ROW_HALF_MIRROR>(v));
    v = max(v, dpp_i<DPP_ROW_MIRROR>(v));
    return v;
}
__device__ __forceinline__ int grp_min16(int v) {
    v = min(v, dpp_i<DPP_QP_1032>(v));
    v = min(v, dpp_i<DPP_QP_2301>(v));
    v = min(v, dpp_i<DPP_ROW_HALF_MIRROR>(v));
    v = min(v, dpp_i<DPP_ROW_MIRROR>(v));
    return v;
}

// lanes of the groups whose bit is set in gm (bit g -> lanes 16g..16g+15)
__device__ __forceinline__ unsigned long long grp_lanes(unsigned gm) {
    unsigned long long m = 0ull;
#pragma unroll
    for (int g = 0; g < 4; g++)
        if (gm & (1u << g)) m |= 0xFFFFull << (16 * g);
    return m;
}

// b if s else a, on values (a select of array element addresses would keep the
// row arrays in scratch memory)
__device__ __forceinline__ cf csel(bool s, cf a, cf b) { return cmk(s ? b.x : a.x, s ? b.y : a.y); }
__device__ __forceinline__ pf2 psel(bool s, cf a, cf b) { return pf2{s ? b.x : a.x, s ? b.y : a.y}; }

struct PivSel4 {
    bool p0, p1;          // this lane's slot 0 / slot 1 row is its system's pivot
    float piv_abs;        // |re| + |im| of the pivot of this lane's system (NaN if a NaN won)
    bool dense;           // 1/pivot outside the fast range in some active system
    unsigned long long t; // ballot of the pivot lanes (one per active system)
};

// the pivot search of step I; v0, v1 = cabs1 of the lane's column-I entries
template <int I>
__device__ __forceinline__ PivSel4 lu4_search(float v0, float v1, int rowid0, int rowid1, bool all_dense,
                                              unsigned long long act_lanes) {
    PivSel4 p;
    const bool e0 = rowid0 >= I && rowid0 < NV, e1 = rowid1 >= I && rowid1 < NV;
    const int k0 = e0 ? __float_as_int(v0) : -1, k1 = e1 ? __float_as_int(v1) : -1;
    const int mx = grp_max16(max(k0, k1));
    const unsigned long long m0 = __builtin_amdgcn_ballot_w64(k0 == mx), m1 = __builtin_amdgcn_ballot_w64(k1 == mx);
    const unsigned long long bad = __builtin_amdgcn_ballot_w64(!rcp_fast_bits(mx)) & act_lanes;
    const unsigned long long t = m0 | m1;
    // every group's field of t is non-zero (the maximum is attained), so the
    // per-field subtraction below borrows inside its field only: a field with
    // two or more bits, or a lane whose two rows both attain it, is a tie
    const unsigned long long tie = ((t & (t - 0x0001000100010001ull)) | (m0 & m1)) & act_lanes;
    if (__builtin_expect(tie != 0ull || bad != 0ull || all_dense, 0)) {
        // rare: NaN at position I wins (:57-64); exact ties: first position wins
        const bool n0 = v0 != v0, n1 = v1 != v1;
        const int kk0 = (e0 && !n0) ? __float_as_int(v0) : -1, kk1 = (e1 && !n1) ? __float_as_int(v1) : -1;
        const int mx2 = grp_max16(max(kk0, kk1));
        const int c0 = (kk0 >= 0 && kk0 == mx2) ? rowid0 : (1 << 20);
        const int c1 = (kk1 >= 0 && kk1 == mx2) ? rowid1 : (1 << 20);
        const int mn = grp_min16(min(c0, c1));
        const bool i0 = n0 && rowid0 == I, i1 = n1 && rowid1 == I;
        const bool nan_at_i = grp_max16((i0 || i1) ? 1 : 0) != 0;
        p.p0 = nan_at_i ? i0 : (mn < (1 << 20) && c0 == mn);
        p.p1 = nan_at_i ? i1 : (mn < (1 << 20) && c1 == mn);
        p.piv_abs = nan_at_i ? __builtin_nanf("") : __int_as_float(mx2);
        p.t = __builtin_amdgcn_ballot_w64(p.p0 || p.p1);
        p.dense = all_dense ||
                  (__builtin_amdgcn_ballot_w64(!rcp_fast_bits(__float_as_int(p.piv_abs))) & act_lanes) != 0ull;
    } else {
        p.p0 = k0 == mx;
        p.p1 = k1 == mx;
        p.piv_abs = __int_as_float(mx);
        p.t = t;
        p.dense = false;
    }
    return p;
}

// pivot lanes: the groups of step I (LuChunks<LU_CHUNK>) that are non-zero in
// some pivot row of the wave, from the pivot slot (sel) into the buffer
template <int I, int K>
__device__ __forceinline__ void lu4_put_row(const cf (&a0)[NV], const cf (&a1)[NV], bool sel, uint32_t pmw,
                                            LUBuf4 &L) {
    using C = LuChunks<LU_CHUNK>;
    if constexpr (K < C::count(I)) {
        constexpr int J = C::start(I, K), N = C::len(I, K);
        if (pmw & C::mask(I, K)) {
            if constexpr (N == 1) {
                L.row[J] = csel(sel, a0[J], a1[J]);
            } else {
#pragma unroll
                for (int q = 0; q < N; q += 2)
                    st4(&L.row[J + q], csel(sel, a0[J + q], a1[J + q]), csel(sel, a0[J + q + 1], a1[J + q + 1]));
            }
        }
        lu4_put_row<I, K + 1>(a0, a1, sel, pmw, L);
    }
}

// rows below the pivot in either slot: a_j -= l * u_j for the groups K.. of step I
template <int I, int K>
__device__ __forceinline__ void lu4_update(cf (&a0)[NV], cf (&a1)[NV], const pf2 &l0, const pf2 &l1, bool b0,
                                           bool b1, uint32_t pmw, const LUBuf4 &L) {
    using C = LuChunks<LU_CHUNK>;
    if constexpr (K < C::count(I)) {
        constexpr int J = C::start(I, K), N = C::len(I, K);
        if (pmw & C::mask(I, K)) {
            cf u[N];
            if constexpr (N == 1) {
                u[0] = L.row[J];
            } else {
#pragma unroll
                for (int q = 0; q < N; q += 2) ld4(&L.row[J + q], u[q], u[q + 1]);
            }
            if (b0) {
#pragma unroll
                for (int q = 0; q < N; q++) {
                    const pf2 v = pcmsub(pf2{a0[J + q].x, a0[J + q].y}, l0, pf2{u[q].x, u[q].y});
                    a0[J + q] = cmk(v.x, v.y);
                }
            }
            if (b1) {
#pragma unroll
                for (int q = 0; q < N; q++) {
                    const pf2 v = pcmsub(pf2{a1[J + q].x, a1[J + q].y}, l1, pf2{u[q].x, u[q].y});
                    a1[J + q] = cmk(v.x, v.y);
                }
            }
        }
        __builtin_amdgcn_sched_barrier(0);
        lu4_update<I, K + 1>(a0, a1, l0, l1, b0, b1, pmw, L);
    }
}

struct Lu4Row {   // per-slot state of the solve
    int rowid;
    uint32_t pat;
    PivF my;
};

template <int I>
__device__ __forceinline__ void lu4_forward(cf (&a0)[NV], cf (&a1)[NV], cf &b0, cf &b1, Lu4Row &s0, Lu4Row &s1,
                                            bool all_dense, unsigned long long act_lanes, LUBuf4 &L) {
    if constexpr (I < NV) {
        const float v0 = __builtin_fabsf(a0[I].x) + __builtin_fabsf(a0[I].y);          // :55
        const float v1 = __builtin_fabsf(a1[I].x) + __builtin_fabsf(a1[I].y);
        const PivSel4 p = lu4_search<I>(v0, v1, s0.rowid, s1.rowid, all_dense, act_lanes);
        const bool piv = p.p0 || p.p1, sel = p.p1;
        // structural patterns of the pivot rows (wave-uniform union)
        const int ppat = (int)(sel ? s1.pat : s0.pat);
        uint32_t pu = 0u;
#pragma unroll
        for (int g = 0; g < 4; g++) {
            const unsigned long long f = p.t & (0xFFFFull << (16 * g));
            if (f != 0ull) pu |= (uint32_t)__builtin_amdgcn_readlane(ppat, __builtin_ctzll(f));
        }
        constexpr uint32_t FULL = 0xFFFFFFFFu << (I + 1);
        const uint32_t pmw = p.dense ? FULL : (pu & FULL);
        if (piv) {                                                 // pivot rows -> the group buffers
            lu4_put_row<I, 0>(a0, a1, sel, pmw, L);
            st4(&L.row[30], csel(sel, a0[I], a1[I]), csel(sel, b0, b1));
            L.pos = sel ? s1.rowid : s0.rowid;
        }
        wave_lds_sync();
        cf sxi, sB0;
        ld4(&L.row[30], sxi, sB0);
        const int piv_pos = L.pos;
        // 1 / pivot as cuCdivf(1, pivot) (:84); the pivot slot keeps the factors
        cf reg;
        divf f;
        if (__builtin_expect(!p.dense, 1)) {
            pf2 oo;
            const pf2 rg = recip_fast(pf2{sxi.x, sxi.y}, p.piv_abs, oo);
            reg = cmk(rg.x, rg.y);
            f.o1 = oo.x;
            f.o2 = oo.y;
        } else {
            f = cdiv_factors(sxi);
            reg = (p.piv_abs == 0.0f) ? cmk(1.0f, 0.0f) : cdiv_apply(cmk(1.0f, 0.0f), f);   // :66
        }
        if (p.p0) s0.my.oo = pf2{f.o1, f.o2};
        if (p.p1) s1.my.oo = pf2{f.o1, f.o2};
        asm volatile("" : "+v"(s0.my.oo), "+v"(s1.my.oo));
        if (p.p0) s0.rowid = I;                                    // :70-82
        else if (s0.rowid == I) s0.rowid = piv_pos;
        if (p.p1) s1.rowid = I;
        else if (s1.rowid == I) s1.rowid = piv_pos;
        const bool bl0 = s0.rowid > I && s0.rowid < NV, bl1 = s1.rowid > I && s1.rowid < NV;   // :86-93
        const uint32_t pmwd = p.dense ? 0xFFFFFFFFu : pmw;
        pf2 l0 = pf2{0.0f, 0.0f}, l1 = pf2{0.0f, 0.0f};
        if (bl0) {
            l0 = pcmul(pf2{a0[I].x, a0[I].y}, pf2{reg.x, reg.y});
            const pf2 t = pcmsub(pf2{b0.x, b0.y}, l0, pf2{sB0.x, sB0.y});
            b0 = cmk(t.x, t.y);
            s0.pat |= (((s0.pat >> I) & 1u) != 0u || p.dense) ? pmwd : 0u;
        }
        if (bl1) {
            l1 = pcmul(pf2{a1[I].x, a1[I].y}, pf2{reg.x, reg.y});
            const pf2 t = pcmsub(pf2{b1.x, b1.y}, l1, pf2{sB0.x, sB0.y});
            b1 = cmk(t.x, t.y);
            s1.pat |= (((s1.pat >> I) & 1u) != 0u || p.dense) ? pmwd : 0u;
        }
        if (bl0 || bl1) lu4_update<I, 0>(a0, a1, l0, l1, bl0, bl1, pmw, L);
        lu4_forward<I + 1>(a0, a1, b0, b1, s0, s1, all_dense, act_lanes, L);
    }
}

// back substitution (:97-106): the slot whose final rowid is I owns position
// I, divides with the factors kept from the forward step and publishes x_I in
// its group's buffer; rows above subtract
template <int I>
__device__ __forceinline__ void lu4_backward(const cf (&a0)[NV], const cf (&a1)[NV], cf &b0, cf &b1,
                                             const Lu4Row &s0, const Lu4Row &s1, LUBuf4 &L) {
    if constexpr (I >= 0) {
        const bool o0 = s0.rowid == I, o1 = s1.rowid == I;
        if (o0 || o1) {
            const PivF my{o1 ? s1.my.oo : s0.my.oo};
            const pf2 q = pcdiv_apply(psel(o1, b0, b1), psel(o1, a0[I], a1[I]), my);
            L.x[I] = cmk(q.x, q.y);
        }
        wave_lds_sync();
        const cf xi = L.x[I];
        if (s0.rowid < I) {
            const pf2 w = pcmsub(pf2{b0.x, b0.y}, pf2{xi.x, xi.y}, pf2{a0[I].x, a0[I].y});
            b0 = cmk(w.x, w.y);
        }
        if (s1.rowid < I) {
            const pf2 w = pcmsub(pf2{b1.x, b1.y}, pf2{xi.x, xi.y}, pf2{a1[I].x, a1[I].y});
            b1 = cmk(w.x, w.y);
        }
        lu4_backward<I - 1>(a0, a1, b0, b1, s0, s1, L);
    }
}

// Solves the system of each 16-lane group: lane q holds rows q (a0, b0) and
// q + 16 (a1, b1; q < 14) with their structural patterns.  Returns x_q in x0
// and x_{q+16} in x1.  act_groups: bit g set when group g holds a system (the
// others' data is ignored by the tie / range tests).  L: this group's buffer.
__device__ __forceinline__ void lu_solve4(cf (&a0)[NV], cf (&a1)[NV], cf b0, cf b1, int lane, uint32_t pat0,
                                          uint32_t pat1, unsigned act_groups, LUBuf4 &L, cf &x0, cf &x1) {
    const int q = lane & 15;
    const bool r1ok = q < NV - 16;
    // wave-uniform by contract; readfirstlane tells the compiler (a mask it
    // takes for divergent turns every pivot-step branch into an EXEC branch)
    const unsigned long long act_lanes = grp_lanes((unsigned)__builtin_amdgcn_readfirstlane((int)act_groups));
    bool ok = true;
#pragma unroll
    for (int c = 0; c < NV; c++) {
        ok = ok && __builtin_fabsf(a0[c].x) < 0x1p88f && __builtin_fabsf(a0[c].y) < 0x1p88f;
        ok = ok && (!r1ok || (__builtin_fabsf(a1[c].x) < 0x1p88f && __builtin_fabsf(a1[c].y) < 0x1p88f));
    }
    const bool all_dense = (__builtin_amdgcn_ballot_w64(!ok) & act_lanes) != 0ull;   // then every step is dense
    Lu4Row s0{q, pat0, PivF{pf2{0.0f, 0.0f}}};
    Lu4Row s1{r1ok ? q + 16 : 99, r1ok ? pat1 : 0u, PivF{pf2{0.0f, 0.0f}}};
    lu4_forward<0>(a0, a1, b0, b1, s0, s1, all_dense, act_lanes, L);
    lu4_backward<NV - 1>(a0, a1, b0, b1, s0, s1, L);
    x0 = L.x[q];
    x1 = L.x[r1ok ? q + 16 : 0];
}

}  // namespace hc
