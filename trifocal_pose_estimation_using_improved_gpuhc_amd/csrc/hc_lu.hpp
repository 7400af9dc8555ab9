// hc_lu.hpp -- the tracker's batched 30x30 complex LU solve, two systems per
// wavefront (one per 32-lane half; lane r owns row r in 60 VGPRs).
//
// Semantics: magmaHC/dev-cgesv-batched-small.cuh:38-107 -- partial pivoting
// on cabs1 = |re| + |im| with first-maximum ties (the pivot search scans the
// eligible positions in order with a strict '>'), rows relabelled through
// rowid instead of moved, a zero pivot skips the elimination with recip = 1,
// back substitution with cuCdivf.  Op for op the spec of DESIGN.md §4, up to
// the sign of exact zeros (the equivalence class DESIGN.md §4 documents).
//
// How one pivot step I runs (common path, both halves at once):
//  * search: key = bits of |re|+|im| (non-negative floats order like ints),
//    max over the half with 4 DPP steps + v_permlane16_swap, ballot of the
//    maxima.  NaN keys take part (positive NaN bits order above every finite
//    value); a maximum outside the fast reciprocal range (NaN, inf, zero,
//    tiny, huge) or a tie in either half sends the step to the exact rare
//    path (NaN at position I wins, first position among ties);
//  * 1/pivot: every lane computes cuCdivf(1, a_rI) of its own candidate
//    while the search runs (round 4: off the step's critical path), with
//    v_rcp_f32 + one Newton step, which is the IEEE quotient for s in
//    [2^-90, 2^120) (exhaustively verified, scripts/rcp_check.hip,
//    profiles/r1_rcp_check.json); the pivot lane's is the step's 1/pivot, and
//    it keeps the factors (o1, o2) for the back substitution;
//  * broadcast: the pivot lane writes 1/pivot (in the pivot element's slot),
//    rhs and rowid into its half's LDS buffer, every lane reads them back;
//  * one exec region of the eligible rows (the rows below and the pivot row,
//    whose multiplier is zero; round 5): multiplier, right-hand side and
//    fill-in pattern, then per column group (one uniform test) every eligible
//    lane writes the group of its row (ds_write_b128; the pivot lane to the
//    buffer, the others to their own scratch window) and reads the pivot
//    row's group back (broadcast ds_read_b128) and updates, 2 v_pk_fma_f32 per
//    element.  The abort kernel's latency mode also writes the pivot row's
//    1/pivot, rhs and rowid from every lane (no exec region at all).
//
// Structural sparsity.  The trifocal Jacobian is sparse (170 of 900 entries
// carry terms) and partial-pivot elimination fills it in only partly: on
// tracker Jacobians 64 % of the pivot-row entries a step broadcasts are exact
// zeros.  Each lane keeps the structural pattern of its row (bit c: column c
// may be non-zero) -- initially the columns with index terms, then OR-ed with
// the pivot rows' patterns whenever the row takes a multiple of one
// (fill-in).  A chunk of columns that is zero in both pivot rows of the wave
// is neither written, read nor used in the update (one uniform branch).
// Exactness: a structurally zero entry holds an exact zero while no product
// is infinite or NaN, and a - l*0 == a up to the sign of a zero.  Guarantees:
//  * the solve runs sparse only if every entry is finite with |re|, |im| <
//    2^64 (wave-uniform check on sums of squares; the argument below needs
//    2^88).  Pivoting on |re|+|im| bounds every multiplier by sqrt(2) and the
//    element growth by (1+sqrt(2))^29 < 2^37, so no intermediate can overflow;
//  * and only while every 1/pivot stays in the fast range (|pivot| < 2^-90:
//    1/pivot may overflow; zero or NaN pivot).
// Otherwise the sparse solve reports `redo` and the caller solves the rebuilt
// system with the dense instantiation (every column, the IEEE reciprocal):
// the reference algorithm step for step.  So the sparse steps carry no dense
// tests at all (a per-step `dense` flag cost ~12 SALU and 3 branches a step).
//
// The buffer is the path slot's SlotLDS::lu; the scratch windows are the dH/dx
// entry block (SlotLDS::ent), dead once gathered into the registers (a dense
// re-solve evaluates dH/dx again).
#pragma once

#include "hc_eval.hpp"

namespace hc {

typedef float f4v __attribute__((ext_vector_type(4)));

struct alignas(16) LUBuf {
    cf row[32];    // current pivot row: [0..29] A, [30] rhs, [31].x = rowid (int bits); x in the back sub
};
static_assert(sizeof(LUBuf) == sizeof(SlotLDS::lu), "LUBuf is SlotLDS::lu");
static_assert(offsetof(SlotLDS, lu) % 16 == 0, "SlotLDS::lu must be 16-B aligned");

// columns per skippable group (the template parameter CH below): 2, where the
// LDS stores of dead columns are what a wider group costs
// (profiles/r3u_ab_oo_rz_gs_chunk2.jsonl: 33.55 -> 31.78 ms per config-2
// launch).  The abort kernel used groups of 4 in two loops until round 5, for
// its lone-wave latency; groups of 2 in the eligible rows' region are as fast
// there, and its latency mode faster (profiles/r5j_ttfp_abort_lu_variants.jsonl,
// r5n_ttfp.jsonl)
constexpr int LU_CHUNK = 2;

// Correctly rounded 1/s for s in [2^-90, 2^120): v_rcp_f32 plus one Newton
// step (bit-identical to hipcc's div_scale / div_fmas / div_fixup sequence
// for every float in that range).
__device__ __forceinline__ float rcp_rn(float s) {
    const float r0 = __builtin_amdgcn_rcpf(s);
    const float e0 = __builtin_fmaf(-s, r0, 1.0f);
    return __builtin_fmaf(e0, r0, r0);
}
// s in the fast reciprocal range, on the bit pattern of a non-negative float
// (NaN and the -1 "no candidate" key fall outside)
__device__ __forceinline__ bool rcp_fast_bits(int bits) {
    return (uint32_t)(bits - 0x12800000) < (uint32_t)(0x7B800000 - 0x12800000);
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

// x & (c | c << 32) as two s_and_b32 with a literal (no 64-bit constant
// materialised in SGPRs)
template <uint32_t C>
__device__ __forceinline__ unsigned long long and_halves(unsigned long long x) {
    uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
    asm("s_and_b32 %0, %0, %2\n\ts_and_b32 %1, %1, %2" : "+s"(lo), "+s"(hi) : "i"(C) : "scc");
    return (unsigned long long)lo | ((unsigned long long)hi << 32);
}
// max over the DPP span of lu_search_span (4: half_max_int_p16)
template <int SPAN>
__device__ __forceinline__ int half_max_int_span(int v) {
    if constexpr (SPAN >= 4) {
        return half_max_int_p16(v);
    } else {
        v = max(v, dpp_i<DPP_QP_1032>(v));
        v = max(v, dpp_i<DPP_QP_2301>(v));
        if constexpr (SPAN >= 2) v = max(v, dpp_i<DPP_ROW_HALF_MIRROR>(v));
        if constexpr (SPAN >= 3) v = max(v, dpp_i<DPP_ROW_MIRROR>(v));
        return v;
    }
}

__device__ __forceinline__ int half_min_int_p16(int v) {
    v = min(v, dpp_i<DPP_QP_1032>(v));
    v = min(v, dpp_i<DPP_QP_2301>(v));
    v = min(v, dpp_i<DPP_ROW_HALF_MIRROR>(v));
    v = min(v, dpp_i<DPP_ROW_MIRROR>(v));
    const auto sw = __builtin_amdgcn_permlane16_swap((unsigned)v, (unsigned)v, false, false);
    return min((int)sw[0], (int)sw[1]);
}

// reciprocals (o1, o2) of the cuCdivf factors of the pivot a lane owns, kept
// from the forward step that chose it (brs, bis = pivot * o1 are recomputed
// from the pivot element, which stays in the owner's rA)
struct PivF { pf2 oo; };

// cuCdivf(1, y) for s = |y.re| + |y.im| in the fast range, in packed FP32 with
// the spec's ops: o1 = 1/s, (brs, bis) = y*o1, o2 = 1/(brs*brs + bis*bis),
// 1/y = ((o1*brs)*o2, (-(o1*bis))*o2); -(o1*bis) is computed as o1*(-bis)
// (IEEE: the same value).  oo returns (o1, o2).  (Computing o2 straight into
// the high half of o1's pair saves the pivot lane one move per step but
// raised the tracking kernel's spills from 11 to 53 VGPRs; round 6.)
__device__ __forceinline__ pf2 recip_fast(pf2 y, float s, pf2 &oo) {
    // o1 and o2 each in a pair of their own (low half), broadcast by op_sel:
    // no copy to place them side by side
    pf2 o1p, o2p, bb, sq, q, r;
    o1p.x = rcp_rn(s);
    asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[1,0]" : "=v"(bb) : "v"(y), "v"(o1p));
    asm("v_pk_mul_f32 %0, %1, %1" : "=v"(sq) : "v"(bb));
    o2p.x = rcp_rn(sq.x + sq.y);
    asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1] neg_hi:[0,1]" : "=v"(q) : "v"(o1p), "v"(bb));
    asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[1,0]" : "=v"(r) : "v"(q), "v"(o2p));
    oo.x = o1p.x;
    oo.y = o2p.x;
    return r;
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

// Column groups of step I: a leading single column when I+1 is odd, then
// groups of CH (even) columns.  The pivot lanes write, and the update reads,
// exactly these groups.
template <int CH>
struct LuChunks {
    static constexpr int single(int I) { return ((I + 1) & 1) && (I + 1 < NV) ? 1 : 0; }
    static constexpr int start(int I, int k) { return k < single(I) ? I + 1 : I + 1 + single(I) + (k - single(I)) * CH; }
    static constexpr int len(int I, int k) {
        return k < single(I) ? 1 : ((NV - start(I, k)) < CH ? (NV - start(I, k)) : CH);
    }
    static constexpr int count(int I) { return single(I) + (NV - (I + 1 + single(I)) + CH - 1) / CH; }
    static constexpr uint32_t mask(int I, int k) { return ((1u << len(I, k)) - 1u) << start(I, k); }
};

// The tracker's column groups by class (round 5).  The sparse LU tests a
// group live when a pivot row of the wave may be non-zero there; for this
// problem's Jacobian most outcomes are fixed in advance:
//  * dead: the symbolic fill-in bound -- at step I every row pattern is within
//    the row's bound cur[r], the pivot rows' within S_I = OR of the bounds of
//    the rows that may hold column I, and a row that may hold column I grows
//    by at most S_I -- has no column of the group: the test can never pass
//    (101 of the 225 groups of a solve);
//  * always: live in every one of the 1.2 M sampled wave-solves of datasets
//    000/001/002 (profiles/r5lv_live.jsonl; 16 of the 40 provably, from the
//    rows that must hold column I): no test, the update runs.  Running a group
//    that happens to be dead is exact: the pivot rows hold zeros there, and a
//    - l * 0 == a (up to the sign of a zero; l is finite in the sparse solve);
//  * tested: the other 84.
// Only the tracker's solves (STRUCT) use the classes: k_tables checks that the
// loaded problem's structural patterns lie within LU_STRUCT_PAT; the component
// LU (k_cgesv) takes any matrix and tests every group.
constexpr uint32_t LU_STRUCT_PAT[NV] = {
    0x7040004u, 0x7080004u, 0x7100004u, 0x7040009u, 0x7080009u, 0x7100009u, 0x7040012u, 0x7080012u,
    0x7100012u, 0x38200020u, 0x38400020u, 0x38800020u, 0x38200041u, 0x38400041u, 0x38800041u, 0x38200082u,
    0x38400082u, 0x38800082u, 0x7003100u, 0x7003100u, 0x7001100u, 0x7018400u, 0x7018400u, 0x7008400u,
    0x38005200u, 0x38005200u, 0x38001200u, 0x38028800u, 0x38028800u, 0x38008800u};
constexpr uint16_t LU_ALWAYS[NV] = {0x2000, 0x1000, 0x1800, 0xc00, 0xc00, 0xd00, 0xc00, 0x600, 0x304, 0x302,
                                    0x184,  0x182,  0x80,   0x60,  0xc0,  0x21,  0x30,  0x30,  0x18,  0,
                                    0,      0,      0,      0,     0,     0,     0,     0,     0,     0};
struct LuBound { uint32_t s[NV], cand[NV]; };   // cand[I]: the rows that may hold column I at step I
constexpr LuBound lu_struct_bound() {
    LuBound b{};
    uint32_t cur[NV] = {};
    for (int r = 0; r < NV; r++) cur[r] = LU_STRUCT_PAT[r];
    for (int i = 0; i < NV; i++) {
        const uint32_t above = (0xFFFFFFFFu << (i + 1)) & ((1u << NV) - 1u);
        uint32_t u = 0u;
        for (int r = 0; r < NV; r++)
            if ((cur[r] >> i) & 1u) { u |= cur[r]; b.cand[i] |= 1u << r; }
        b.s[i] = u & above;
        for (int r = 0; r < NV; r++)
            if ((cur[r] >> i) & 1u) cur[r] |= u & above;
    }
    return b;
}
constexpr LuBound LU_BOUND = lu_struct_bound();
enum : int { GRP_TESTED = 0, GRP_DEAD = 1, GRP_ALWAYS = 2 };
template <int CH>
constexpr int lu_group_class(int I, int K) {
    return (LU_BOUND.s[I] & LuChunks<CH>::mask(I, K)) == 0u ? GRP_DEAD
           : ((LU_ALWAYS[I] >> K) & 1u)                     ? GRP_ALWAYS
                                                              : GRP_TESTED;
}
// The pivot search of the tracker's step I need only reduce over the lanes
// (rows) that may hold column I: every other row's entry is an exact zero.
// Span of the DPP reduction that covers them: 1 a quad (two quad_perm
// steps), 2 a half-row (+ row_half_mirror), 3 a 16-lane row (+ row_mirror),
// 4 the half-wave (+ v_permlane16_swap).  Steps 0..17 need 1 to 3.
constexpr int lu_search_span(int I) {
    const uint32_t c = LU_BOUND.cand[I];
    if (c == 0u) return 4;
    int lo = 0, hi = 31;
    while (!((c >> lo) & 1u)) lo++;
    while (!((c >> hi) & 1u)) hi--;
    return (lo >> 2) == (hi >> 2) ? 1 : (lo >> 3) == (hi >> 3) ? 2 : (lo >> 4) == (hi >> 4) ? 3 : 4;
}
template <int CH>
constexpr bool lu_classes_consistent() {   // no measured-always group is provably dead
    for (int i = 0; i < NV - 1; i++)
        for (int k = 0; k < LuChunks<CH>::count(i); k++)
            if (((LU_ALWAYS[i] >> k) & 1u) && (LU_BOUND.s[i] & LuChunks<CH>::mask(i, k)) == 0u) return false;
    return true;
}
static_assert(lu_classes_consistent<2>(), "LU_ALWAYS names a provably dead group");

// Group tests on one bit: gbits = pmw | pmw >> 1 | pmw >> 2 | pmw >> 3, so bit J
// says "some column of J..J+3 may be non-zero" and a group test is s_bitcmp1
// + s_cbranch (the compiler keeps an s_cmp after a multi-bit s_and).
template <int CH>
__device__ __forceinline__ uint32_t group_bits(uint32_t pmw) {
    uint32_t t = pmw;
#pragma unroll
    for (int k = 1; k < CH; k++) t |= pmw >> k;
    return t;
}
template <int I, int K, int CH>
__device__ __forceinline__ bool group_live(uint32_t pmw, uint32_t gb) {
    using C = LuChunks<CH>;
    constexpr int J = C::start(I, K), N = C::len(I, K);
    if constexpr (N == 1) return (pmw >> J) & 1u;
    else return (gb >> J) & 1u;
}

#ifdef HC_DIAG_LUWORK
// diagnostic build: rank-1 update elements the solves execute (sum over the
// executed column groups of columns x active lanes), and the solves
// [0] executed elements, [1] completed sparse solves, [2] dense solves (path
// solves); wave-level: [3] sparse wave-solves, [4] live column groups, [5] rare
// pivot steps; [6..8] stages whose right-hand side ran the mixed / dH/dt-only /
// H-only evaluation, [9] stages that rebuilt the prefix tables (k_track)
constexpr int DIAG_LUWORK_WORDS = 10;
__device__ unsigned long long g_diag_luwork[DIAG_LUWORK_WORDS];
struct LuWork { unsigned long long acc, mask, groups, rare, excl; };   // mask: lanes whose work counts (active
                                                                      // path slots); excl: lanes that update by l = 0
#define HC_LU_WORK(ncols) (lu_work_acc.acc += (unsigned long long)(ncols) * \
    (unsigned long long)__builtin_popcountll(__builtin_amdgcn_read_exec() & lu_work_acc.mask & ~lu_work_acc.excl))
#define HC_LU_WORK_ARG , LuWork &lu_work_acc
#define HC_LU_WORK_PASS , lu_work_acc
#else
#define HC_LU_WORK(ncols) do { } while (0)
#define HC_LU_WORK_ARG
#define HC_LU_WORK_PASS
#endif

#ifdef HC_DIAG_PHASES
__device__ unsigned long long g_diag_lu_mid[65536];   // per (workgroup, wave): see lu_solve
#endif

#ifdef HC_DIAG_LIVE
// diagnostic build: how often each column group of each pivot step is live
// (wave-level test), sampled on every eighth workgroup: [I][K] live count,
// [I][LIVE_SOLVES] sparse wave-solves that reached step I
constexpr int LIVE_SOLVES = 16;
__device__ unsigned long long g_diag_live[NV][LIVE_SOLVES + 1];
#define HC_DIAG_LIVE_HIT(I, K) do { if (lane_fresh() == 0 && (blockIdx.x & 7u) == 0u) \
    atomicAdd(&g_diag_live[I][K], 1ull); } while (0)
#else
#define HC_DIAG_LIVE_HIT(I, K) do { } while (0)
#endif

// the column groups K.. of step I: one uniform test per group (round 4; the
// pivot row's stores and the update each tested every group before: 2.2 %
// faster, profiles/r4o_ab_fused_group_tests.jsonl); the pivot lanes write the
// group, the rows below read it back and take a_j -= l * u_j
template <int I, int K, int CH>
__device__ __forceinline__ void lu_store_update(cf (&rA)[NV], const cf &l, uint32_t pmw, uint32_t gb, LUBuf &L,
                                                bool is_piv, bool below HC_LU_WORK_ARG) {
    using C = LuChunks<CH>;
    if constexpr (K < C::count(I)) {
        constexpr int J = C::start(I, K), N = C::len(I, K);
        if (__builtin_expect(group_live<I, K, CH>(pmw, gb), 1)) {
            if (is_piv) {
                if constexpr (N == 1) {
                    L.row[J] = rA[J];
                } else {
#pragma unroll
                    for (int q = 0; q < N; q += 2) st4(&L.row[J + q], rA[J + q], rA[J + q + 1]);
                }
            }
            wave_lds_sync();
            if (below) {
                HC_LU_WORK(N);
#ifdef HC_DIAG_LUWORK
                lu_work_acc.groups++;
#endif
                cf u[N];
                if constexpr (N == 1) {
                    u[0] = L.row[J];
                } else {
#pragma unroll
                    for (int q = 0; q < N; q += 2) ld4(&L.row[J + q], u[q], u[q + 1]);
                }
#pragma unroll
                for (int q = 0; q < N; q++) {
                    const pf2 v = pcmsub(pf2{rA[J + q].x, rA[J + q].y}, pf2{l.x, l.y}, pf2{u[q].x, u[q].y});
                    rA[J + q] = cmk(v.x, v.y);
                }
            }
        }
        __builtin_amdgcn_sched_barrier(0);
        lu_store_update<I, K + 1, CH>(rA, l, pmw, gb, L, is_piv, below HC_LU_WORK_PASS);
    }
}

// The column groups K.. of step I inside the eligible rows' exec region (the
// rows below and the pivot row; round 5): one uniform test per group, then
// every eligible lane writes the group of its row -- the pivot lane to the
// pivot-row buffer, the others to their own 16-B window of a scratch area
// (wrow, chosen per step: row r's window for group J is scratch[2r + J], so
// one instruction's windows are disjoint), so the store needs no exec switch
// -- reads the pivot row's group back and takes a_j -= l * u_j.  The pivot
// lane has l = 0: its row is unchanged up to the sign of zeros (sparse solves
// only: every entry is finite there, so 0 * u is a zero).  A live group is
// one SALU test and one branch besides its store, read and FMAs; the round-4
// group (the pivot lane's store and the update of the rows below, each in its
// own exec region) took four more SALU and one more branch.
// (profiles/r5c_ab_lu_elig_groups.jsonl: config-2 launch -2.0 %, lone sample
// -5 %; a variant whose pivot row also went through a window, its address
// exchanged with 1/pivot, issued fewer instructions and ran 1 % slower,
// profiles/r5h_ab_lu_windows.jsonl.)
template <int I, int K, int CH, bool STRUCT, bool PAIRS = false>
__device__ __forceinline__ void lu_group_elig(cf (&rA)[NV], const pf2 &l, uint32_t pmw, uint32_t gb, cf *wrow,
                                              const LUBuf &L HC_LU_WORK_ARG) {
    using C = LuChunks<CH>;
    constexpr bool PAIR = PAIRS && STRUCT && K + 1 < C::count(I) && lu_group_class<CH>(I, K) == GRP_ALWAYS &&
                          lu_group_class<CH>(I, K + 1) == GRP_ALWAYS && C::len(I, K) == 2 && C::len(I, K + 1) == 2;
    if constexpr (PAIR) {
        // latency mode (the abort kernel): two always-live groups, both stores,
        // both reads, one wait (profiles/r5lp_ttfp_lat_pairs.jsonl: time to the
        // first pose -1.6 %; the tracking kernel measured 0.7 % slower with it,
        // three more VGPR spills: profiles/r5st_ab_lu_group_classes.jsonl, pr1)
        constexpr int J = C::start(I, K), J2 = C::start(I, K + 1);
        st4(&wrow[J], rA[J], rA[J + 1]);
        st4(&wrow[J2], rA[J2], rA[J2 + 1]);
        wave_lds_sync();
        HC_LU_WORK(4);
        HC_DIAG_LIVE_HIT(I, K);
        HC_DIAG_LIVE_HIT(I, K + 1);
#ifdef HC_DIAG_LUWORK
        lu_work_acc.groups += 2;
#endif
        cf u[4];
        ld4(&L.row[J], u[0], u[1]);
        ld4(&L.row[J2], u[2], u[3]);
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const int c = q < 2 ? J + q : J2 + q - 2;
            const pf2 v = pcmsub(pf2{rA[c].x, rA[c].y}, l, pf2{u[q].x, u[q].y});
            rA[c] = cmk(v.x, v.y);
        }
        __builtin_amdgcn_sched_barrier(0);
        lu_group_elig<I, K + 2, CH, STRUCT, PAIRS>(rA, l, pmw, gb, wrow, L HC_LU_WORK_PASS);
    } else if constexpr (K < C::count(I)) {
        constexpr int J = C::start(I, K), N = C::len(I, K);
        constexpr int CLS = STRUCT ? lu_group_class<CH>(I, K) : GRP_TESTED;
        if (CLS != GRP_DEAD && (CLS == GRP_ALWAYS || __builtin_expect(group_live<I, K, CH>(pmw, gb), 1))) {
            if constexpr (N == 1) {
                wrow[J] = rA[J];
            } else {
#pragma unroll
                for (int q = 0; q < N; q += 2) st4(&wrow[J + q], rA[J + q], rA[J + q + 1]);
            }
            wave_lds_sync();
            HC_LU_WORK(N);
            HC_DIAG_LIVE_HIT(I, K);
#ifdef HC_DIAG_LUWORK
            lu_work_acc.groups++;
#endif
            cf u[N];
            if constexpr (N == 1) {
                u[0] = L.row[J];
            } else {
#pragma unroll
                for (int q = 0; q < N; q += 2) ld4(&L.row[J + q], u[q], u[q + 1]);
            }
#pragma unroll
            for (int q = 0; q < N; q++) {
                const pf2 v = pcmsub(pf2{rA[J + q].x, rA[J + q].y}, l, pf2{u[q].x, u[q].y});
                rA[J + q] = cmk(v.x, v.y);
            }
        }
        __builtin_amdgcn_sched_barrier(0);
        lu_group_elig<I, K + 1, CH, STRUCT, PAIRS>(rA, l, pmw, gb, wrow, L HC_LU_WORK_PASS);
    }
}

// Batched latency mode (round 6; the abort kernel with the problem's structure,
// whose time to the first pose is a lone path's latency).  Every column group
// the fill-in bound leaves alive (124 of 225 per solve) runs without a test --
// a group that happens to be zero in the pivot row is exact, as for the
// always-live groups -- so a pivot step needs no pattern bookkeeping, and it
// makes ONE LDS round trip instead of one per live group: every lane writes
// 1/pivot, rhs, rowid and all those groups (the pivot lane into the buffer,
// the others into their scratch windows), then every lane reads them back
// together, then the eligible rows update.
#ifndef HC_LU_LATB
#define HC_LU_LATB 1
#endif
template <int CH>
struct LatCols {   // the columns of step I's live-able groups, packed in group order
    static constexpr int off(int I, int K) {
        int n = 0;
        for (int k = 0; k < K; k++)
            if (lu_group_class<CH>(I, k) != GRP_DEAD) n += LuChunks<CH>::len(I, k);
        return n;
    }
    static constexpr int total(int I) { return off(I, LuChunks<CH>::count(I)); }
};
template <int I, int K, int CH>
__device__ __forceinline__ void lat_store(const cf (&rA)[NV], cf *wrow) {
    using C = LuChunks<CH>;
    if constexpr (K < C::count(I)) {
        if constexpr (lu_group_class<CH>(I, K) != GRP_DEAD) {
            constexpr int J = C::start(I, K), N = C::len(I, K);
            if constexpr (N == 1) wrow[J] = rA[J];
            else st4(&wrow[J], rA[J], rA[J + 1]);
        }
        lat_store<I, K + 1, CH>(rA, wrow);
    }
}
// the groups whose packed columns start in [LO, HI) (a batch: its reads are
// issued together, its updates follow)
template <int I, int K, int CH, int LO, int HI, int M>
__device__ __forceinline__ void lat_load(cf (&u)[M], const LUBuf &L) {
    using C = LuChunks<CH>;
    if constexpr (K < C::count(I)) {
        constexpr int O = LatCols<CH>::off(I, K);
        if constexpr (lu_group_class<CH>(I, K) != GRP_DEAD && O >= LO && O < HI) {
            constexpr int J = C::start(I, K), N = C::len(I, K);
            if constexpr (N == 1) u[O - LO] = L.row[J];
            else ld4(&L.row[J], u[O - LO], u[O - LO + 1]);
        }
        lat_load<I, K + 1, CH, LO, HI>(u, L);
    }
}
template <int I, int K, int CH, int LO, int HI, int M>
__device__ __forceinline__ void lat_fma(cf (&rA)[NV], const pf2 &l, const cf (&u)[M]) {
    using C = LuChunks<CH>;
    if constexpr (K < C::count(I)) {
        constexpr int O = LatCols<CH>::off(I, K);
        if constexpr (lu_group_class<CH>(I, K) != GRP_DEAD && O >= LO && O < HI) {
            constexpr int J = C::start(I, K), N = C::len(I, K);
#pragma unroll
            for (int q = 0; q < N; q++) {
                const pf2 v = pcmsub(pf2{rA[J + q].x, rA[J + q].y}, l, pf2{u[O - LO + q].x, u[O - LO + q].y});
                rA[J + q] = cmk(v.x, v.y);
            }
        }
        lat_fma<I, K + 1, CH, LO, HI>(rA, l, u);
    }
}
// columns read in the step's first batch (with 1/pivot and rhs); the rest
// follow in batches of the same size: the lu_solve template parameter LAT
// (the abort kernel has 128 VGPRs: 8, profiles/r6c_ttfp_ab_latb_cols.jsonl)
#ifndef HC_LU_LATB_COLS
#define HC_LU_LATB_COLS 8
#endif
template <int I, int LO, int CH, int B>
__device__ __forceinline__ void lat_batches(cf (&rA)[NV], const pf2 &l, const LUBuf &L) {
    constexpr int T = LatCols<CH>::total(I);
    if constexpr (LO < T) {
        constexpr int HI = LO + B;
        cf u[B + 1];
        lat_load<I, 0, CH, LO, HI>(u, L);
        lat_fma<I, 0, CH, LO, HI>(rA, l, u);
        lat_batches<I, HI, CH, B>(rA, l, L);
    }
}

// The rest of pivot step I once the pivots are chosen: broadcast, relabel,
// 1/pivot, update.  DENSE (the whole solve of a matrix that is not provably
// finite or that met a pivot outside the fast reciprocal range): every column
// group and the IEEE reciprocal.  The sparse solve carries no dense tests: it
// reports such a solve, and the caller solves the system again densely.
template <int I, bool DENSE, int CH, int LAT, bool STRUCT>
__device__ __forceinline__ void lu_step_body(cf (&rA)[NV], cf &rB, int &rowid, uint32_t &pat, PivF &my, LUBuf &L,
                                             cf *scr, bool is_piv, int pl0, int pl1, pf2 reg_s, pf2 oo_s,
                                             bool elig HC_LU_WORK_ARG) {
    if constexpr (HC_LU_LATB && LAT > 0 && STRUCT && CH == 2 && !DENSE) {
        HC_ISA_MARK_I("lu_store", I);
        cf *wrow = is_piv ? L.row : scr;
        wrow[I] = cmk(reg_s.x, reg_s.y);
        st4(&wrow[30], rB, cmk(__int_as_float(rowid), 0.0f));
        lat_store<I, 0, CH>(rA, wrow);
        wave_lds_sync();
        HC_ISA_MARK_I("lu_rcp", I);
        // (the pivot lane reading an exact zero from a zero slot instead, so that
        // its multiplier needs no selects, issued fewer instructions and measured
        // no faster: profiles/r6f_ttfp_ab_zero_slot.jsonl)
        const cf reg = L.row[I];
        cf sB0, pr;
        ld4(&L.row[30], sB0, pr);
        cf u[LAT + 1];
        lat_load<I, 0, CH, 0, LAT>(u, L);
        const int piv_pos = __float_as_int(pr.x);
        rowid = is_piv ? I : (rowid == I ? piv_pos : rowid);   // :70-82
        my.oo.x = is_piv ? oo_s.x : my.oo.x;
        my.oo.y = is_piv ? oo_s.y : my.oo.y;
        asm volatile("" : "+v"(my.oo));
        HC_ISA_MARK_I("lu_update", I);
        if (elig) {   // the rows below and the pivot row (multiplier 0: unchanged up to the sign of zeros)
            HC_ISA_MARK_I("lu_mult", I);
            const pf2 lq = pcmul(pf2{rA[I].x, rA[I].y}, pf2{reg.x, reg.y});
            const pf2 lp = {is_piv ? 0.0f : lq.x, is_piv ? 0.0f : lq.y};
            const pf2 bp = pcmsub(pf2{rB.x, rB.y}, lp, pf2{sB0.x, sB0.y});
            rB = cmk(bp.x, bp.y);
            lat_fma<I, 0, CH, 0, LAT>(rA, lp, u);
            lat_batches<I, LAT, CH, LAT>(rA, lp, L);
        }
        return;
    }
    constexpr uint32_t FULL = 0xFFFFFFFFu << (I + 1);
    uint32_t pmw = FULL;
    if constexpr (!DENSE) {
        // structural patterns of the two pivot rows (wave-uniform)
        const uint32_t pp0 = (uint32_t)__builtin_amdgcn_readlane((int)pat, pl0);
        const uint32_t pp1 = (uint32_t)__builtin_amdgcn_readlane((int)pat, pl1);
        pmw = (pp0 | pp1) & FULL;
    }
    const uint32_t gb = group_bits<CH>(pmw);
    HC_ISA_MARK_I("lu_store", I);
    // latency mode (LAT, the abort kernel): every lane writes, the pivot lane to
    // the buffer, the others to their scratch windows -- no exec region, at the
    // price of LDS bandwidth (profiles/r5m_ab_lu_x.jsonl: lone sample -2 %,
    // loaded launch +0.8 %)
    constexpr bool X1 = LAT > 0 && CH == 2 && !DENSE;
    cf *wrow = nullptr;
    if constexpr (X1) {
        wrow = is_piv ? L.row : scr;
        wrow[I] = cmk(reg_s.x, reg_s.y);
        st4(&wrow[30], rB, cmk(__int_as_float(rowid), 0.0f));
    } else if (is_piv) {                                   // pivot row -> buffer, 1/pivot in the pivot's slot
        L.row[I] = cmk(reg_s.x, reg_s.y);
        L.row[30] = rB;
        L.row[31].x = __int_as_float(rowid);
    }
    wave_lds_sync();
    HC_ISA_MARK_I("lu_rcp", I);
    const cf reg = L.row[I];
    cf sB0, pr;
    ld4(&L.row[30], sB0, pr);
    const int piv_pos = __float_as_int(pr.x);
    if constexpr (X1) {
        rowid = is_piv ? I : (rowid == I ? piv_pos : rowid);   // :70-82
        my.oo.x = is_piv ? oo_s.x : my.oo.x;
        my.oo.y = is_piv ? oo_s.y : my.oo.y;
    } else {
        if (is_piv) rowid = I;                                 // :70-82
        else if (rowid == I) rowid = piv_pos;
        // the pivot lane keeps its factors (computed in the search, lu_forward)
        if (is_piv) my.oo = oo_s;
    }
    // opaque: the select chain must be resolved here, not carried as 30
    // per-step factor pairs into the back substitution
    asm volatile("" : "+v"(my.oo));
    // :86-93: rowid > I after the relabel, i.e. an eligible row that is not the
    // pivot (the displaced row takes the pivot's old id > I); known from the
    // search, so the exec region does not wait for the read-back (padding lanes,
    // never eligible, stay out: their rows are not part of the system)
    const bool below = elig && !is_piv;
    // one exec-masked region per step: multiplier, right-hand side,
    // fill-in pattern (branch-free) and the rank-1 update.  Fill-in: a row
    // below whose column I may be non-zero takes the pivot patterns (both
    // halves': a superset of its own pivot row's).
    if constexpr (CH == 2 && !DENSE) {
        // the multiplier, right-hand side and fill-in pattern in the eligible
        // rows' region too (the pivot lane's multiplier is zeroed: its rhs and
        // row stay, up to the sign of zeros), one exec region per step
        // (profiles/r5m_ab_lu_x.jsonl: -0.4 %, lone sample -1.5 %)
        HC_ISA_MARK_I("lu_update", I);
        if constexpr (!X1) wrow = is_piv ? L.row : scr;
#ifdef HC_DIAG_LUWORK
        lu_work_acc.excl = __builtin_amdgcn_ballot_w64(is_piv);
#endif
        HC_DIAG_LIVE_HIT(I, LIVE_SOLVES);
        if (elig) {
            HC_ISA_MARK_I("lu_mult", I);
            // (the pivot lane's multiplier is zeroed by two selects: reading an
            // exact zero from a zero slot instead held one more address in a VGPR
            // across the solve: 11 -> 20 spills; round 6)
            const pf2 lq = pcmul(pf2{rA[I].x, rA[I].y}, pf2{reg.x, reg.y});
            const pf2 lp = {is_piv ? 0.0f : lq.x, is_piv ? 0.0f : lq.y};
            const pf2 bp = pcmsub(pf2{rB.x, rB.y}, lp, pf2{sB0.x, sB0.y});
            rB = cmk(bp.x, bp.y);
            pat |= (uint32_t)__builtin_amdgcn_sbfe((int)pat, I, 1) & pmw;
            lu_group_elig<I, 0, CH, STRUCT, (LAT > 0)>(rA, lp, pmw, gb, wrow, L HC_LU_WORK_PASS);
        }
        return;
    }
    pf2 lp = {0.0f, 0.0f};
    if (below) {
        HC_ISA_MARK_I("lu_mult", I);
        lp = pcmul(pf2{rA[I].x, rA[I].y}, pf2{reg.x, reg.y});
        const pf2 bp = pcmsub(pf2{rB.x, rB.y}, lp, pf2{sB0.x, sB0.y});
        rB = cmk(bp.x, bp.y);
        // v_bfe_i32 + v_and_or_b32
        if constexpr (!DENSE) pat |= (uint32_t)__builtin_amdgcn_sbfe((int)pat, I, 1) & pmw;
    }
    HC_ISA_MARK_I("lu_update", I);
    // the dense re-solve: one test per group for the pivot lane's store and the
    // update of the rows below (round 4; the dense steps may hold inf and NaN,
    // so the pivot row cannot take a zero multiplier there)
    lu_store_update<I, 0, CH>(rA, cmk(lp.x, lp.y), pmw, gb, L, is_piv, below HC_LU_WORK_PASS);
}

// One pivot step: the pivot search, then lu_step_body.  !DENSE: a pivot
// outside the fast reciprocal range sets `redo` (the solve goes on with
// garbage, the caller discards it and solves densely).
template <int I, bool DENSE, int CH, int LAT, bool STRUCT>
__device__ __forceinline__ void lu_forward(cf (&rA)[NV], cf &rB, int &rowid, uint32_t &pat, int lane, int r, int hb,
                                           bool row_lane, PivF &my, LUBuf &L, cf *scr, bool &redo,
                                           unsigned long long elig_m HC_LU_WORK_ARG) {
    if constexpr (I < NV) {
        HC_ISA_MARK_I("lu_search", I);
        const float v = __builtin_fabsf(rA[I].x) + __builtin_fabsf(rA[I].y);          // :55
        // 1 / own candidate as cuCdivf(1, a_rI) (:66, :84), off the step's critical path:
        // the pivot lane's is the step's 1/pivot (same ops on the same value)
        pf2 reg_s, oo_s;
        if constexpr (!DENSE) {
            reg_s = recip_fast(pf2{rA[I].x, rA[I].y}, v, oo_s);
        } else {
            const divf f = cdiv_factors(rA[I]);
            const cf rg = (v == 0.0f) ? cmk(1.0f, 0.0f) : cdiv_apply(cmk(1.0f, 0.0f), f);
            reg_s = pf2{rg.x, rg.y};
            oo_s = pf2{f.o1, f.o2};
        }
        // eligible rows (not pivoted yet; :86-93), carried from the previous
        // step as a lane mask, elig & ~pivots (SALU), instead of a rowid
        // compare after the relabel (profiles/r5e1_ab_lu_elig_carry.jsonl: -0.6 %)
        const bool elig = __builtin_amdgcn_inverse_ballot_w64(elig_m);
        bool is_piv;
        float piv_abs;
        int pl0, pl1;   // pivot lanes of the two halves
        unsigned long long piv_m;   // the two pivot lanes
        // the tracker's steps 0..17 reduce over the candidate rows' quad,
        // half-row or row only (lu_search_span): every other row's entry is an
        // exact zero (key 0, or -1 when not eligible), so the candidates'
        // group holds the maximum whenever it is a fast-range (positive) key,
        // and the ballots keep the candidate lanes only (other groups match
        // their own maxima).  bad == 0 then means each half's maximum is a
        // candidate's, so popcount(m) == 2 is still one pivot per half.
        constexpr int SPAN = (STRUCT && !DENSE) ? lu_search_span(I) : 4;
        const int key = elig ? __float_as_int(v) : -1;
        const int mx = half_max_int_span<SPAN>(key);
        unsigned long long m = __builtin_amdgcn_ballot_w64(key == mx);
        unsigned long long bad = __builtin_amdgcn_ballot_w64(!rcp_fast_bits(mx));
        if constexpr (SPAN < 4) {
            m = and_halves<LU_BOUND.cand[I]>(m);
            bad = and_halves<LU_BOUND.cand[I]>(bad);
        }
        const unsigned mlo = (unsigned)m, mhi = (unsigned)(m >> 32);
        // common: one maximum per half (two in the wave; s_bcnt1, where the
        // per-half m & (m - 1) tests took six SALU), both in the fast range
        // the pivot steps where exact ties are frequent on this problem's Jacobians
        // (steps 18, 19, 21, 22: 79, 29, 51, 32 % of solves) resolve them inline
        // with one more half-wave min reduction (lowest row id among the maxima)
        // instead of taking the rare path (profiles/r4f_ab_trims.jsonl)
        constexpr bool TIE = I == 18 || I == 19 || I == 21 || I == 22;
        const bool rare = DENSE || (TIE ? (bad != 0ull) : ((__builtin_popcountll(m) != 2) | (bad != 0ull)));
        if (__builtin_expect(rare, 0)) {
            HC_ISA_MARK_I("lu_rare", I);
#ifdef HC_DIAG_LUWORK
            lu_work_acc.rare++;
#endif
            // rare: NaN at position I wins (:57-64); exact ties: first position wins
            const bool isn = v != v;
            const unsigned long long nanb = __builtin_amdgcn_ballot_w64(isn);
            // the maximum over the non-NaN candidates: the first search's unless
            // some lane holds a NaN (ties and out-of-range pivots need no second
            // reduction) or the search was narrowed to the candidate rows
            int mx2 = mx;
            unsigned long long m2 = m;
            if constexpr (SPAN < 4) {
                mx2 = half_max_int_p16(key);
                m2 = __builtin_amdgcn_ballot_w64(key == mx2);
            }
            if (__builtin_expect(nanb != 0ull, 0)) {
                const int key2 = (elig && !isn) ? __float_as_int(v) : -1;
                mx2 = half_max_int_p16(key2);
                m2 = __builtin_amdgcn_ballot_w64(key2 == mx2);
            }
            const unsigned long long nanm = nanb & __builtin_amdgcn_ballot_w64(rowid == I);
            const unsigned nlo = (unsigned)nanm, nhi = (unsigned)(nanm >> 32);
            const unsigned mine_m = hb ? (unsigned)(m2 >> 32) : (unsigned)m2, mine_n = hb ? nhi : nlo;
            const int c2 = ((mine_m >> r) & 1u) ? rowid : (1 << 20);
            const int mn = half_min_int_p16(c2);
            const unsigned long long w = __builtin_amdgcn_ballot_w64(row_lane && rowid == mn);
            const unsigned wm = hb ? (unsigned)(w >> 32) : (unsigned)w;
            const int pl = mine_n ? hb + __builtin_ctz(mine_n) : hb + (wm ? __builtin_ctz(wm) : 0);
            is_piv = lane == pl;
            piv_abs = mine_n ? __builtin_nanf("") : __int_as_float(mx2);
            const unsigned long long pm = __builtin_amdgcn_ballot_w64(is_piv);
            piv_m = pm;
            pl0 = __builtin_ctz((unsigned)pm | 0x80000000u);
            pl1 = 32 + __builtin_ctz((unsigned)(pm >> 32) | 0x80000000u);
            if constexpr (!DENSE)
                redo = redo || __builtin_amdgcn_ballot_w64(!rcp_fast_bits(__float_as_int(piv_abs))) != 0ull;
        } else if constexpr (TIE) {
            // first position (lowest row id) among each half's maxima
            const int c2 = key == mx ? rowid : (1 << 20);
            const int mn = half_min_int_p16(c2);
            is_piv = key == mx && rowid == mn;
            piv_abs = __int_as_float(mx);
            const unsigned long long w = __builtin_amdgcn_ballot_w64(is_piv);
            piv_m = w;
            pl0 = __builtin_ctz((unsigned)w);
            pl1 = 32 + __builtin_ctz((unsigned)(w >> 32));
        } else {
            // (the narrowed search: only the candidate lanes' matches count)
            is_piv = __builtin_amdgcn_inverse_ballot_w64(m);   // (one bit per half: m is the pivot mask)
            piv_m = m;
            piv_abs = __int_as_float(mx);
            pl0 = __builtin_ctz(mlo);        // exactly one bit per half here
            pl1 = 32 + __builtin_ctz(mhi);
        }
        HC_ISA_MARK_I("lu_pattern", I);
        lu_step_body<I, DENSE, CH, LAT, STRUCT>(rA, rB, rowid, pat, my, L, scr, is_piv, pl0, pl1, reg_s, oo_s,
                                                elig HC_LU_WORK_PASS);
        lu_forward<I + 1, DENSE, CH, LAT, STRUCT>(rA, rB, rowid, pat, lane, r, hb, row_lane, my, L, scr, redo,
                                                  elig_m & ~piv_m HC_LU_WORK_PASS);
    }
}

// back substitution (:97-106): the lane whose final rowid is I owns position I
// and divides with the factors it kept from the forward step; x_I reaches the
// lanes of its half with v_readlane (owner lane of each half found by a
// ballot of the final row ids), and lanes I and 32 + I -- which return x_I --
// capture it with one exec-masked move (static lanes: no compare, no select,
// no LDS redistribution at the end).  The owner's rB is final at its step
// (every step J > I has updated it) and dead after it, so the later steps
// J < I may update it unmasked.
template <int I>
__device__ __forceinline__ void lu_backward(const cf (&rA)[NV], cf &rB, int rowid, const PivF &my, pf2 &res) {
    if constexpr (I >= 0) {
        HC_ISA_MARK_I("lu_back", I);
        const unsigned long long own = __builtin_amdgcn_ballot_w64(rowid == I);
        const int o0 = __builtin_ctz((unsigned)own);          // one owner per half
        const int o1 = 32 + __builtin_ctz((unsigned)(own >> 32));
        const pf2 q = pcdiv_apply(pf2{rB.x, rB.y}, pf2{rA[I].x, rA[I].y}, my);
        const float x0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(q.x), o0));
        const float y0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(q.y), o0));
        const float x1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(q.x), o1));
        const float y1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(q.y), o1));
        // x_I of each half from its SGPR pair: one v_mov_b64 for all lanes, one
        // more with the low half masked off, one into res of lanes I, 32 + I
        // (exec saved and restored)
        const pf2 xs0 = {x0, y0}, xs1 = {x1, y1};
        pf2 xv;
        unsigned long long tmp;
        asm volatile("s_nop 1\n\ts_mov_b64 %2, exec\n\tv_mov_b64 %0, %3\n\ts_mov_b32 exec_lo, 0\n\t"
                     "v_mov_b64 %0, %4\n\ts_mov_b32 exec_lo, %5\n\ts_mov_b32 exec_hi, %5\n\t"
                     "v_mov_b64 %1, %0\n\ts_mov_b64 exec, %2"
                     : "=&v"(xv), "+v"(res), "=&s"(tmp) : "s"(xs0), "s"(xs1), "i"(1u << I));
        // rows above position I take b -= x_I * a_I; the update runs unmasked
        // (no compare, no exec region): the rows at or below I are solved, so
        // their rB is dead (profiles/r3aa_ab_backsub_unmasked.jsonl)
        if constexpr (I > 0) {
            const pf2 w = pcmsub(pf2{rB.x, rB.y}, xv, pf2{rA[I].x, rA[I].y});
            rB = cmk(w.x, w.y);
        }
        lu_backward<I - 1>(rA, rB, rowid, my, res);
    }
}

// Solves the system of each half: lane r holds row r of A in rA and b_r in
// rB; pattern = the structural pattern of row r.  Returns x_r in lane r.  L is
// this half's buffer (16-B aligned).  DENSE = false: the structurally sparse
// solve, which sets `redo` (wave-uniform) instead of handling a matrix that is
// not provably finite or a pivot outside the fast reciprocal range: the
// caller then rebuilds the system and calls the DENSE solve, the reference
// algorithm step for step (both exact).
// scratch: this half's LU_SCRATCH_CF entries (16-B aligned) that the sparse
// solve with groups of 2 may overwrite: the store windows of the eligible
// rows (row r writes column group J at scratch[2r + J]); the caller's data
// there is lost.
constexpr int LU_SCRATCH_CF = 2 * 31 + 32;   // 94: lane r's window scratch[2r .. 2r + 31]
template <bool DENSE, int CH = LU_CHUNK, int LAT = 0, bool STRUCT = false>
__device__ __forceinline__ cf lu_solve(cf (&rA)[NV], cf rB, int lane, uint32_t pattern, LUBuf &L, cf *scratch,
                                      bool &redo, unsigned long long count_mask = ~0ull);
template <bool DENSE, int CH, int LAT, bool STRUCT>
__device__ __forceinline__ cf lu_solve(cf (&rA)[NV], cf rB, int lane, uint32_t pattern, LUBuf &L, cf *scratch,
                                      bool &redo, unsigned long long count_mask) {
    static_assert(CH == 2, "column groups of 2 (the scratch windows are 16 B)");
    (void)count_mask;   // diagnostic builds (HC_DIAG_LUWORK): lanes whose executed work is counted
    const int r = lane & 31, hb = lane & 32;
    const bool row_lane = r < NV;
    redo = false;
    if constexpr (DENSE) HC_ISA_MARK("lu_dense");   // (scripts/isa_phases.py: the dense re-solve's copy)
    else HC_ISA_MARK("lu_sparse");
    HC_ISA_MARK("lu_finite");
    if constexpr (!DENSE) {
        // every entry finite and below 2^64 in magnitude (inside the 2^88 the
        // sparse path needs): the per-component sums of squares (v_pk_fma_f32, 30
        // VALU) stay finite only then -- NaN propagates, an inf or |entry| >= 2^64
        // makes a square overflow.  A sum that overflows from many entries below
        // 2^64 only sends the solve to the dense path, which is exact as well.
        pf2 sq = {0.0f, 0.0f};
#pragma unroll
        for (int c = 0; c < NV; c++) {
            const pf2 e = {rA[c].x, rA[c].y};
            asm("v_pk_fma_f32 %0, %1, %1, %0" : "+v"(sq) : "v"(e));
        }
        const bool ok = sq.x + sq.y < __builtin_inff();
        if (__builtin_expect(__builtin_amdgcn_ballot_w64(!ok) != 0ull, 0)) {
            redo = true;
            return cmk(0.0f, 0.0f);
        }
    }
    int rowid = row_lane ? r : 99;   // padding lanes never pivot
    uint32_t pat = row_lane ? pattern : 0u;
    PivF my{pf2{0.0f, 0.0f}};
#ifdef HC_DIAG_LUWORK
    LuWork lu_work_acc{0ull, count_mask, 0ull, 0ull, 0ull};
    lu_forward<0, DENSE, CH, LAT, STRUCT>(rA, rB, rowid, pat, lane, r, hb, row_lane, my, L, scratch + 2 * r, redo,
                                          __builtin_amdgcn_ballot_w64(row_lane), lu_work_acc);
    const unsigned long long solves = (unsigned long long)__builtin_popcountll(count_mask & __builtin_amdgcn_ballot_w64(row_lane)) / NV;
    if (lane == 0 && !DENSE && !redo) {   // sparse solves that completed, and their work
        atomicAdd(&g_diag_luwork[0], lu_work_acc.acc);
        atomicAdd(&g_diag_luwork[1], solves);
        atomicAdd(&g_diag_luwork[3], 1ull);
        atomicAdd(&g_diag_luwork[4], lu_work_acc.groups);
        atomicAdd(&g_diag_luwork[5], lu_work_acc.rare);
    }
    if (lane == 0 && DENSE) atomicAdd(&g_diag_luwork[2], solves);   // dense (re-)solves
#else
    lu_forward<0, DENSE, CH, LAT, STRUCT>(rA, rB, rowid, pat, lane, r, hb, row_lane, my, L, scratch + 2 * r, redo,
                                          __builtin_amdgcn_ballot_w64(row_lane));
#endif
#ifdef HC_DIAG_PHASES
    // diagnostic build: the forward / back-substitution boundary of this wave's
    // solve (s_memtime), read by k_track after the solve (g_diag_lu_mid)
    if ((lane & 63) == 0 && blockIdx.x < 16384u) g_diag_lu_mid[blockIdx.x * 4 + (threadIdx.x >> 6)] = __builtin_amdgcn_s_memtime();
#endif
    // lane r returns x_r (captured at back-substitution step r; padding lanes 0)
    HC_ISA_MARK("lu_back_init");
    pf2 res = {0.0f, 0.0f};
    lu_backward<NV - 1>(rA, rB, rowid, my, res);
    return cmk(res.x, res.y);
}

}  // namespace hc
