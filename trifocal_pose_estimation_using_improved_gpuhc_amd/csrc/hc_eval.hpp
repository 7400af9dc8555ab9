// hc_eval.hpp -- polynomial evaluation of the two-paths-per-wave tracker.
//
// Same terms, same operation order as the reference and the oracle:
// gpu-idx-evals/dev-eval-indxing-trifocal_2op1p_30x30_LimUnroll_L2Cache.cuh
// :57-88 (dH/dx), :91-119 (dH/dt), :122-148 (H).  Lane r of a half-wave
// evaluates equation row r of its path from compacted per-row term lists:
//
//  * term words carry LDS byte offsets relative to the path slot (SlotLDS), so
//    an operand address is one add (prefix offsets in 16-bit halves, x
//    offsets in bytes) instead of shift + mask + add;
//  * prefix tables (round 4): a term's parameter part depends only on its
//    (coef, a, b) -- (c * p[a]) * p[b] for dH/dx and H, c * (d[a]*p[b] +
//    d[b]*p[a]) for dH/dt -- and p(t) changes only with t, so each slot keeps
//    the 93 distinct (c * p[a]) * p[b] and the 38 distinct d[a]*p[b] +
//    d[b]*p[a] of this problem in LDS (SlotLDS::tp, qp), rebuilt by
//    build_prefixes when its t or sample changes (about 0.4 times per stage),
//    and a term reads its prefix instead of two or four parameters: the same
//    operations on the same values, so the results are bit-identical;
//  * the complex products use packed FP32 (v_pk_mul_f32 / v_pk_fma_f32): two
//    instructions per complex multiply / multiply-add, each component computed
//    by the same fma chain as the scalar spec;
//  * no per-term select: a lane's padding terms come after its last real term
//    and use coef 0 with p[33] = x[30] = 1, so they add exact zeros to a +0
//    accumulator (dH/dx) or to the finished sum (dH/dt, H; the reference also
//    evaluates its padding terms);
//  * dH/dx terms are grouped by entry into slots of fixed capacity (below), so
//    every entry ends at a compile-time term position on every lane; the
//    entries are packed over all 32 lanes of a half (any lane may compute any
//    row's entry), not one row per lane.
#pragma once

#include <stddef.h>

#include "hc_slot.hpp"

namespace hc {

typedef float pf2 __attribute__((ext_vector_type(2)));

// dH/dx terms grouped by entry.  A Jacobian entry (one row, one column: the
// sum of its 1..8 terms, in table order) is computed by one lane of the half
// in one of its entry slots; slot s holds at most HX_GCAP[s] terms.  Since
// every lane stores its slot s at the same compile-time term position, the
// term loop has one store per slot (no per-term address or reset selects);
// shorter entries are padded with coefficient-0 terms on unit operands
// (p[33] = x[30] = 1), as the reference pads its 8-term lists.  The 170
// entries of this problem (12 x 8, 8 x 6, 36 x 5, 4 x 4, 54 x 3, 56 x 1
// terms) are bin-packed by k_prep_tables over all 32 lanes, so the loop is
// 21 terms long (8 + 5 + 3 + 3 + 1 + 1) instead of the 25 that one row per
// lane needs (rows of 11 to 23 terms in slots of 8, 5, 5, 5, 1, 1).  An entry
// goes to its row's block in SlotLDS::ent at the byte offset the lane's
// destination word holds for that slot (unused slots: the LU buffer's last
// word, which the LU rewrites before it reads it).
constexpr int HX_GCAP[6] = {8, 5, 3, 3, 1, 1};
constexpr int HX_SLOT_CAP = 21;
constexpr int HX_NSLOT = 6;
__host__ __device__ constexpr int hx_gend(int s) { return s < 0 ? 0 : hx_gend(s - 1) + HX_GCAP[s]; }   // end of slot s
__host__ __device__ constexpr bool hx_is_gend(int k) {
    return k + 1 == hx_gend(0) || k + 1 == hx_gend(1) || k + 1 == hx_gend(2) || k + 1 == hx_gend(3) ||
           k + 1 == hx_gend(4) || k + 1 == hx_gend(5);
}
__host__ __device__ constexpr int hx_gslot(int k) {
    return k < hx_gend(0) ? 0 : k < hx_gend(1) ? 1 : k < hx_gend(2) ? 2 : k < hx_gend(3) ? 3 : k < hx_gend(4) ? 4 : 5;
}
static_assert(hx_gend(5) == HX_SLOT_CAP, "slot capacities");
constexpr int SLOT_OFF_X = (int)offsetof(SlotLDS, x);
constexpr int SLOT_OFF_ENT = (int)offsetof(SlotLDS, ent);
constexpr int SLOT_OFF_ENTZERO = SLOT_OFF_ENT + 8 * (ENT_CAP - 1);        // the structural zero
// while the prefixes are built, p(t) is staged in ent[0..33] and the diff
// params in ent[34..67] (the entries are rewritten by the stage's dH/dx)
constexpr int SLOT_OFF_STG = SLOT_OFF_ENT;
constexpr int SLOT_STG_DIF_DELTA = 8 * NPP;
constexpr int SLOT_OFF_TP = (int)offsetof(SlotLDS, tp);
constexpr int SLOT_OFF_QP = (int)offsetof(SlotLDS, qp);
constexpr int SLOT_OFF_HXDUMMY = (int)offsetof(SlotLDS, lu) + 8 * 31;   // unused entry / prefix slots store here
static_assert(SLOT_OFF_QP + 8 * QP_CAP < 65536 && SLOT_OFF_HXDUMMY < 65536, "slot offsets must fit 16 bits");
static_assert(SLOT_OFF_X + 8 * 31 < 256, "x offsets must fit a byte");
static_assert(2 * NPP <= ENT_CAP - 1, "the staging area lies below the structural zero");

// Compacted tables, built by k_prep_tables from the reference's padded
// unified index (Data_Reader.cpp:167-189) and kept in the workspace.
//  gm[q][r]   (row r): SlotLDS byte offsets of row r's entries in columns 2q
//             (bits 0..15) and 2q+1 (bits 16..31); the structural zero for
//             columns without terms
//  pat[r]     structural pattern of row r (bit c: column c has terms)
//  hx[k][l]   (lane l's k-th dH/dx term, entry slot hx_gslot(k)):
//             off(tp[i]) | off(x[u]) << 16 | off(x[v]) << 24, i = its (c, a, b)
//  hxd[q][l]  (lane l): SlotLDS byte offsets its slots 2q (bits 0..15) and 2q+1 (bits 16..31) store to
//  ht[j][r]   (row r's j-th dH/dt / H term): .x = off(tp[i]) | off(qp[m]) << 16, i its (c, a, b), m its (a, b)
//                                            .y = off(x[u]) | off(x[v]) << 8 | off(x[w]) << 16 | (int8)coef << 24
//  pre[k][l]  build_prefixes' job of lane l in round k (rounds 0..2: tp, 3..4: qp):
//             .x = off(p[a]) | off(p[b]) << 16 in the staging area, .y = destination | (int8)coef << 16
//             (padding jobs: a = b = 33, coef 0, destination SLOT_OFF_HXDUMMY)
constexpr int GM_WORDS = NV / 2;
constexpr int PRE_TP_ROUNDS = (TP_CAP + 31) / 32, PRE_ROUNDS = PRE_TP_ROUNDS + (QP_CAP + 31) / 32;
// the coefficient in byte 2 of a word, in one SDWA convert (the compiler's
// form took a v_alignbit first)
__device__ __forceinline__ float coef_b2(uint32_t w) {
    float co;
    asm("v_cvt_f32_i32_sdwa %0, sext(%1) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_2" : "=v"(co) : "v"(w));
    return co;
}
__device__ __forceinline__ float coef_ht(const uint2 &w) { return (float)((int)w.y >> 24); }
struct EvalTables {
    int hx_len;
    int status;
    unsigned magic;                   // TAB_MAGIC once built: the tables persist in the workspace
    unsigned lu_struct;               // 1: the dH/dx structure lies within the tracker LU's (hc_lu.hpp LU_STRUCT_PAT)
    unsigned long long src_hash;      // hash of the unified index they were built from
    unsigned long long pad2;
    uint32_t gm[GM_WORDS][32];
    uint32_t pat[32];
    uint32_t hxd[HX_NSLOT / 2][32];
    uint32_t ht_acc_mask[4];          // eval_rhs: lanes (of a half) that accumulate in help term q
    uint32_t ht_light_mask[4];        // eval_rhs: lanes that accumulate a helper's product in light term q
    uint2 pre[PRE_ROUNDS][32];
    uint32_t hx[HX_SLOT_CAP * 32];
    uint2 ht[HT_TERMS * 32];
};

__device__ __forceinline__ pf2 ldp(const char *base, uint32_t off) {
    return *reinterpret_cast<const pf2 *>(base + off);
}
// Packed complex primitives: two VOP3P instructions each, op_sel / neg
// modifiers spelled out (the compiler does not fold per-element negation into
// neg_lo / neg_hi).  Each component is the same fma chain as the scalar spec in
// hc_device.hpp (cmul / cmadd / cmsub), so results are bit-identical.
// a*b: re = fma(a.x,b.x,-(a.y*b.y)), im = fma(a.x,b.y,a.y*b.x)
__device__ __forceinline__ pf2 pcmul(pf2 a, pf2 b) {
    pf2 t, r;
    asm("v_pk_mul_f32 %0, %1, %2 op_sel:[1,1] op_sel_hi:[1,0] neg_lo:[1,0]" : "=v"(t) : "v"(a), "v"(b));
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[0,1,1]" : "=v"(r) : "v"(a), "v"(b), "v"(t));
    return r;
}
// acc + a*b: re = fma(-a.y,b.y, fma(a.x,b.x,acc.x)), im = fma(a.y,b.x, fma(a.x,b.y,acc.y))
__device__ __forceinline__ pf2 pcmadd(pf2 acc, pf2 a, pf2 b) {
    pf2 s, r;
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[0,1,1]" : "=v"(s) : "v"(a), "v"(b), "v"(acc));
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[1,0,0]" : "=v"(r) : "v"(a), "v"(b), "v"(s));
    return r;
}
// acc - a*b: re = fma(a.y,b.y, fma(-a.x,b.x,acc.x)), im = fma(-a.y,b.x, fma(-a.x,b.y,acc.y))
__device__ __forceinline__ pf2 pcmsub(pf2 acc, pf2 a, pf2 b) {
    pf2 s, r;
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[0,1,1] neg_lo:[1,0,0] neg_hi:[1,0,0]" : "=v"(s) : "v"(a), "v"(b), "v"(acc));
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_hi:[1,0,0]" : "=v"(r) : "v"(a), "v"(b), "v"(s));
    return r;
}

// Software-pipelined term loops.  A term's table word is read EV_WAHEAD terms
// and its operands EV_AHEAD terms before it is computed, in program order
// ahead of the previous terms' entry stores (which the compiler may not move
// loads across), so a lane has several terms' LDS reads in flight instead of
// one round trip per term, with few registers held.
#ifndef HC_EV_AHEAD
#define HC_EV_AHEAD 2
#endif
constexpr int EV_AHEAD = HC_EV_AHEAD;
constexpr int EV_WAHEAD = EV_AHEAD + 2;

struct HxOps { pf2 t, xu, xv; };
__device__ __forceinline__ HxOps hx_ops(const char *sb, uint32_t w) {
    return HxOps{ldp(sb, w & 0xFFFFu), ldp(sb, (w >> 16) & 0xFFu), ldp(sb, w >> 24)};
}

// the term loop of eval_hx: operands are read through sb (the slot's prefix
// table tp and x), each finished entry is stored at sb + the lane's
// destination offset.  A term is ((c * p[a]) * p[b]) * x[u] accumulated with
// x[v] (:57-88); its prefix (c * p[a]) * p[b] comes from tp (build_prefixes).
__device__ __forceinline__ void eval_hx_terms(const uint32_t *s_hx, const uint32_t *s_hxd, char *sb, int r) {
    uint32_t w[HX_SLOT_CAP];
    uint32_t dst[HX_NSLOT / 2];
#pragma unroll
    for (int q = 0; q < HX_NSLOT / 2; q++) dst[q] = s_hxd[q * 32 + r];
#pragma unroll
    for (int k = 0; k < EV_WAHEAD; k++) w[k] = s_hx[k * 32 + r];
    HxOps o[EV_AHEAD + 1];
#pragma unroll
    for (int k = 0; k < EV_AHEAD; k++) o[k] = hx_ops(sb, w[k]);
    pf2 acc = {0.0f, 0.0f};
#pragma unroll
    for (int k = 0; k < HX_SLOT_CAP; k++) {
        if (k + EV_WAHEAD < HX_SLOT_CAP) w[k + EV_WAHEAD] = s_hx[(k + EV_WAHEAD) * 32 + r];
        if (k + EV_AHEAD < HX_SLOT_CAP) o[(k + EV_AHEAD) % (EV_AHEAD + 1)] = hx_ops(sb, w[k + EV_AHEAD]);
        const HxOps &q = o[k % (EV_AHEAD + 1)];
        const pf2 P = pcmul(q.t, q.xu);
        acc = pcmadd(acc, P, q.xv);
        if (hx_is_gend(k)) {                 // static: the entry in slot hx_gslot(k) ends here on every lane
            const int sl = hx_gslot(k);
            const uint32_t off = (sl & 1) ? (dst[sl >> 1] >> 16) : (dst[sl >> 1] & 0xFFFFu);
            *reinterpret_cast<pf2 *>(sb + off) = acc;
            acc = pf2{0.0f, 0.0f};
        }
        __builtin_amdgcn_sched_barrier(0);
    }
}

// dH/dx: row r of both paths' Jacobians into rA.  The term loop is fully
// unrolled over the padded table (HX_SLOT_CAP words per lane) and branch-free,
// so several terms' LDS reads stay in flight; each entry slot is stored once,
// where its group of terms ends, and 30 gathers through the row's gather map
// rebuild the register row.  The gather map of row r (EvalTables::gm): half c %
// 2 of word c / 2 = the SlotLDS byte offset of column c's entry in the packed
// entry block (or of the structural zero), so a gather address is one SDWA
// add, as the evaluations' operand addresses.  Its 15 words are read from LDS
// (stride 32 words) where the gather runs.
__device__ __forceinline__ void gather_hx(cf (&rA)[NV], const uint32_t *gmw, const SlotLDS &S, int r) {
    const char *sb = reinterpret_cast<const char *>(&S);
    uint32_t g[GM_WORDS];
#pragma unroll
    for (int q = 0; q < GM_WORDS; q++) g[q] = gmw[q * 32 + r];
#pragma unroll
    for (int c = 0; c < NV; c++) {
        const pf2 v = ldp(sb, (c & 1) ? (g[c / 2] >> 16) : (g[c / 2] & 0xFFFFu));
        rA[c] = cmk(v.x, v.y);
    }
}

__device__ __forceinline__ void eval_hx(cf (&rA)[NV], const uint32_t *s_hx, const uint32_t *s_hxd,
                                        const uint32_t *gmw, SlotLDS &S, int r) {
    eval_hx_terms(s_hx, s_hxd, reinterpret_cast<char *>(&S), r);
    wave_lds_sync();
    HC_ISA_MARK("ev_gather");
    gather_hx(rA, gmw, S, r);
}

// The slot's prefix tables (round 4).  p and the diff params are staged in
// the entry block (ent[0..33], ent[34..67]), then every lane runs its jobs
// (EvalTables::pre): (c * p[a]) * p[b] into tp and d[a]*p[b] + d[b]*p[a] into
// qp, with the operations of the term loops they replace (:57-148).  The two
// halves build their own slots' tables in the same instructions.
template <typename PW>
__device__ __forceinline__ void build_prefix_rounds(SlotLDS &S, int r, const PW *pre) {
    char *sb = reinterpret_cast<char *>(&S);
    wave_lds_sync();
#pragma unroll
    for (int k = 0; k < PRE_TP_ROUNDS; k++) {
        const uint2 w = pre[k * 32 + r];
        const pf2 pa = ldp(sb, w.x & 0xFFFFu), pb = ldp(sb, w.x >> 16);
        const float co = coef_b2(w.y);
        const pf2 t = pcmul(pa * pf2{co, co}, pb);                                     // (c * p[a]) * p[b]
        *reinterpret_cast<pf2 *>(sb + (w.y & 0xFFFFu)) = t;
    }
#pragma unroll
    for (int k = PRE_TP_ROUNDS; k < PRE_ROUNDS; k++) {
        const uint2 w = pre[k * 32 + r];
        const uint32_t oa = w.x & 0xFFFFu, ob = w.x >> 16;
        const pf2 pa = ldp(sb, oa), pb = ldp(sb, ob);
        const pf2 da = ldp(sb + SLOT_STG_DIF_DELTA, oa), db = ldp(sb + SLOT_STG_DIF_DELTA, ob);
        const pf2 q = pcmadd(pcmul(da, pb), db, pa);                                   // d[a]*p[b] + d[b]*p[a]
        *reinterpret_cast<pf2 *>(sb + (w.y & 0xFFFFu)) = q;
    }
    wave_lds_sync();
}
// The tracker's: lane r stages p[r] = t * target[r] + (1 - t) * start[r] (lane
// 0 also p[32]; p[33] = 1; ..._TrunPaths.cu:181 via the p(t) helper of
// dev-eval-indxing-..._LimUnroll_L2Cache.cuh:40-54) and d[r] from the slot's
// sample (global memory, L2-resident); sp: the start params (LDS).
template <typename PW>
__device__ __forceinline__ void build_prefixes(SlotLDS &S, int r, const PW *pre, const cf *target, const cf *diff,
                                               const cf *sp, float t0) {
    cf *stg = S.ent;
    const float omt = (float)(1.0 - (double)t0);
    stg[r] = cadd(cscale(target[r], t0), cscale(sp[r], omt));
    stg[NPP + r] = diff[r];
    if (r == 0) {
        stg[32] = cadd(cscale(target[32], t0), cscale(sp[32], omt));
        stg[33] = cmk(1.0f, 0.0f);
        stg[NPP + 32] = diff[32];
        stg[NPP + 33] = diff[33];
    }
    build_prefix_rounds(S, r, pre);
}

// dH/dt, H and the merged pass share one loop (eval_rhs).
//  * dH/dt: b = -sum_j c*(d[a]*p[b] + d[b]*p[a])*x[u]*x[v]*x[w]  (:91-119),
//    d[a]*p[b] + d[b]*p[a] from the slot's qp table;
//  * H:     b =  sum_j c*p[a]*p[b]*x[u]*x[v]*x[w]               (:122-148),
//    (c*p[a])*p[b] from the slot's tp table (build_prefixes);
//  * merged (RHS_MIXED): dH/dt in the halves with ht_half, H in the others, in
//    one pass, for a wave whose two paths run different stage kinds
//    (predictor | corrector: 44 % of the wave-stages of config 2) instead of
//    both loops.  A term's x part ((prefix * x[u]) * x[v], accumulated with
//    x[w]) is the same in both; the prefix is per half: dH/dt's
//    -(c * (d[a]*p[b] + d[b]*p[a])), negated so that both accumulate acc +
//    P*x[w] (acc - P*x[w] == acc + (-P)*x[w] bit for bit, and the negation
//    passes through the products exactly), or H's (c * p[a]) * p[b].
//
// Balanced rows.  A row's terms form one sequential chain, and the rows of
// this problem have 10 (rows 0..17), 13 or 16 terms, so a loop over the
// longest row left most lanes idle for 6 terms.  The loop now runs
// HT_FULL = 13 full terms and HT_HELP = 3 "light" ones: a row with 14..16
// terms (an owner) computes its first 13 terms itself; the products P of its
// last terms (everything but the accumulation with x[w]) are computed by its
// partner lane (lane ^ 16, a row of at most 10 terms: a helper) in the
// helper's full terms 10 + q, and handed over with one v_permlane16_swap per
// dword (lane i <-> i ^ 16, no LDS); the owner then
// accumulates them, in order, in its light terms (one x[w] read each).  Lanes
// mask the accumulation they must not do (k_prep_tables' masks: helpers in
// their help terms, everyone but owners in the light terms).  Bit-exact: the
// owner's chain is the same sequence of operations on the same values.
enum : int { RHS_HT = 0, RHS_H = 1, RHS_MIXED = 2 };
constexpr int HT_FULL = 13, HT_HELP = HT_TERMS - HT_FULL;
constexpr int HT_HELP_FIRST = HT_FULL - HT_HELP;   // the helpers' own terms end here

// acc +/- a*b in the lanes of m only (exec-masked packed fma pair, pcmadd /
// pcmsub operation for operation; the other lanes keep acc)
template <bool SUB>
__device__ __forceinline__ pf2 pcmacc_masked(pf2 acc, pf2 a, pf2 b, unsigned long long m) {
    pf2 t;
    unsigned long long sv;
    if constexpr (SUB)
        asm("s_mov_b64 %2, exec\n\ts_mov_b64 exec, %3\n\t"
            "v_pk_fma_f32 %1, %4, %5, %0 op_sel_hi:[0,1,1] neg_lo:[1,0,0] neg_hi:[1,0,0]\n\t"
            "s_nop 0\n\t"
            "v_pk_fma_f32 %0, %4, %5, %1 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_hi:[1,0,0]\n\t"
            "s_mov_b64 exec, %2"
            : "+v"(acc), "=&v"(t), "=&s"(sv) : "s"(m), "v"(a), "v"(b));
    else
        asm("s_mov_b64 %2, exec\n\ts_mov_b64 exec, %3\n\t"
            "v_pk_fma_f32 %1, %4, %5, %0 op_sel_hi:[0,1,1]\n\t"
            "s_nop 0\n\t"
            "v_pk_fma_f32 %0, %4, %5, %1 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[1,0,0]\n\t"
            "s_mov_b64 exec, %2"
            : "+v"(acc), "=&v"(t), "=&s"(sv) : "s"(m), "v"(a), "v"(b));
    return acc;
}
// the partner's value: lane i <-> lane i ^ 16 within each half (rows of 16
// lanes swapped in pairs: v_permlane16_swap with one register as both
// operands, one VALU per dword and no copy)
__device__ __forceinline__ pf2 from_partner(pf2 v) {
    asm("v_permlane16_swap_b32 %0, %0\n\tv_permlane16_swap_b32 %1, %1" : "+v"(v.x), "+v"(v.y));
    return v;
}
struct RhsMasks { unsigned long long acc[HT_HELP], light[HT_HELP]; };

__device__ __forceinline__ RhsMasks rhs_masks(const EvalTables *T) {
    RhsMasks m;
#pragma unroll
    for (int q = 0; q < HT_HELP; q++) {
        // uniform by construction; readfirstlane tells the compiler (SGPR operands)
        const unsigned long long a = (uint32_t)__builtin_amdgcn_readfirstlane((int)T->ht_acc_mask[q]),
                                 l = (uint32_t)__builtin_amdgcn_readfirstlane((int)T->ht_light_mask[q]);
        m.acc[q] = a | (a << 32);
        m.light[q] = l | (l << 32);
    }
    return m;
}

template <int KIND>
struct RhsOps { pf2 t, q, xu, xv, xw; };
template <int KIND, typename TW>
__device__ __forceinline__ RhsOps<KIND> rhs_ops(const char *sb, const TW &w) {
    RhsOps<KIND> o;
    if constexpr (KIND != RHS_HT) o.t = ldp(sb, w.x & 0xFFFFu);     // (c * p[a]) * p[b]
    if constexpr (KIND != RHS_H) o.q = ldp(sb, w.x >> 16);          // d[a]*p[b] + d[b]*p[a]
    o.xu = ldp(sb, w.y & 0xFFu);
    o.xv = ldp(sb, (w.y >> 8) & 0xFFu);
    o.xw = ldp(sb, (w.y >> 16) & 0xFFu);
    return o;
}

template <int KIND, typename TW>
__device__ __forceinline__ cf eval_rhs(const TW *s_ht, const SlotLDS &S, int r, bool ht_half, const RhsMasks &mk) {
    const char *sb = reinterpret_cast<const char *>(&S);
    constexpr bool SUB = KIND == RHS_HT;
    TW w[HT_TERMS];
#pragma unroll
    for (int j = 0; j < EV_WAHEAD; j++) w[j] = s_ht[j * 32 + r];
    RhsOps<KIND> o[EV_AHEAD + 1];
#pragma unroll
    for (int j = 0; j < EV_AHEAD; j++) o[j] = rhs_ops<KIND>(sb, w[j]);
    pf2 acc = {0.0f, 0.0f};
    pf2 hp[HT_HELP];
#pragma unroll
    for (int j = 0; j < HT_FULL; j++) {
        if (j + EV_WAHEAD < HT_TERMS) w[j + EV_WAHEAD] = s_ht[(j + EV_WAHEAD) * 32 + r];
        if (j + EV_AHEAD < HT_FULL) o[(j + EV_AHEAD) % (EV_AHEAD + 1)] = rhs_ops<KIND>(sb, w[j + EV_AHEAD]);
        const RhsOps<KIND> &q = o[j % (EV_AHEAD + 1)];
        const float co = coef_ht(w[j]);
        pf2 P;
        if constexpr (KIND == RHS_HT) {
            const pf2 s = q.q * pf2{co, co};
            P = pcmul(pcmul(s, q.xu), q.xv);
        } else if constexpr (KIND == RHS_H) {
            P = pcmul(pcmul(q.t, q.xu), q.xv);
        } else {
            const pf2 s = q.q * pf2{-co, -co};
            const pf2 pre = {ht_half ? s.x : q.t.x, ht_half ? s.y : q.t.y};
            P = pcmul(pcmul(pre, q.xu), q.xv);
        }
        if (j < HT_HELP_FIRST) {
            acc = SUB ? pcmsub(acc, P, q.xw) : pcmadd(acc, P, q.xw);
        } else {   // helpers compute a partner's product here instead of accumulating
            hp[j - HT_HELP_FIRST] = P;
            acc = pcmacc_masked<SUB>(acc, P, q.xw, mk.acc[j - HT_HELP_FIRST]);
        }
        __builtin_amdgcn_sched_barrier(0);   // keep the look-ahead reads ahead (no sinking to their uses)
    }
#pragma unroll
    for (int q = 0; q < HT_HELP; q++) {     // owners: the partner's products, in order
        const pf2 P = from_partner(hp[q]);
        const pf2 xw = ldp(sb, (w[HT_FULL + q].y >> 16) & 0xFFu);
        acc = pcmacc_masked<SUB>(acc, P, xw, mk.light[q]);
    }
    return cmk(acc.x, acc.y);
}

}  // namespace hc
