// hc_eval.hpp -- polynomial evaluation of the two-paths-per-wave tracker.
//
// Same terms, same operation order as the reference and the oracle:
// gpu-idx-evals/dev-eval-indxing-trifocal_2op1p_30x30_LimUnroll_L2Cache.cuh
// :57-88 (dH/dx), :91-119 (dH/dt), :122-148 (H).  Lane r of a half-wave
// evaluates equation row r of its path from compacted per-row term lists:
//
//  * term words carry LDS byte offsets relative to the path slot (SlotLDS), so
//    an operand address is one add (p offsets in 16-bit halves, x offsets in
//    bytes) instead of shift + mask + add;
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
constexpr int SLOT_OFF_P = (int)offsetof(SlotLDS, p);
constexpr int SLOT_DIF_DELTA = (int)offsetof(SlotLDS, dif) - (int)offsetof(SlotLDS, p);
constexpr int SLOT_OFF_ENT = (int)offsetof(SlotLDS, ent);
constexpr int SLOT_OFF_HXDUMMY = (int)offsetof(SlotLDS, lu) + 8 * 31;   // unused entry slots store here
static_assert(SLOT_OFF_ENT + 8 * NV * 7 < 65536 && SLOT_OFF_HXDUMMY < 65536, "entry offsets must fit 16 bits");
static_assert(SLOT_OFF_X + 8 * 31 < 256, "x offsets must fit a byte");
static_assert(SLOT_OFF_P + 8 * NPP < 65536, "p offsets must fit 16 bits");

// Compacted tables, built once per launch by k_prep_tables from the
// reference's padded unified index (Data_Reader.cpp:167-189).
//  map[q][r]  (row r): column c -> entry slot of row r's block in SlotLDS::ent
//             (3 bits x 10 columns per word, 6 = structural zero)
//  hx[k][l] (lane l's k-th dH/dx term, entry slot hx_gslot(k)): .x = off(p[a]) | off(p[b]) << 16
//                                      .y = off(x[u]) | off(x[v]) << 8 | (int8)coef << 16
//  hxd[q][l]  (lane l): SlotLDS byte offsets its slots 2q (bits 0..15) and 2q+1 (bits 16..31) store to
//  ht[j][r] (row r's j-th dH/dt / H term): .x = off(p[a]) | off(p[b]) << 16
//                                      .y = off(x[u]) | off(x[v]) << 8 | off(x[w]) << 16 | (int8)coef << 24
struct EvalTables {
    int hx_len;
    int status;
    unsigned magic;                   // TAB_MAGIC once built: the tables persist in the workspace
    unsigned pad;
    unsigned long long src_hash;      // hash of the unified index they were built from
    unsigned long long pad2;
    uint32_t map[3][32];
    uint32_t hxd[HX_NSLOT / 2][32];
    uint2 hx[HX_SLOT_CAP * 32];
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
constexpr int EV_AHEAD = 2;
constexpr int EV_WAHEAD = EV_AHEAD + 2;

struct HxOps { pf2 pa, pb, xu, xv; };
__device__ __forceinline__ HxOps hx_ops(const char *sb, uint2 w) {
    return HxOps{ldp(sb, w.x & 0xFFFFu), ldp(sb, w.x >> 16), ldp(sb, w.y & 0xFFu), ldp(sb, (w.y >> 8) & 0xFFu)};
}

// the term loop of eval_hx: operands are read through sb (x, p of the slot),
// each finished entry is stored at sb + the lane's destination offset
__device__ __forceinline__ void eval_hx_terms(const uint2 *s_hx, const uint32_t *s_hxd, char *sb, int r) {
    uint2 w[HX_SLOT_CAP];
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
        // (float)(int8_t)(w.y >> 16) in one SDWA convert (the compiler's form
        // took a v_alignbit first)
        float co;
        asm("v_cvt_f32_i32_sdwa %0, sext(%1) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_2"
            : "=v"(co) : "v"(w[k].y));
        pf2 P = q.pa * pf2{co, co};
        P = pcmul(P, q.pb);
        P = pcmul(P, q.xu);
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
// where its group of terms ends, slot 6 (structural zero) is zeroed, and 30
// gathers through the column -> slot map rebuild the register row.
// the register row r of dH/dx from the lane's entry block (S.ent row r)
__device__ __forceinline__ void gather_hx(cf (&rA)[NV], const uint32_t (&map)[3], const SlotLDS &S, int r) {
    const cf *ent_row = S.ent + (r < NV ? r : 0) * 7;
    // opaque copy: keeps LICM from hoisting the 30 decoded gather addresses out
    // of the path loop (30 VGPRs held across the LU, then spilled)
    uint32_t m[3] = {map[0], map[1], map[2]};
    asm volatile("" : "+v"(m[0]), "+v"(m[1]), "+v"(m[2]));
    // slot = v_bfe_u32, address = v_lshl_add_u32 (2 VALU per column, not 3)
    const char *eb = reinterpret_cast<const char *>(ent_row);
#pragma unroll
    for (int c = 0; c < NV; c++) {
        uint32_t code;   // asm: the compiler would turn bfe + shift back into shift + and + add
        asm("v_bfe_u32 %0, %1, %2, 3" : "=v"(code) : "v"(m[c / 10]), "i"(3 * (c % 10)));
        rA[c] = *reinterpret_cast<const cf *>(eb + (code << 3));
    }
}

__device__ __forceinline__ void eval_hx(cf (&rA)[NV], const uint2 *s_hx, const uint32_t *s_hxd,
                                        const uint32_t (&map)[3], SlotLDS &S, int r) {
    cf *ent_row = S.ent + (r < NV ? r : 0) * 7;
    eval_hx_terms(s_hx, s_hxd, reinterpret_cast<char *>(&S), r);
    float z;   // a fresh zero (a hoisted zero pair gets spilled in abort mode)
    asm volatile("v_mov_b32 %0, 0" : "=v"(z));
    if (r < NV) ent_row[6] = cmk(z, z);   // structural zero
    wave_lds_sync();
    gather_hx(rA, map, S, r);
}

struct HtOps { pf2 pa, pb, da, db, xu, xv, xw; };
__device__ __forceinline__ HtOps ht_ops(const char *sb, uint2 w) {
    const uint32_t oa = w.x & 0xFFFFu, ob = w.x >> 16;
    return HtOps{ldp(sb, oa), ldp(sb, ob), ldp(sb + SLOT_DIF_DELTA, oa), ldp(sb + SLOT_DIF_DELTA, ob),
                 ldp(sb, w.y & 0xFFu), ldp(sb, (w.y >> 8) & 0xFFu), ldp(sb, (w.y >> 16) & 0xFFu)};
}

// dH/dt: b = -sum_j c*(d[a]*p[b] + d[b]*p[a])*x[u]*x[v]*x[w]
__device__ __forceinline__ cf eval_ht(const uint2 *s_ht, const SlotLDS &S, int r) {
    const char *sb = reinterpret_cast<const char *>(&S);
    uint2 w[HT_TERMS];
#pragma unroll
    for (int j = 0; j < EV_WAHEAD; j++) w[j] = s_ht[j * 32 + r];
    HtOps o[EV_AHEAD + 1];
#pragma unroll
    for (int j = 0; j < EV_AHEAD; j++) o[j] = ht_ops(sb, w[j]);
    pf2 acc = {0.0f, 0.0f};
#pragma unroll
    for (int j = 0; j < HT_TERMS; j++) {
        if (j + EV_WAHEAD < HT_TERMS) w[j + EV_WAHEAD] = s_ht[(j + EV_WAHEAD) * 32 + r];
        if (j + EV_AHEAD < HT_TERMS) o[(j + EV_AHEAD) % (EV_AHEAD + 1)] = ht_ops(sb, w[j + EV_AHEAD]);
        const HtOps &q = o[j % (EV_AHEAD + 1)];
        const float co = (float)((int)w[j].y >> 24);
        pf2 s = pcmadd(pcmul(q.da, q.pb), q.db, q.pa);
        s = s * pf2{co, co};
        const pf2 P = pcmul(pcmul(s, q.xu), q.xv);
        acc = pcmsub(acc, P, q.xw);
        __builtin_amdgcn_sched_barrier(0);   // keep the look-ahead reads ahead (no sinking to their uses)
    }
    return cmk(acc.x, acc.y);
}

// dH/dt in the halves with ht_half, H in the others, in one pass: for a wave
// whose two paths run different stage kinds (predictor | corrector: 44 % of
// the wave-stages of config 2), instead of both full loops.  A term's x part
// ((prefix * x[u]) * x[v], accumulated with x[w]) is the same in both; the
// prefix is per half:
//   dH/dt: -(c * (d[a]*p[b] + d[b]*p[a])), negated so that the accumulation
//          is acc + P*x[w] in both (acc - P*x[w] == acc + (-P)*x[w] bit for
//          bit, and the negation passes through the products exactly);
//   H:     (c * p[a]) * p[b].
__device__ __forceinline__ cf eval_hth(const uint2 *s_ht, const SlotLDS &S, int r, bool ht_half) {
    const char *sb = reinterpret_cast<const char *>(&S);
    uint2 w[HT_TERMS];
#pragma unroll
    for (int j = 0; j < EV_WAHEAD; j++) w[j] = s_ht[j * 32 + r];
    HtOps o[EV_AHEAD + 1];
#pragma unroll
    for (int j = 0; j < EV_AHEAD; j++) o[j] = ht_ops(sb, w[j]);
    pf2 acc = {0.0f, 0.0f};
#pragma unroll
    for (int j = 0; j < HT_TERMS; j++) {
        if (j + EV_WAHEAD < HT_TERMS) w[j + EV_WAHEAD] = s_ht[(j + EV_WAHEAD) * 32 + r];
        if (j + EV_AHEAD < HT_TERMS) o[(j + EV_AHEAD) % (EV_AHEAD + 1)] = ht_ops(sb, w[j + EV_AHEAD]);
        const HtOps &q = o[j % (EV_AHEAD + 1)];
        const float co = (float)((int)w[j].y >> 24);
        pf2 s = pcmadd(pcmul(q.da, q.pb), q.db, q.pa);
        s = s * pf2{-co, -co};
        const pf2 h = pcmul(q.pa * pf2{co, co}, q.pb);
        const pf2 pre = {ht_half ? s.x : h.x, ht_half ? s.y : h.y};
        const pf2 P = pcmul(pcmul(pre, q.xu), q.xv);
        acc = pcmadd(acc, P, q.xw);
        __builtin_amdgcn_sched_barrier(0);
    }
    return cmk(acc.x, acc.y);
}

struct HOps { pf2 pa, pb, xu, xv, xw; };
__device__ __forceinline__ HOps h_ops(const char *sb, uint2 w) {
    return HOps{ldp(sb, w.x & 0xFFFFu), ldp(sb, w.x >> 16), ldp(sb, w.y & 0xFFu), ldp(sb, (w.y >> 8) & 0xFFu),
                ldp(sb, (w.y >> 16) & 0xFFu)};
}

// H: b = sum_j c*p[a]*p[b]*x[u]*x[v]*x[w]
__device__ __forceinline__ cf eval_h(const uint2 *s_ht, const SlotLDS &S, int r) {
    const char *sb = reinterpret_cast<const char *>(&S);
    uint2 w[HT_TERMS];
#pragma unroll
    for (int j = 0; j < EV_WAHEAD; j++) w[j] = s_ht[j * 32 + r];
    HOps o[EV_AHEAD + 1];
#pragma unroll
    for (int j = 0; j < EV_AHEAD; j++) o[j] = h_ops(sb, w[j]);
    pf2 acc = {0.0f, 0.0f};
#pragma unroll
    for (int j = 0; j < HT_TERMS; j++) {
        if (j + EV_WAHEAD < HT_TERMS) w[j + EV_WAHEAD] = s_ht[(j + EV_WAHEAD) * 32 + r];
        if (j + EV_AHEAD < HT_TERMS) o[(j + EV_AHEAD) % (EV_AHEAD + 1)] = h_ops(sb, w[j + EV_AHEAD]);
        const HOps &q = o[j % (EV_AHEAD + 1)];
        const float co = (float)((int)w[j].y >> 24);
        pf2 P = q.pa * pf2{co, co};
        P = pcmul(pcmul(pcmul(P, q.pb), q.xu), q.xv);
        acc = pcmadd(acc, P, q.xw);
        __builtin_amdgcn_sched_barrier(0);
    }
    return cmk(acc.x, acc.y);
}

}  // namespace hc
