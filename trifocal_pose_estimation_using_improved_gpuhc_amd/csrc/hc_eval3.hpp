// hc_eval3.hpp -- v3 polynomial evaluation of the two-paths-per-wave tracker.
//
// Same terms, same operation order as eval_hx2 / eval_ht / eval_h (and the
// oracle): gpu-idx-evals/dev-eval-indxing-trifocal_2op1p_30x30_LimUnroll_L2Cache.cuh
// :57-88 (dH/dx), :91-119 (dH/dt), :122-148 (H).  What changes is the
// instruction count (profiles/r1_v3w4_pmc_summary.json: VALU issue 73 % busy):
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
//  * the end-of-entry flag of a dH/dx term is the sign bit of its second word.
#pragma once

#include <stddef.h>

#include "hc_track2.hpp"

namespace hc {

typedef float pf2 __attribute__((ext_vector_type(2)));

constexpr int HX3_SLOT_CAP = 24;   // per-lane dH/dx terms (this problem: 23); keeps LDS <= 40 KB/WG
constexpr int SLOT_OFF_X = (int)offsetof(SlotLDS, x);
constexpr int SLOT_OFF_P = (int)offsetof(SlotLDS, p);
constexpr int SLOT_DIF_DELTA = (int)offsetof(SlotLDS, dif) - (int)offsetof(SlotLDS, p);
static_assert(SLOT_OFF_X + 8 * 31 < 256, "x offsets must fit a byte");
static_assert(SLOT_OFF_P + 8 * NPP < 65536, "p offsets must fit 16 bits");

// v3 tables, built by the prep kernel next to the v1/v2 tables.
//  hx[k][r] (row r's k-th dH/dx term): .x = off(p[a]) | off(p[b]) << 16
//                                      .y = off(x[u]) | off(x[v]) << 8 | (int8)coef << 16 | 8*slot << 24 | last << 31
//  ht[j][r] (row r's j-th dH/dt / H term): .x = off(p[a]) | off(p[b]) << 16
//                                      .y = off(x[u]) | off(x[v]) << 8 | off(x[w]) << 16 | (int8)coef << 24
struct TableWS3 {
    int hx_len;
    int status;
    int pad[2];
    uint2 hx[HX3_SLOT_CAP * 32];
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

// dH/dx: row r of both paths' Jacobians into rA
__device__ __forceinline__ void eval_hx3(cf (&rA)[NV], const uint2 *s_hx3, int hx_len, const uint32_t (&map)[3],
                                         SlotLDS &S, int r) {
    const char *sb = reinterpret_cast<const char *>(&S);
    cf *ent_row = S.ent + (r < NV ? r : 0) * 7;
    char *eb = reinterpret_cast<char *>(ent_row);
    if (r < NV) ent_row[6] = cmk(0.0f, 0.0f);   // structural zero (the v3 LU reuses this block)
    pf2 acc = {0.0f, 0.0f};
    for (int k = 0; k < hx_len; k++) {
        const uint2 w = s_hx3[k * 32 + r];
        const pf2 pa = ldp(sb, w.x & 0xFFFFu), pb = ldp(sb, w.x >> 16);
        const pf2 xu = ldp(sb, w.y & 0xFFu), xv = ldp(sb, (w.y >> 8) & 0xFFu);
        const float co = (float)(int)(int8_t)(uint8_t)(w.y >> 16);
        pf2 P = pa * pf2{co, co};
        P = pcmul(P, pb);
        P = pcmul(P, xu);
        acc = pcmadd(acc, P, xv);
        if ((int)w.y < 0) {             // last term of an entry (never set on padding terms)
            *reinterpret_cast<pf2 *>(eb + ((w.y >> 24) & 0x7Fu)) = acc;
            acc = pf2{0.0f, 0.0f};
        }
    }
    wave_lds_sync();
#pragma unroll
    for (int c = 0; c < NV; c++) {
        const uint32_t code = (map[c / 10] >> (3 * (c % 10))) & 7u;
        rA[c] = ent_row[code];
    }
}

// dH/dt: b = -sum_j c*(d[a]*p[b] + d[b]*p[a])*x[u]*x[v]*x[w]
__device__ __forceinline__ cf eval_ht3(const uint2 *s_ht3, const SlotLDS &S, int r) {
    const char *sb = reinterpret_cast<const char *>(&S);
    pf2 acc = {0.0f, 0.0f};
#pragma unroll 4
    for (int j = 0; j < HT_TERMS; j++) {
        const uint2 w = s_ht3[j * 32 + r];
        const uint32_t oa = w.x & 0xFFFFu, ob = w.x >> 16;
        const pf2 pa = ldp(sb, oa), pb = ldp(sb, ob);
        const pf2 da = ldp(sb + SLOT_DIF_DELTA, oa), db = ldp(sb + SLOT_DIF_DELTA, ob);
        const pf2 xu = ldp(sb, w.y & 0xFFu), xv = ldp(sb, (w.y >> 8) & 0xFFu), xw = ldp(sb, (w.y >> 16) & 0xFFu);
        const float co = (float)((int)w.y >> 24);
        pf2 s = pcmadd(pcmul(da, pb), db, pa);
        s = s * pf2{co, co};
        const pf2 P = pcmul(pcmul(s, xu), xv);
        acc = pcmsub(acc, P, xw);
    }
    return cmk(acc.x, acc.y);
}

// H: b = sum_j c*p[a]*p[b]*x[u]*x[v]*x[w]
__device__ __forceinline__ cf eval_h3(const uint2 *s_ht3, const SlotLDS &S, int r) {
    const char *sb = reinterpret_cast<const char *>(&S);
    pf2 acc = {0.0f, 0.0f};
#pragma unroll 4
    for (int j = 0; j < HT_TERMS; j++) {
        const uint2 w = s_ht3[j * 32 + r];
        const pf2 pa = ldp(sb, w.x & 0xFFFFu), pb = ldp(sb, w.x >> 16);
        const pf2 xu = ldp(sb, w.y & 0xFFu), xv = ldp(sb, (w.y >> 8) & 0xFFu), xw = ldp(sb, (w.y >> 16) & 0xFFu);
        const float co = (float)((int)w.y >> 24);
        pf2 P = pa * pf2{co, co};
        P = pcmul(pcmul(pcmul(P, pb), xu), xv);
        acc = pcmadd(acc, P, xw);
    }
    return cmk(acc.x, acc.y);
}

}  // namespace hc
