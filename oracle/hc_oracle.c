/*
 * hc_oracle.c -- TEST INFRASTRUCTURE ONLY (see hc_oracle.h for the rules).
 *
 * Plain-C restatement of the reference path tracker for trifocal_2op1p_30x30.
 * Every function cites the reference file:line it restates (paths relative to
 * the reference repository root).  Build: oracle/Makefile, with
 * -ffp-contract=off so the only fused multiply-adds are the explicit fmaf()
 * calls of the arithmetic spec (DESIGN.md "Arithmetic specification"); the
 * HIP kernel implements the identical spec, so the two agree bit for bit
 * (up to the sign of exact zeros, which never reaches a non-zero value or a
 * branch -- DESIGN.md explains why).
 */
#include "hc_oracle.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define NV ORC_NV
#define NPP (ORC_NP + 1) /* 34 */
#define NT ORC_NTRACK

/* ====================================================================== */
/* complex arithmetic spec (MAGMA magma_operators.h / cuComplex restated)  */
/* ====================================================================== */
typedef struct { float x, y; } cf;

static inline cf cmk(float x, float y) { cf r; r.x = x; r.y = y; return r; }
static inline cf cadd(cf a, cf b) { return cmk(a.x + b.x, a.y + b.y); }
static inline cf csub(cf a, cf b) { return cmk(a.x - b.x, a.y - b.y); }
static inline cf cscale(cf a, float s) { return cmk(a.x * s, a.y * s); }
static inline cf cdivs(cf a, float s) { return cmk(a.x / s, a.y / s); }
#ifdef ORC_PLAIN_OPS
/* Experiment build only (libhc_oracle_plain.so, tests/cpuhc_pin.py): the
   reference's host operators as plain expressions (MAGMA magma_operators.h
   order), compiled like the reference CPU build (-O3 with GCC's default
   -ffp-contract=fast, CMakeLists.txt:36,57; -march=x86-64-v3 for the reference's
   -march=native: FMA available), so the compiler chooses the FMAs as it did
   for CPU_HC_Solver. */
static inline cf cmul(cf a, cf b) { return cmk(a.x * b.x - a.y * b.y, a.y * b.x + a.x * b.y); }
static inline cf cmadd(cf acc, cf a, cf b) { return cadd(acc, cmul(a, b)); }
static inline cf cmsub(cf acc, cf a, cf b) { return csub(acc, cmul(a, b)); }
#else
/* a*b with the two documented FMAs */
static inline cf cmul(cf a, cf b) {
    return cmk(fmaf(a.x, b.x, -(a.y * b.y)), fmaf(a.x, b.y, a.y * b.x));
}
/* acc + a*b */
static inline cf cmadd(cf acc, cf a, cf b) {
    return cmk(fmaf(-a.y, b.y, fmaf(a.x, b.x, acc.x)), fmaf(a.y, b.x, fmaf(a.x, b.y, acc.y)));
}
/* acc - a*b */
static inline cf cmsub(cf acc, cf a, cf b) {
    return cmk(fmaf(a.y, b.y, fmaf(-a.x, b.x, acc.x)), fmaf(-a.y, b.x, fmaf(-a.x, b.y, acc.y)));
}
#endif
/* MAGMA_C_DIV == cuCdivf (CUDA cuComplex.h), literal, no FMA */
static inline cf cdiv(cf a, cf b) {
    float s = fabsf(b.x) + fabsf(b.y);
    float oos = 1.0f / s;
    float ars = a.x * oos, ais = a.y * oos;
    float brs = b.x * oos, bis = b.y * oos;
    s = (brs * brs) + (bis * bis);
    oos = 1.0f / s;
    return cmk(((ars * brs) + (ais * bis)) * oos, ((ais * brs) - (ars * bis)) * oos);
}

static inline cf ld(const float *p, int i) { return cmk(p[2 * i], p[2 * i + 1]); }
static inline void st(float *p, int i, cf v) { p[2 * i] = v.x; p[2 * i + 1] = v.y; }

int orc_max_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

/* ====================================================================== */
/* readers -- magmaHC/Data_Reader.cpp:37-60,104-165,191-338                */
/* (iostream `>> float` == strtof correct rounding == fscanf("%f"))        */
/* ====================================================================== */
int orc_read_start_sols(const char *file, float *ss) {
    /* Data_Reader.cpp:37-60 -- 9360 "re im" lines, track-major; x[30] = 1 */
    FILE *f = fopen(file, "r");
    if (!f) return -1;
    float re, im;
    int d = 0, i = 0, n = 0;
    while (fscanf(f, "%f %f", &re, &im) == 2) {
        if (i >= NT) { fclose(f); return -2; }
        ss[(i * (NV + 1) + d) * 2] = re;
        ss[(i * (NV + 1) + d) * 2 + 1] = im;
        n++;
        if (d < NV - 1) d++; else { d = 0; i++; }
    }
    fclose(f);
    for (int k = 0; k < NT; k++) { ss[(k * (NV + 1) + NV) * 2] = 1.0f; ss[(k * (NV + 1) + NV) * 2 + 1] = 0.0f; }
    return n;
}

int orc_read_start_params(const char *file, float *sp) {
    /* Data_Reader.cpp:104-121 -- 33 "re im" pairs, p[33] = 1 */
    FILE *f = fopen(file, "r");
    if (!f) return -1;
    float re, im;
    int d = 0;
    while (d < NPP && fscanf(f, "%f %f", &re, &im) == 2) { sp[2 * d] = re; sp[2 * d + 1] = im; d++; }
    fclose(f);
    sp[2 * ORC_NP] = 1.0f; sp[2 * ORC_NP + 1] = 0.0f;
    return d;
}

int orc_read_ints(const char *file, int *out, int max_count) {
    /* Data_Reader.cpp:123-165 */
    FILE *f = fopen(file, "r");
    if (!f) return -1;
    int v, d = 0;
    while (d < max_count && fscanf(f, "%d", &v) == 1) out[d++] = v;
    fclose(f);
    return d;
}

int orc_read_floats(const char *file, float *out, int max_count) {
    /* Data_Reader.cpp:191-270 (poses, intrinsic matrix) */
    FILE *f = fopen(file, "r");
    if (!f) return -1;
    float v;
    int d = 0;
    while (d < max_count && fscanf(f, "%f", &v) == 1) out[d++] = v;
    fclose(f);
    return d;
}

int orc_count_triplet_edgels(const char *file) {
    /* Data_Reader.cpp:273-305 -- 12 floats per complete record */
    FILE *f = fopen(file, "r");
    if (!f) return 0;
    float v[12];
    int n = 0;
    for (;;) {
        int k = 0;
        while (k < 12 && fscanf(f, "%f", &v[k]) == 1) k++;
        if (k < 12) break;
        n++;
    }
    fclose(f);
    return n;
}

int orc_read_triplet_edgels(const char *file, float *loc, float *tan, int max_edgels) {
    /* Data_Reader.cpp:288-324: x1 y1 tx1 ty1 x2 y2 tx2 ty2 x3 y3 tx3 ty3 */
    FILE *f = fopen(file, "r");
    if (!f) return -1;
    float v[12];
    int n = 0;
    while (n < max_edgels) {
        int k = 0;
        while (k < 12 && fscanf(f, "%f", &v[k]) == 1) k++;
        if (k < 12) break;
        for (int view = 0; view < 3; view++) {
            loc[n * 6 + 2 * view] = v[4 * view + 0];
            loc[n * 6 + 2 * view + 1] = v[4 * view + 1];
            tan[n * 6 + 2 * view] = v[4 * view + 2];
            tan[n * 6 + 2 * view + 1] = v[4 * view + 3];
        }
        n++;
    }
    fclose(f);
    return n;
}

/* ====================================================================== */
/* sample generation -- magmaHC/GPU_HC_Solver.cpp:252-306                  */
/* ====================================================================== */
void orc_prepare_target_params(unsigned seed, int num_gpus, const int *sub,
                               const float *loc, const float *tan, int E,
                               const float *start_params, float *tgt, float *dif, int *picked) {
    unsigned idx[3];
    srand(seed);                                   /* :260 */
    int k = 0;
    for (int g = 0; g < num_gpus; g++) {           /* :263 gpu-major */
        for (int ti = 0; ti < sub[g]; ti++, k++) { /* :265 sample-minor */
            for (;;) {                             /* :268-271 -- i0 == i2 is NOT rejected */
                for (int ri = 0; ri < 3; ri++) idx[ri] = (unsigned)(rand() % E);
                if (idx[0] != idx[1] && idx[0] != idx[1] && idx[1] != idx[2]) break;
            }
            if (picked) for (int i = 0; i < 3; i++) picked[k * 3 + i] = (int)idx[i];
            float *tp = tgt + (size_t)k * NPP * 2;
            for (int i = 0; i < 3; i++)            /* :276-281 locations */
                for (int j = 0; j < 6; j++) { tp[2 * (i * 6 + j)] = loc[idx[i] * 6 + j]; tp[2 * (i * 6 + j) + 1] = 0.0f; }
            for (int i = 0; i < 2; i++)            /* :283-288 tangents */
                for (int j = 0; j < 6; j++) { tp[2 * (i * 6 + j + 18)] = tan[idx[i] * 6 + j]; tp[2 * (i * 6 + j + 18) + 1] = 0.0f; }
            tp[60] = 1.0f; tp[61] = 0.0f;          /* :289-292 */
            tp[62] = 0.5f; tp[63] = 0.0f;
            tp[64] = 1.0f; tp[65] = 0.0f;
            tp[66] = 1.0f; tp[67] = 0.0f;
            float *dp = dif + (size_t)k * NPP * 2;
            for (int i = 0; i < NPP; i++) st(dp, i, csub(ld(tp, i), ld(start_params, i))); /* :295-296 */
        }
    }
}

/* ====================================================================== */
/* evaluations -- gpu-idx-evals/dev-eval-indxing-..._LimUnroll_L2Cache.cuh */
/* ====================================================================== */
/* :40-54 -- p_i = target_i*t + start_i*(1.0-t), i < 33; p[33] = 1 (TrunPaths.cu:122) */
void orc_param_homotopy_gpu(float t, const float *sp, const float *tp, float *p) {
    float omt = (float)(1.0 - (double)t);
    for (int i = 0; i < ORC_NP; i++) st(p, i, cadd(cscale(ld(tp, i), t), cscale(ld(sp, i), omt)));
    p[2 * ORC_NP] = 1.0f; p[2 * ORC_NP + 1] = 0.0f;
}

/* CPU_HC_Solver.hpp:102-106 -- all 34 entries (p[33] = t + (1-t), may be != 1) */
static void param_homotopy_cpu(float t, const float *sp, const float *tp, cf *p) {
    float omt = (float)(1.0 - (double)t);
    for (int i = 0; i <= ORC_NP; i++) p[i] = cadd(cscale(ld(tp, i), t), cscale(ld(sp, i), omt));
}

/* :57-88 -- A[r][c] = sum_j c*p[a]*p[b]*x[u]*x[v]; entry ((c*8+j)*5+part)*30 + r.
   Padding terms (coef 0, p33, p33, x30, x30) are exact (+0,+0) and are skipped
   (only the sign of an exact zero can differ). */
static inline cf hx_entry(const int *T, int r, int c, const cf *x, const cf *p) {
    cf acc = cmk(0.0f, 0.0f);
    for (int j = 0; j < ORC_HX_TERMS; j++) {
        const int base = (c * ORC_HX_TERMS + j) * ORC_HX_PARTS * NV + r;
        const int co = T[base];
        if (co == 0) continue;
        const cf P = cmul(cmul(cscale(p[T[base + NV]], (float)co), p[T[base + 2 * NV]]), x[T[base + 3 * NV]]);
        acc = cmadd(acc, P, x[T[base + 4 * NV]]);
    }
    return acc;
}
/* :91-119 -- b[r] = -sum_j c*(d[a]*p[b] + d[b]*p[a])*x[u]*x[v]*x[w]; entry (j*6+part)*30 + r */
static inline cf ht_row(const int *D, int r, const cf *x, const cf *p, const cf *d) {
    cf acc = cmk(0.0f, 0.0f);
    for (int j = 0; j < ORC_HT_TERMS; j++) {
        const int base = j * ORC_HT_PARTS * NV + r;
        const int co = D[base];
        if (co == 0) continue;
        const int a = D[base + NV], b = D[base + 2 * NV];
        cf s = cmadd(cmul(d[a], p[b]), d[b], p[a]);
        s = cscale(s, (float)co);
        const cf P = cmul(cmul(s, x[D[base + 3 * NV]]), x[D[base + 4 * NV]]);
        acc = cmsub(acc, P, x[D[base + 5 * NV]]);
    }
    return acc;
}
/* :122-148 -- b[r] = sum_j c*p[a]*p[b]*x[u]*x[v]*x[w] */
static inline cf h_row(const int *D, int r, const cf *x, const cf *p) {
    cf acc = cmk(0.0f, 0.0f);
    for (int j = 0; j < ORC_HT_TERMS; j++) {
        const int base = j * ORC_HT_PARTS * NV + r;
        const int co = D[base];
        if (co == 0) continue;
        const cf P = cmul(cmul(cmul(cscale(p[D[base + NV]], (float)co), p[D[base + 2 * NV]]), x[D[base + 3 * NV]]),
                          x[D[base + 4 * NV]]);
        acc = cmadd(acc, P, x[D[base + 5 * NV]]);
    }
    return acc;
}

void orc_eval_hx(const int *dHdx, const float *xf, const float *pf, float *A) {
    cf x[NV + 1], p[NPP];
    for (int i = 0; i <= NV; i++) x[i] = ld(xf, i);
    for (int i = 0; i < NPP; i++) p[i] = ld(pf, i);
    for (int r = 0; r < NV; r++)
        for (int c = 0; c < NV; c++) st(A, r * NV + c, hx_entry(dHdx, r, c, x, p));
}
void orc_eval_ht(const int *dHdt, const float *xf, const float *pf, const float *df, float *b) {
    cf x[NV + 1], p[NPP], d[NPP];
    for (int i = 0; i <= NV; i++) x[i] = ld(xf, i);
    for (int i = 0; i < NPP; i++) { p[i] = ld(pf, i); d[i] = ld(df, i); }
    for (int r = 0; r < NV; r++) st(b, r, ht_row(dHdt, r, x, p, d));
}
void orc_eval_h(const int *dHdt, const float *xf, const float *pf, float *b) {
    cf x[NV + 1], p[NPP];
    for (int i = 0; i <= NV; i++) x[i] = ld(xf, i);
    for (int i = 0; i < NPP; i++) p[i] = ld(pf, i);
    for (int r = 0; r < NV; r++) st(b, r, h_row(dHdt, r, x, p));
}

/* ====================================================================== */
/* LU -- magmaHC/dev-cgesv-batched-small.cuh:38-107 (GPU semantics)        */
/* Thread r owns original row r (rA[r][*], rB[r]); rowid[r] is its logical */
/* position; pivoting relabels positions instead of moving rows.           */
/* ====================================================================== */
static void cgesv_gpu(cf rA[NV][NV], cf *rB, cf *xout) {
    int rowid[NV];
    float dsx[NV];
    cf sx[NV], sB[NV];
    for (int r = 0; r < NV; r++) rowid[r] = r;
    for (int i = 0; i < NV; i++) {
        for (int r = 0; r < NV; r++) dsx[rowid[r]] = fabsf(rA[r][i].x) + fabsf(rA[r][i].y); /* :55 */
        float mx = dsx[i];                                                                   /* :57 */
        int mid = i;
        for (int j = i + 1; j < NV; j++) if (dsx[j] > mx) { mid = j; mx = dsx[j]; }          /* :59-64 */
        const int zero = (mx == 0.0f);                                                      /* :66 */
        const float update = zero ? 0.0f : 1.0f;                                            /* :68 */
        int pl = -1, ql = -1;
        for (int r = 0; r < NV; r++) { if (rowid[r] == mid) pl = r; if (rowid[r] == i) ql = r; }
        for (int j = i; j < NV; j++) sx[j] = cscale(rA[pl][j], update);                     /* :73-76 */
        const cf sB0 = rB[pl];                                                              /* :77 */
        rowid[pl] = i;                                                                      /* :72 */
        if (ql != pl) rowid[ql] = mid;                                                      /* :79-81 */
        const cf reg = zero ? cmk(1.0f, 0.0f) : cdiv(cmk(1.0f, 0.0f), sx[i]);               /* :84 */
        for (int r = 0; r < NV; r++) {                                                      /* :86-93 */
            if (rowid[r] > i) {
                rA[r][i] = cmul(rA[r][i], reg);
                for (int j = i + 1; j < NV; j++) rA[r][j] = cmsub(rA[r][j], rA[r][i], sx[j]);
                rB[r] = cmsub(rB[r], rA[r][i], sB0);
            }
        }
    }
    for (int r = 0; r < NV; r++) sB[rowid[r]] = rB[r];                                      /* :97 */
    for (int i = NV - 1; i >= 0; i--) {                                                     /* :99-106 */
        for (int r = 0; r < NV; r++) sx[rowid[r]] = rA[r][i];
        const cf reg = cdiv(sB[i], sx[i]);
        for (int t = 0; t < i; t++) sB[t] = cmsub(sB[t], reg, sx[t]);
        sB[i] = reg;
    }
    for (int i = 0; i < NV; i++) xout[i] = sB[i];
}

void orc_cgesv_gpu(float *Af, const float *bf, float *xf) {
    cf A[NV][NV], b[NV], x[NV];
    for (int r = 0; r < NV; r++) { for (int c = 0; c < NV; c++) A[r][c] = ld(Af, r * NV + c); b[r] = ld(bf, r); }
    cgesv_gpu(A, b, x);
    for (int r = 0; r < NV; r++) { st(xf, r, x[r]); for (int c = 0; c < NV; c++) st(Af, r * NV + c, A[r][c]); }
}

/* ====================================================================== */
/* GPU tracker -- gpu-kernels/kernel_GPUHC_..._PH_CodeOpt_TrunPaths.cu:45-290 */
/* ====================================================================== */
/* the 32-slot __shfl_down_sync tree of :235-238 (slots 30, 31 read as 0)  */
static inline float tree_sum(const float *v) {
    float a[16], b[8], c[4], d[2];
    for (int l = 0; l < 16; l++) a[l] = v[l] + ((l + 16 < NV) ? v[l + 16] : 0.0f);
    for (int l = 0; l < 8; l++) b[l] = a[l] + a[l + 8];
    for (int l = 0; l < 4; l++) c[l] = b[l] + b[l + 4];
    for (int l = 0; l < 2; l++) d[l] = c[l] + c[l + 2];
    return d[0] + d[1];
}

static void gpuhc_one_path(const orc_hc_settings *s, int bid, const float *ssf, const float *spf,
                           const float *tpf, const float *dpf, const int *U, float *tracks,
                           uint8_t *conv_o, uint8_t *inf_o, orc_path_stats *st_o) {
    const int k = bid % NT, smp = bid / NT;           /* :67-69 */
    const int *dHdx = U, *dHdt = U + ORC_HX_SIZE;
    cf x[NV + 1], xl[NV + 1], sols[NV + 1], p[NPP], dif[NPP];
    cf A[NV][NV], B[NV], kk[NV];
    float *trk = tracks + (size_t)bid * (NV + 1) * 2;
    for (int i = 0; i < NV; i++) {                    /* :101-103 */
        sols[i] = ld(ssf + (size_t)k * (NV + 1) * 2, i);
        x[i] = ld(trk, i);
        xl[i] = x[i];
    }
    sols[NV] = x[NV] = xl[NV] = cmk(1.0f, 0.0f);      /* :119-121 */
    for (int i = 0; i < NPP; i++) dif[i] = ld(dpf + (size_t)smp * NPP * 2, i); /* :107-118 */
    p[ORC_NP] = cmk(1.0f, 0.0f);                      /* :122 */

    int succ = 0;                                     /* sipiv[30], :123 */
    float t0 = 0.0f, t_step = 0.0f, delta_t = 0.01f;  /* :80 */
    int end_zone = 0, check_depths = s->no_truncation ? 0 : 1;   /* 0: archived ..._PH_CodeOpt.cu */
    int isSucc = 0, isInf = 0;
    int nsteps = 0, ncorr = 0;
    float vs[NV], vc[NV];
    static const unsigned char scales[3] = {1, 0, 1};

    for (int step = 0; step <= s->max_steps; step++) {                     /* :138 */
        if (!((double)t0 < 1.0 && (1.0 - (double)t0 > 0.0000001))) break; /* :139, :277 */
        if (!end_zone && (double)fabsf(1.0f - t0) <= 0.0500001) end_zone = 1; /* :144 */
        if (check_depths) {                                               /* :149-153 */
            int allpos = 1;
            for (int i = 0; i < 8; i++) allpos &= (x[i].x > 0.0f);
            if (t0 > 0.0f) check_depths = allpos ? 0 : 1;
        }
        if ((double)t0 > 0.95 && check_depths) break;                     /* :154 */
        if (end_zone) {                                                   /* :156-162 */
            if (delta_t > fabsf(1.0f - t0)) delta_t = fabsf(1.0f - t0);
        } else if ((double)delta_t > fabs(0.95 - (double)t0)) {
            delta_t = (float)fabs(0.95 - (double)t0);
        }
        t_step = t0;                                                      /* :164 */
        const float h2 = (float)(0.5 * (double)delta_t);                  /* :165 */
        float scale = 0.0f;
        int coef = 1;
        nsteps++;
        for (int rk = 0; rk < 4; rk++) {                                  /* :178 */
            orc_param_homotopy_gpu(t0, spf, tpf + (size_t)smp * NPP * 2, (float *)p);
            for (int r = 0; r < NV; r++) {
                for (int c = 0; c < NV; c++) A[r][c] = hx_entry(dHdx, r, c, x, p);
                B[r] = ht_row(dHdt, r, x, p, dif);
            }
            cgesv_gpu(A, B, kk);                                          /* :188 */
            if (rk < 3 && s->explicit_rk) {
                /* archived ..._PH.cu with dev-get-new-data.cuh:37-71 (gc = MAGMA_C_ONE):
                   s += ((k*dt)*gc*1.0)/(6|3); x = (rk ? x_last : x) + k*((h2|dt)*gc) */
                const cf one = cmk(1.0f, 0.0f);
                const float dv = rk == 0 ? 6.0f : 3.0f;
                const cf g = cmk(rk == 2 ? delta_t : h2, 0.0f);
                for (int r = 0; r < NV; r++) {
                    sols[r] = cadd(sols[r], cdivs(cscale(cmul(cscale(kk[r], delta_t), one), 1.0f), dv));
                    if (rk > 0) x[r] = xl[r];
                    x[r] = cadd(x[r], cmul(kk[r], g));
                }
                if (rk != 1) t0 += h2;
            } else if (rk < 3) {                                          /* :191-205 */
                const float w = (float)((double)coef * 1.0 / 6.0);
                for (int r = 0; r < NV; r++) {
                    sols[r] = cadd(sols[r], cscale(cscale(kk[r], delta_t), w));
                    if (coef > 1) x[r] = xl[r];
                }
                scale += (float)scales[rk] * h2;
                coef <<= scales[rk];
                for (int r = 0; r < NV; r++) x[r] = cadd(x[r], cscale(kk[r], scale));
                t0 += (float)scales[rk] * h2;
            }
        }
        for (int r = 0; r < NV; r++) {                                    /* :209-210 */
            sols[r] = cadd(sols[r], cdivs(cscale(cscale(kk[r], delta_t), 1.0f), 6.0f));
            x[r] = sols[r];
        }
        for (int c = 0; c < s->max_corrections; c++) {                    /* :217-250 */
            for (int r = 0; r < NV; r++) {
                for (int cc = 0; cc < NV; cc++) A[r][cc] = hx_entry(dHdx, r, cc, x, p);
                B[r] = h_row(dHdt, r, x, p);
            }
            cgesv_gpu(A, B, kk);
            ncorr++;
            for (int r = 0; r < NV; r++) {
                x[r] = csub(x[r], kk[r]);
                vs[r] = kk[r].x * kk[r].x + kk[r].y * kk[r].y;
                vc[r] = x[r].x * x[r].x + x[r].y * x[r].y;
            }
            const float ns = tree_sum(vs), nc = tree_sum(vc);
            isSucc = (double)ns < 0.000001 * (double)nc;                  /* :241 */
            isInf = (double)nc > 1e14;                                    /* :242 */
            if (isInf) break;
            if (isSucc) break;
        }
        if (isInf) break;                                                 /* :252 */
        if (!isSucc) {                                                    /* :257-265 */
            delta_t = (float)((double)delta_t * 0.5);
            for (int r = 0; r < NV; r++) { x[r] = xl[r]; sols[r] = xl[r]; }
            succ = 0;
            t0 = t_step;
        } else {                                                          /* :266-275 */
            succ++;
            for (int r = 0; r < NV; r++) { xl[r] = x[r]; sols[r] = x[r]; }
            if (succ >= s->inc_steps) { succ = 0; delta_t *= 2.0f; }
        }
    }
    for (int i = 0; i < NV; i++) st(trk, i, x[i]);                        /* :282 */
    conv_o[bid] = ((double)t0 >= 1.0 || (1.0 - (double)t0 <= 0.0000001)) ? 1 : 0; /* :284 */
    inf_o[bid] = isInf ? 1 : 0;                                           /* :285 */
    if (st_o) { st_o[bid].steps = nsteps; st_o[bid].corrections = ncorr; st_o[bid].inliers21 = 0; st_o[bid].inliers31 = 0; }
}

void orc_gpuhc_track(const orc_hc_settings *s, int N, const float *ss, const float *sp,
                     const float *tp, const float *dp, const int *U, float *tracks,
                     uint8_t *conv, uint8_t *inf, orc_path_stats *stats) {
    const int total = N * NT;
#ifdef _OPENMP
    const int nth = s->num_threads > 0 ? s->num_threads : omp_get_max_threads();
#pragma omp parallel for schedule(dynamic) num_threads(nth)
#endif
    for (int b = 0; b < total; b++) gpuhc_one_path(s, b, ss, sp, tp, dp, U, tracks, conv, inf, stats);
}

void orc_gpuhc_track_subset(const orc_hc_settings *s, int n, const int *ids, const float *ss,
                            const float *sp, const float *tp, const float *dp, const int *U,
                            float *tracks, uint8_t *conv, uint8_t *inf, orc_path_stats *stats) {
#ifdef _OPENMP
    const int nth = s->num_threads > 0 ? s->num_threads : omp_get_max_threads();
#pragma omp parallel for schedule(dynamic) num_threads(nth)
#endif
    for (int i = 0; i < n; i++) gpuhc_one_path(s, ids[i], ss, sp, tp, dp, U, tracks, conv, inf, stats);
}

/* ====================================================================== */
/* hypothesis scoring -- magmaHC/dev-trifocal_2op1p-eval.cuh:28-250        */
/* rnorm3df(a,b,c) -> 1/sqrtf(a*a+b*b+c*c); hypotf(x,y) -> sqrtf(x*x+y*y); */
/* fdividef -> IEEE division (documented deviations).           */
/* ====================================================================== */
static inline float rnorm3(float a, float b, float c) { return 1.0f / sqrtf(a * a + b * b + c * c); }
static inline float hyp(float a, float b) { return sqrtf(a * a + b * b); }

int orc_score_hypothesis(const float *xf, int E, const float *loc, const float *K, int *in21, int *in31) {
    *in21 = 0; *in31 = 0;
    for (int i = 18; i < 30; i++)                                        /* :46-51 */
        if (!((double)fabsf(xf[2 * i + 1]) < 1e-5)) return 0;
    float d[NV], R[18];
    for (int i = 0; i < NV; i++) d[i] = xf[2 * i];                       /* :61 */
    for (int m = 0; m < 2; m++) {                                        /* :64-92 */
        const float a = d[m * 3 + 24], b = d[m * 3 + 25], c = d[m * 3 + 26];
        float *r = R + m * 9;
        r[0] = 1.0f + a * a - (b * b + c * c);
        r[1] = 2.0f * (a * b - c);
        r[2] = 2.0f * (a * c + b);
        r[3] = 2.0f * (a * b + c);
        r[4] = 1.0f + b * b - (a * a + c * c);
        r[5] = 2.0f * (b * c - a);
        r[6] = 2.0f * (a * c - b);
        r[7] = 2.0f * (b * c + a);
        r[8] = 1.0f + c * c - (a * a + b * b);
        const float n0 = rnorm3(r[0], r[3], r[6]);
        const float n1 = rnorm3(r[1], r[4], r[7]);
        const float n2 = rnorm3(r[2], r[5], r[8]);
        r[0] *= n0; r[1] *= n0; r[2] *= n0;
        r[3] *= n1; r[4] *= n1; r[5] *= n1;
        r[6] *= n2; r[7] *= n2; r[8] *= n2;
    }
    const float fx = K[0], fy = K[4], cx = K[3] /* reference bug, :140 */, cy = K[5];
    int c21 = 0, c31 = 0;
    for (int e = 0; e < E; e++) {                                        /* :105-231 */
        const float *g = loc + (size_t)e * 6;
        float num, den, v0, v1, v2, ex, ey;
        num = d[20] * (R[2] * g[2] + R[5] * g[3] + R[8]) - (R[2] * d[18] + R[5] * d[19] + R[8] * d[20]);
        den = 1.0f - (R[6] * g[0] + R[7] * g[1] + R[8]) * (R[2] * g[2] + R[5] * g[3] + R[8]);
        v2 = num * (R[6] * g[0] + R[7] * g[1] + R[8]) + den * d[20];
        v0 = (num * (R[0] * g[0] + R[1] * g[1] + R[2]) + den * d[18]) / v2;
        v1 = (num * (R[3] * g[0] + R[4] * g[1] + R[5]) + den * d[19]) / v2;
        ex = (v0 * fx + cx) - (g[2] * fx + cx);
        ey = (v1 * fy + cy) - (g[3] * fy + cy);
        if (hyp(ex, ey) < 2.0f) c21++;
        num = d[23] * (R[11] * g[4] + R[14] * g[5] + R[17]) - (R[11] * d[21] + R[14] * d[22] + R[17] * d[23]);
        den = 1.0f - (R[15] * g[0] + R[16] * g[1] + R[17]) * (R[11] * g[4] + R[14] * g[5] + R[17]);
        v2 = num * (R[15] * g[0] + R[16] * g[1] + R[17]) + den * d[23];
        v0 = (num * (R[9] * g[0] + R[10] * g[1] + R[11]) + den * d[21]) / v2;
        v1 = (num * (R[12] * g[0] + R[13] * g[1] + R[14]) + den * d[22]) / v2;
        ex = (v0 * fx + cx) - (g[4] * fx + cx);
        ey = (v1 * fy + cy) - (g[5] * fy + cy);
        if (hyp(ex, ey) < 2.0f) c31++;
    }
    *in21 = c21; *in31 = c31;
    const float r21 = (float)c21 / (float)E, r31 = (float)c31 / (float)E; /* :241-242 */
    return ((double)r21 >= 0.90 && (double)r31 >= 0.90) ? 1 : 0;
}

/* ====================================================================== */
/* Pose recovery + maximal-support selection:       */
/* Evaluations::Transform_GPUHC_Sols_to_Trifocal_Relative_Pose            */
/* (Evaluations.cpp:298-358), get_Solution_with_Maximal_Support (:382-504) */
/* and the util.hpp helpers they call, written in the reference's own      */
/* structure: a candidate list in batch-id order, then a loop over         */
/* candidates x edgels with the running ">=" maximum.                      */
/* ====================================================================== */
/* util.hpp:104-112 get_Matrix_Vector_Product<3> (accumulates from 0.0)   */
static void u_matvec(const float *M, const float *V, float *MV) {
    for (int i = 0; i < 3; i++) {
        MV[i] = 0.0f;
        for (int j = 0; j < 3; j++) MV[i] += M[i * 3 + j] * V[j];
    }
}
/* util.hpp:114-124 get_Matrix_Transpose<3> (in place)                    */
static void u_transpose(float *R) {
    float T[9];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) T[i * 3 + j] = R[j * 3 + i];
    for (int i = 0; i < 9; i++) R[i] = T[i];
}
/* util.hpp:76-78 get_Vector_Norm                                         */
static float u_norm(const float *v) { return sqrtf(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]); }
/* util.hpp:69-74 Normalize_Translation_Vector                            */
static void u_normalize_t(float *t) {
    const float n = u_norm(t);
    t[0] /= n; t[1] /= n; t[2] /= n;
}
/* util.hpp:31-66 Cayley_To_Rotation_Matrix + Normalize_Rotation_Matrix   */
static void u_cayley(const float *r, float *R) {
    R[0] = 1 + r[0] * r[0] - (r[1] * r[1] + r[2] * r[2]);
    R[1] = 2 * (r[0] * r[1] - r[2]);
    R[2] = 2 * (r[0] * r[2] + r[1]);
    R[3] = 2 * (r[0] * r[1] + r[2]);
    R[4] = 1 + r[1] * r[1] - (r[0] * r[0] + r[2] * r[2]);
    R[5] = 2 * (r[1] * r[2] - r[0]);
    R[6] = 2 * (r[0] * r[2] - r[1]);
    R[7] = 2 * (r[1] * r[2] + r[0]);
    R[8] = 1 + r[2] * r[2] - (r[0] * r[0] + r[1] * r[1]);
    const float n1 = sqrtf(R[0] * R[0] + R[3] * R[3] + R[6] * R[6]);
    const float n2 = sqrtf(R[1] * R[1] + R[4] * R[4] + R[7] * R[7]);
    const float n3 = sqrtf(R[2] * R[2] + R[5] * R[5] + R[8] * R[8]);
    R[0] /= n1; R[3] /= n1; R[6] /= n1;
    R[1] /= n2; R[4] /= n2; R[7] /= n2;
    R[2] /= n3; R[5] /= n3; R[8] /= n3;
}
/* util.hpp:169-186 get_depth_rho                                         */
static float u_depth_rho(const float *g1, const float *g2, float *R, const float *T) {
    float mvp[3], Rg2[3], rho;
    u_transpose(R);
    u_matvec(R, g2, mvp);
    for (int i = 0; i < 3; i++) Rg2[i] = mvp[i];
    rho = T[2] * Rg2[2];
    u_matvec(R, T, mvp);
    rho -= mvp[2];
    u_transpose(R);
    u_matvec(R, g1, mvp);
    rho /= (float)(1 - mvp[2] * Rg2[2]);
    return rho;
}
/* util.hpp:188-209 get_Reprojection_Pixels_Error (gamma2 scaled in place) */
static float u_reproj_px(const float *g1, float *g2, const float *R, const float *T, const float *K, float rho1) {
    float mvp[3];
    u_matvec(R, g1, mvp);
    for (int i = 0; i < 3; i++) { mvp[i] *= rho1; mvp[i] += T[i]; }
    mvp[0] /= mvp[2];
    mvp[1] /= mvp[2];
    mvp[0] = mvp[0] * K[0] + K[2];
    mvp[1] = mvp[1] * K[4] + K[5];
    g2[0] = g2[0] * K[0] + K[2];
    g2[1] = g2[1] * K[4] + K[5];
    mvp[0] -= g2[0];
    mvp[1] -= g2[1];
    mvp[2] = 0.0f;
    return u_norm(mvp);
}

typedef struct { float R21[9], t21[3], R31[9], t31[3]; } orc_pose;

/* Evaluations.cpp:235-265 from the 31-complex track x                    */
static void convert_pose(const float *x, orc_pose *P) {
    for (int i = 0; i < 3; i++) { P->t21[i] = x[2 * (18 + i)]; P->t31[i] = x[2 * (21 + i)]; }
    u_normalize_t(P->t21);
    u_normalize_t(P->t31);
    float r[3];
    for (int i = 0; i < 3; i++) r[i] = x[2 * (24 + i)];
    u_cayley(r, P->R21);
    for (int i = 0; i < 3; i++) r[i] = x[2 * (27 + i)];
    u_cayley(r, P->R31);
}

int orc_pose_support(int num_paths, const float *tracks, const uint8_t *conv, int E, const float *loc,
                     const float *K, int quirks, int32_t *inliers, orc_pose_selection *sel) {
    /* ---- Transform_GPUHC_Sols_to_Trifocal_Relative_Pose (:298-358) ---- */
    int *cand = (int *)malloc(sizeof(int) * (size_t)(num_paths > 0 ? num_paths : 1));
    orc_pose *poses = (orc_pose *)malloc(sizeof(orc_pose) * (size_t)(num_paths > 0 ? num_paths : 1));
    int nc = 0;
    for (int bs = 0; bs < num_paths; bs++) {
        inliers[2 * bs] = inliers[2 * bs + 1] = -1;
        const int r = bs / ORC_NTRACK;
        const long ci = quirks ? (long)ORC_NTRACK * r + bs : bs;          /* :317 */
        if (ci >= num_paths || !conv[ci]) continue;
        const float *x = tracks + (size_t)bs * (ORC_NV + 1) * 2;
        int small_imag = 0, pos_depth = 0;
        for (int vi = 0; vi < 6; vi++)                                    /* :324-327 */
            if ((double)fabsf(x[2 * (24 + vi) + 1]) < 1e-5) small_imag++;
        if (small_imag < 6) continue;
        for (int di = 0; di < 8; di++)                                    /* :330-332 */
            if (x[2 * di] >= 0) pos_depth++;
        if (pos_depth < 8) continue;
        convert_pose(quirks ? tracks : x, &poses[nc]);                    /* :334-341 */
        cand[nc++] = bs;
    }
    /* ---- get_Solution_with_Maximal_Support (:382-504) ---- */
    int max21 = 0, max31 = 0, pick21 = -1, pick31 = -1;
    for (int cp = 0; cp < nc; cp++) {
        int n21 = 0, n31 = 0;
        orc_pose *P = &poses[cp];
        for (int ei = 0; ei < E; ei++) {
            float g1[3] = {loc[ei * 6 + 0], loc[ei * 6 + 1], 1.0f};
            float g2[3] = {loc[ei * 6 + 2], loc[ei * 6 + 3], 1.0f};
            float g3[3] = {loc[ei * 6 + 4], loc[ei * 6 + 5], 1.0f};
            const float rho21 = u_depth_rho(g1, g2, P->R21, P->t21);
            const float e21 = u_reproj_px(g1, g2, P->R21, P->t21, K, rho21);
            const float rho31 = u_depth_rho(g1, g3, P->R31, P->t31);
            const float e31 = u_reproj_px(g1, g3, P->R31, P->t31, K, rho31);
            if (e21 < 2) n21++;                                           /* REPROJ_ERROR_INLIER_THRESH */
            if (e31 < 2) n31++;
        }
        inliers[2 * cand[cp]] = n21;
        inliers[2 * cand[cp] + 1] = n31;
        /* :455-467: push when >= the running max; the reference then reads element
           [0] (quirks), its commented-out rule keeps the latest one (default) */
        if (n21 >= max21) { max21 = n21; if (!quirks || pick21 < 0) pick21 = cp; }
        if (n31 >= max31) { max31 = n31; if (!quirks || pick31 < 0) pick31 = cp; }
    }
    memset(sel, 0, sizeof(*sel));
    sel->num_candidates = nc;
    sel->path21 = pick21 >= 0 ? cand[pick21] : -1;
    sel->path31 = pick31 >= 0 ? cand[pick31] : -1;
    sel->inliers21 = pick21 >= 0 ? inliers[2 * cand[pick21]] : -1;
    sel->inliers31 = pick31 >= 0 ? inliers[2 * cand[pick31] + 1] : -1;
    if (pick21 >= 0) { memcpy(sel->R21, poses[pick21].R21, 36); memcpy(sel->t21, poses[pick21].t21, 12); }
    if (pick31 >= 0) { memcpy(sel->R31, poses[pick31].R31, 36); memcpy(sel->t31, poses[pick31].t31, 12); }
    free(cand);
    free(poses);
    return nc > 0;                                                       /* :490-503 */
}

/* Evaluations.cpp:360-380 + :523-543 (Measure_Relative_Pose_Error)       */
static float rot_residual(const float *gt, const float *R) {
    float G[9], M[9];
    for (int i = 0; i < 9; i++) G[i] = gt[i];
    u_transpose(G);
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
            M[i * 3 + j] = 0;
            for (int k = 0; k < 3; k++) M[i * 3 + j] += G[i * 3 + k] * R[k * 3 + j];
        }
    float tr = 0.0f;
    for (int i = 0; i < 3; i++) tr += M[i * 3 + i];
    return (float)acos(0.5 * (tr - 1.0));
}
static float transl_residual(const float *gt_t, const float *t) {
    float g[3] = {gt_t[0], gt_t[1], gt_t[2]};
    u_normalize_t(g);
    float dot = 0.0f;
    for (int i = 0; i < 3; i++) dot += g[i] * t[i];
    return (float)fabs(dot - 1.0);
}
int orc_pose_residuals(const float *gt21, const float *gt31, const orc_pose_selection *sel, float *out4) {
    out4[0] = rot_residual(gt21, sel->R21);
    out4[1] = rot_residual(gt31, sel->R31);
    out4[2] = transl_residual(gt21 + 9, sel->t21);
    out4[3] = transl_residual(gt31 + 9, sel->t31);
    return out4[2] < 1e-1 && out4[3] < 1e-1 && out4[0] < 1e-1 && out4[1] < 1e-1;
}

/* ====================================================================== */
/* Noisy synthcurves.  Restates the C++ standard     */
/* library pieces the product uses (include/hc_host.h hc_add_pixel_noise):  */
/* std::mt19937_64 (the standard's parameters), generate_canonical<double, */
/* 53> over it, and libstdc++'s normal_distribution<double> (Marsaglia     */
/* polar method, second variate cached).                                   */
/* ====================================================================== */
typedef struct { uint64_t mt[312]; int i; } orc_mt64;
static void mt64_seed(orc_mt64 *g, uint64_t seed) {
    g->mt[0] = seed;
    for (int i = 1; i < 312; i++) g->mt[i] = 6364136223846793005ULL * (g->mt[i - 1] ^ (g->mt[i - 1] >> 62)) + (uint64_t)i;
    g->i = 312;
}
static uint64_t mt64_next(orc_mt64 *g) {
    if (g->i >= 312) {
        for (int k = 0; k < 312; k++) {
            const uint64_t y = (g->mt[k] & 0xFFFFFFFF80000000ULL) | (g->mt[(k + 1) % 312] & 0x7FFFFFFFULL);
            g->mt[k] = g->mt[(k + 156) % 312] ^ (y >> 1) ^ ((y & 1ULL) ? 0xB5026F5AA96619E9ULL : 0ULL);
        }
        g->i = 0;
    }
    uint64_t z = g->mt[g->i++];
    z ^= (z >> 29) & 0x5555555555555555ULL;
    z ^= (z << 17) & 0x71D67FFFEDA60000ULL;
    z ^= (z << 37) & 0xFFF7EEE000000000ULL;
    z ^= z >> 43;
    return z;
}
static double canonical53(orc_mt64 *g) {
    const double r = (double)(mt64_next(g)) / 18446744073709551616.0;   /* one 64-bit draw / 2^64 */
    return r >= 1.0 ? nextafter(1.0, 0.0) : r;
}
typedef struct { orc_mt64 g; int saved_ok; double saved; } orc_normal;
static double normal_next(orc_normal *n, double sigma) {
    double ret;
    if (n->saved_ok) {
        n->saved_ok = 0;
        ret = n->saved;
    } else {
        double x, y, r2;
        do {
            x = 2.0 * canonical53(&n->g) - 1.0;
            y = 2.0 * canonical53(&n->g) - 1.0;
            r2 = x * x + y * y;
        } while (r2 > 1.0 || r2 == 0.0);
        const double mult = sqrt(-2 * log(r2) / r2);
        n->saved = x * mult;
        n->saved_ok = 1;
        ret = y * mult;
    }
    return ret * sigma + 0.0;
}
void orc_add_pixel_noise(int E, const float *loc, const float *K, double sigma, uint64_t seed, float *out) {
    orc_normal n;
    mt64_seed(&n.g, seed);
    n.saved_ok = 0;
    n.saved = 0.0;
    const double fx = K[0], cx = K[2], fy = K[4], cy = K[5];
    for (int e = 0; e < E; e++)
        for (int v = 0; v < 3; v++) {
            const double u = (double)loc[e * 6 + 2 * v] * fx + cx + normal_next(&n, sigma);
            const double w = (double)loc[e * 6 + 2 * v + 1] * fy + cy + normal_next(&n, sigma);
            out[e * 6 + 2 * v] = (float)((u - cx) / fx);
            out[e * 6 + 2 * v + 1] = (float)((w - cy) / fy);
        }
}

/* ====================================================================== */
/* LAPACK cgesv semantics (call sites CPUHC_Generic_Solver_Eval_by_Indx.cpp:93,100,107,114,127) */
/* cgetf2 (right-looking, icamax on cabs1, first max) + cgetrs: the test  */
/* build's LU.  The reference links OpenBLAS 0.3.23, whose kernels differ  */
/* in FMA use; orc_set_external_cgesv routes the CPU-HC solves through that */
/* library (tests/cpuhc_pin.py), which with the plain-operator build     */
/* reproduces CPU_Sols_Statistics.txt exactly (tests/test_oracle_kat.py).  */
/* ====================================================================== */
static int cgesv_lapack(cf *A /* col-major 30x30 */, cf *B) {
    int ipiv[NV], info = 0;
#define AA(i, j) A[(j) * NV + (i)]
    for (int j = 0; j < NV; j++) {
        int jp = j;
        float mx = fabsf(AA(j, j).x) + fabsf(AA(j, j).y);
        for (int i = j + 1; i < NV; i++) {
            const float v = fabsf(AA(i, j).x) + fabsf(AA(i, j).y);
            if (v > mx) { mx = v; jp = i; }
        }
        ipiv[j] = jp;
        if (AA(jp, j).x != 0.0f || AA(jp, j).y != 0.0f) {
            if (jp != j)
                for (int c = 0; c < NV; c++) { cf t = AA(j, c); AA(j, c) = AA(jp, c); AA(jp, c) = t; }
            const cf r = cdiv(cmk(1.0f, 0.0f), AA(j, j));
            for (int i = j + 1; i < NV; i++) AA(i, j) = cmul(AA(i, j), r);
        } else if (info == 0) {
            info = j + 1;
        }
        for (int c = j + 1; c < NV; c++) {
            const cf u = AA(j, c);
            for (int i = j + 1; i < NV; i++) AA(i, c) = cmsub(AA(i, c), AA(i, j), u);
        }
    }
    if (info != 0) return info;                       /* cgesv: no getrs when singular */
    for (int j = 0; j < NV; j++) if (ipiv[j] != j) { cf t = B[j]; B[j] = B[ipiv[j]]; B[ipiv[j]] = t; }
    for (int j = 0; j < NV; j++)                      /* L y = Pb (unit lower) */
        for (int i = j + 1; i < NV; i++) B[i] = cmsub(B[i], B[j], AA(i, j));
    for (int j = NV - 1; j >= 0; j--) {               /* U x = y */
        B[j] = cdiv(B[j], AA(j, j));
        for (int i = 0; i < j; i++) B[i] = cmsub(B[i], B[j], AA(i, j));
    }
#undef AA
    return 0;
}

int orc_cgesv_lapack(float *Af, float *Bf) {
    cf A[NV * NV], B[NV];
    for (int i = 0; i < NV * NV; i++) A[i] = ld(Af, i);
    for (int i = 0; i < NV; i++) B[i] = ld(Bf, i);
    const int info = cgesv_lapack(A, B);
    for (int i = 0; i < NV * NV; i++) st(Af, i, A[i]);
    for (int i = 0; i < NV; i++) st(Bf, i, B[i]);
    return info;
}


/* Experiment hook (tests/cpuhc_pin.py only): route the CPU-HC solves through
   an external LAPACK cgesv with the ILP64 interface (OpenBLAS `cgesv_64_`),
   the library the reference links (CPUHC_Generic_Solver_Eval_by_Indx.cpp:93). */
typedef void (*orc_ext_cgesv64)(const long long *n, const long long *nrhs, void *A, const long long *lda,
                                long long *ipiv, void *B, const long long *ldb, long long *info);
static orc_ext_cgesv64 g_ext_cgesv = 0;
void orc_set_external_cgesv(void *fn) { g_ext_cgesv = (orc_ext_cgesv64)fn; }
static inline void cpu_lu(cf *A, cf *B) {
    if (g_ext_cgesv) {
        const long long n = NV, nrhs = 1, ld = NV;
        long long ipiv[NV], info = 0;
        g_ext_cgesv(&n, &nrhs, A, &ld, ipiv, B, &ld, &info);
        return;
    }
    cgesv_lapack(A, B);
}

/* ====================================================================== */
/* CPU-HC -- cpuhc-solvers/CPUHC_Generic_Solver_Eval_by_Indx.cpp:22-251     */
/* cpu-jacobian-evals/cpu-eval-indx_trifocal_2op1p_30x30.hpp:22-89 (column-major A) */
/* ====================================================================== */
static void cpuhc_one_path(const orc_hc_settings *s, int bid, const float *ssf, const float *spf,
                           const float *tpf, const float *dpf, const int *dHdx, const int *dHdt,
                           float *tracks, uint8_t *conv_o, uint8_t *inf_o, orc_path_stats *st_o) {
    const int k = bid % NT, smp = bid / NT;                               /* :40-41 */
    cf x[NV + 1], inter[NV + 1], last[NV + 1], p[NPP], dif[NPP];
    cf A[NV * NV], B[NV];
    const float *tpp = tpf + (size_t)smp * NPP * 2;
    for (int i = 0; i <= NV; i++) {                                       /* Feed_Start_Sols x3 */
        x[i] = ld(ssf + (size_t)k * (NV + 1) * 2, i);
        inter[i] = x[i];
        last[i] = x[i];
    }
    for (int i = 0; i < NPP; i++) dif[i] = ld(dpf + (size_t)smp * NPP * 2, i);
    int succ = 0, isSucc = 0, isInf = 0, end_zone = 0, nsteps = 0, ncorr = 0;
    float t0 = 0.0f, t_step = 0.0f, delta_t = 0.01f;
#define EVAL_HX()                                                                        \
    for (int r = 0; r < NV; r++)                                                         \
        for (int c = 0; c < NV; c++) A[c * NV + r] = hx_entry(dHdx, r, c, x, p)
#define EVAL_HT() for (int r = 0; r < NV; r++) B[r] = ht_row(dHdt, r, x, p, dif)
    for (int step = 0; step <= s->max_steps; step++) {                    /* :67 */
        if (!((double)t0 < 1.0 && (1.0 - (double)t0 > 0.0000001))) break;
        if (!end_zone && (double)fabsf(1.0f - t0) <= 0.0500001) end_zone = 1; /* :73 */
        if (end_zone) {
            if (delta_t > fabsf(1.0f - t0)) delta_t = fabsf(1.0f - t0);
        } else if ((double)delta_t > fabs(0.95 - (double)t0)) {
            delta_t = (float)fabs(0.95 - (double)t0);
        }
        t_step = t0;
        const float h2 = (float)(0.5 * (double)delta_t);                  /* :84 */
        nsteps++;
        /* (i) :90-94 + k2 helper :180-191 */
        param_homotopy_cpu(t0, spf, tpp, p); EVAL_HX(); EVAL_HT(); cpu_lu(A, B);
        for (int i = 0; i < NV; i++) {
            inter[i] = cadd(inter[i], cdivs(cscale(cscale(B[i], delta_t), 1.0f), 6.0f));
            B[i] = cscale(B[i], h2);
            x[i] = cadd(x[i], B[i]);
        }
        t0 += h2;
        /* (ii) :97-101 + k3 helper :193-205 */
        param_homotopy_cpu(t0, spf, tpp, p); EVAL_HX(); EVAL_HT(); cpu_lu(A, B);
        for (int i = 0; i < NV; i++) {
            inter[i] = cadd(inter[i], cdivs(cscale(cscale(B[i], delta_t), 1.0f), 3.0f));
            x[i] = last[i];
            B[i] = cscale(B[i], h2);
            x[i] = cadd(x[i], B[i]);
        }
        /* (iii) :104-108 + k4 helper :207-220 */
        param_homotopy_cpu(t0, spf, tpp, p); EVAL_HX(); EVAL_HT(); cpu_lu(A, B);
        for (int i = 0; i < NV; i++) {
            inter[i] = cadd(inter[i], cdivs(cscale(cscale(B[i], delta_t), 1.0f), 3.0f));
            x[i] = last[i];
            B[i] = cscale(B[i], delta_t);
            x[i] = cadd(x[i], B[i]);
        }
        t0 += h2;
        /* (iv) :111-117 + prediction :222-230 */
        param_homotopy_cpu(t0, spf, tpp, p); EVAL_HX(); EVAL_HT(); cpu_lu(A, B);
        for (int i = 0; i < NV; i++) {
            inter[i] = cadd(inter[i], cdivs(cscale(cscale(B[i], delta_t), 1.0f), 6.0f));
            x[i] = inter[i];
        }
        for (int c = 0; c < s->max_corrections; c++) {                    /* :122-135 */
            EVAL_HX();
            for (int r = 0; r < NV; r++) B[r] = h_row(dHdt, r, x, p);
            cpu_lu(A, B);
            ncorr++;
            float sq_sols = 0.0f, sq_corr = 0.0f;                         /* :232-251 */
            for (int i = 0; i < NV; i++) {
                x[i] = csub(x[i], B[i]);
                sq_sols += B[i].x * B[i].x + B[i].y * B[i].y;
                sq_corr += x[i].x * x[i].x + x[i].y * x[i].y;
            }
            isSucc = (double)sq_sols < 0.000001 * (double)sq_corr;
            isInf = (double)sq_corr > 1e14;
            if (isSucc) break;
            if (isInf) break;
        }
        if (isInf) break;                                                 /* :138-141 */
        if (!isSucc) {                                                    /* :146-155 */
            succ = 0;
            delta_t = (float)((double)delta_t * 0.5);
            t0 = t_step;
            for (int i = 0; i < NV; i++) { x[i] = last[i]; inter[i] = last[i]; }
        } else {                                                          /* :156-166 */
            for (int i = 0; i < NV; i++) { last[i] = x[i]; inter[i] = x[i]; }
            succ++;
            if (succ >= s->inc_steps) { succ = 0; delta_t *= 2.0f; }
        }
    }
#undef EVAL_HX
#undef EVAL_HT
    float *trk = tracks + (size_t)bid * (NV + 1) * 2;
    for (int i = 0; i < NV; i++) st(trk, i, x[i]);
    trk[2 * NV] = 1.0f; trk[2 * NV + 1] = 0.0f;
    conv_o[bid] = ((double)t0 >= 1.0 || (1.0 - (double)t0 <= 0.0000001)) ? 1 : 0; /* :172 */
    inf_o[bid] = isInf ? 1 : 0;                                           /* :139 */
    if (st_o) { st_o[bid].steps = nsteps; st_o[bid].corrections = ncorr; st_o[bid].inliers21 = 0; st_o[bid].inliers31 = 0; }
}

double orc_cpuhc_track(const orc_hc_settings *s, int N, const float *ss, const float *sp,
                       const float *tp, const float *dp, const int *dHdx, const int *dHdt,
                       float *tracks, uint8_t *conv, uint8_t *inf, orc_path_stats *stats) {
    const int total = N * NT;
#ifdef _OPENMP
    const int nth = s->num_threads > 0 ? s->num_threads : omp_get_max_threads();
    const double t0 = omp_get_wtime();
#pragma omp parallel for schedule(dynamic) num_threads(nth)
#endif
    for (int b = 0; b < total; b++) cpuhc_one_path(s, b, ss, sp, tp, dp, dHdx, dHdt, tracks, conv, inf, stats);
#ifdef _OPENMP
    return omp_get_wtime() - t0;
#else
    return 0.0;
#endif
}

/* ====================================================================== */
/* counts -- magmaHC/Evaluations.cpp:145-182                                */
/* ====================================================================== */
void orc_count_solutions(int N, const float *tracks, const uint8_t *conv, const uint8_t *inf, int *out) {
    int nc = 0, nr = 0, ni = 0;
    for (int b = 0; b < N * NT; b++) {
        if (conv[b]) nc++;
        if (inf[b]) ni++;
        if (conv[b]) {
            int real = 0;
            for (int v = 0; v < NV; v++)
                if ((double)fabsf(tracks[((size_t)b * (NV + 1) + v) * 2 + 1]) <= 1e-4) real++;
            if (real == NV) nr++;
        }
    }
    out[0] = nc; out[1] = nr; out[2] = ni;
}
