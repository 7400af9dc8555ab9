// hc_kernels.hip -- MI355X (gfx950) GPU-HC tracker kernels + the C-ABI of
// include/hc_trifocal.h.
//
// Replaces magmaHC/gpu-kernels/kernel_GPUHC_trifocal_2op1p_30x30_PH_CodeOpt_TrunPaths[_TrunRANSAC][_Volta].cu
// (the four CUDA/MAGMA kernels + launchers, magmaHC-kernels.hpp:24-105).
//
// Design: a persistent grid of 256-thread workgroups; each of the
// 4 wavefronts pulls path ids b = sample*312 + track from a device work queue
// (one agent-scope atomicAdd per path) and tracks that path alone: lane r < 30
// owns Jacobian row r, RHS r and x_r in VGPRs.  One predictor/corrector
// "stage" = p(t) (LDS) + dH/dx + dH/dt|H from the LDS-resident compacted index
// tables + the register LU.  Early abort (TrunRANSAC) scores converged paths
// with all 64 lanes and raises an agent-scope flag.
#include "hc_device.hpp"
#include "hc_lu3.hpp"
#include "hc_track4.hpp"
#include "hc_lu3s.hpp"
#include "hc_lu9.hpp"
#include "../../include/hc_trifocal.h"

#include <atomic>
#include <cstdlib>
#include <mutex>

namespace hc {

thread_local hipError_t g_last_hip_error = hipSuccess;   // shared with hc_pose.hip (hc_last_error_string)
static inline hcStatus launch_status(hcStatus on_fail) {
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) { g_last_hip_error = e; return on_fail; }
    return HC_SUCCESS;
}

// Longest-processing-time-first dequeue order (scripts/make_track_order.py):
// queue position q -> track c_track_order[q / N], sample q % N.  Results are
// per batch id, so the order only changes when a path runs, not what it computes.
__constant__ int c_track_order[NTRK] = {
#include "hc_track_order.inc"
};
__device__ __forceinline__ int path_of_queue_pos(int q, int num_paths, int ordered) {
    if (!ordered) return q;
    const int n = num_paths / NTRK;          // samples in this launch
    const int rank = q / n;
    return (q - rank * n) * NTRK + c_track_order[rank];
}

constexpr int WG_THREADS = 256;
constexpr int WAVES_PER_WG = WG_THREADS / WAVE;

struct KArgs {
    int num_paths;
    int ordered;        // dequeue track-major in c_track_order (abort mode off)
    int max_steps, max_corr, inc_steps;
    const cf *start_sols;
    const cf *const *start_sols_array;
    cf *tracks;
    cf *const *track_array;
    const cf *start_params;
    const cf *target_params;
    const cf *diff_params;
    uint8_t *conv;
    uint8_t *inf;
    hcPathStats *stats;
    TableWS *ws;
    TableWS2 *ws2;
    TableWS3 *ws3;
    // abort mode
    int num_edgels;
    const float *edgels;
    const float *K;
    uint8_t *found_flag;
    int32_t *batch_index;
};

// ---------------------------------------------------------------- table prep
// Compacts the reference's padded unified index (38880 ints) into the slot
// tables of TableWS.  One workgroup, thread r < 30 = equation row r.
__global__ void __launch_bounds__(64) k_prep_tables(const int32_t *__restrict__ U, TableWS *ws,
                                                    const uint8_t *found_in) {
    __shared__ int cnt[NV][32];
    __shared__ int s_nslot[NV], s_base[NV + 1];
    const int r = threadIdx.x;
    if (r < NV) {
        for (int c = 0; c < NV; c++) {
            int n = 0;
            for (int j = 0; j < HX_TERMS; j++) n += U[(c * HX_TERMS + j) * HX_PARTS * NV + r] != 0;
            cnt[c][r] = n;
        }
    }
    __syncthreads();
    if (r == 0) {
        int base = 0;
        for (int c = 0; c < NV; c++) {
            int mx = 0;
            for (int q = 0; q < NV; q++) mx = max(mx, cnt[c][q]);
            s_nslot[c] = mx;
            s_base[c] = base;
            base += mx;
        }
        s_base[NV] = base;
        for (int c = 0; c < NV; c++) { ws->nslot[c] = s_nslot[c]; ws->slot_base[c] = s_base[c]; }
        ws->nslot[NV] = base;
        if (base > HX_SLOT_CAP) ws->status = HC_ERROR_TABLE;
        if (found_in) ws->found = found_in[0] ? 1u : 0u;
    }
    __syncthreads();
    const bool overflow = s_base[NV] > HX_SLOT_CAP;
    if (r < 32 && !overflow) {
        for (int c = 0; c < NV; c++) {
            int k = 0;
            if (r < NV) {
                for (int j = 0; j < HX_TERMS; j++) {
                    const int base = (c * HX_TERMS + j) * HX_PARTS * NV + r;
                    const int co = U[base];
                    if (co == 0) continue;
                    const uint32_t w = (uint32_t)(co & 0xF) | ((uint32_t)U[base + NV] << 4) |
                                       ((uint32_t)U[base + 2 * NV] << 10) | ((uint32_t)U[base + 3 * NV] << 16) |
                                       ((uint32_t)U[base + 4 * NV] << 21);
                    ws->hx[(s_base[c] + k) * 32 + r] = w;
                    k++;
                }
            }
            for (; k < s_nslot[c]; k++) ws->hx[(s_base[c] + k) * 32 + r] = 0u;
        }
        const int32_t *D = U + HX_SIZE;
        int k = 0;
        if (r < NV) {
            for (int j = 0; j < HT_TERMS; j++) {
                const int base = j * HT_PARTS * NV + r;
                const int co = D[base];
                if (co == 0) continue;
                const uint32_t w = (uint32_t)(co & 0xF) | ((uint32_t)D[base + NV] << 4) | ((uint32_t)D[base + 2 * NV] << 10) |
                                   ((uint32_t)D[base + 3 * NV] << 16) | ((uint32_t)D[base + 4 * NV] << 21) |
                                   ((uint32_t)D[base + 5 * NV] << 26);
                ws->ht[k * 32 + r] = w;
                k++;
            }
        }
        for (; k < HT_TERMS; k++) ws->ht[k * 32 + r] = 0u;
    }
    // ---- v2: per-lane dH/dx term lists + column -> entry-slot map
    __shared__ int s_len[32];
    TableWS2 *w2 = (TableWS2 *)((char *)ws + ((sizeof(TableWS) + 255) & ~(size_t)255));
    if (r < 32) {
        int n = 0, slot = 0;
        uint32_t map[3] = {0u, 0u, 0u};
        for (int c = 0; c < NV; c++) map[c / 10] |= 6u << (3 * (c % 10));
        if (r < NV) {
            for (int c = 0; c < NV; c++) {
                int last_j = -1;
                for (int j = 0; j < HX_TERMS; j++)
                    if (U[(c * HX_TERMS + j) * HX_PARTS * NV + r] != 0) last_j = j;
                if (last_j < 0) continue;
                for (int j = 0; j <= last_j; j++) {
                    const int base = (c * HX_TERMS + j) * HX_PARTS * NV + r;
                    const int co = U[base];
                    if (co == 0) continue;
                    if (n < HX2_SLOT_CAP && slot < 6)
                        w2->hx[n * 32 + r] = (uint32_t)(co & 0xF) | ((uint32_t)U[base + NV] << 4) |
                                             ((uint32_t)U[base + 2 * NV] << 10) | ((uint32_t)U[base + 3 * NV] << 16) |
                                             ((uint32_t)U[base + 4 * NV] << 21) | ((uint32_t)slot << 26) |
                                             ((uint32_t)(j == last_j) << 29);
                    n++;
                }
                map[c / 10] = (map[c / 10] & ~(7u << (3 * (c % 10)))) | ((uint32_t)slot << (3 * (c % 10)));
                slot++;
            }
        }
        for (int q = 0; q < 3; q++) w2->map[q][r] = map[q];
        s_len[r] = (slot > 6) ? (1 << 20) : n;
    }
    __syncthreads();
    if (r == 0) {
        int mx = 0;
        for (int q = 0; q < 32; q++) mx = max(mx, s_len[q]);
        w2->hx_len = mx;
        w2->status = (mx > HX2_SLOT_CAP) ? HC_ERROR_TABLE : 0;
    }
    __syncthreads();
    if (r < 32) {
        const int len = min(w2->hx_len, HX2_SLOT_CAP);
        for (int k2 = s_len[r]; k2 < len; k2++) w2->hx[k2 * 32 + r] = 0u;
    }
    // ---- v3: the same per-lane term lists as LDS byte offsets (hc_eval3.hpp)
    TableWS3 *w3 = (TableWS3 *)((char *)w2 + ((sizeof(TableWS2) + 255) & ~(size_t)255));
    __shared__ int s_bad;
    if (r == 0) s_bad = 0;
    __syncthreads();
    const uint2 pad_hx = make_uint2((uint32_t)(SLOT_OFF_P + 8 * 33) | ((uint32_t)(SLOT_OFF_P + 8 * 33) << 16),
                                    (uint32_t)(SLOT_OFF_X + 8 * 30) | ((uint32_t)(SLOT_OFF_X + 8 * 30) << 8));
    if (r < 32) {
        int n = 0, slot = 0;
        bool bad = false;
        if (r < NV) {
            for (int c = 0; c < NV; c++) {
                int last_j = -1;
                for (int j = 0; j < HX_TERMS; j++)
                    if (U[(c * HX_TERMS + j) * HX_PARTS * NV + r] != 0) last_j = j;
                if (last_j < 0) continue;
                for (int j = 0; j <= last_j; j++) {
                    const int base = (c * HX_TERMS + j) * HX_PARTS * NV + r;
                    const int co = U[base], a = U[base + NV], b = U[base + 2 * NV], u = U[base + 3 * NV],
                              v = U[base + 4 * NV];
                    if (co == 0) continue;
                    bad |= co < -128 || co > 127 || a < 0 || a >= NPP || b < 0 || b >= NPP || u < 0 || u > NV ||
                           v < 0 || v > NV || slot >= 6;
                    if (n < HX3_SLOT_CAP && !bad)
                        w3->hx[n * 32 + r] = make_uint2(
                            (uint32_t)(SLOT_OFF_P + 8 * a) | ((uint32_t)(SLOT_OFF_P + 8 * b) << 16),
                            (uint32_t)(SLOT_OFF_X + 8 * u) | ((uint32_t)(SLOT_OFF_X + 8 * v) << 8) |
                                (((uint32_t)co & 0xFFu) << 16) | ((uint32_t)(8 * slot) << 24) |
                                ((uint32_t)(j == last_j) << 31));
                    n++;
                }
                slot++;
            }
        }
        if (n > HX3_SLOT_CAP) bad = true;
        for (int k2 = n; k2 < HX3_SLOT_CAP; k2++) w3->hx[k2 * 32 + r] = pad_hx;
        s_len[r] = n;
        const int32_t *D = U + HX_SIZE;
        int k = 0;
        if (r < NV) {
            for (int j = 0; j < HT_TERMS; j++) {
                const int base = j * HT_PARTS * NV + r;
                const int co = D[base], a = D[base + NV], b = D[base + 2 * NV], u = D[base + 3 * NV],
                          v = D[base + 4 * NV], x3 = D[base + 5 * NV];
                if (co == 0) continue;
                bad |= co < -128 || co > 127 || a < 0 || a >= NPP || b < 0 || b >= NPP || u < 0 || u > NV ||
                       v < 0 || v > NV || x3 < 0 || x3 > NV;
                if (!bad)
                    w3->ht[k * 32 + r] = make_uint2(
                        (uint32_t)(SLOT_OFF_P + 8 * a) | ((uint32_t)(SLOT_OFF_P + 8 * b) << 16),
                        (uint32_t)(SLOT_OFF_X + 8 * u) | ((uint32_t)(SLOT_OFF_X + 8 * v) << 8) |
                            ((uint32_t)(SLOT_OFF_X + 8 * x3) << 16) | (((uint32_t)co & 0xFFu) << 24));
                k++;
            }
        }
        for (; k < HT_TERMS; k++) w3->ht[k * 32 + r] = make_uint2(pad_hx.x, pad_hx.y | ((uint32_t)(SLOT_OFF_X + 8 * 30) << 16));
        if (bad) atomicOr(&s_bad, 1);
    }
    __syncthreads();
    if (r == 0) {
        int mx = 0;
        for (int q = 0; q < 32; q++) mx = max(mx, s_len[q]);
        w3->hx_len = mx;
        w3->status = s_bad ? HC_ERROR_TABLE : 0;
    }
}

__host__ __device__ __forceinline__ TableWS2 *ws2_of(TableWS *ws) {
    return (TableWS2 *)((char *)ws + ((sizeof(TableWS) + 255) & ~(size_t)255));
}
__host__ __device__ __forceinline__ TableWS3 *ws3_of(TableWS *ws) {
    return (TableWS3 *)((char *)ws2_of(ws) + ((sizeof(TableWS2) + 255) & ~(size_t)255));
}

// per-workgroup LDS
struct WaveLDS {
    cf x[32];     // current track, x[30] = 1
    cf p[NPP];    // p(t)
    cf tgt[NPP];  // target params of the current sample
    cf dif[NPP];  // diff params of the current sample
};
struct BlockLDS {
    uint32_t hx[HX_SLOT_CAP * 32];
    uint32_t ht[HT_TERMS * 32];
    cf sp[NPP];
    WaveLDS w[WAVES_PER_WG];
};

__device__ __forceinline__ void load_tables(BlockLDS &L, const TableWS *ws, const cf *start_params) {
    const int S = ws->nslot[NV];
    for (int i = threadIdx.x; i < S * 32; i += WG_THREADS) L.hx[i] = ws->hx[i];
    for (int i = threadIdx.x; i < HT_TERMS * 32; i += WG_THREADS) L.ht[i] = ws->ht[i];
    if (threadIdx.x < NPP) L.sp[threadIdx.x] = start_params[threadIdx.x];
    __syncthreads();
}

// ---------------------------------------------------------------- tracker
// kernel_GPUHC_trifocal_pose_PH_CodeOpt_TrunPaths (.cu:45-290) and, with
// ABORT, ..._TrunPaths_TrunRANSAC (.cu:45-327).
template <bool ABORT>
__global__ void __launch_bounds__(WG_THREADS) k_track(KArgs a) {
    __shared__ BlockLDS L;
    TableWS *ws = a.ws;
    if (ws->status != 0u) return;
    load_tables(L, ws, a.start_params);
    if (ABORT && threadIdx.x == 0) {
        const unsigned long long now = __builtin_amdgcn_s_memrealtime();
        atomicCAS(&ws->t_start, 0ull, now);
    }
    const int lane = lane_id();
    const int l32 = lane & 31;
    const int wid = threadIdx.x / WAVE;
    WaveLDS &W = L.w[wid];
    const int *__restrict__ g_nslot = ws->nslot;
    const int *__restrict__ g_base = ws->slot_base;
    if (lane == 30) W.x[30] = cmk(1.0f, 0.0f);
    if (lane == 31) W.x[31] = cmk(0.0f, 0.0f);
    if (lane == 33) W.p[33] = cmk(1.0f, 0.0f);
    int cur_smp = -1;

    for (;;) {
        int b = 0;
        if (lane == 0) b = (int)atomicAdd(&ws->queue, 1u);
        b = uni(b);
        if (b >= a.num_paths) break;
        const int trk = b % NTRK, smp = b / NTRK;                          // :67-69
        cf *dtrack = a.track_array ? a.track_array[b] : a.tracks + (size_t)b * (NV + 1);
        if (ABORT) {                                                       // TrunRANSAC.cu:152
            const unsigned f = __hip_atomic_load(&ws->found, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (uni((int)f) != 0) {                                        // skipped: x stays start, conv 0
                if (lane == 0) {
                    a.conv[b] = 0;
                    a.inf[b] = 0;
                    if (a.stats) a.stats[b] = hcPathStats{0, 0, 0, 0};
                }
                continue;
            }
        }
        if (smp != cur_smp) {                                              // :107-118
            if (lane < NPP) {
                W.tgt[lane] = a.target_params[(size_t)smp * NPP + lane];
                W.dif[lane] = a.diff_params[(size_t)smp * NPP + lane];
            }
            cur_smp = smp;
        }
        const cf *dstart = a.start_sols_array ? a.start_sols_array[trk] : a.start_sols + (size_t)trk * (NV + 1);
        const bool rl = lane < NV;
        cf x = rl ? dtrack[lane] : cmk(0.0f, 0.0f);                      // :101-103
        cf sols = rl ? dstart[lane] : cmk(0.0f, 0.0f);
        cf xl = x;
        wave_lds_sync();

        float t0 = 0.0f, t_step = 0.0f, delta_t = 0.01f;                   // :80
        bool end_zone = false, check_depths = true, isSucc = false, isInf = false;
        int succ = 0, nsteps = 0, ncorr = 0;

        for (int step = 0; step <= a.max_steps; step++) {                  // :138
            if (!((double)t0 < 1.0 && (1.0 - (double)t0 > 0.0000001))) break;
            if (!end_zone && (double)__builtin_fabsf(1.0f - t0) <= 0.0500001) end_zone = true;  // :144
            if (check_depths) {                                            // :149-153
                const unsigned long long pos = __ballot(lane < 8 && x.x > 0.0f);
                const bool allpos = (pos & 0xFFull) == 0xFFull;
                if (t0 > 0.0f) check_depths = !allpos;
            }
            if ((double)t0 > 0.95 && check_depths) break;                  // :154
            if (end_zone) {                                                // :156-162
                if (delta_t > __builtin_fabsf(1.0f - t0)) delta_t = __builtin_fabsf(1.0f - t0);
            } else if ((double)delta_t > __builtin_fabs(0.95 - (double)t0)) {
                delta_t = (float)__builtin_fabs(0.95 - (double)t0);
            }
            t_step = t0;
            const float h2 = (float)(0.5 * (double)delta_t);               // :165
            float scale = 0.0f;
            int coef = 1;
            nsteps++;
            // one stage per iteration: s = 0..3 predictor (RK4), s >= 4 corrector
            for (int s = 0;; s++) {
                const bool pred = s < 4;
                if (pred) {                                                // :181
                    const float omt = (float)(1.0 - (double)t0);
                    if (lane < NPP - 1) W.p[lane] = cadd(cscale(W.tgt[lane], t0), cscale(L.sp[lane], omt));
                }
                if (rl) W.x[lane] = x;
                wave_lds_sync();
                cf rA[NV];
                eval_hx(rA, L.hx, g_nslot, g_base, W.x, W.p, l32);         // :184 / :220
                const cf rB = pred ? eval_ht(L.ht, W.x, W.p, W.dif, l32)   // :185
                                   : eval_h(L.ht, W.x, W.p, l32);          // :221
                wave_lds_sync();
                const cf k = lu_solve(rA, rB, lane);                       // :188 / :224
                if (pred) {
                    if (s < 3) {                                           // :191-205
                        const float w = (float)((double)coef * 1.0 / 6.0);
                        sols = cadd(sols, cscale(cscale(k, delta_t), w));
                        if (coef > 1) x = xl;
                        const int sc = (s == 1) ? 0 : 1;                   // scales {1,0,1}
                        scale += (float)sc * h2;
                        coef <<= sc;
                        x = cadd(x, cscale(k, scale));
                        t0 += (float)sc * h2;
                    } else {                                               // :209-210
                        sols = cadd(sols, cdivs(cscale(cscale(k, delta_t), 1.0f), 6.0f));
                        x = sols;
                    }
                    if (a.max_corr <= 0 && s == 3) break;
                } else {                                                   // :228-249
                    x = csub(x, k);
                    ncorr++;
                    const float vs = rl ? k.x * k.x + k.y * k.y : 0.0f;
                    const float vc = rl ? x.x * x.x + x.y * x.y : 0.0f;
                    const float ns = tree_sum32(vs), nc = tree_sum32(vc);
                    isSucc = (double)ns < 0.000001 * (double)nc;
                    isInf = (double)nc > 1e14;
                    if (isInf || isSucc || (s - 4) + 1 >= a.max_corr) break;
                }
            }
            if (isInf) break;                                              // :252
            if (!isSucc) {                                                 // :257-265
                delta_t = (float)((double)delta_t * 0.5);
                x = xl;
                sols = xl;
                succ = 0;
                t0 = t_step;
            } else {                                                       // :266-275
                succ++;
                xl = x;
                sols = x;
                if (succ >= a.inc_steps) { succ = 0; delta_t *= 2.0f; }
            }
        }
        // write back (:282-286)
        const bool converged = ((double)t0 >= 1.0 || (1.0 - (double)t0 <= 0.0000001));
        if (rl) dtrack[lane] = x;
        int2 inl = make_int2(0, 0);
        if (ABORT && converged) {                                          // TrunRANSAC.cu:312-322
            if (rl) W.x[lane] = x;
            wave_lds_sync();
            const unsigned long long im_ok =
                __ballot(lane >= 18 && lane < NV && (double)__builtin_fabsf(x.y) < 1e-5);
            if ((im_ok & 0x3FFC0000ull) == 0x3FFC0000ull) {                // lanes 18..29, eval.cuh:46-53
                Hyp h;
                make_hypothesis(W.x, h);
                const float fx = a.K[0], fy = a.K[4], cx = a.K[3] /* eval quirk */, cy = a.K[5];
                inl = score_hypothesis(h, a.edgels, a.num_edgels, fx, fy, cx, cy, lane);
                const float r21 = (float)inl.x / (float)a.num_edgels;
                const float r31 = (float)inl.y / (float)a.num_edgels;
                if ((double)r21 >= 0.90 && (double)r31 >= 0.90 && lane == 0) {   // :241-246
                    __hip_atomic_store(&ws->found, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    a.found_flag[0] = 1;
                    a.batch_index[b] = b;
                    atomicCAS(&ws->t_found, 0ull, (unsigned long long)__builtin_amdgcn_s_memrealtime());
                }
            }
            wave_lds_sync();
        }
        if (lane == 0) {
            a.conv[b] = converged ? 1 : 0;
            a.inf[b] = isInf ? 1 : 0;
            if (a.stats) a.stats[b] = hcPathStats{nsteps, ncorr, inl.x, inl.y};
        }
    }
}

// ---------------------------------------------------------------- tracker v2
// Two paths per wavefront (hc_track2.hpp).  Each half-wave is a path slot with
// its own stage machine; one loop iteration runs one stage (p(t), dH/dx,
// dH/dt|H, LU) for both slots.  Phases of a slot:
enum : int { PH_DEQ = 0, PH_BEGIN = 1, PH_STAGE = 2, PH_FINISH = 3, PH_IDLE = 4 };

__device__ __forceinline__ int half_sum_i(int v) {
    v += dpp_i<DPP_QP_1032>(v);
    v += dpp_i<DPP_QP_2301>(v);
    v += dpp_i<DPP_ROW_HALF_MIRROR>(v);
    v += dpp_i<DPP_ROW_MIRROR>(v);
    v += swz_xor16_i(v);
    return v;
}

// Abort-mode scoring of one half's converged path (dev-trifocal_2op1p-eval.cuh:
// 28-250, 32 lanes per path): inlier counts of views 2 and 3 over all triplet
// edgels.  Out of line: it runs once per converged path, and inlined its
// registers weigh on the stage loop's allocation (72 VGPR spills).
template <int VIEW>   // 0: view 2 (edgel columns 2, 3), 1: view 3 (columns 4, 5)
__device__ __forceinline__ int score_view(const float *R, float da, float db, float dc, const float *edgels,
                                          int num_edgels, float fx, float fy, float cx, float cy, int r) {
    int c = 0;
    for (int e = r; e < num_edgels; e += 32) {
        const float *g = edgels + (size_t)e * 6;
        const float g0 = g[0], g1 = g[1], gu = g[2 + 2 * VIEW], gv = g[3 + 2 * VIEW];
        const float num = dc * (R[2] * gu + R[5] * gv + R[8]) - (R[2] * da + R[5] * db + R[8] * dc);
        const float den = 1.0f - (R[6] * g0 + R[7] * g1 + R[8]) * (R[2] * gu + R[5] * gv + R[8]);
        const float v2 = num * (R[6] * g0 + R[7] * g1 + R[8]) + den * dc;
        const float v0 = (num * (R[0] * g0 + R[1] * g1 + R[2]) + den * da) / v2;
        const float v1 = (num * (R[3] * g0 + R[4] * g1 + R[5]) + den * db) / v2;
        const float ex = (v0 * fx + cx) - (gu * fx + cx);
        const float ey = (v1 * fy + cy) - (gv * fy + cy);
        c += (__builtin_sqrtf(ex * ex + ey * ey) < 2.0f) ? 1 : 0;
    }
    return c;
}
// The two views are scored in separate passes, each from its own evaluation
// of the hypothesis (12 live values instead of 24): the abort kernel's register
// allocation is otherwise set by this cold path.
__device__ __forceinline__ int2 score_half(const cf *sx, const float *edgels, int num_edgels,
                                           const float *K, int r) {
    const float fx = K[0], fy = K[4], cx = K[3] /* eval quirk */, cy = K[5];
    int c21, c31;
    {
        Hyp hy;
        make_hypothesis(sx, hy);
        c21 = score_view<0>(hy.R, hy.T[0], hy.T[1], hy.T[2], edgels, num_edgels, fx, fy, cx, cy, r);
    }
    {
        const cf *sx2 = sx;
        asm volatile("" : "+v"(sx2));   // a second evaluation, not the first one kept live
        Hyp hy;
        make_hypothesis(sx2, hy);
        c31 = score_view<1>(hy.R + 9, hy.T[3], hy.T[4], hy.T[5], edgels, num_edgels, fx, fy, cx, cy, r);
    }
    return make_int2(half_sum_i(c21), half_sum_i(c31));
}

#ifdef HC_DIAG_PHASES
// diagnostic build: per-phase shader cycles summed over waves (k_track2):
// [0] slot phases, [1] park + p(t), [2] dH/dx, [3] dH/dt | H, [4] LU forward,
// [5] LU backward, [6] stage update, [7] wave lifetime, [8] waves; with
// HC_DIAG_LU the forward steps' parts [9] pivot search, [10] row broadcast,
// [11] reciprocal + multipliers, [12] rank-1 update
__device__ unsigned long long g_diag_phase[13];
#endif

// GTAB: the term tables are read from the workspace (global, L1/L2-resident)
// instead of being staged in LDS (10 KB less LDS per workgroup; experiment)
template <bool ABORT, int MINW, int V, int WGT = WG_THREADS, bool GTAB = false>
__global__ void __launch_bounds__(WGT, MINW) k_track2(KArgs a) {
    // V = 2: bpermute LU + v2 evals; V = 3: LDS-broadcast LU + packed v3 evals;
    // V = 8: v3 evals + the structurally sparse LU of hc_lu3s.hpp
    constexpr bool EV3 = V >= 3;
    constexpr int TAB_BYTES = GTAB ? 16 : EV3 ? (int)(sizeof(uint2) * (HX3_SLOT_CAP + HT_TERMS) * 32)
                                     : (int)(sizeof(uint32_t) * (HX2_SLOT_CAP + HT_TERMS) * 32);
    __shared__ __attribute__((aligned(16))) char s_tab[TAB_BYTES];
    __shared__ cf s_sp[NPP];
    __shared__ SlotLDS s_slot[2 * (WGT / WAVE)];
    TableWS *ws = a.ws;
    TableWS2 *w2 = a.ws2;
    TableWS3 *w3 = a.ws3;
    if ((ws->status | (unsigned)w2->status | (EV3 ? (unsigned)w3->status : 0u)) != 0u) return;
    const int hx_len = EV3 ? w3->hx_len : w2->hx_len;
    uint32_t *s_hx2 = reinterpret_cast<uint32_t *>(s_tab);
    uint32_t *s_ht = s_hx2 + HX2_SLOT_CAP * 32;
    const uint2 *s_hx3 = GTAB ? w3->hx : reinterpret_cast<const uint2 *>(s_tab);
    const uint2 *s_ht3 = GTAB ? w3->ht : reinterpret_cast<const uint2 *>(s_tab) + HX3_SLOT_CAP * 32;
    if constexpr (GTAB) {
    } else if constexpr (EV3) {
        uint2 *t_hx3 = reinterpret_cast<uint2 *>(s_tab), *t_ht3 = t_hx3 + HX3_SLOT_CAP * 32;
        for (int i = threadIdx.x; i < HX3_SLOT_CAP * 32; i += WGT) t_hx3[i] = w3->hx[i];   // padded table
        for (int i = threadIdx.x; i < HT_TERMS * 32; i += WGT) t_ht3[i] = w3->ht[i];
    } else {
        for (int i = threadIdx.x; i < hx_len * 32; i += WGT) s_hx2[i] = w2->hx[i];
        for (int i = threadIdx.x; i < HT_TERMS * 32; i += WGT) s_ht[i] = ws->ht[i];
    }
    if (threadIdx.x < NPP) s_sp[threadIdx.x] = a.start_params[threadIdx.x];
    {
        float *z = reinterpret_cast<float *>(s_slot);
        for (int i = threadIdx.x; i < (int)(sizeof(s_slot) / 4); i += WGT) z[i] = 0.0f;
    }
    __syncthreads();
    if (ABORT && threadIdx.x == 0) atomicCAS(&ws->t_start, 0ull, (unsigned long long)__builtin_amdgcn_s_memrealtime());
    const int lane = lane_id();
    const int r = lane & 31, hb = lane & 32;
    const int wid = threadIdx.x / WAVE;
    SlotLDS &S = s_slot[wid * 2 + (hb >> 5)];
    if (r == 30) S.x[30] = cmk(1.0f, 0.0f);
    if (r == 0) S.p[33] = cmk(1.0f, 0.0f);
    // per-row constants (column->slot maps, structural pattern) live in LDS and
    // are re-read every stage: held in VGPRs across the loop they spill (abort mode)
    __shared__ uint32_t s_rowc[4][32];
    if (threadIdx.x < 32) {
        const uint32_t m0[3] = {w2->map[0][threadIdx.x], w2->map[1][threadIdx.x], w2->map[2][threadIdx.x]};
        s_rowc[0][threadIdx.x] = m0[0];
        s_rowc[1][threadIdx.x] = m0[1];
        s_rowc[2][threadIdx.x] = m0[2];
        s_rowc[3][threadIdx.x] = V >= 8 ? row_pattern(m0) : 0u;   // structural pattern of row r (v8 LU)
    }
    __syncthreads();
    const bool rl = r < NV;
    wave_lds_sync();

    // per-slot state (uniform within a half)
    int ph = PH_DEQ, b = -1, smp_loaded = -1;
    unsigned found_seen = 0u;   // abort mode: the found flag as of the last stage
#ifdef HC_DIAG_TIMES
    int diag_t0 = 0;
#endif
    int s = 0, stepidx = 0, coef = 1, succ = 0, nsteps = 0, ncorr = 0;
    float t0 = 0.0f, t_step = 0.0f, dt = 0.01f, h2 = 0.0f, scale = 0.0f;
    bool end_zone = false, check = true, isSucc = false, isInf = false;
    cf x = cmk(0.0f, 0.0f), xl = x, sols = x;

#ifdef HC_DIAG_PHASES
    uint64_t dg[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#ifdef HC_DIAG_LU
    uint64_t lgd[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#else
    uint64_t *lgd = nullptr;
#endif
    uint64_t dt_ = __builtin_amdgcn_s_memtime(), dt0_ = dt_;
#define HC_DIAG_MARK(k) do { const uint64_t n_ = __builtin_amdgcn_s_memtime(); dg[k] += n_ - dt_; dt_ = n_; } while (0)
#else
#define HC_DIAG_MARK(k) do { } while (0)
#endif
    for (;;) {
        HC_DIAG_MARK(6);
        // ---------------- resolve slot phases until every slot is at a stage or idle
        for (;;) {
            if (ph == PH_FINISH) {                                            // :282-286
                const bool conv = ((double)t0 >= 1.0 || (1.0 - (double)t0 <= 0.0000001));
                cf *dtrack = a.track_array ? a.track_array[b] : a.tracks + (size_t)b * (NV + 1);
                if (rl) dtrack[r] = x;
                int in21 = 0, in31 = 0;
                if (ABORT && conv) {                                          // TrunRANSAC.cu:312-322
                    if (rl) S.x[r] = x;
                    wave_lds_sync();
                    const unsigned long long im = __ballot(r >= 18 && rl && (double)__builtin_fabsf(x.y) < 1e-5);
                    if (((unsigned)(im >> hb) & 0x3FFC0000u) == 0x3FFC0000u) {   // eval.cuh:46-53
                        const int2 c = score_half(S.x, a.edgels, a.num_edgels, a.K, r);
                        in21 = c.x;
                        in31 = c.y;
                        const float r21 = (float)in21 / (float)a.num_edgels, r31 = (float)in31 / (float)a.num_edgels;
                        if ((double)r21 >= 0.90 && (double)r31 >= 0.90 && r == 0) {   // eval.cuh:241-246
                            __hip_atomic_store(&ws->found, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                            a.found_flag[0] = 1;
                            a.batch_index[b] = b;
                            atomicCAS(&ws->t_found, 0ull, (unsigned long long)__builtin_amdgcn_s_memrealtime());
                        }
                    }
                }
                if (r == 0) {
                    a.conv[b] = conv ? 1 : 0;
                    a.inf[b] = isInf ? 1 : 0;
#ifdef HC_DIAG_TIMES
                    // diagnostic build: dequeue / finish device timestamps (100 MHz) of each path
                    in21 = diag_t0;
                    in31 = (int)__builtin_amdgcn_s_memrealtime();
#endif
                    if (a.stats) a.stats[b] = hcPathStats{nsteps, ncorr, in21, in31};
                }
                ph = PH_DEQ;
            }
            if (ph == PH_DEQ) {
                int nb = 0;
                if (r == 0) nb = (int)atomicAdd(&ws->queue, 1u);
                nb = bperm_i(nb, hb);
                if (nb >= a.num_paths) {
                    ph = PH_IDLE;
                    b = -1;
                } else {
                    b = path_of_queue_pos(nb, a.num_paths, a.ordered);
                    bool skip = false;
                    if (ABORT) {                                              // TrunRANSAC.cu:152
                        skip = __hip_atomic_load(&ws->found, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u;
                        skip = bperm_i((int)skip, hb) != 0;
                        if (skip && r == 0) {
                            a.conv[b] = 0;
                            a.inf[b] = 0;
                            if (a.stats) a.stats[b] = hcPathStats{0, 0, 0, 0};
                        }
                    }
                    if (!skip) {
                        const int trk = b % NTRK, smp = b / NTRK;            // :67-69
                        if (smp != smp_loaded && r < NPP) {
                            S.tgt[r] = a.target_params[(size_t)smp * NPP + r];
                            S.dif[r] = a.diff_params[(size_t)smp * NPP + r];
                        }
                        if (smp != smp_loaded && r < NPP - 32) {
                            S.tgt[r + 32] = a.target_params[(size_t)smp * NPP + r + 32];
                            S.dif[r + 32] = a.diff_params[(size_t)smp * NPP + r + 32];
                        }
                        smp_loaded = smp;
#ifdef HC_DIAG_TIMES
                        diag_t0 = (int)__builtin_amdgcn_s_memrealtime();
#endif
                        const cf *dtrack = a.track_array ? a.track_array[b] : a.tracks + (size_t)b * (NV + 1);
                        const cf *dstart = a.start_sols_array ? a.start_sols_array[trk]
                                                              : a.start_sols + (size_t)trk * (NV + 1);
                        x = rl ? dtrack[r] : cmk(0.0f, 0.0f);                 // :101-103
                        sols = rl ? dstart[r] : cmk(0.0f, 0.0f);
                        xl = x;
                        t0 = 0.0f; t_step = 0.0f; dt = 0.01f;                 // :80
                        end_zone = false; check = true; isSucc = false; isInf = false;
                        succ = 0; nsteps = 0; ncorr = 0; stepidx = 0;
                        ph = PH_BEGIN;
                    }
                }
            }
            if (ABORT && ph == PH_BEGIN && stepidx > 0 && found_seen != 0u) {
                // a pose was found: a path in flight stops at its step boundary and
                // reports like a skipped one (track untouched, conv = 0).  The
                // reference's in-flight blocks run on (..._TrunRANSAC.cu:152 only
                // gates the start); their results are not read once found.
                if (r == 0) {
                    a.conv[b] = 0;
                    a.inf[b] = 0;
                    if (a.stats) a.stats[b] = hcPathStats{0, 0, 0, 0};
                }
                ph = PH_DEQ;
            }
            if (ph == PH_BEGIN) {                                             // :138-165
                bool done = stepidx > a.max_steps;
                if (!done) done = !((double)t0 < 1.0 && (1.0 - (double)t0 > 0.0000001));
                if (!done) {
                    if (!end_zone && (double)__builtin_fabsf(1.0f - t0) <= 0.0500001) end_zone = true;
                    if (check) {
                        const unsigned long long pos = __ballot(r < 8 && x.x > 0.0f);
                        const bool allpos = ((unsigned)(pos >> hb) & 0xFFu) == 0xFFu;
                        if (t0 > 0.0f) check = !allpos;
                    }
                    done = (double)t0 > 0.95 && check;
                }
                if (!done) {
                    if (end_zone) {
                        if (dt > __builtin_fabsf(1.0f - t0)) dt = __builtin_fabsf(1.0f - t0);
                    } else if ((double)dt > __builtin_fabs(0.95 - (double)t0)) {
                        dt = (float)__builtin_fabs(0.95 - (double)t0);
                    }
                    t_step = t0;
                    h2 = (float)(0.5 * (double)dt);
                    scale = 0.0f;
                    coef = 1;
                    s = 0;
                    nsteps++;
                }
                ph = done ? PH_FINISH : PH_STAGE;
            }
            if (__ballot(ph == PH_FINISH || ph == PH_DEQ || ph == PH_BEGIN) == 0ull) break;
        }
        if (__ballot(ph == PH_STAGE) == 0ull) break;
        HC_DIAG_MARK(0);
        // the found flag for the next step boundary: read now, used after the stage
#ifndef HC_NO_INFLIGHT_STOP
        if (ABORT) found_seen = __hip_atomic_load(&ws->found, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#endif

        // ---------------- one stage for both slots
        // park the slot state in LDS so it does not occupy VGPRs across eval + LU
        if (r == 0) {
            SlotState q;
            q.t0 = t0; q.t_step = t_step; q.dt = dt; q.h2 = h2; q.scale = scale;
            q.s = s; q.stepidx = stepidx; q.coef = coef; q.succ = succ; q.nsteps = nsteps; q.ncorr = ncorr;
            q.b = b; q.smp = smp_loaded; q.ph = ph;
            q.flags = (end_zone ? 1 : 0) | (check ? 2 : 0) | (isSucc ? 4 : 0) | (isInf ? 8 : 0);
            q.pad = 0;
            S.st = q;
        }
        if (rl) { S.x[r] = x; S.xl[r] = xl; S.sols[r] = sols; }
        {
            const bool act0 = ph == PH_STAGE;
            const bool pred0 = act0 && s < 4;
            if (pred0 && r < NPP - 1) {                                      // :181 p(t), i < 33
                const float omt = (float)(1.0 - (double)t0);
                const cf *sp = s_sp;   // opaque base: the address is not hoisted and held across the loop
                asm volatile("" : "+v"(sp));
                S.p[r] = cadd(cscale(S.tgt[r], t0), cscale(sp[r], omt));
            }
            if (pred0 && r == 0) S.p[32] = cadd(cscale(S.tgt[32], t0), cscale(s_sp[32], (float)(1.0 - (double)t0)));
        }
        wave_lds_sync();
        const int s_in = s, ph_in = ph;
        asm volatile("" :: "v"(s_in), "v"(ph_in));
        // opaque lane id: keeps LICM from hoisting ~30 lane-derived per-pivot
        // constants (bpermute addresses, r == i masks) out of the path loop
        int lane_v = lane_id();   // recomputed (2 VALU), not held across the loop
        asm volatile("" : "+v"(lane_v));
        const int r_v = lane_v & 31;
        const uint32_t map[3] = {s_rowc[0][r_v], s_rowc[1][r_v], s_rowc[2][r_v]};
        const uint32_t row_pat = s_rowc[3][r_v];
        const bool act = ph_in == PH_STAGE;
        const bool pred = act && s_in < 4;
        HC_DIAG_MARK(1);
        // right-hand side first: dH/dt | H need no Jacobian registers, so their
        // LDS gathers can run many terms ahead
        cf rB = cmk(0.0f, 0.0f);
        if (__ballot(pred) != 0ull) {                                        // :185
            const cf t = EV3 ? eval_ht3(s_ht3, S, r_v) : eval_ht2(s_ht, S, r_v);
            if (pred) rB = t;
        }
        if (__ballot(act && !pred) != 0ull) {                                // :221
            const cf t = EV3 ? eval_h3(s_ht3, S, r_v) : eval_h2(s_ht, S, r_v);
            if (!pred) rB = t;
        }
        HC_DIAG_MARK(3);
        cf rA[NV];
        if constexpr (EV3) eval_hx3(rA, s_hx3, hx_len, map, S, r_v);     // :184 / :220
        else eval_hx2(rA, s_hx2, hx_len, map, S, r_v);
        wave_lds_sync();
        HC_DIAG_MARK(2);
        cf k;                                                                // :188 / :224
#ifdef HC_DIAG_PHASES
        if constexpr (V == 8) { uint64_t tm_; k = lu_solve3s(rA, rB, lane_v, row_pat, *reinterpret_cast<LUBuf *>(S.ent), &tm_, lgd); dg[4] += tm_ - dt_; dt_ = tm_; }
        else
#endif
        if constexpr (V == 9) k = lu_solve9<LU9_PROD>(rA, rB, lane_v, row_pat, *reinterpret_cast<LUBuf *>(S.ent));
        else if constexpr (V == 8) k = lu_solve3s(rA, rB, lane_v, row_pat, *reinterpret_cast<LUBuf *>(S.ent));
        else if constexpr (V == 3) k = lu_solve3(rA, rB, lane_v, *reinterpret_cast<LUBuf *>(S.ent));
        else k = lu_solve2(rA, rB, lane_v);
        wave_lds_sync();
        HC_DIAG_MARK(5);
        {
            const SlotState q = S.st;
            t0 = q.t0; t_step = q.t_step; dt = q.dt; h2 = q.h2; scale = q.scale;
            s = q.s; stepidx = q.stepidx; coef = q.coef; succ = q.succ; nsteps = q.nsteps; ncorr = q.ncorr;
            b = q.b; smp_loaded = q.smp; ph = q.ph;
            end_zone = q.flags & 1; check = q.flags & 2; isSucc = q.flags & 4; isInf = q.flags & 8;
            x = rl ? S.x[r] : cmk(0.0f, 0.0f);
            xl = rl ? S.xl[r] : cmk(0.0f, 0.0f);
            sols = rl ? S.sols[r] : cmk(0.0f, 0.0f);
        }
        if (act) {
            bool step_end = false;
            if (pred) {
                if (s < 3) {                                                 // :191-205
                    const float w = (float)((double)coef * 1.0 / 6.0);
                    sols = cadd(sols, cscale(cscale(k, dt), w));
                    if (coef > 1) x = xl;
                    const int sc = (s == 1) ? 0 : 1;
                    scale += (float)sc * h2;
                    coef <<= sc;
                    x = cadd(x, cscale(k, scale));
                    t0 += (float)sc * h2;
                } else {                                                     // :209-210
                    sols = cadd(sols, cdivs(cscale(cscale(k, dt), 1.0f), 6.0f));
                    x = sols;
                }
                s++;
                if (s == 4 && a.max_corr <= 0) step_end = true;
            } else {                                                         // :228-249
                x = csub(x, k);
                ncorr++;
                const float vs = rl ? k.x * k.x + k.y * k.y : 0.0f;
                const float vc = rl ? x.x * x.x + x.y * x.y : 0.0f;
                const float ns = tree_sum_half(vs), nc = tree_sum_half(vc);
                isSucc = (double)ns < 0.000001 * (double)nc;
                isInf = (double)nc > 1e14;
                if (isInf || isSucc || (s - 4) + 1 >= a.max_corr) step_end = true;
                else s++;
            }
            if (step_end) {
                if (isInf) {                                                 // :252
                    ph = PH_FINISH;
                } else {
                    if (!isSucc) {                                           // :257-265
                        dt = (float)((double)dt * 0.5);
                        x = xl;
                        sols = xl;
                        succ = 0;
                        t0 = t_step;
                    } else {                                                 // :266-275
                        succ++;
                        xl = x;
                        sols = x;
                        if (succ >= a.inc_steps) { succ = 0; dt *= 2.0f; }
                    }
                    stepidx++;
                    ph = PH_BEGIN;
                }
            }
        }
    }
#ifdef HC_DIAG_PHASES
    HC_DIAG_MARK(0);
    if (lane == 0) {
        dg[7] = __builtin_amdgcn_s_memtime() - dt0_;
        for (int q = 0; q < 8; q++) atomicAdd(&g_diag_phase[q], (unsigned long long)dg[q]);
        atomicAdd(&g_diag_phase[8], 1ull);
#ifdef HC_DIAG_LU
        for (int q = 0; q < 4; q++) atomicAdd(&g_diag_phase[9 + q], (unsigned long long)lgd[q]);
#endif
    }
#endif
#undef HC_DIAG_MARK
}

// ---------------------------------------------------------------- tracker v4
// Four paths per wavefront (hc_track4.hpp): each 16-lane DPP row is a path
// slot with its own stage machine (t, step size, stage, path id uniform per
// row); lane r owns rows / unknowns r and r + 16.  One loop iteration runs one
// predictor or corrector stage (p(t), dH/dx, dH/dt|H, LU) for all four slots.
// The stage logic is k_track2's (..._TrunPaths.cu:138-280) per row.
template <bool ABORT>
#ifndef HC_V4_MINW
#define HC_V4_MINW 2
#endif
__global__ void __launch_bounds__(WG_THREADS, HC_V4_MINW) k_track4(KArgs a) {
    constexpr int TAB_BYTES = (int)(sizeof(uint2) * (HX3_SLOT_CAP + HT_TERMS) * 32);
    __shared__ __attribute__((aligned(16))) char s_tab[TAB_BYTES];
    __shared__ cf s_sp[NPP];
    __shared__ SlotLDS4 s_slot[4 * WAVES_PER_WG];
    TableWS *ws = a.ws;
    TableWS2 *w2 = a.ws2;
    TableWS3 *w3 = a.ws3;
    if ((ws->status | (unsigned)w2->status | (unsigned)w3->status) != 0u) return;
    const int hx_len = w3->hx_len;
    uint2 *s_hx3 = reinterpret_cast<uint2 *>(s_tab);
    uint2 *s_ht3 = s_hx3 + HX3_SLOT_CAP * 32;
    for (int i = threadIdx.x; i < hx_len * 32; i += WG_THREADS) s_hx3[i] = rebase_p_offsets(w3->hx[i]);
    for (int i = threadIdx.x; i < HT_TERMS * 32; i += WG_THREADS) s_ht3[i] = rebase_p_offsets(w3->ht[i]);
    if (threadIdx.x < NPP) s_sp[threadIdx.x] = a.start_params[threadIdx.x];
    {
        float *z = reinterpret_cast<float *>(s_slot);
        for (int i = threadIdx.x; i < (int)(sizeof(s_slot) / 4); i += WG_THREADS) z[i] = 0.0f;
    }
    __syncthreads();
    if (ABORT && threadIdx.x == 0) atomicCAS(&ws->t_start, 0ull, (unsigned long long)__builtin_amdgcn_s_memrealtime());
    const int lane = lane_id();
    const int r = lane & 15, qb = lane & 48;
    const int wid = threadIdx.x / WAVE;
    SlotLDS4 &S = s_slot[wid * 4 + (qb >> 4)];
    if (r == 0) { S.x[30] = cmk(1.0f, 0.0f); S.p[33] = cmk(1.0f, 0.0f); }
    const uint32_t map0[3] = {w2->map[0][r], w2->map[1][r], w2->map[2][r]};
    const uint32_t map1[3] = {w2->map[0][r + QL], w2->map[1][r + QL], w2->map[2][r + QL]};
    const bool v1 = r + QL < NV;   // slot 1 holds a real row / unknown
    wave_lds_sync();

    int ph = PH_DEQ, b = -1, smp_loaded = -1;
    int s = 0, stepidx = 0, coef = 1, succ = 0, nsteps = 0, ncorr = 0;
    float t0 = 0.0f, t_step = 0.0f, dt = 0.01f, h2 = 0.0f, scale = 0.0f;
    bool end_zone = false, check = true, isSucc = false, isInf = false;
    const cf z0 = cmk(0.0f, 0.0f);
    cf x0 = z0, x1 = z0, xl0 = z0, xl1 = z0, so0 = z0, so1 = z0;
    cf tg0 = z0, tg1 = z0, tg2 = z0;   // target params r, r + 16, 32 of the slot's sample

    for (;;) {
        for (;;) {
            if (ph == PH_FINISH) {                                            // :282-286
                const bool conv = ((double)t0 >= 1.0 || (1.0 - (double)t0 <= 0.0000001));
                cf *dtrack = a.track_array ? a.track_array[b] : a.tracks + (size_t)b * (NV + 1);
                dtrack[r] = x0;
                if (v1) dtrack[r + QL] = x1;
                int in21 = 0, in31 = 0;
                if (ABORT && conv) {                                          // TrunRANSAC.cu:312-322
                    S.x[r] = x0;
                    if (v1) S.x[r + QL] = x1;
                    wave_lds_sync();
                    const unsigned long long im =
                        __ballot(v1 && r >= 2 && (double)__builtin_fabsf(x1.y) < 1e-5);   // x[18..29]
                    if (((unsigned)(im >> qb) & 0x3FFCu) == 0x3FFCu) {       // eval.cuh:46-53
                        Hyp hy;
                        make_hypothesis(S.x, hy);
                        const float fx = a.K[0], fy = a.K[4], cx = a.K[3] /* eval quirk */, cy = a.K[5];
                        const float *R = hy.R;
                        const float d18 = hy.T[0], d19 = hy.T[1], d20 = hy.T[2], d21 = hy.T[3], d22 = hy.T[4], d23 = hy.T[5];
                        int c21 = 0, c31 = 0;
                        for (int e = r; e < a.num_edgels; e += QL) {
                            const float *g = a.edgels + (size_t)e * 6;
                            const float g0 = g[0], g1 = g[1], g2 = g[2], g3 = g[3], g4 = g[4], g5 = g[5];
                            float num, den, w0v, w1v, w2v, ex, ey;
                            num = d20 * (R[2] * g2 + R[5] * g3 + R[8]) - (R[2] * d18 + R[5] * d19 + R[8] * d20);
                            den = 1.0f - (R[6] * g0 + R[7] * g1 + R[8]) * (R[2] * g2 + R[5] * g3 + R[8]);
                            w2v = num * (R[6] * g0 + R[7] * g1 + R[8]) + den * d20;
                            w0v = (num * (R[0] * g0 + R[1] * g1 + R[2]) + den * d18) / w2v;
                            w1v = (num * (R[3] * g0 + R[4] * g1 + R[5]) + den * d19) / w2v;
                            ex = (w0v * fx + cx) - (g2 * fx + cx);
                            ey = (w1v * fy + cy) - (g3 * fy + cy);
                            c21 += (__builtin_sqrtf(ex * ex + ey * ey) < 2.0f) ? 1 : 0;
                            num = d23 * (R[11] * g4 + R[14] * g5 + R[17]) - (R[11] * d21 + R[14] * d22 + R[17] * d23);
                            den = 1.0f - (R[15] * g0 + R[16] * g1 + R[17]) * (R[11] * g4 + R[14] * g5 + R[17]);
                            w2v = num * (R[15] * g0 + R[16] * g1 + R[17]) + den * d23;
                            w0v = (num * (R[9] * g0 + R[10] * g1 + R[11]) + den * d21) / w2v;
                            w1v = (num * (R[12] * g0 + R[13] * g1 + R[14]) + den * d22) / w2v;
                            ex = (w0v * fx + cx) - (g4 * fx + cx);
                            ey = (w1v * fy + cy) - (g5 * fy + cy);
                            c31 += (__builtin_sqrtf(ex * ex + ey * ey) < 2.0f) ? 1 : 0;
                        }
                        in21 = row_sum_i(c21);
                        in31 = row_sum_i(c31);
                        const float r21 = (float)in21 / (float)a.num_edgels, r31 = (float)in31 / (float)a.num_edgels;
                        if ((double)r21 >= 0.90 && (double)r31 >= 0.90 && r == 0) {   // eval.cuh:241-246
                            __hip_atomic_store(&ws->found, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                            a.found_flag[0] = 1;
                            a.batch_index[b] = b;
                            atomicCAS(&ws->t_found, 0ull, (unsigned long long)__builtin_amdgcn_s_memrealtime());
                        }
                    }
                }
                if (r == 0) {
                    a.conv[b] = conv ? 1 : 0;
                    a.inf[b] = isInf ? 1 : 0;
                    if (a.stats) a.stats[b] = hcPathStats{nsteps, ncorr, in21, in31};
                }
                ph = PH_DEQ;
            }
            if (ph == PH_DEQ) {
                int nb = 0;
                if (r == 0) nb = (int)atomicAdd(&ws->queue, 1u);
                nb = qbcast0_i(nb);
                if (nb >= a.num_paths) {
                    ph = PH_IDLE;
                    b = -1;
                } else {
                    b = path_of_queue_pos(nb, a.num_paths, a.ordered);
                    bool skip = false;
                    if (ABORT) {                                              // TrunRANSAC.cu:152
                        int f = 0;
                        if (r == 0) f = (int)__hip_atomic_load(&ws->found, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        skip = qbcast0_i(f) != 0;
                        if (skip && r == 0) {
                            a.conv[b] = 0;
                            a.inf[b] = 0;
                            if (a.stats) a.stats[b] = hcPathStats{0, 0, 0, 0};
                        }
                    }
                    if (!skip) {
                        const int trk = b % NTRK, smp = b / NTRK;            // :67-69
                        if (smp != smp_loaded) {
                            const cf *tp = a.target_params + (size_t)smp * NPP;
                            const cf *dp = a.diff_params + (size_t)smp * NPP;
                            tg0 = tp[r]; tg1 = tp[r + QL]; tg2 = tp[2 * QL];
                            S.dif[r] = dp[r];
                            S.dif[r + QL] = dp[r + QL];
                            if (r < NPP - 2 * QL) S.dif[r + 2 * QL] = dp[r + 2 * QL];
                        }
                        smp_loaded = smp;
                        const cf *dtrack = a.track_array ? a.track_array[b] : a.tracks + (size_t)b * (NV + 1);
                        const cf *dstart = a.start_sols_array ? a.start_sols_array[trk]
                                                              : a.start_sols + (size_t)trk * (NV + 1);
                        x0 = dtrack[r];                                       // :101-103
                        x1 = v1 ? dtrack[r + QL] : z0;
                        so0 = dstart[r];
                        so1 = v1 ? dstart[r + QL] : z0;
                        xl0 = x0; xl1 = x1;
                        t0 = 0.0f; t_step = 0.0f; dt = 0.01f;                 // :80
                        end_zone = false; check = true; isSucc = false; isInf = false;
                        succ = 0; nsteps = 0; ncorr = 0; stepidx = 0;
                        ph = PH_BEGIN;
                    }
                }
            }
            if (ph == PH_BEGIN) {                                             // :138-165
                bool done = stepidx > a.max_steps;
                if (!done) done = !((double)t0 < 1.0 && (1.0 - (double)t0 > 0.0000001));
                if (!done) {
                    if (!end_zone && (double)__builtin_fabsf(1.0f - t0) <= 0.0500001) end_zone = true;
                    if (check) {
                        const unsigned long long pos = __ballot(r < 8 && x0.x > 0.0f);
                        const bool allpos = ((unsigned)(pos >> qb) & 0xFFu) == 0xFFu;
                        if (t0 > 0.0f) check = !allpos;
                    }
                    done = (double)t0 > 0.95 && check;
                }
                if (!done) {
                    if (end_zone) {
                        if (dt > __builtin_fabsf(1.0f - t0)) dt = __builtin_fabsf(1.0f - t0);
                    } else if ((double)dt > __builtin_fabs(0.95 - (double)t0)) {
                        dt = (float)__builtin_fabs(0.95 - (double)t0);
                    }
                    t_step = t0;
                    h2 = (float)(0.5 * (double)dt);
                    scale = 0.0f;
                    coef = 1;
                    s = 0;
                    nsteps++;
                }
                ph = done ? PH_FINISH : PH_STAGE;
            }
            if (__ballot(ph == PH_FINISH || ph == PH_DEQ || ph == PH_BEGIN) == 0ull) break;
        }
        if (__ballot(ph == PH_STAGE) == 0ull) break;

        // ---------------- one stage for all four slots
        S.x[r] = x0;
        if (v1) S.x[r + QL] = x1;
        const bool act = ph == PH_STAGE;
        const bool pred = act && s < 4;
        if (pred) {                                                           // :181 p(t), i < 33
            const float omt = (float)(1.0 - (double)t0);
            S.p[r] = cadd(cscale(tg0, t0), cscale(s_sp[r], omt));
            S.p[r + QL] = cadd(cscale(tg1, t0), cscale(s_sp[r + QL], omt));
            if (r == 0) S.p[32] = cadd(cscale(tg2, t0), cscale(s_sp[32], omt));
        }
        wave_lds_sync();
        // opaque lane id: keeps LICM from hoisting lane-derived per-pivot constants
        int lane_v = lane;
        asm volatile("" : "+v"(lane_v));
        const int r_v = lane_v & 15;
        cf A0[NV], A1[NV];
        eval_hx4(A0, A1, s_hx3, hx_len, map0, map1, S, r_v);                 // :184 / :220
        cf b0 = z0, b1 = z0;
        if (__ballot(pred) != 0ull) {                                         // :185
            cf t0v, t1v;
            eval_ht4(s_ht3, S, r_v, t0v, t1v);
            if (pred) { b0 = t0v; b1 = t1v; }
        }
        if (__ballot(act && !pred) != 0ull) {                                 // :221
            cf t0v, t1v;
            eval_h4(s_ht3, S, r_v, t0v, t1v);
            if (!pred) { b0 = t0v; b1 = t1v; }
        }
        wave_lds_sync();
        cf k0, k1;                                                            // :188 / :224
        lu_solve4(A0, A1, b0, b1, lane_v, *reinterpret_cast<LUBuf *>(S.ent), k0, k1);
        wave_lds_sync();
        if (act) {
            bool step_end = false;
            if (pred) {
                if (s < 3) {                                                  // :191-205
                    const float w = (float)((double)coef * 1.0 / 6.0);
                    so0 = cadd(so0, cscale(cscale(k0, dt), w));
                    so1 = cadd(so1, cscale(cscale(k1, dt), w));
                    if (coef > 1) { x0 = xl0; x1 = xl1; }
                    const int sc = (s == 1) ? 0 : 1;
                    scale += (float)sc * h2;
                    coef <<= sc;
                    x0 = cadd(x0, cscale(k0, scale));
                    x1 = cadd(x1, cscale(k1, scale));
                    t0 += (float)sc * h2;
                } else {                                                      // :209-210
                    so0 = cadd(so0, cdivs(cscale(cscale(k0, dt), 1.0f), 6.0f));
                    so1 = cadd(so1, cdivs(cscale(cscale(k1, dt), 1.0f), 6.0f));
                    x0 = so0;
                    x1 = so1;
                }
                if (!v1) { x1 = z0; so1 = z0; }
                s++;
                if (s == 4 && a.max_corr <= 0) step_end = true;
            } else {                                                          // :228-249
                x0 = csub(x0, k0);
                x1 = v1 ? csub(x1, k1) : z0;
                ncorr++;
                const float vs = (k0.x * k0.x + k0.y * k0.y) + (v1 ? k1.x * k1.x + k1.y * k1.y : 0.0f);
                const float vc = (x0.x * x0.x + x0.y * x0.y) + (v1 ? x1.x * x1.x + x1.y * x1.y : 0.0f);
                const float ns = tree_sum_q(vs), nc = tree_sum_q(vc);
                isSucc = (double)ns < 0.000001 * (double)nc;
                isInf = (double)nc > 1e14;
                if (isInf || isSucc || (s - 4) + 1 >= a.max_corr) step_end = true;
                else s++;
            }
            if (step_end) {
                if (isInf) {                                                  // :252
                    ph = PH_FINISH;
                } else {
                    if (!isSucc) {                                            // :257-265
                        dt = (float)((double)dt * 0.5);
                        x0 = xl0; x1 = xl1;
                        so0 = xl0; so1 = xl1;
                        succ = 0;
                        t0 = t_step;
                    } else {                                                  // :266-275
                        succ++;
                        xl0 = x0; xl1 = x1;
                        so0 = x0; so1 = x1;
                        if (succ >= a.inc_steps) { succ = 0; dt *= 2.0f; }
                    }
                    stepidx++;
                    ph = PH_BEGIN;
                }
            }
        }
    }
}

// ---------------------------------------------------------------- components
__global__ void __launch_bounds__(WG_THREADS) k_cgesv(int n, const cf *__restrict__ A, const cf *__restrict__ B,
                                                      cf *__restrict__ X) {
    const int lane = lane_id();
    const int sys = blockIdx.x * WAVES_PER_WG + threadIdx.x / WAVE;
    if (sys >= n) return;   // wave-uniform
    cf rA[NV];
    const bool rl = lane < NV;
#pragma unroll
    for (int c = 0; c < NV; c++) rA[c] = rl ? A[((size_t)sys * NV + lane) * NV + c] : cmk(0.0f, 0.0f);
    const cf rB = rl ? B[(size_t)sys * NV + lane] : cmk(0.0f, 0.0f);
    const cf x = lu_solve(rA, rB, lane);
    if (rl) X[(size_t)sys * NV + lane] = x;
}

__global__ void __launch_bounds__(WG_THREADS) k_eval(int n, const TableWS *ws, const cf *__restrict__ X,
                                                     const cf *__restrict__ P, const cf *__restrict__ D,
                                                     cf *__restrict__ HX, cf *__restrict__ HT, cf *__restrict__ H) {
    __shared__ BlockLDS L;
    load_tables(L, ws, P);
    const int lane = lane_id();
    const int wid = threadIdx.x / WAVE;
    const int sys = blockIdx.x * WAVES_PER_WG + wid;
    if (sys >= n) return;
    WaveLDS &W = L.w[wid];
    if (lane < 31) W.x[lane] = X[(size_t)sys * 31 + lane];
    if (lane == 31) W.x[31] = cmk(0.0f, 0.0f);
    if (lane < NPP) { W.p[lane] = P[(size_t)sys * NPP + lane]; W.dif[lane] = D[(size_t)sys * NPP + lane]; }
    wave_lds_sync();
    cf rA[NV];
    eval_hx(rA, L.hx, ws->nslot, ws->slot_base, W.x, W.p, lane & 31);
    const cf ht = eval_ht(L.ht, W.x, W.p, W.dif, lane & 31);
    const cf h = eval_h(L.ht, W.x, W.p, lane & 31);
    if (lane < NV) {
#pragma unroll
        for (int c = 0; c < NV; c++) HX[((size_t)sys * NV + lane) * NV + c] = rA[c];
        HT[(size_t)sys * NV + lane] = ht;
        H[(size_t)sys * NV + lane] = h;
    }
}

__global__ void __launch_bounds__(WG_THREADS) k_cgesv2(int n, const cf *__restrict__ A, const cf *__restrict__ B,
                                                       cf *__restrict__ X) {
    const int lane = lane_id();
    const int r = lane & 31;
    const int sys = (blockIdx.x * WAVES_PER_WG + threadIdx.x / WAVE) * 2 + (lane >> 5);
    const bool ok = sys < n && r < NV;
    cf rA[NV];
#pragma unroll
    for (int c = 0; c < NV; c++) rA[c] = ok ? A[((size_t)sys * NV + r) * NV + c] : cmk(0.0f, 0.0f);
    const cf rB = ok ? B[(size_t)sys * NV + r] : cmk(0.0f, 0.0f);
    const cf x = lu_solve2(rA, rB, lane);
    if (ok) X[(size_t)sys * NV + r] = x;
}

__global__ void __launch_bounds__(WG_THREADS) k_cgesv3(int n, const cf *__restrict__ A, const cf *__restrict__ B,
                                                       cf *__restrict__ X) {
    __shared__ LUBuf s_lu[2 * WAVES_PER_WG];
    const int lane = lane_id();
    const int r = lane & 31;
    const int sys = (blockIdx.x * WAVES_PER_WG + threadIdx.x / WAVE) * 2 + (lane >> 5);
    const bool ok = sys < n && r < NV;
    cf rA[NV];
#pragma unroll
    for (int c = 0; c < NV; c++) rA[c] = ok ? A[((size_t)sys * NV + r) * NV + c] : cmk(0.0f, 0.0f);
    const cf rB = ok ? B[(size_t)sys * NV + r] : cmk(0.0f, 0.0f);
    const cf x = lu_solve3(rA, rB, lane, s_lu[(threadIdx.x / WAVE) * 2 + (lane >> 5)]);
    if (ok) X[(size_t)sys * NV + r] = x;
}

__global__ void __launch_bounds__(WG_THREADS) k_eval2(int n, TableWS *ws, const cf *__restrict__ X,
                                                      const cf *__restrict__ P, const cf *__restrict__ D,
                                                      cf *__restrict__ HX, cf *__restrict__ HT, cf *__restrict__ H) {
    __shared__ uint32_t s_hx2[HX2_SLOT_CAP * 32];
    __shared__ uint32_t s_ht[HT_TERMS * 32];
    __shared__ SlotLDS s_slot[2 * WAVES_PER_WG];
    const TableWS2 *w2 = ws2_of(ws);
    const int hx_len = w2->hx_len;
    for (int i = threadIdx.x; i < hx_len * 32; i += WG_THREADS) s_hx2[i] = w2->hx[i];
    for (int i = threadIdx.x; i < HT_TERMS * 32; i += WG_THREADS) s_ht[i] = ws->ht[i];
    {
        float *z = reinterpret_cast<float *>(s_slot);
        for (int i = threadIdx.x; i < (int)(sizeof(s_slot) / 4); i += WG_THREADS) z[i] = 0.0f;
    }
    __syncthreads();
    const int lane = lane_id();
    const int r = lane & 31;
    const int sys = (blockIdx.x * WAVES_PER_WG + threadIdx.x / WAVE) * 2 + (lane >> 5);
    SlotLDS &S = s_slot[(threadIdx.x / WAVE) * 2 + (lane >> 5)];
    const bool ok = sys < n;
    if (ok && r < 31) S.x[r] = X[(size_t)sys * 31 + r];
    if (ok) {
        S.p[r] = P[(size_t)sys * NPP + r];
        S.dif[r] = D[(size_t)sys * NPP + r];
        if (r < NPP - 32) { S.p[r + 32] = P[(size_t)sys * NPP + r + 32]; S.dif[r + 32] = D[(size_t)sys * NPP + r + 32]; }
    }
    const uint32_t map[3] = {w2->map[0][r], w2->map[1][r], w2->map[2][r]};
    wave_lds_sync();
    cf rA[NV];
    eval_hx2(rA, s_hx2, hx_len, map, S, r);
    const cf ht = eval_ht2(s_ht, S, r);
    const cf h = eval_h2(s_ht, S, r);
    if (ok && r < NV) {
#pragma unroll
        for (int c = 0; c < NV; c++) HX[((size_t)sys * NV + r) * NV + c] = rA[c];
        HT[(size_t)sys * NV + r] = ht;
        H[(size_t)sys * NV + r] = h;
    }
}

__global__ void __launch_bounds__(WG_THREADS) k_eval3(int n, TableWS *ws, const cf *__restrict__ X,
                                                      const cf *__restrict__ P, const cf *__restrict__ D,
                                                      cf *__restrict__ HX, cf *__restrict__ HT, cf *__restrict__ H) {
    __shared__ uint2 s_hx3[HX3_SLOT_CAP * 32];
    __shared__ uint2 s_ht3[HT_TERMS * 32];
    __shared__ SlotLDS s_slot[2 * WAVES_PER_WG];
    const TableWS2 *w2 = ws2_of(ws);
    const TableWS3 *w3 = ws3_of(ws);
    if (w3->status != 0) return;
    const int hx_len = w3->hx_len;
    for (int i = threadIdx.x; i < HX3_SLOT_CAP * 32; i += WG_THREADS) s_hx3[i] = w3->hx[i];   // padded table
    for (int i = threadIdx.x; i < HT_TERMS * 32; i += WG_THREADS) s_ht3[i] = w3->ht[i];
    {
        float *z = reinterpret_cast<float *>(s_slot);
        for (int i = threadIdx.x; i < (int)(sizeof(s_slot) / 4); i += WG_THREADS) z[i] = 0.0f;
    }
    __syncthreads();
    const int lane = lane_id();
    const int r = lane & 31;
    const int sys = (blockIdx.x * WAVES_PER_WG + threadIdx.x / WAVE) * 2 + (lane >> 5);
    SlotLDS &S = s_slot[(threadIdx.x / WAVE) * 2 + (lane >> 5)];
    const bool ok = sys < n;
    if (ok && r < 31) S.x[r] = X[(size_t)sys * 31 + r];
    if (ok) {
        S.p[r] = P[(size_t)sys * NPP + r];
        S.dif[r] = D[(size_t)sys * NPP + r];
        if (r < NPP - 32) { S.p[r + 32] = P[(size_t)sys * NPP + r + 32]; S.dif[r + 32] = D[(size_t)sys * NPP + r + 32]; }
    }
    const uint32_t map[3] = {w2->map[0][r], w2->map[1][r], w2->map[2][r]};
    wave_lds_sync();
    cf rA[NV];
    eval_hx3(rA, s_hx3, hx_len, map, S, r);
    const cf ht = eval_ht3(s_ht3, S, r);
    const cf h = eval_h3(s_ht3, S, r);
    if (ok && r < NV) {
#pragma unroll
        for (int c = 0; c < NV; c++) HX[((size_t)sys * NV + r) * NV + c] = rA[c];
        HT[(size_t)sys * NV + r] = ht;
        H[(size_t)sys * NV + r] = h;
    }
}

// v8 / v9 LU standalone: the structural pattern of a row is its non-zero entries
template <bool V9>
__global__ void __launch_bounds__(WG_THREADS) k_cgesv8(int n, const cf *__restrict__ A, const cf *__restrict__ B,
                                                       cf *__restrict__ X) {
    __shared__ LUBuf s_lu[2 * WAVES_PER_WG];
    const int lane = lane_id();
    const int r = lane & 31;
    const int sys = (blockIdx.x * WAVES_PER_WG + threadIdx.x / WAVE) * 2 + (lane >> 5);
    const bool ok = sys < n && r < NV;
    cf rA[NV];
    uint32_t pat = 0;
#pragma unroll
    for (int c = 0; c < NV; c++) {
        rA[c] = ok ? A[((size_t)sys * NV + r) * NV + c] : cmk(0.0f, 0.0f);
        if (rA[c].x != 0.0f || rA[c].y != 0.0f) pat |= 1u << c;   // NaN counts as non-zero
    }
    const cf rB = ok ? B[(size_t)sys * NV + r] : cmk(0.0f, 0.0f);
    const cf x = V9 ? lu_solve9<LU9_PROD>(rA, rB, lane, pat, s_lu[(threadIdx.x / WAVE) * 2 + (lane >> 5)])
                    : lu_solve3s(rA, rB, lane, pat, s_lu[(threadIdx.x / WAVE) * 2 + (lane >> 5)]);
    if (ok) X[(size_t)sys * NV + r] = x;
}

// v4 component kernels: one system / evaluation point per 16-lane row
__global__ void __launch_bounds__(WG_THREADS) k_cgesv4(int n, const cf *__restrict__ A, const cf *__restrict__ B,
                                                       cf *__restrict__ X) {
    __shared__ LUBuf s_lu[4 * WAVES_PER_WG];
    const int lane = lane_id();
    const int r = lane & 15;
    const int sys = (blockIdx.x * WAVES_PER_WG + threadIdx.x / WAVE) * 4 + (lane >> 4);
    const bool ok = sys < n;
    const bool v1 = r + QL < NV;
    cf A0[NV], A1[NV];
#pragma unroll
    for (int c = 0; c < NV; c++) {
        A0[c] = ok ? A[((size_t)sys * NV + r) * NV + c] : cmk(0.0f, 0.0f);
        A1[c] = (ok && v1) ? A[((size_t)sys * NV + r + QL) * NV + c] : cmk(0.0f, 0.0f);
    }
    const cf b0 = ok ? B[(size_t)sys * NV + r] : cmk(0.0f, 0.0f);
    const cf b1 = (ok && v1) ? B[(size_t)sys * NV + r + QL] : cmk(0.0f, 0.0f);
    cf x0, x1;
    lu_solve4(A0, A1, b0, b1, lane, s_lu[(threadIdx.x / WAVE) * 4 + (lane >> 4)], x0, x1);
    if (ok) {
        X[(size_t)sys * NV + r] = x0;
        if (v1) X[(size_t)sys * NV + r + QL] = x1;
    }
}

__global__ void __launch_bounds__(WG_THREADS) k_eval4(int n, TableWS *ws, const cf *__restrict__ X,
                                                      const cf *__restrict__ P, const cf *__restrict__ D,
                                                      cf *__restrict__ HX, cf *__restrict__ HT, cf *__restrict__ H) {
    __shared__ uint2 s_hx3[HX3_SLOT_CAP * 32];
    __shared__ uint2 s_ht3[HT_TERMS * 32];
    __shared__ SlotLDS4 s_slot[4 * WAVES_PER_WG];
    const TableWS2 *w2 = ws2_of(ws);
    const TableWS3 *w3 = ws3_of(ws);
    if (w3->status != 0) return;
    const int hx_len = w3->hx_len;
    for (int i = threadIdx.x; i < hx_len * 32; i += WG_THREADS) s_hx3[i] = rebase_p_offsets(w3->hx[i]);
    for (int i = threadIdx.x; i < HT_TERMS * 32; i += WG_THREADS) s_ht3[i] = rebase_p_offsets(w3->ht[i]);
    {
        float *z = reinterpret_cast<float *>(s_slot);
        for (int i = threadIdx.x; i < (int)(sizeof(s_slot) / 4); i += WG_THREADS) z[i] = 0.0f;
    }
    __syncthreads();
    const int lane = lane_id();
    const int r = lane & 15;
    const int sys = (blockIdx.x * WAVES_PER_WG + threadIdx.x / WAVE) * 4 + (lane >> 4);
    SlotLDS4 &S = s_slot[(threadIdx.x / WAVE) * 4 + (lane >> 4)];
    const bool ok = sys < n;
    const bool v1 = r + QL < NV;
    if (ok) {
        for (int i = r; i < 31; i += QL) S.x[i] = X[(size_t)sys * 31 + i];
        for (int i = r; i < NPP; i += QL) { S.p[i] = P[(size_t)sys * NPP + i]; S.dif[i] = D[(size_t)sys * NPP + i]; }
    }
    const uint32_t map0[3] = {w2->map[0][r], w2->map[1][r], w2->map[2][r]};
    const uint32_t map1[3] = {w2->map[0][r + QL], w2->map[1][r + QL], w2->map[2][r + QL]};
    wave_lds_sync();
    cf A0[NV], A1[NV], t0, t1, h0, h1;
    eval_hx4(A0, A1, s_hx3, hx_len, map0, map1, S, r);
    eval_ht4(s_ht3, S, r, t0, t1);
    eval_h4(s_ht3, S, r, h0, h1);
    if (ok) {
#pragma unroll
        for (int c = 0; c < NV; c++) HX[((size_t)sys * NV + r) * NV + c] = A0[c];
        HT[(size_t)sys * NV + r] = t0;
        H[(size_t)sys * NV + r] = h0;
        if (v1) {
#pragma unroll
            for (int c = 0; c < NV; c++) HX[((size_t)sys * NV + r + QL) * NV + c] = A1[c];
            HT[(size_t)sys * NV + r + QL] = t1;
            H[(size_t)sys * NV + r + QL] = h1;
        }
    }
}

// ---------------------------------------------------------------- host side
// HC_TRIFOCAL_KERNEL=v1|v2|v3|v4|v8 selects another tracker generation (A/B
// baselines, all bit-identical); default v9 = v3 evals + the structurally
// sparse LU with lean pivot steps (hc_lu9.hpp); v8 = the sparse LU of
// hc_lu3s.hpp.  v4: four paths per wave (hc_track4.hpp).
static int v9_waves() {
    static int w = -1;
    if (w < 0) {
        const char *e = getenv("HC_TRIFOCAL_V9_WAVES");
        w = (e && e[0] == '4') ? 4 : 5;
    }
    return w;
}
static int kernel_version() {
    static int v = -1;
    if (v < 0) {
        const char *e = getenv("HC_TRIFOCAL_KERNEL");
        v = (e && e[0] == 'v' && e[1] == '1') ? 1 : (e && e[0] == 'v' && e[1] == '2') ? 2
          : (e && e[0] == 'v' && e[1] == '3') ? 3 : (e && e[0] == 'v' && e[1] == '4') ? 4
          : (e && e[0] == 'v' && e[1] == '8') ? 8 : 9;
    }
    return v;
}
// HC_TRIFOCAL_MINWAVES=3|4: register budget of the v3 tracker (waves per SIMD);
// 4 (<= 128 VGPRs) measured 8 % faster than 3 on MI355X (r6) and is the default
static int v3_minwaves() {
    static int w = -1;
    if (w < 0) {
        const char *e = getenv("HC_TRIFOCAL_MINWAVES");
        w = (e && e[0] == '3') ? 3 : 4;
    }
    return w;
}
// HC_TRIFOCAL_ORDER=natural: dequeue in batch-id order (A/B baseline); default
// longest-track-first (abort mode always dequeues sample-major, so whole
// hypotheses finish as early as possible)
static bool path_order_ltf() {
    static int o = -1;
    if (o < 0) {
        const char *e = getenv("HC_TRIFOCAL_ORDER");
        o = (e && e[0] == 'n') ? 0 : 1;
    }
    return o == 1;
}
static size_t ws_bytes_needed() {
    return ((sizeof(TableWS) + 255) & ~(size_t)255) + ((sizeof(TableWS2) + 255) & ~(size_t)255) +
           ((sizeof(TableWS3) + 255) & ~(size_t)255);
}

static int grid_for(int waves_needed, const void *kernel, int wg_threads = WG_THREADS) {
    static std::mutex mu;
    static int cache_dev = -1, cache_blocks = 0, cache_cus = 0;
    static const void *cache_k = nullptr;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return -1;
    {
        std::lock_guard<std::mutex> g(mu);
        if (dev != cache_dev || kernel != cache_k) {
            int cus = 0, per_cu = 0;
            if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return -1;
            if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, wg_threads, 0) != hipSuccess) per_cu = 1;
            cache_dev = dev; cache_k = kernel; cache_cus = cus; cache_blocks = per_cu < 1 ? 1 : per_cu;
        }
    }
    const int wpg = wg_threads / WAVE;
    const int want = (waves_needed + wpg - 1) / wpg;
    int per_cu = cache_blocks;
    // HC_TRIFOCAL_WGS_PER_CU: fewer resident workgroups per CU than the occupancy
    // limit (experiment: fewer path slots, more paths per slot)
    static const char *cap_env = getenv("HC_TRIFOCAL_WGS_PER_CU");
    if (cap_env && atoi(cap_env) > 0 && atoi(cap_env) < per_cu) per_cu = atoi(cap_env);
    const int cap = cache_cus * per_cu;
    return want < cap ? want : cap;
}

static hcStatus launch_track(const hcTrackArgs *t, const hcAbortArgs *ab, void *workspace, size_t wsb,
                             hcStream stream, bool abort_mode) {
    if (!t || t->sub_ransac_iters < 0) return HC_ERROR_INVALID_VALUE;
    if (!workspace || wsb < ws_bytes_needed()) return HC_ERROR_WORKSPACE;
    if (t->sub_ransac_iters == 0) return HC_SUCCESS;
    if ((!t->start_sols && !t->start_sols_array) || (!t->tracks && !t->track_array) || !t->start_params ||
        !t->target_params || !t->diff_params || !t->unified_index || !t->converge || !t->infinity)
        return HC_ERROR_INVALID_VALUE;
    if (t->settings.max_steps < 0 || t->settings.max_corrections < 0 || t->settings.delta_t_inc_steps < 0)
        return HC_ERROR_INVALID_VALUE;
    if (abort_mode && (!ab || ab->num_triplet_edgels <= 0 || !ab->triplet_edge_locations || !ab->intrinsic_matrix ||
                       !ab->found_trifocal_sols || !ab->trifocal_sols_batch_index))
        return HC_ERROR_INVALID_VALUE;
    const long long paths = (long long)t->sub_ransac_iters * NTRK;
    if (paths > 0x7FFFFFFFll) return HC_ERROR_INVALID_VALUE;
    hipStream_t s = (hipStream_t)stream;
    TableWS *ws = (TableWS *)workspace;
    (void)hipGetLastError();  // errors of earlier, unrelated calls are not ours
    if ((g_last_hip_error = hipMemsetAsync(ws, 0, 64, s)) != hipSuccess) return HC_ERROR_LAUNCH;
    hipLaunchKernelGGL(k_prep_tables, dim3(1), dim3(64), 0, s, t->unified_index, ws,
                       abort_mode ? ab->found_trifocal_sols : nullptr);
    if (launch_status(HC_ERROR_LAUNCH) != HC_SUCCESS) return HC_ERROR_LAUNCH;
    KArgs k{};
    k.num_paths = (int)paths;
    k.ordered = (!abort_mode && path_order_ltf()) ? 1 : 0;
    k.max_steps = t->settings.max_steps;
    k.max_corr = t->settings.max_corrections;
    k.inc_steps = t->settings.delta_t_inc_steps;
    k.start_sols = (const cf *)t->start_sols;
    k.start_sols_array = (const cf *const *)t->start_sols_array;
    k.tracks = (cf *)t->tracks;
    k.track_array = (cf *const *)t->track_array;
    k.start_params = (const cf *)t->start_params;
    k.target_params = (const cf *)t->target_params;
    k.diff_params = (const cf *)t->diff_params;
    k.conv = t->converge;
    k.inf = t->infinity;
    k.stats = t->stats;
    k.ws = ws;
    k.ws2 = ws2_of(ws);
    k.ws3 = ws3_of(ws);
    const int ver = kernel_version();
    const bool w4 = v3_minwaves() == 4;
#ifdef HC_TRACK_W5
    // experiment: 5 waves/SIMD with 640-thread workgroups (LDS: 2 per CU)
    const bool w5 = ver == 9 && !abort_mode && getenv("HC_TRIFOCAL_OCC") && getenv("HC_TRIFOCAL_OCC")[0] == '5';
#else
    const bool w5 = false;
#endif
    const void *kern = ver == 9   ? (abort_mode ? (const void *)k_track2<true, 4, 9> : (const void *)k_track2<false, 4, 9>)
                       : ver == 8 ? (abort_mode ? (const void *)k_track2<true, 4, 8> : (const void *)k_track2<false, 4, 8>)
                       : ver == 4 ? (abort_mode ? (const void *)k_track4<true> : (const void *)k_track4<false>)
                       : ver == 1 ? (abort_mode ? (const void *)k_track<true> : (const void *)k_track<false>)
                       : ver == 2 ? (abort_mode ? (const void *)k_track2<true, 3, 2> : (const void *)k_track2<false, 3, 2>)
                       : w4       ? (abort_mode ? (const void *)k_track2<true, 4, 3> : (const void *)k_track2<false, 4, 3>)
                                  : (abort_mode ? (const void *)k_track2<true, 3, 3> : (const void *)k_track2<false, 3, 3>);
    int wg_threads = WG_THREADS;
#ifdef HC_TRACK_W5
    if (w5) { kern = (const void *)k_track2<false, 5, 9, 640>; wg_threads = 640; }
#endif
    // v9 tracking (abort off): term tables read from the workspace (L1/L2) instead of
    // LDS, which leaves 27.5 KB LDS and 96 VGPRs per 4-wave workgroup: 5 waves/SIMD.
    // HC_TRIFOCAL_V9_WAVES=4 selects the 4-wave kernel with LDS-staged tables.
    if (ver == 9 && !abort_mode && v9_waves() == 5) kern = (const void *)k_track2<false, 5, 9, 256, true>;
    (void)w5;
    const int grid = grid_for(ver == 4 ? (int)((paths + 3) / 4) : ver >= 2 ? (int)((paths + 1) / 2) : (int)paths,
                              kern, wg_threads);
    if (grid <= 0) return HC_ERROR_DEVICE;
    if (abort_mode) {
        k.num_edgels = ab->num_triplet_edgels;
        k.edgels = ab->triplet_edge_locations;
        k.K = ab->intrinsic_matrix;
        k.found_flag = ab->found_trifocal_sols;
        k.batch_index = ab->trifocal_sols_batch_index;
    }
    void *kargs[] = {&k};
    g_last_hip_error = hipLaunchKernel(kern, dim3(grid), dim3(wg_threads), kargs, 0, s);
    if (g_last_hip_error != hipSuccess) return HC_ERROR_LAUNCH;
    return launch_status(HC_ERROR_LAUNCH);
}

}  // namespace hc

extern "C" {
#ifdef HC_DIAG_PHASES
int hc_diag_phases(unsigned long long *out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(hc::g_diag_phase), sizeof(unsigned long long) * 13) != hipSuccess) return -1;
    if (reset) {
        static const unsigned long long z[13] = {0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(hc::g_diag_phase), z, sizeof(z)) != hipSuccess) return -1;
    }
    return 0;
}
#endif

size_t hc_trifocal_workspace_size(void) { return hc::ws_bytes_needed(); }

hcStatus hc_trifocal_2op1p_30x30_track(const hcTrackArgs *args, void *workspace, size_t workspace_bytes,
                                       hcStream stream) {
    return hc::launch_track(args, nullptr, workspace, workspace_bytes, stream, false);
}

hcStatus hc_trifocal_2op1p_30x30_track_abort(const hcTrackArgs *args, const hcAbortArgs *abort_args,
                                             void *workspace, size_t workspace_bytes, hcStream stream) {
    return hc::launch_track(args, abort_args, workspace, workspace_bytes, stream, true);
}

hcStatus hc_trifocal_read_timings(const void *workspace, double *first_found_seconds) {
    if (!workspace || !first_found_seconds) return HC_ERROR_INVALID_VALUE;
    hc::TableWS h;
    if (hipMemcpy(&h, workspace, 64, hipMemcpyDeviceToHost) != hipSuccess) return HC_ERROR_DEVICE;
    // s_memrealtime ticks at a constant 100 MHz on gfx9 parts
    *first_found_seconds = (h.t_found && h.t_start) ? (double)(long long)(h.t_found - h.t_start) / 100.0e6 : -1.0;
    return HC_SUCCESS;
}

hcStatus hc_trifocal_read_timestamps(const void *workspace, uint64_t *start_ticks, uint64_t *found_ticks,
                                     double *tick_hz) {
    if (!workspace || !start_ticks || !found_ticks || !tick_hz) return HC_ERROR_INVALID_VALUE;
    hc::TableWS h;
    if (hipMemcpy(&h, workspace, 64, hipMemcpyDeviceToHost) != hipSuccess) return HC_ERROR_DEVICE;
    *start_ticks = h.t_start;
    *found_ticks = h.t_found;
    *tick_hz = 100.0e6;   // s_memrealtime: constant 100 MHz on gfx9
    return HC_SUCCESS;
}

hcStatus hc_cgesv_30x30_batched(int n, const hcComplex *A, const hcComplex *b, hcComplex *x, hcStream stream) {
    if (n < 0 || (n > 0 && (!A || !b || !x))) return HC_ERROR_INVALID_VALUE;
    if (n == 0) return HC_SUCCESS;
    (void)hipGetLastError();
    if (hc::kernel_version() >= 8) {
        const int per = 2 * hc::WAVES_PER_WG;
        hipLaunchKernelGGL(hc::kernel_version() == 9 ? hc::k_cgesv8<true> : hc::k_cgesv8<false>,
                           dim3((n + per - 1) / per), dim3(hc::WG_THREADS), 0, (hipStream_t)stream, n,
                           (const hc::cf *)A, (const hc::cf *)b, (hc::cf *)x);
    } else if (hc::kernel_version() == 4) {
        const int per = 4 * hc::WAVES_PER_WG;
        hipLaunchKernelGGL(hc::k_cgesv4, dim3((n + per - 1) / per), dim3(hc::WG_THREADS), 0, (hipStream_t)stream, n,
                           (const hc::cf *)A, (const hc::cf *)b, (hc::cf *)x);
    } else if (hc::kernel_version() == 3) {
        const int per = 2 * hc::WAVES_PER_WG;
        hipLaunchKernelGGL(hc::k_cgesv3, dim3((n + per - 1) / per), dim3(hc::WG_THREADS), 0, (hipStream_t)stream, n,
                           (const hc::cf *)A, (const hc::cf *)b, (hc::cf *)x);
    } else if (hc::kernel_version() == 2) {
        const int per = 2 * hc::WAVES_PER_WG;
        hipLaunchKernelGGL(hc::k_cgesv2, dim3((n + per - 1) / per), dim3(hc::WG_THREADS), 0, (hipStream_t)stream, n,
                           (const hc::cf *)A, (const hc::cf *)b, (hc::cf *)x);
    } else {
        const int grid = (n + hc::WAVES_PER_WG - 1) / hc::WAVES_PER_WG;
        hipLaunchKernelGGL(hc::k_cgesv, dim3(grid), dim3(hc::WG_THREADS), 0, (hipStream_t)stream, n,
                           (const hc::cf *)A, (const hc::cf *)b, (hc::cf *)x);
    }
    return hc::launch_status(HC_ERROR_LAUNCH);
}

hcStatus hc_trifocal_eval_batched(int n, const int32_t *unified_index, const hcComplex *x, const hcComplex *p,
                                  const hcComplex *d, hcComplex *Hx, hcComplex *Ht, hcComplex *H, void *workspace,
                                  size_t workspace_bytes, hcStream stream) {
    if (n < 0 || !unified_index || (n > 0 && (!x || !p || !d || !Hx || !Ht || !H))) return HC_ERROR_INVALID_VALUE;
    if (!workspace || workspace_bytes < hc::ws_bytes_needed()) return HC_ERROR_WORKSPACE;
    if (n == 0) return HC_SUCCESS;
    hipStream_t s = (hipStream_t)stream;
    hc::TableWS *ws = (hc::TableWS *)workspace;
    (void)hipGetLastError();
    if ((hc::g_last_hip_error = hipMemsetAsync(ws, 0, 64, s)) != hipSuccess) return HC_ERROR_LAUNCH;
    hipLaunchKernelGGL(hc::k_prep_tables, dim3(1), dim3(64), 0, s, unified_index, ws, nullptr);
    if (hc::launch_status(HC_ERROR_LAUNCH) != HC_SUCCESS) return HC_ERROR_LAUNCH;
    if (hc::kernel_version() == 4) {
        const int per = 4 * hc::WAVES_PER_WG;
        hipLaunchKernelGGL(hc::k_eval4, dim3((n + per - 1) / per), dim3(hc::WG_THREADS), 0, s, n, ws,
                           (const hc::cf *)x, (const hc::cf *)p, (const hc::cf *)d, (hc::cf *)Hx, (hc::cf *)Ht,
                           (hc::cf *)H);
    } else if (hc::kernel_version() == 3 || hc::kernel_version() >= 8) {
        const int per = 2 * hc::WAVES_PER_WG;
        hipLaunchKernelGGL(hc::k_eval3, dim3((n + per - 1) / per), dim3(hc::WG_THREADS), 0, s, n, ws,
                           (const hc::cf *)x, (const hc::cf *)p, (const hc::cf *)d, (hc::cf *)Hx, (hc::cf *)Ht,
                           (hc::cf *)H);
    } else if (hc::kernel_version() == 2) {
        const int per = 2 * hc::WAVES_PER_WG;
        hipLaunchKernelGGL(hc::k_eval2, dim3((n + per - 1) / per), dim3(hc::WG_THREADS), 0, s, n, ws,
                           (const hc::cf *)x, (const hc::cf *)p, (const hc::cf *)d, (hc::cf *)Hx, (hc::cf *)Ht,
                           (hc::cf *)H);
    } else {
        const int grid = (n + hc::WAVES_PER_WG - 1) / hc::WAVES_PER_WG;
        hipLaunchKernelGGL(hc::k_eval, dim3(grid), dim3(hc::WG_THREADS), 0, s, n, ws, (const hc::cf *)x,
                           (const hc::cf *)p, (const hc::cf *)d, (hc::cf *)Hx, (hc::cf *)Ht, (hc::cf *)H);
    }
    return hc::launch_status(HC_ERROR_LAUNCH);
}

const char *hc_last_error_string(void) { return hipGetErrorString(hc::g_last_hip_error); }

const char *hc_trifocal_version(void) {
    switch (hc::kernel_version()) {
    case 1: return "hc_trifocal gfx950 v1 (wave-per-path, register LU)";
    case 2: return "hc_trifocal gfx950 v2 (2 paths/wave, bpermute LU, per-lane term lists)";
    case 9: return hc::v9_waves() == 5 ? "hc_trifocal gfx950 v9 (2 paths/wave, structurally sparse LDS-broadcast LU with lean pivot steps and readlane back substitution, pipelined evals, 5 waves/SIMD)"
                                   : "hc_trifocal gfx950 v9 (2 paths/wave, structurally sparse LDS-broadcast LU with lean pivot steps and readlane back substitution, pipelined evals, 4 waves/SIMD)";
    case 8: return "hc_trifocal gfx950 v8 (2 paths/wave, structurally sparse LDS-broadcast LU, packed evals, 4 waves/SIMD)";
    case 4: return "hc_trifocal gfx950 v4 (4 paths/wave, 2 rows/lane, LDS-broadcast LU, packed evals, 2 waves/SIMD)";
    default:
        return hc::v3_minwaves() == 4 ? "hc_trifocal gfx950 v3.1 (2 paths/wave, LDS-broadcast LU, permlane16 pivot search, packed evals, 4 waves/SIMD)"
                                      : "hc_trifocal gfx950 v3.1 (2 paths/wave, LDS-broadcast LU, permlane16 pivot search, packed evals, 3 waves/SIMD)";
    }
}

}  // extern "C"
