// hc_host.cpp -- host data layer of the trifocal GPU-HC framework (include/hc_host.h).
//
// Reads the reference's problem / RANSAC text formats with the same std::istream
// extraction the reference uses (magmaHC/Data_Reader.cpp), generates the RANSAC
// target parameters with the host libc srand()/rand() exactly like
// GPU_HC_Solver::Prepare_Target_Params, and counts solutions like
// Evaluations::Evaluate_HC_Sols; merges per-GPU pose selections and measures
// the relative-pose error against the ground truth like Evaluations.cpp:360-543.
#include "../../include/hc_host.h"
#include "../../include/hc_pose.h"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <fstream>
#include <iomanip>
#include <string>

namespace {
constexpr int NV = 30, NPP = 34, NT = 312;
}

extern "C" {

int hc_read_start_sols(const char *file, float *ss) {
    // Data_Reader.cpp:37-60
    std::ifstream f(file);
    if (!f) return -1;
    float re, im;
    int d = 0, i = 0, n = 0;
    while (f >> re >> im) {
        if (i >= NT) return -2;
        ss[(i * (NV + 1) + d) * 2] = re;
        ss[(i * (NV + 1) + d) * 2 + 1] = im;
        n++;
        if (d < NV - 1) d++;
        else { d = 0; i++; }
    }
    for (int k = 0; k < NT; k++) {
        ss[(k * (NV + 1) + NV) * 2] = 1.0f;
        ss[(k * (NV + 1) + NV) * 2 + 1] = 0.0f;
    }
    return n;
}

int hc_read_start_params(const char *file, float *sp) {
    // Data_Reader.cpp:104-121
    std::ifstream f(file);
    if (!f) return -1;
    float re, im;
    int d = 0;
    while (d < NPP && (f >> re >> im)) { sp[2 * d] = re; sp[2 * d + 1] = im; d++; }
    sp[2 * (NPP - 1)] = 1.0f;
    sp[2 * (NPP - 1) + 1] = 0.0f;
    return d;
}

int hc_read_int_table(const char *file, int32_t *out, int max_count) {
    // Data_Reader.cpp:123-165
    std::ifstream f(file);
    if (!f) return -1;
    int v, d = 0;
    while (d < max_count && (f >> v)) out[d++] = v;
    return d;
}

int hc_read_float_table(const char *file, float *out, int max_count) {
    // Data_Reader.cpp:191-270
    std::ifstream f(file);
    if (!f) return -1;
    float v;
    int d = 0;
    while (d < max_count && (f >> v)) out[d++] = v;
    return d;
}

int hc_count_triplet_edgels(const char *file) {
    // Data_Reader.cpp:273-305
    std::ifstream f(file);
    if (!f) return 0;
    float v[12];
    int n = 0;
    while (f >> v[0] >> v[1] >> v[2] >> v[3] >> v[4] >> v[5] >> v[6] >> v[7] >> v[8] >> v[9] >> v[10] >> v[11]) n++;
    return n;
}

int hc_read_triplet_edgels(const char *file, float *loc, float *tan, int max_edgels) {
    // Data_Reader.cpp:288-324: x1 y1 tx1 ty1 x2 y2 tx2 ty2 x3 y3 tx3 ty3
    std::ifstream f(file);
    if (!f) return -1;
    float v[12];
    int n = 0;
    while (n < max_edgels &&
           (f >> v[0] >> v[1] >> v[2] >> v[3] >> v[4] >> v[5] >> v[6] >> v[7] >> v[8] >> v[9] >> v[10] >> v[11])) {
        for (int view = 0; view < 3; view++) {
            loc[n * 6 + 2 * view] = v[4 * view];
            loc[n * 6 + 2 * view + 1] = v[4 * view + 1];
            tan[n * 6 + 2 * view] = v[4 * view + 2];
            tan[n * 6 + 2 * view + 1] = v[4 * view + 3];
        }
        n++;
    }
    return n;
}

void hc_split_samples(int num_samples, int num_gpus, int *sub) {
    // GPU_HC_Solver.cpp:85-88
    for (int g = 0; g < num_gpus; g++) sub[g] = num_samples / num_gpus + ((g < num_samples % num_gpus) ? 1 : 0);
}

void hc_prepare_target_params(unsigned seed, int num_gpus, const int *sub, const float *loc, const float *tan,
                              int E, const float *sp, float *tgt, float *dif, int32_t *picked) {
    // GPU_HC_Solver.cpp:252-306 (FEED_RANDOM_SEED false: srand(seed))
    unsigned idx[3] = {0, 0, 0};
    std::srand(seed);
    int k = 0;
    for (int g = 0; g < num_gpus; g++) {
        for (int ti = 0; ti < sub[g]; ti++, k++) {
            while (true) {
                for (int ri = 0; ri < 3; ri++) idx[ri] = (unsigned)(std::rand() % E);
                // the reference tests (0,1) twice and never (0,2): kept for parity
                if ((idx[0] != idx[1]) && (idx[0] != idx[1]) && (idx[1] != idx[2])) break;
            }
            if (picked) for (int i = 0; i < 3; i++) picked[k * 3 + i] = (int32_t)idx[i];
            float *tp = tgt + (size_t)k * NPP * 2;
            for (int i = 0; i < 3; i++)
                for (int j = 0; j < 6; j++) { tp[2 * (i * 6 + j)] = loc[idx[i] * 6 + j]; tp[2 * (i * 6 + j) + 1] = 0.0f; }
            for (int i = 0; i < 2; i++)
                for (int j = 0; j < 6; j++) {
                    tp[2 * (i * 6 + j + 18)] = tan[idx[i] * 6 + j];
                    tp[2 * (i * 6 + j + 18) + 1] = 0.0f;
                }
            tp[60] = 1.0f; tp[61] = 0.0f;
            tp[62] = 0.5f; tp[63] = 0.0f;
            tp[64] = 1.0f; tp[65] = 0.0f;
            tp[66] = 1.0f; tp[67] = 0.0f;
            float *dp = dif + (size_t)k * NPP * 2;
            for (int i = 0; i < NPP; i++) {
                dp[2 * i] = tp[2 * i] - sp[2 * i];
                dp[2 * i + 1] = tp[2 * i + 1] - sp[2 * i + 1];
            }
        }
    }
}

void hc_count_solutions(int N, const float *tracks, const uint8_t *conv, const uint8_t *inf, int32_t *out) {
    // Evaluations.cpp:145-182 (ZERO_IMAG_PART_TOL_FOR_SP = 1e-4)
    int nc = 0, nr = 0, ni = 0;
    for (long b = 0; b < (long)N * NT; b++) {
        if (conv[b]) nc++;
        if (inf[b]) ni++;
        if (conv[b]) {
            int real = 0;
            for (int v = 0; v < NV; v++)
                if (std::fabs(tracks[(b * (NV + 1) + v) * 2 + 1]) <= 1e-4) real++;
            if (real == NV) nr++;
        }
    }
    out[0] = nc; out[1] = nr; out[2] = ni;
}

int hc_write_converged_sols(const char *file, int N, const float *tracks, const uint8_t *conv) {
    // Evaluations.cpp:120-143 (same stream manipulators, same layout)
    std::ofstream f(file);
    if (!f) return -1;
    int counter = 0, written = 0;
    for (int ri = 0; ri < N; ri++) {
        f << "-------------------- RANSAC Iteration " << ri + 1 << " --------------------\n\n";
        for (int bs = 0; bs < NT; bs++) {
            f << std::setprecision(10);
            const long b = (long)ri * NT + bs;
            if (conv[b] == 1) {
                f << counter << "\n";
                for (int vs = 0; vs < NV; vs++)
                    f << std::setprecision(20) << tracks[(b * (NV + 1) + vs) * 2] << "\t" << std::setprecision(20)
                      << tracks[(b * (NV + 1) + vs) * 2 + 1] << "\n";
                f << "\n";
                written++;
            }
            counter++;
        }
        f << "\n";
    }
    return written;
}

void hc_add_pixel_noise(int E, const float *loc, const float *K, double sigma, uint64_t seed, float *out) {
    std::mt19937_64 gen(seed);
    std::normal_distribution<double> noise(0.0, sigma);
    const double fx = K[0], cx = K[2], fy = K[4], cy = K[5];
    for (int e = 0; e < E; e++)
        for (int v = 0; v < 3; v++) {
            const double u = (double)loc[e * 6 + 2 * v] * fx + cx + noise(gen);
            const double w = (double)loc[e * 6 + 2 * v + 1] * fy + cy + noise(gen);
            out[e * 6 + 2 * v] = (float)((u - cx) / fx);
            out[e * 6 + 2 * v + 1] = (float)((w - cy) / fy);
        }
}

int hc_write_triplet_edgels(const char *file, int E, const float *loc, const float *tan) {
    FILE *f = std::fopen(file, "w");
    if (!f) return -1;
    for (int e = 0; e < E; e++) {
        for (int v = 0; v < 3; v++)
            std::fprintf(f, "%.9g %.9g %.9g %.9g%s", loc[e * 6 + 2 * v], loc[e * 6 + 2 * v + 1], tan[e * 6 + 2 * v],
                         tan[e * 6 + 2 * v + 1], v < 2 ? " " : "\n");
    }
    std::fclose(f);
    return E;
}

void hc_pose_merge(int n, const hcPoseSelection *parts, const int32_t *off, int flags, hcPoseSelection *out) {
    // one launch over all paths would have max-reduced the same keys (hc_pose.hip)
    const bool quirks = (flags & HC_POSE_REFERENCE_QUIRKS) != 0;
    hcPoseSelection r{};
    r.path21 = r.path31 = -1;
    r.inliers21 = r.inliers31 = -1;
    bool have[2] = {false, false};
    for (int i = 0; i < n; i++) {
        const hcPoseSelection &p = parts[i];
        r.num_candidates += p.num_candidates;
        if (p.num_candidates <= 0) continue;
        for (int v = 0; v < 2; v++) {
            const uint64_t k = v == 0 ? p.key21 : p.key31;
            const uint64_t g = quirks ? k - (uint64_t)(uint32_t)off[i]
                                      : ((k >> 32) << 32) | (uint64_t)((uint32_t)k + (uint32_t)off[i]);
            uint64_t &best = v == 0 ? r.key21 : r.key31;
            if (!have[v] || g > best) {
                have[v] = true;
                best = g;
                if (v == 0) {
                    r.path21 = p.path21 + off[i]; r.inliers21 = p.inliers21;
                    for (int j = 0; j < 9; j++) r.R21[j] = p.R21[j];
                    for (int j = 0; j < 3; j++) r.t21[j] = p.t21[j];
                } else {
                    r.path31 = p.path31 + off[i]; r.inliers31 = p.inliers31;
                    for (int j = 0; j < 9; j++) r.R31[j] = p.R31[j];
                    for (int j = 0; j < 3; j++) r.t31[j] = p.t31[j];
                }
            }
        }
    }
    *out = r;
}

namespace {
// Evaluations.cpp:360-374: acos(0.5 * (trace(R_gt' R) - 1.0)), float matrix product / trace
float rotation_residual(const float *gt, const float *R) {
    float M[9];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
            float acc = 0.0f;
            for (int k = 0; k < 3; k++) acc += gt[k * 3 + i] * R[k * 3 + j];   // (R_gt')(i,k) = gt(k,i)
            M[i * 3 + j] = acc;
        }
    float tr = 0.0f;
    for (int i = 0; i < 3; i++) tr += M[i * 3 + i];
    return (float)std::acos(0.5 * ((double)tr - 1.0));
}
// Evaluations.cpp:376-380 with the GT translation normalised (util.hpp:69-78)
float translation_residual(const float *gt_t, const float *t) {
    float g[3] = {gt_t[0], gt_t[1], gt_t[2]};
    const float n = std::sqrt((g[0] * g[0] + g[1] * g[1]) + g[2] * g[2]);
    g[0] /= n; g[1] /= n; g[2] /= n;
    float dot = 0.0f;
    for (int i = 0; i < 3; i++) dot += g[i] * t[i];
    return (float)std::fabs((double)dot - 1.0);
}
}  // namespace

int hc_pose_residuals(const float *gt21, const float *gt31, const float *R21, const float *t21, const float *R31,
                      const float *t31, float *out) {
    // Evaluations.cpp:523-543 (Measure_Relative_Pose_Error)
    out[0] = rotation_residual(gt21, R21);
    out[1] = rotation_residual(gt31, R31);
    out[2] = translation_residual(gt21 + 9, t21);
    out[3] = translation_residual(gt31 + 9, t31);
    return ((double)out[2] < 1e-1 && (double)out[3] < 1e-1 && (double)out[0] < 1e-1 && (double)out[1] < 1e-1) ? 1 : 0;
}

}  // extern "C"
