// hc_host.cpp -- host data layer of the trifocal GPU-HC framework (include/hc_host.h).
//
// Reads the reference's problem / RANSAC text formats with the same std::istream
// extraction the reference uses (magmaHC/Data_Reader.cpp), generates the RANSAC
// target parameters with the host libc srand()/rand() exactly like
// GPU_HC_Solver::Prepare_Target_Params, and counts solutions like
// Evaluations::Evaluate_HC_Sols.
#include "../../include/hc_host.h"

#include <cmath>
#include <cstdlib>
#include <fstream>
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

}  // extern "C"
