/*
 * hc_host.h -- host-side C-ABI of the trifocal GPU-HC framework: the reference's
 * data formats, RANSAC sample generation and solution statistics, exported
 * with plain C types so Python (ctypes) and other FFIs can drive the same code
 * the C++ GPU_HC_Solver uses.
 *
 *   hc_read_*                 magmaHC/Data_Reader.cpp:37-338 (identical parsing:
 *                             std::istream >> float / >> int)
 *   hc_prepare_target_params  GPU_HC_Solver::Prepare_Target_Params
 *                             (magmaHC/GPU_HC_Solver.cpp:252-306), glibc srand/rand
 *   hc_split_samples          GPU_HC_Solver ctor sample split (GPU_HC_Solver.cpp:85-88)
 *   hc_count_solutions        Evaluations::Evaluate_HC_Sols (magmaHC/Evaluations.cpp:145-182)
 *   hc_write_converged_sols   Evaluations::Write_Converged_Sols (magmaHC/Evaluations.cpp:120-143)
 *   hc_add_pixel_noise,       noisy synthcurves in the
 *   hc_write_triplet_edgels   Triplet_Edgels format of Data_Reader.cpp:273-324
 * All complex arrays are interleaved float (re, im) == hcComplex.
 */
#ifndef HC_HOST_H
#define HC_HOST_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Return value: number of items read, or <0 when the file cannot be opened. */
int hc_read_start_sols(const char *file, float *start_sols /* 312 x 31 x 2, x[30] = 1 */);
int hc_read_start_params(const char *file, float *start_params /* 34 x 2, p[33] = 1 */);
int hc_read_int_table(const char *file, int32_t *out, int max_count);
int hc_read_float_table(const char *file, float *out, int max_count);
int hc_count_triplet_edgels(const char *file);
int hc_read_triplet_edgels(const char *file, float *locations /* E x 6 */,
                           float *tangents /* E x 6 */, int max_edgels);

/* Num_Of_Tracks / Num_Of_Vars fixed at 312 / 30.  sub_ransac_iters[g] for g < num_gpus. */
void hc_split_samples(int num_samples, int num_gpus, int *sub_ransac_iters);

/* Samples k = 0..N-1 (N = sum of sub_ransac_iters) in the reference's gpu-major
   order; target/diff: N x 34 x 2; picked (optional) N x 3 edgel indices. */
void hc_prepare_target_params(unsigned seed, int num_gpus, const int *sub_ransac_iters,
                              const float *locations, const float *tangents, int num_edgels,
                              const float *start_params, float *target_params,
                              float *diff_params, int32_t *picked);

/* counts[0] converged, counts[1] real (converged, all |Im| <= 1e-4), counts[2] inf. */
void hc_count_solutions(int num_samples, const float *tracks /* 312N x 31 x 2 */,
                        const uint8_t *converge, const uint8_t *infinity, int32_t *counts);

/* Writes <file> in the byte layout of Evaluations::Write_Converged_Sols: per
   sample a "---- RANSAC Iteration k ----" header, then for every converged
   path its global batch id and 30 "re\tim" lines (std::setprecision(20)).
   Returns the number of paths written, <0 if the file cannot be opened. */
int hc_write_converged_sols(const char *file, int num_samples, const float *tracks /* 312N x 31 x 2 */,
                            const uint8_t *converge);

/* Noisy synthcurves (not in the reference, which ships noiseless data only):
   every point of every view is moved by N(0, sigma_px^2) pixel noise and
   converted back to metric, tangents unchanged.  Pixel u = x*K[0] + K[2],
   v = y*K[4] + K[5] in double; draws from std::mt19937_64(seed) through
   std::normal_distribution<double>(0, sigma_px), edgel-major, views 1..3, u
   then v; x' = (float)((u' - K[2]) / K[0]), y' = (float)((v' - K[5]) / K[4]). */
void hc_add_pixel_noise(int num_edgels, const float *locations /* E x 6 */, const float *K, double sigma_px,
                        uint64_t seed, float *noisy_locations /* E x 6 */);
/* Writes E lines "x1 y1 tx1 ty1 x2 y2 tx2 ty2 x3 y3 tx3 ty3" (%.9g: reads back
   bit-exactly through hc_read_triplet_edgels).  Returns E, <0 on open failure. */
int hc_write_triplet_edgels(const char *file, int num_edgels, const float *locations, const float *tangents);

#ifdef __cplusplus
}
#endif
#endif
