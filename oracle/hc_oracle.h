/*
 * hc_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement ("oracle") of the reference GPU-HC / CPU-HC path tracker for
 * trifocal_2op1p_30x30.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library -- as the checker / CPU baseline,
 * never as the product path.  The product path (HIP kernels behind
 * include/hc_trifocal.h) never links or calls anything in oracle/.
 *
 * Pinning: the reference cannot be built or run here (the
 * CUDA/MAGMA GPU path is unbuildable; running the CPU-HC sources was DENIED
 * and that denial binds every round).  The oracle is pinned against
 *   (1) the reference's own committed data through known-answer tests
 *       (H(start_sols, start_params) ~ 0, dH/dx == finite differences of H),
 *   (2) the committed aggregate counts Output_Write_Files/CPU_Sols_Statistics.txt
 *       (11098 converged / 521 real / 6577 inf over 100 samples, srand(0)),
 *   (3) numpy linear algebra for the LU solve.
 * See DESIGN.md "Arithmetic specification" for the op-level spec both the
 * oracle and the HIP kernel implement (FMA only at the documented sites).
 */
#ifndef HC_ORACLE_H
#define HC_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORC_NV      30      /* Num_Of_Vars                                  */
#define ORC_NP      33      /* Num_Of_Params (34 with the homogenising 1)   */
#define ORC_NTRACK  312     /* Num_Of_Tracks                                */
#define ORC_HX_TERMS 8      /* dHdx_Max_Terms                               */
#define ORC_HX_PARTS 5      /* dHdx_Max_Parts                               */
#define ORC_HT_TERMS 16     /* dHdt_Max_Terms                               */
#define ORC_HT_PARTS 6      /* dHdt_Max_Parts                               */
#define ORC_HX_SIZE (ORC_NV * ORC_NV * ORC_HX_TERMS * ORC_HX_PARTS) /* 36000 */
#define ORC_HT_SIZE (ORC_NV * ORC_HT_TERMS * ORC_HT_PARTS)          /* 2880  */

/* ---------------- data readers (Data_Reader.cpp semantics) ---------------- */
/* All complex arrays are interleaved float (re, im).                          */
int orc_read_start_sols(const char *file, float *start_sols /* 312*31*2 */);
int orc_read_start_params(const char *file, float *start_params /* 34*2 */);
int orc_read_ints(const char *file, int *out, int max_count);
int orc_read_floats(const char *file, float *out, int max_count);
int orc_count_triplet_edgels(const char *file);
int orc_read_triplet_edgels(const char *file, float *loc /* E*6 */, float *tan /* E*6 */, int max_edgels);

/* ---------------- RANSAC sample generation (Prepare_Target_Params) -------- */
void orc_prepare_target_params(unsigned seed, int num_gpus, const int *sub_ransac_iters,
                               const float *loc, const float *tan, int num_edgels,
                               const float *start_params, float *target_params,
                               float *diff_params, int *picked /* N*3, may be NULL */);

/* ---------------- evaluations (exposed for KATs) --------------------------- */
void orc_param_homotopy_gpu(float t, const float *start_params, const float *target_params,
                            float *p /* 34*2 */);
void orc_eval_hx(const int *dHdx, const float *x /* 31*2 */, const float *p /* 34*2 */,
                 float *A /* row-major 30x30x2 */);
void orc_eval_ht(const int *dHdt, const float *x, const float *p, const float *diff,
                 float *b /* 30*2 */);
void orc_eval_h(const int *dHdt, const float *x, const float *p, float *b /* 30*2 */);
/* register-resident LU of dev-cgesv-batched-small.cuh (GPU semantics).
   A row-major 30x30 complex (destroyed), b in, x out (30 complex). */
void orc_cgesv_gpu(float *A, const float *b, float *x);
/* LAPACK cgesv (getrf + getrs) semantics used by CPU-HC. A column-major.
   Returns info (0 = ok; >0 singular, B untouched as in LAPACK cgesv). */
int orc_cgesv_lapack(float *A_colmajor, float *B);

/* ---------------- path trackers ------------------------------------------- */
typedef struct {
    int max_steps;          /* GPUHC_Max_Steps (80)                     */
    int max_corrections;    /* GPUHC_Max_Correction_Steps (3)           */
    int inc_steps;          /* GPUHC_Num_Of_Steps_to_Increase_Delta_t   */
    int num_threads;        /* OpenMP threads (<=0: runtime default)    */
    int no_truncation;      /* GPU-HC only: 1 = PH_CodeOpt, no depth-sign truncation */
    int explicit_rk;        /* GPU-HC only: 1 = archived ..._PH RK arithmetic (dev-get-new-data.cuh) */
} orc_hc_settings;

/* Per-path statistics (same layout as hcPathStats in include/hc_trifocal.h). */
typedef struct {
    int32_t steps;          /* predictor (RK4) executions               */
    int32_t corrections;    /* corrector iterations executed            */
    int32_t inliers21;      /* abort mode: reprojection inliers view 2  */
    int32_t inliers31;      /* abort mode: reprojection inliers view 3  */
} orc_path_stats;

/* GPU-HC semantics (kernel_GPUHC_trifocal_pose_PH_CodeOpt_TrunPaths).
   tracks: (312*N) x 31 complex, ld 31, in/out (x[30] is not written).
   Path b = sample*312 + track.  start_sols: 312 x 31.  params: 34 per sample. */
void orc_gpuhc_track(const orc_hc_settings *s, int num_samples,
                     const float *start_sols, const float *start_params,
                     const float *target_params, const float *diff_params,
                     const int *unified_index /* 38880 */,
                     float *tracks, uint8_t *conv, uint8_t *inf, orc_path_stats *stats);

/* Subset version for tests: track only the listed paths (path ids b).  Arrays
   are indexed by b exactly as in orc_gpuhc_track. */
void orc_gpuhc_track_subset(const orc_hc_settings *s, int num_paths, const int *path_ids,
                            const float *start_sols, const float *start_params,
                            const float *target_params, const float *diff_params,
                            const int *unified_index,
                            float *tracks, uint8_t *conv, uint8_t *inf, orc_path_stats *stats);

/* Hypothesis scoring of dev-trifocal_2op1p-eval.cuh for one converged track.
   Returns 1 if the hypothesis passes the 0.90 inlier-ratio test, writes the
   inlier counts (0/0 if the imaginary-part gate fails).  x: 31 complex.      */
int orc_score_hypothesis(const float *x, int num_edgels, const float *loc,
                         const float *K, int *inliers21, int *inliers31);

/* CPU-HC semantics (CPUHC_Generic_Solver_Eval_by_Indx): no depth-sign
   truncation, LAPACK cgesv.  Same array layouts as orc_gpuhc_track.  Returns
   wall seconds of the path loop (omp_get_wtime around it, like the reference). */
double orc_cpuhc_track(const orc_hc_settings *s, int num_samples,
                       const float *start_sols, const float *start_params,
                       const float *target_params, const float *diff_params,
                       const int *dHdx, const int *dHdt,
                       float *tracks, uint8_t *conv, uint8_t *inf, orc_path_stats *stats);

/* Route orc_cpuhc_track's solves through an external ILP64 LAPACK cgesv
   (OpenBLAS `cgesv_64_`; NULL restores the restated getf2/getrs).  Pin
   experiments only (tests/cpuhc_pin.py). */
void orc_set_external_cgesv(void *cgesv64);

/* Evaluations::Evaluate_HC_Sols counts over 312*N paths:
   out[0] converged, out[1] real (all 30 |Im| <= 1e-4 among converged), out[2] inf. */
void orc_count_solutions(int num_samples, const float *tracks, const uint8_t *conv,
                         const uint8_t *inf, int *out3);

/* Pose recovery + maximal-support selection (Evaluations.cpp:298-504, util.hpp):
   candidates = converged, |Im x[24..29]| < 1e-5, Re x[0..7] >= 0, in batch-id
   order; inliers (2 per path, -1 for non-candidates); selection = last
   candidate with the maximal count per view, or with quirks != 0 the
   reference's literal behaviour (flag index b + 312*(b/312), pose of path 0,
   list element [0]).  Returns 1 if there is a candidate. */
typedef struct {
    int32_t num_candidates, path21, inliers21, path31, inliers31, pad;
    uint64_t key21, key31;                  /* unused by the oracle (0)       */
    float R21[9], t21[3], R31[9], t31[3];
} orc_pose_selection;                       /* == hcPoseSelection layout      */
int orc_pose_support(int num_paths, const float *tracks, const uint8_t *conv, int num_edgels,
                     const float *loc, const float *K, int quirks, int32_t *inliers,
                     orc_pose_selection *sel);
/* Measure_Relative_Pose_Error: out4 = rot res 21, 31, transl res 21, 31; 1 = success */
int orc_pose_residuals(const float *gt_pose21, const float *gt_pose31, const orc_pose_selection *sel,
                       float *out4);

/* Noisy synthcurves: N(0, sigma_px^2) pixel noise on every point of every view
   from std::mt19937_64(seed) + libstdc++ normal_distribution<double> (restated). */
void orc_add_pixel_noise(int num_edgels, const float *loc, const float *K, double sigma_px, uint64_t seed,
                         float *noisy);

int orc_max_threads(void);

#ifdef __cplusplus
}
#endif
#endif
