/*
 * hc_pose.h -- pose recovery and maximal-support hypothesis selection on the
 * device, after a tracking launch.
 *
 * Replaces the host-side post-processing that GPU_HC_Solver::Solve_by_GPU_HC
 * runs after every RANSAC round (magmaHC/GPU_HC_Solver.cpp:526-527):
 *   Evaluations::Transform_GPUHC_Sols_to_Trifocal_Relative_Pose
 *                                    (magmaHC/Evaluations.cpp:298-358)
 *     candidate = converged && |Im x[24..29]| < IMAG_PART_TOL (1e-5)
 *                 && Re x[0..7] >= 0;  R = Cayley(Re x[24..26] | x[27..29])
 *                 with unit columns, t = Re x[18..20] | x[21..23] normalised
 *                 (util.hpp:31-79)
 *   Evaluations::get_Solution_with_Maximal_Support (Evaluations.cpp:382-504)
 *     for every candidate and every triplet edgel: depth rho (util.hpp:169-186)
 *     and pixel reprojection error (util.hpp:188-209) for views 1-2 and 1-3;
 *     inlier if < REPROJ_ERROR_INLIER_THRESH (2 px, definitions.hpp:17); the
 *     views are selected independently by maximal support (:455-500)
 * and the relative-pose error against the ground truth
 *   Evaluations::Measure_Relative_Pose_Error (Evaluations.cpp:523-543),
 *   get_Rotation_Residual / get_Translation_Residual (:360-380).
 *
 * Selection rule.  The reference pushes every candidate whose count is >= the
 * running maximum and then reads element [0] of that list, i.e. always the
 * first candidate; together with Appendix C item 7 of SURVEY.md (the pose is
 * converted from the base pointer = path 0, and the converged flag is read at
 * index b + 312*(b/312)) its host selection is not meaningful.  The default
 * here is the rule the reference's own commented-out line states
 * (Evaluations.cpp:460,466, `Index = cp_i` under `>=`): the LAST candidate (in
 * batch-id order) that attains the maximal count.  HC_POSE_REFERENCE_QUIRKS
 * reproduces the reference literally (flag index b + 312*(b/312), out of range
 * = not converged; every candidate's pose taken from path 0; element [0]).
 *
 * Conventions as in hc_trifocal.h: caller-owned device buffers, asynchronous on
 * the caller's stream and current device, hcStatus errors, batch id b.
 */
#ifndef HC_POSE_H
#define HC_POSE_H

#include "hc_trifocal.h"

#ifdef __cplusplus
extern "C" {
#endif

#define HC_POSE_REFERENCE_QUIRKS 1   /* flags bit: literal reference selection */

/* Result of one selection (device memory, written by the entry point). */
typedef struct {
    int32_t num_candidates;   /* real-rotation, positive-depth converged paths      */
    int32_t path21;           /* batch id selected for views 1-2 (-1: none)         */
    int32_t inliers21;
    int32_t path31;           /* batch id selected for views 1-3 (-1: none)         */
    int32_t inliers31;
    int32_t pad;
    uint64_t key21;           /* selection keys: (count << 32 | b), or 0xFFFFFFFF - b
                                 with HC_POSE_REFERENCE_QUIRKS; the larger key wins */
    uint64_t key31;
    float R21[9], t21[3];     /* pose of path21: R row-major, unit t                */
    float R31[9], t31[3];     /* pose of path31                                     */
} hcPoseSelection;

/* Candidate filter, pose conversion, inlier scoring of every candidate over all
 * triplet edgels and maximal-support selection for num_paths = 312*N tracks.
 *   tracks      (312N) x 31 complex, ld 31 (the tracker's output)
 *   converge    312N bytes
 *   locations   E x 6 floats (x1 y1 x2 y2 x3 y3), metric
 *   K           9 floats, row-major intrinsics
 *   inliers     2 x 312N int32 out: (inliers21, inliers31) per path, -1 for
 *               non-candidates
 *   selection   one hcPoseSelection out */
hcStatus hc_trifocal_pose_support(int num_paths, const hcComplex *tracks, const uint8_t *converge,
                                  int num_edgels, const float *locations, const float *K, int flags,
                                  int32_t *inliers, hcPoseSelection *selection, hcStream stream);

/* Host: merges the selections of several launches / GPUs (each over its own
 * batch-id range starting at path_offsets[i]) into one, with global batch ids:
 * the keys are re-based and the maximal key wins per view, exactly as if one
 * launch had covered all paths.  parts are host copies. */
void hc_pose_merge(int n, const hcPoseSelection *parts, const int32_t *path_offsets, int flags,
                   hcPoseSelection *out);

/* Host: relative pose error of a selected pose against ground-truth poses
 * (12 floats each: R row-major then t, GT_Poses21/31 files).
 * out[0..3] = rotation residual 21, 31 (rad), translation residual 21, 31;
 * returns 1 when all four are below ROT/TRANSL_RESIDUAL_TOL (0.1), else 0. */
int hc_pose_residuals(const float *gt_pose21, const float *gt_pose31, const float *R21, const float *t21,
                      const float *R31, const float *t31, float *out4);

#ifdef __cplusplus
}
#endif

#endif /* HC_POSE_H */
