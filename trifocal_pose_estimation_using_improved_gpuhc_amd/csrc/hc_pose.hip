// hc_pose.hip -- device pose recovery + maximal-support selection (include/hc_pose.h).
//
// Replaces the host post-processing of every RANSAC round
// (magmaHC/GPU_HC_Solver.cpp:526-527):
//   Evaluations::Transform_GPUHC_Sols_to_Trifocal_Relative_Pose (Evaluations.cpp:298-358)
//   Evaluations::get_Solution_with_Maximal_Support              (Evaluations.cpp:382-504)
// with the multiview helpers of magmaHC/util.hpp restated op for op (FP32,
// no contraction: -ffp-contract=off; IEEE division and sqrt).
//
// Layout: one wavefront per batch id b (grid-stride).  Non-converged paths
// cost one byte load.  A candidate's pose is computed redundantly by every
// lane (uniform loads of x[18..29]), then the 64 lanes stride over the
// triplet edgels (E x 24 B, L2-resident after the first candidate) and the two
// inlier counts are wave-reduced.  Selection is a single 64-bit atomicMax per
// view on key = count << 32 | b (largest count, ties -> largest b = the last
// candidate attaining the maximum, the rule of Evaluations.cpp:460,466); a
// one-wave epilogue decodes the keys and writes the selected poses.
#include "../../include/hc_pose.h"
#include "hc_device.hpp"

namespace hc {

extern thread_local hipError_t g_last_hip_error;   // hc_kernels.hip

namespace {

struct Pose {
    float R[18];   // R21 row-major, R31 row-major
    float t[6];    // unit t21, unit t31
};

// util.hpp:31-66: Cayley_To_Rotation_Matrix + Normalize_Rotation_Matrix
// (all three column norms first, then the divisions)
__device__ __forceinline__ void cayley_unit(float a, float b, float c, float *R) {
    R[0] = (1.0f + a * a) - (b * b + c * c);
    R[1] = 2.0f * (a * b - c);
    R[2] = 2.0f * (a * c + b);
    R[3] = 2.0f * (a * b + c);
    R[4] = (1.0f + b * b) - (a * a + c * c);
    R[5] = 2.0f * (b * c - a);
    R[6] = 2.0f * (a * c - b);
    R[7] = 2.0f * (b * c + a);
    R[8] = (1.0f + c * c) - (a * a + b * b);
    const float n0 = __builtin_sqrtf((R[0] * R[0] + R[3] * R[3]) + R[6] * R[6]);
    const float n1 = __builtin_sqrtf((R[1] * R[1] + R[4] * R[4]) + R[7] * R[7]);
    const float n2 = __builtin_sqrtf((R[2] * R[2] + R[5] * R[5]) + R[8] * R[8]);
    R[0] /= n0; R[3] /= n0; R[6] /= n0;
    R[1] /= n1; R[4] /= n1; R[7] /= n1;
    R[2] /= n2; R[5] /= n2; R[8] /= n2;
}

// util.hpp:69-78: Normalize_Translation_Vector
__device__ __forceinline__ void unit3(float *t) {
    const float n = __builtin_sqrtf((t[0] * t[0] + t[1] * t[1]) + t[2] * t[2]);
    t[0] /= n; t[1] /= n; t[2] /= n;
}

// Evaluations.cpp:235-265 (Convert_Trifocal_Translation / _Rotation) from x = 31 complex
__device__ __forceinline__ void make_pose(const cf *__restrict__ x, Pose &P) {
#pragma unroll
    for (int i = 0; i < 6; i++) P.t[i] = x[18 + i].x;
    unit3(P.t);
    unit3(P.t + 3);
    cayley_unit(x[24].x, x[25].x, x[26].x, P.R);
    cayley_unit(x[27].x, x[28].x, x[29].x, P.R + 9);
}

// util.hpp:169-209 for one view pair: depth rho of gamma1 (get_depth_rho), then
// the pixel reprojection error of gamma2 (get_Reprojection_Pixels_Error).
// gamma = (g.x, g.y, 1); matrix-vector products accumulate from 0.0f as the
// reference's get_Matrix_Vector_Product does.
__device__ __forceinline__ bool reproj_inlier(float g0, float g1, float h0, float h1, const float *R, const float *T,
                                              float K0, float K2, float K4, float K5) {
    const float Rg2_2 = ((0.0f + R[2] * h0) + R[5] * h1) + R[8] * 1.0f;   // (R' gamma2)_2
    float rho = T[2] * Rg2_2;
    const float RtT_2 = ((0.0f + R[2] * T[0]) + R[5] * T[1]) + R[8] * T[2];   // (R' T)_2
    rho -= RtT_2;
    float m0 = ((0.0f + R[0] * g0) + R[1] * g1) + R[2] * 1.0f;            // R gamma1
    float m1 = ((0.0f + R[3] * g0) + R[4] * g1) + R[5] * 1.0f;
    float m2 = ((0.0f + R[6] * g0) + R[7] * g1) + R[8] * 1.0f;
    rho /= (1.0f - m2 * Rg2_2);
    m0 *= rho; m0 += T[0];
    m1 *= rho; m1 += T[1];
    m2 *= rho; m2 += T[2];
    m0 /= m2;
    m1 /= m2;
    m0 = m0 * K0 + K2;
    m1 = m1 * K4 + K5;
    const float p0 = h0 * K0 + K2, p1 = h1 * K4 + K5;
    m0 -= p0;
    m1 -= p1;
    const float err = __builtin_sqrtf((m0 * m0 + m1 * m1) + 0.0f * 0.0f);
    return err < 2.0f;   // REPROJ_ERROR_INLIER_THRESH (definitions.hpp:17)
}

__device__ __forceinline__ bool is_converged(const uint8_t *conv, int b, int num_paths, bool quirks) {
    if (!quirks) return conv[b] != 0;
    const long long ci = (long long)b + (long long)NTRK * (b / NTRK);   // Evaluations.cpp:317
    return ci < num_paths && conv[ci] != 0;
}

__device__ __forceinline__ uint64_t sel_key(int count, int b, bool quirks) {
    return quirks ? (uint64_t)(0xFFFFFFFFu - (uint32_t)b) : (((uint64_t)(uint32_t)count << 32) | (uint32_t)b);
}

__global__ void __launch_bounds__(256) k_pose_support(int num_paths, const cf *__restrict__ tracks,
                                                      const uint8_t *__restrict__ conv, int E,
                                                      const float *__restrict__ loc, const float *__restrict__ K,
                                                      int flags, int32_t *__restrict__ inl, hcPoseSelection *sel) {
    const int lane = lane_id();
    const int nw = gridDim.x * (blockDim.x / WAVE);
    const bool quirks = (flags & HC_POSE_REFERENCE_QUIRKS) != 0;
    const float K0 = K[0], K2 = K[2], K4 = K[4], K5 = K[5];
    for (int b = blockIdx.x * (blockDim.x / WAVE) + threadIdx.x / WAVE; b < num_paths; b += nw) {
        int c21 = -1, c31 = -1;
        if (is_converged(conv, b, num_paths, quirks)) {
            const cf *x = tracks + (size_t)b * (NV + 1);
            const cf xv = lane < NV ? x[lane] : cmk(0.0f, 0.0f);
            // Evaluations.cpp:322-331: |Im x[24..29]| < IMAG_PART_TOL, Re x[0..7] >= 0
            const unsigned long long im = __ballot(lane >= 24 && lane < NV && (double)__builtin_fabsf(xv.y) < 1e-5);
            const unsigned long long dp = __ballot(lane < 8 && xv.x >= 0.0f);
            if ((im & 0x3F000000ull) == 0x3F000000ull && (dp & 0xFFull) == 0xFFull) {
                Pose P;
                make_pose(quirks ? tracks : x, P);   // quirk: converted from the base pointer (:334-341)
                int a21 = 0, a31 = 0;
                for (int e = lane; e < E; e += WAVE) {
                    const float2 g01 = *reinterpret_cast<const float2 *>(loc + (size_t)e * 6);
                    const float2 g23 = *reinterpret_cast<const float2 *>(loc + (size_t)e * 6 + 2);
                    const float2 g45 = *reinterpret_cast<const float2 *>(loc + (size_t)e * 6 + 4);
                    a21 += reproj_inlier(g01.x, g01.y, g23.x, g23.y, P.R, P.t, K0, K2, K4, K5) ? 1 : 0;
                    a31 += reproj_inlier(g01.x, g01.y, g45.x, g45.y, P.R + 9, P.t + 3, K0, K2, K4, K5) ? 1 : 0;
                }
                c21 = wave_sum_i(a21);
                c31 = wave_sum_i(a31);
                if (lane == 0) {
                    atomicAdd(&sel->num_candidates, 1);
                    atomicMax(reinterpret_cast<unsigned long long *>(&sel->key21),
                              (unsigned long long)sel_key(c21, b, quirks));
                    atomicMax(reinterpret_cast<unsigned long long *>(&sel->key31),
                              (unsigned long long)sel_key(c31, b, quirks));
                }
            }
        }
        if (lane == 0) {
            inl[2 * (size_t)b] = c21;
            inl[2 * (size_t)b + 1] = c31;
        }
    }
}

// decode the keys; pose of the selected path (Evaluations.cpp:496-501)
__global__ void __launch_bounds__(64) k_pose_final(int num_paths, const cf *__restrict__ tracks,
                                                   const int32_t *__restrict__ inl, int flags, hcPoseSelection *sel) {
    if (threadIdx.x != 0) return;
    const bool quirks = (flags & HC_POSE_REFERENCE_QUIRKS) != 0;
    const bool any = sel->num_candidates > 0;
    for (int v = 0; v < 2; v++) {
        const uint64_t key = v == 0 ? sel->key21 : sel->key31;
        int b = -1, cnt = -1;
        if (any) {
            b = quirks ? (int)(0xFFFFFFFFu - (uint32_t)key) : (int)(uint32_t)key;
            cnt = (b >= 0 && b < num_paths) ? inl[2 * (size_t)b + v] : -1;
        }
        Pose P;
        for (int i = 0; i < 18; i++) P.R[i] = 0.0f;
        for (int i = 0; i < 6; i++) P.t[i] = 0.0f;
        if (b >= 0 && b < num_paths) make_pose(quirks ? tracks : tracks + (size_t)b * (NV + 1), P);
        float *R = v == 0 ? sel->R21 : sel->R31;
        float *t = v == 0 ? sel->t21 : sel->t31;
        for (int i = 0; i < 9; i++) R[i] = P.R[v * 9 + i];
        for (int i = 0; i < 3; i++) t[i] = P.t[v * 3 + i];
        if (v == 0) { sel->path21 = b; sel->inliers21 = cnt; }
        else { sel->path31 = b; sel->inliers31 = cnt; }
    }
}

}  // namespace

}  // namespace hc

extern "C" hcStatus hc_trifocal_pose_support(int num_paths, const hcComplex *tracks, const uint8_t *converge,
                                             int num_edgels, const float *locations, const float *K, int flags,
                                             int32_t *inliers, hcPoseSelection *selection, hcStream stream) {
    using namespace hc;
    if (num_paths < 0 || num_edgels < 0 || !selection || (flags & ~HC_POSE_REFERENCE_QUIRKS) != 0)
        return HC_ERROR_INVALID_VALUE;
    if (num_paths > 0 && (!tracks || !converge || !inliers || !K || (num_edgels > 0 && !locations)))
        return HC_ERROR_INVALID_VALUE;
    hipStream_t s = (hipStream_t)stream;
    (void)hipGetLastError();
    if ((g_last_hip_error = hipMemsetAsync(selection, 0, sizeof(hcPoseSelection), s)) != hipSuccess) return HC_ERROR_LAUNCH;
    if (num_paths > 0) {
        int dev = 0, cus = 256;
        if (hipGetDevice(&dev) != hipSuccess) return HC_ERROR_DEVICE;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return HC_ERROR_DEVICE;
        const long long waves = num_paths < cus * 32 ? num_paths : (long long)cus * 32;
        const int blocks = (int)((waves + 3) / 4);
        hipLaunchKernelGGL(k_pose_support, dim3(blocks), dim3(256), 0, s, num_paths, (const cf *)tracks, converge,
                           num_edgels, locations, K, flags, inliers, selection);
        if ((g_last_hip_error = hipGetLastError()) != hipSuccess) return HC_ERROR_LAUNCH;
    }
    hipLaunchKernelGGL(k_pose_final, dim3(1), dim3(64), 0, s, num_paths, (const cf *)tracks, (const int32_t *)inliers,
                       flags, selection);
    if ((g_last_hip_error = hipGetLastError()) != hipSuccess) return HC_ERROR_LAUNCH;
    return HC_SUCCESS;
}
