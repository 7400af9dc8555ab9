// magmaHC-kernels.hpp -- the reference's four GPU-HC launcher declarations
// (magmaHC/gpu-kernels/magmaHC-kernels.hpp:24-105) and the two archived
// ..._PH_CodeOpt[_Volta] ablation launchers
// and ..._PH (arxived_GPU_code/gpu-kernels/magmaHC-kernels.hpp:42-96), restated so that the shim
// (hc_trifocal_shim.cpp) compiles against exactly the signatures
// GPU_HC_Solver::Solve_by_GPU_HC calls (GPU_HC_Solver.cpp:390-436): C++
// linkage, MAGMA types, the same parameter order.  In a real integration the
// reference's own header is used and this file is not needed.
#pragma once

#include "magma_v2.h"

// Ampere and above, abort off (..._TrunPaths.cu:292-386)
real_Double_t kernel_GPUHC_trifocal_2op1p_30x30_PH_CodeOpt_TrunPaths(
    magma_queue_t my_queue, int sub_RANSAC_iters, int HC_max_steps, int HC_max_correction_steps,
    int HC_delta_t_incremental_steps, magmaFloatComplex **d_startSols_array, magmaFloatComplex **d_Track_array,
    magmaFloatComplex *d_startParams, magmaFloatComplex *d_targetParams, magmaFloatComplex *d_diffParams,
    int *d_unified_dHdx_dHdt_Index, bool *d_is_GPU_HC_Sol_Converge, bool *d_is_GPU_HC_Sol_Infinity,
    magmaFloatComplex *d_Debug_Purpose);

// Volta, abort off: separate dH/dx and dH/dt index tables
real_Double_t kernel_GPUHC_trifocal_2op1p_30x30_PH_CodeOpt_TrunPaths_Volta(
    magma_queue_t my_queue, int sub_RANSAC_iters, int HC_max_steps, int HC_max_correction_steps,
    int HC_delta_t_incremental_steps, magmaFloatComplex **d_startSols_array, magmaFloatComplex **d_Track_array,
    magmaFloatComplex *d_startParams, magmaFloatComplex *d_targetParams, magmaFloatComplex *d_diffParams,
    int *d_dHdx_indx, int *d_dHdt_indx, bool *d_is_GPU_HC_Sol_Converge, bool *d_is_GPU_HC_Sol_Infinity,
    magmaFloatComplex *d_Debug_Purpose);

// Ampere and above, abort on (..._TrunRANSAC.cu:329-455)
real_Double_t kernel_GPUHC_trifocal_2op1p_30x30_PH_CodeOpt_TrunPaths_TrunRANSAC(
    magma_queue_t my_queue, int sub_RANSAC_iters, int Num_Of_Triplet_Edgels, int HC_max_steps,
    int HC_max_correction_steps, int HC_delta_t_incremental_steps, magmaFloatComplex **d_startSols_array,
    magmaFloatComplex **d_Track_array, magmaFloatComplex *d_startParams, magmaFloatComplex *d_targetParams,
    magmaFloatComplex *d_diffParams, int *d_unified_dHdx_dHdt_Index, float *d_Triplet_Edge_Locations,
    float *d_Intrinsic_Matrix, bool *d_is_GPU_HC_Sol_Converge, bool *d_is_GPU_HC_Sol_Infinity,
    magmaFloatComplex *d_Debug_Purpose, bool *d_Found_Trifocal_Sols, int *d_Trifocal_Sols_Batch_Index);

// Volta, abort on
real_Double_t kernel_GPUHC_trifocal_2op1p_30x30_PH_CodeOpt_TrunPaths_TrunRANSAC_Volta(
    magma_queue_t my_queue, int sub_RANSAC_iters, int Num_Of_Triplet_Edgels, int HC_max_steps,
    int HC_max_correction_steps, int HC_delta_t_incremental_steps, magmaFloatComplex **d_startSols_array,
    magmaFloatComplex **d_Track_array, magmaFloatComplex *d_startParams, magmaFloatComplex *d_targetParams,
    magmaFloatComplex *d_diffParams, int *d_dHdx_indx, int *d_dHdt_indx, float *d_Triplet_Edge_Locations,
    float *d_Intrinsic_Matrix, bool *d_is_GPU_HC_Sol_Converge, bool *d_is_GPU_HC_Sol_Infinity,
    magmaFloatComplex *d_Debug_Purpose, bool *d_Found_Trifocal_Sols, int *d_Trifocal_Sols_Batch_Index);

// archived ablation: no depth-sign path truncation (arxived_GPU_code/gpu-kernels/
// kernel_GPUHC_trifocal_2op1p_30x30_PH_CodeOpt[_Volta].cu)
real_Double_t kernel_GPUHC_trifocal_2op1p_30x30_PH_CodeOpt(
    magma_queue_t my_queue, int sub_RANSAC_iters, int HC_max_steps, int HC_max_correction_steps,
    int HC_delta_t_incremental_steps, magmaFloatComplex **d_startSols_array, magmaFloatComplex **d_Track_array,
    magmaFloatComplex *d_startParams, magmaFloatComplex *d_targetParams, magmaFloatComplex *d_diffParams,
    int *d_unified_dHdx_dHdt_Index, bool *d_is_GPU_HC_Sol_Converge, bool *d_is_GPU_HC_Sol_Infinity,
    magmaFloatComplex *d_Debug_Purpose);

real_Double_t kernel_GPUHC_trifocal_2op1p_30x30_PH_CodeOpt_Volta(
    magma_queue_t my_queue, int sub_RANSAC_iters, int HC_max_steps, int HC_max_correction_steps,
    int HC_delta_t_incremental_steps, magmaFloatComplex **d_startSols_array, magmaFloatComplex **d_Track_array,
    magmaFloatComplex *d_startParams, magmaFloatComplex *d_targetParams, magmaFloatComplex *d_diffParams,
    int *d_dHdx_indx, int *d_dHdt_indx, bool *d_is_GPU_HC_Sol_Converge, bool *d_is_GPU_HC_Sol_Infinity,
    magmaFloatComplex *d_Debug_Purpose);

// archived ablation: direct parameter homotopy with the explicit RK helpers
// (arxived_GPU_code/gpu-kernels/kernel_GPUHC_trifocal_2op1p_30x30_PH.cu)
real_Double_t kernel_GPUHC_trifocal_2op1p_30x30_PH(
    magma_queue_t my_queue, int sub_RANSAC_iters, int HC_max_steps, int HC_max_correction_steps,
    int HC_delta_t_incremental_steps, magmaFloatComplex **d_startSols_array, magmaFloatComplex **d_Track_array,
    magmaFloatComplex *d_startParams, magmaFloatComplex *d_targetParams, magmaFloatComplex *d_diffParams,
    int *d_dHdx_indx, int *d_dHdt_indx, bool *d_is_GPU_HC_Sol_Converge, bool *d_is_GPU_HC_Sol_Infinity,
    magmaFloatComplex *d_Debug_Purpose);
