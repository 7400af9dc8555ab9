// hc_trifocal_shim.cpp -- drop-in replacement of the reference's four GPU-HC
// launchers (magmaHC/gpu-kernels/magmaHC-kernels.hpp:24-105, implemented in
// kernel_GPUHC_trifocal_2op1p_30x30_PH_CodeOpt_TrunPaths[_TrunRANSAC][_Volta].cu)
// and of the archived ablation launchers ..._PH_CodeOpt[_Volta] (no path
// truncation) and ..._PH (explicit RK as well; arxived_GPU_code/gpu-kernels/
// magmaHC-kernels.hpp:42-96)
// on top of this repository's C-ABI (include/hc_trifocal.h).
//
// A maintainer compiles this file in place of the four .cu files and links
// -lhc_trifocal; GPU_HC_Solver::Solve_by_GPU_HC (GPU_HC_Solver.cpp:390-436)
// then runs unchanged.  Semantics kept from the reference:
//  * C++ linkage, MAGMA types, the reference's parameter order;
//  * the reference's pointer arrays (d_startSols_array: one pointer per track,
//    d_Track_array: one per (sample, track)) are passed through as-is;
//  * bool flags (1 byte) are the ABI's uint8_t flags;
//  * the launch is asynchronous on the queue's stream and the return value is
//    0.0 (..._TrunPaths.cu:385); failures are printed like the reference
//    (:383), never exit();
//  * abort mode uses the reference's semantics: paths in flight when a good
//    hypothesis is found run to completion (hcAbortArgs::inflight_stop = 0);
//  * the Volta variants take separate dH/dx and dH/dt tables: the shim
//    concatenates them into the unified layout (Data_Reader.cpp:167-189) on the
//    queue's stream before the launch.
// The ABI never allocates on the hot path; the shim owns one workspace (and one
// unified-table buffer for the Volta variants) per (device, stream), allocated
// by hc_trifocal_shim_reserve (hc_trifocal_shim.h, called from
// GPU_HC_Solver::Allocate_Arrays) and kept for the process lifetime.  A launch
// on a stream that was not reserved, or that needs more than was reserved,
// grows the workspace on the hot path (synchronising the stream) and says so
// once.
#include <cstdio>
#include <map>
#include <mutex>
#include <utility>

#include "hc_trifocal_shim.h"
#include "magmaHC-kernels.hpp"

namespace {

constexpr int kHxInts = 36000, kHtInts = 2880;   // dHdx_Index_Matrix_Size, dHdt_Index_Matrix_Size (..._TrunPaths.cu:311-320)

struct StreamState {
    void *workspace = nullptr;
    size_t ws_bytes = 0;
    int32_t *unified = nullptr;   // Volta variants only
    int hot_grows = 0;            // launches that had to allocate
};

std::mutex g_mu;
std::map<std::pair<int, hipStream_t>, StreamState> g_states;

// (g_mu held) the stream's workspace grown to `need` bytes, the unified buffer if asked
bool ensure(StreamState &st, hipStream_t s, size_t need, bool need_unified) {
    if (st.workspace && st.ws_bytes < need) {
        // the previous launch on this stream may still use it
        if (hipStreamSynchronize(s) != hipSuccess || hipFree(st.workspace) != hipSuccess) return false;
        st.workspace = nullptr;
        st.ws_bytes = 0;
    }
    if (!st.workspace) {
        if (hipMalloc(&st.workspace, need) != hipSuccess) st.workspace = nullptr;
        st.ws_bytes = st.workspace ? need : 0;
    }
    if (need_unified && !st.unified &&
        hipMalloc(reinterpret_cast<void **>(&st.unified), (kHxInts + kHtInts) * sizeof(int32_t)) != hipSuccess)
        st.unified = nullptr;
    return st.workspace && (!need_unified || st.unified);
}

// the library must read the argument structs as this shim lays them out
bool abi_ok() {
    static const bool ok = [] {
        const int v = hc_trifocal_abi_version();
        if (v != HC_TRIFOCAL_ABI_VERSION)
            printf("hc_trifocal_shim: library ABI %d, shim built against %d: not launching\n", v,
                   HC_TRIFOCAL_ABI_VERSION);
        return v == HC_TRIFOCAL_ABI_VERSION;
    }();
    return ok;
}

// the stream's state for a launch of N samples (N = 0: abort mode, the base
// size); reserved streams return at once
StreamState *state_for(hipStream_t s, bool need_unified, int N = 0, int max_steps = 80) {
    if (!abi_ok()) return nullptr;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return nullptr;
    std::lock_guard<std::mutex> g(g_mu);
    StreamState &st = g_states[{dev, s}];
    const size_t need = N > 0 ? hc_trifocal_workspace_size_for_steps(N, max_steps) : hc_trifocal_workspace_size();
    if (st.workspace && st.ws_bytes >= need && (!need_unified || st.unified)) return &st;
    if (st.hot_grows++ == 0)
        printf("hc_trifocal_shim: allocating on the launch path (stream not reserved for %d samples at %d steps; "
               "call hc_trifocal_shim_reserve from Allocate_Arrays)\n", N, max_steps);
    return ensure(st, s, need, need_unified) ? &st : nullptr;
}

hcTrackArgs make_args(int sub_RANSAC_iters, int max_steps, int max_corr, int inc_steps,
                      magmaFloatComplex **d_startSols_array, magmaFloatComplex **d_Track_array,
                      magmaFloatComplex *d_startParams, magmaFloatComplex *d_targetParams,
                      magmaFloatComplex *d_diffParams, const int *d_unified, bool *d_conv, bool *d_inf) {
    hcTrackArgs a{};
    a.sub_ransac_iters = sub_RANSAC_iters;
    a.settings.max_steps = max_steps;
    a.settings.max_corrections = max_corr;
    a.settings.delta_t_inc_steps = inc_steps;
    a.start_sols_array = reinterpret_cast<const hcComplex *const *>(d_startSols_array);
    a.track_array = reinterpret_cast<hcComplex *const *>(d_Track_array);
    a.start_params = reinterpret_cast<const hcComplex *>(d_startParams);
    a.target_params = reinterpret_cast<const hcComplex *>(d_targetParams);
    a.diff_params = reinterpret_cast<const hcComplex *>(d_diffParams);
    a.unified_index = reinterpret_cast<const int32_t *>(d_unified);
    a.converge = reinterpret_cast<uint8_t *>(d_conv);
    a.infinity = reinterpret_cast<uint8_t *>(d_inf);
    return a;
}

void report(hcStatus st, const char *what) {
    if (st != HC_SUCCESS) printf("%s failed: status %d (%s)\n", what, (int)st, hc_last_error_string());
}

const int32_t *unify(StreamState *st, const int *d_dHdx_indx, const int *d_dHdt_indx, hipStream_t s) {
    if (hipMemcpyAsync(st->unified, d_dHdx_indx, kHxInts * sizeof(int32_t), hipMemcpyDeviceToDevice, s) != hipSuccess ||
        hipMemcpyAsync(st->unified + kHxInts, d_dHdt_indx, kHtInts * sizeof(int32_t), hipMemcpyDeviceToDevice, s) !=
            hipSuccess)
        return nullptr;
    return st->unified;
}

real_Double_t track(magma_queue_t q, int N, int max_steps, int max_corr, int inc_steps, magmaFloatComplex **ss,
                    magmaFloatComplex **tracks, magmaFloatComplex *sp, magmaFloatComplex *tp, magmaFloatComplex *dp,
                    const int *unified, const int *d_hx, const int *d_ht, bool *conv, bool *inf, const char *name,
                    bool truncate = true, bool explicit_rk = false) {
    hipStream_t s = magma_queue_get_hip_stream(q);
    StreamState *st = state_for(s, unified == nullptr, N, max_steps);
    if (!st) { report(HC_ERROR_WORKSPACE, name); return 0.0; }
    const int32_t *U = unified ? reinterpret_cast<const int32_t *>(unified) : unify(st, d_hx, d_ht, s);
    if (!U) { report(HC_ERROR_LAUNCH, name); return 0.0; }
    hcTrackArgs a = make_args(N, max_steps, max_corr, inc_steps, ss, tracks, sp, tp, dp, U, conv, inf);
    const size_t wsb = st->ws_bytes;
    report(explicit_rk ? hc_trifocal_2op1p_30x30_track_ph(&a, st->workspace, wsb, (hcStream)s)
           : truncate  ? hc_trifocal_2op1p_30x30_track(&a, st->workspace, wsb, (hcStream)s)
                       : hc_trifocal_2op1p_30x30_track_ph_codeopt(&a, st->workspace, wsb, (hcStream)s),
           name);
    return 0.0;
}

real_Double_t track_abort(magma_queue_t q, int N, int E, int max_steps, int max_corr, int inc_steps,
                          magmaFloatComplex **ss, magmaFloatComplex **tracks, magmaFloatComplex *sp,
                          magmaFloatComplex *tp, magmaFloatComplex *dp, const int *unified, const int *d_hx,
                          const int *d_ht, float *edgels, float *K, bool *conv, bool *inf, bool *found,
                          int *batch_index, const char *name) {
    hipStream_t s = magma_queue_get_hip_stream(q);
    StreamState *st = state_for(s, unified == nullptr);
    if (!st) { report(HC_ERROR_WORKSPACE, name); return 0.0; }
    const int32_t *U = unified ? reinterpret_cast<const int32_t *>(unified) : unify(st, d_hx, d_ht, s);
    if (!U) { report(HC_ERROR_LAUNCH, name); return 0.0; }
    hcTrackArgs a = make_args(N, max_steps, max_corr, inc_steps, ss, tracks, sp, tp, dp, U, conv, inf);
    hcAbortArgs ab{};
    ab.num_triplet_edgels = E;
    ab.triplet_edge_locations = edgels;
    ab.intrinsic_matrix = K;
    ab.found_trifocal_sols = reinterpret_cast<uint8_t *>(found);
    ab.trifocal_sols_batch_index = batch_index;
    ab.inflight_stop = 0;   // the reference's semantics (..._TrunRANSAC.cu:148-152)
    report(hc_trifocal_2op1p_30x30_track_abort(&a, &ab, st->workspace, hc_trifocal_workspace_size(), (hcStream)s),
           name);
    return 0.0;
}

}  // namespace

extern "C" hcStatus hc_trifocal_shim_reserve(magma_queue_t queue, int max_samples, int max_steps) {
    if (!queue || max_samples < 0 || max_steps < 0 || !abi_ok()) return HC_ERROR_INVALID_VALUE;
    const hipStream_t s = magma_queue_get_hip_stream(queue);
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return HC_ERROR_DEVICE;
    std::lock_guard<std::mutex> g(g_mu);
    StreamState &st = g_states[{dev, s}];
    const size_t need = max_samples > 0 ? hc_trifocal_workspace_size_for_steps(max_samples, max_steps)
                                        : hc_trifocal_workspace_size();
    if (!ensure(st, s, need, true)) return HC_ERROR_WORKSPACE;
    return hipStreamSynchronize(s) == hipSuccess ? HC_SUCCESS : HC_ERROR_DEVICE;
}

extern "C" hcStatus hc_trifocal_shim_status(magma_queue_t queue) {
    if (!queue) return HC_ERROR_INVALID_VALUE;
    const hipStream_t s = magma_queue_get_hip_stream(queue);
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return HC_ERROR_DEVICE;
    void *ws = nullptr;
    {
        std::lock_guard<std::mutex> g(g_mu);
        auto it = g_states.find({dev, s});
        if (it == g_states.end() || !it->second.workspace) return HC_SUCCESS;   // nothing launched here
        ws = it->second.workspace;
    }
    if (hipStreamSynchronize(s) != hipSuccess) return HC_ERROR_DEVICE;
    return hc_trifocal_workspace_status(ws);
}

extern "C" hcStatus hc_trifocal_shim_info(magma_queue_t queue, size_t *workspace_bytes, int *hot_path_grows) {
    if (!queue || !workspace_bytes || !hot_path_grows) return HC_ERROR_INVALID_VALUE;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return HC_ERROR_DEVICE;
    std::lock_guard<std::mutex> g(g_mu);
    auto it = g_states.find({dev, magma_queue_get_hip_stream(queue)});
    *workspace_bytes = it == g_states.end() ? 0 : it->second.ws_bytes;
    *hot_path_grows = it == g_states.end() ? 0 : it->second.hot_grows;
    return HC_SUCCESS;
}

real_Double_t kernel_GPUHC_trifocal_2op1p_30x30_PH_CodeOpt_TrunPaths(
    magma_queue_t my_queue, int sub_RANSAC_iters, int HC_max_steps, int HC_max_correction_steps,
    int HC_delta_t_incremental_steps, magmaFloatComplex **d_startSols_array, magmaFloatComplex **d_Track_array,
    magmaFloatComplex *d_startParams, magmaFloatComplex *d_targetParams, magmaFloatComplex *d_diffParams,
    int *d_unified_dHdx_dHdt_Index, bool *d_is_GPU_HC_Sol_Converge, bool *d_is_GPU_HC_Sol_Infinity,
    magmaFloatComplex * /*d_Debug_Purpose*/) {
    return track(my_queue, sub_RANSAC_iters, HC_max_steps, HC_max_correction_steps, HC_delta_t_incremental_steps,
                 d_startSols_array, d_Track_array, d_startParams, d_targetParams, d_diffParams,
                 d_unified_dHdx_dHdt_Index, nullptr, nullptr, d_is_GPU_HC_Sol_Converge, d_is_GPU_HC_Sol_Infinity,
                 "kernel_GPUHC_trifocal_2op1p_30x30_PH_CodeOpt_TrunPaths");
}

real_Double_t kernel_GPUHC_trifocal_2op1p_30x30_PH_CodeOpt_TrunPaths_Volta(
    magma_queue_t my_queue, int sub_RANSAC_iters, int HC_max_steps, int HC_max_correction_steps,
    int HC_delta_t_incremental_steps, magmaFloatComplex **d_startSols_array, magmaFloatComplex **d_Track_array,
    magmaFloatComplex *d_startParams, magmaFloatComplex *d_targetParams, magmaFloatComplex *d_diffParams,
    int *d_dHdx_indx, int *d_dHdt_indx, bool *d_is_GPU_HC_Sol_Converge, bool *d_is_GPU_HC_Sol_Infinity,
    magmaFloatComplex * /*d_Debug_Purpose*/) {
    return track(my_queue, sub_RANSAC_iters, HC_max_steps, HC_max_correction_steps, HC_delta_t_incremental_steps,
                 d_startSols_array, d_Track_array, d_startParams, d_targetParams, d_diffParams, nullptr, d_dHdx_indx,
                 d_dHdt_indx, d_is_GPU_HC_Sol_Converge, d_is_GPU_HC_Sol_Infinity,
                 "kernel_GPUHC_trifocal_2op1p_30x30_PH_CodeOpt_TrunPaths_Volta");
}

real_Double_t kernel_GPUHC_trifocal_2op1p_30x30_PH_CodeOpt_TrunPaths_TrunRANSAC(
    magma_queue_t my_queue, int sub_RANSAC_iters, int Num_Of_Triplet_Edgels, int HC_max_steps,
    int HC_max_correction_steps, int HC_delta_t_incremental_steps, magmaFloatComplex **d_startSols_array,
    magmaFloatComplex **d_Track_array, magmaFloatComplex *d_startParams, magmaFloatComplex *d_targetParams,
    magmaFloatComplex *d_diffParams, int *d_unified_dHdx_dHdt_Index, float *d_Triplet_Edge_Locations,
    float *d_Intrinsic_Matrix, bool *d_is_GPU_HC_Sol_Converge, bool *d_is_GPU_HC_Sol_Infinity,
    magmaFloatComplex * /*d_Debug_Purpose*/, bool *d_Found_Trifocal_Sols, int *d_Trifocal_Sols_Batch_Index) {
    return track_abort(my_queue, sub_RANSAC_iters, Num_Of_Triplet_Edgels, HC_max_steps, HC_max_correction_steps,
                       HC_delta_t_incremental_steps, d_startSols_array, d_Track_array, d_startParams, d_targetParams,
                       d_diffParams, d_unified_dHdx_dHdt_Index, nullptr, nullptr, d_Triplet_Edge_Locations,
                       d_Intrinsic_Matrix, d_is_GPU_HC_Sol_Converge, d_is_GPU_HC_Sol_Infinity,
                       d_Found_Trifocal_Sols, d_Trifocal_Sols_Batch_Index,
                       "kernel_GPUHC_trifocal_2op1p_30x30_PH_CodeOpt_TrunPaths_TrunRANSAC");
}

real_Double_t kernel_GPUHC_trifocal_2op1p_30x30_PH_CodeOpt_TrunPaths_TrunRANSAC_Volta(
    magma_queue_t my_queue, int sub_RANSAC_iters, int Num_Of_Triplet_Edgels, int HC_max_steps,
    int HC_max_correction_steps, int HC_delta_t_incremental_steps, magmaFloatComplex **d_startSols_array,
    magmaFloatComplex **d_Track_array, magmaFloatComplex *d_startParams, magmaFloatComplex *d_targetParams,
    magmaFloatComplex *d_diffParams, int *d_dHdx_indx, int *d_dHdt_indx, float *d_Triplet_Edge_Locations,
    float *d_Intrinsic_Matrix, bool *d_is_GPU_HC_Sol_Converge, bool *d_is_GPU_HC_Sol_Infinity,
    magmaFloatComplex * /*d_Debug_Purpose*/, bool *d_Found_Trifocal_Sols, int *d_Trifocal_Sols_Batch_Index) {
    return track_abort(my_queue, sub_RANSAC_iters, Num_Of_Triplet_Edgels, HC_max_steps, HC_max_correction_steps,
                       HC_delta_t_incremental_steps, d_startSols_array, d_Track_array, d_startParams, d_targetParams,
                       d_diffParams, nullptr, d_dHdx_indx, d_dHdt_indx, d_Triplet_Edge_Locations, d_Intrinsic_Matrix,
                       d_is_GPU_HC_Sol_Converge, d_is_GPU_HC_Sol_Infinity, d_Found_Trifocal_Sols,
                       d_Trifocal_Sols_Batch_Index, "kernel_GPUHC_trifocal_2op1p_30x30_PH_CodeOpt_TrunPaths_TrunRANSAC_Volta");
}

real_Double_t kernel_GPUHC_trifocal_2op1p_30x30_PH_CodeOpt(
    magma_queue_t my_queue, int sub_RANSAC_iters, int HC_max_steps, int HC_max_correction_steps,
    int HC_delta_t_incremental_steps, magmaFloatComplex **d_startSols_array, magmaFloatComplex **d_Track_array,
    magmaFloatComplex *d_startParams, magmaFloatComplex *d_targetParams, magmaFloatComplex *d_diffParams,
    int *d_unified_dHdx_dHdt_Index, bool *d_is_GPU_HC_Sol_Converge, bool *d_is_GPU_HC_Sol_Infinity,
    magmaFloatComplex * /*d_Debug_Purpose*/) {
    return track(my_queue, sub_RANSAC_iters, HC_max_steps, HC_max_correction_steps, HC_delta_t_incremental_steps,
                 d_startSols_array, d_Track_array, d_startParams, d_targetParams, d_diffParams,
                 d_unified_dHdx_dHdt_Index, nullptr, nullptr, d_is_GPU_HC_Sol_Converge, d_is_GPU_HC_Sol_Infinity,
                 "kernel_GPUHC_trifocal_2op1p_30x30_PH_CodeOpt", false);
}

real_Double_t kernel_GPUHC_trifocal_2op1p_30x30_PH_CodeOpt_Volta(
    magma_queue_t my_queue, int sub_RANSAC_iters, int HC_max_steps, int HC_max_correction_steps,
    int HC_delta_t_incremental_steps, magmaFloatComplex **d_startSols_array, magmaFloatComplex **d_Track_array,
    magmaFloatComplex *d_startParams, magmaFloatComplex *d_targetParams, magmaFloatComplex *d_diffParams,
    int *d_dHdx_indx, int *d_dHdt_indx, bool *d_is_GPU_HC_Sol_Converge, bool *d_is_GPU_HC_Sol_Infinity,
    magmaFloatComplex * /*d_Debug_Purpose*/) {
    return track(my_queue, sub_RANSAC_iters, HC_max_steps, HC_max_correction_steps, HC_delta_t_incremental_steps,
                 d_startSols_array, d_Track_array, d_startParams, d_targetParams, d_diffParams, nullptr, d_dHdx_indx,
                 d_dHdt_indx, d_is_GPU_HC_Sol_Converge, d_is_GPU_HC_Sol_Infinity,
                 "kernel_GPUHC_trifocal_2op1p_30x30_PH_CodeOpt_Volta", false);
}

real_Double_t kernel_GPUHC_trifocal_2op1p_30x30_PH(
    magma_queue_t my_queue, int sub_RANSAC_iters, int HC_max_steps, int HC_max_correction_steps,
    int HC_delta_t_incremental_steps, magmaFloatComplex **d_startSols_array, magmaFloatComplex **d_Track_array,
    magmaFloatComplex *d_startParams, magmaFloatComplex *d_targetParams, magmaFloatComplex *d_diffParams,
    int *d_dHdx_indx, int *d_dHdt_indx, bool *d_is_GPU_HC_Sol_Converge, bool *d_is_GPU_HC_Sol_Infinity,
    magmaFloatComplex * /*d_Debug_Purpose*/) {
    return track(my_queue, sub_RANSAC_iters, HC_max_steps, HC_max_correction_steps, HC_delta_t_incremental_steps,
                 d_startSols_array, d_Track_array, d_startParams, d_targetParams, d_diffParams, nullptr, d_dHdx_indx,
                 d_dHdt_indx, d_is_GPU_HC_Sol_Converge, d_is_GPU_HC_Sol_Infinity,
                 "kernel_GPUHC_trifocal_2op1p_30x30_PH", false, true);
}
