// shim_harness.cpp -- TEST HARNESS (tests/test_shim.py only): a concrete
// magma_queue for the types-only stand-in (standin/magma_v2.h) and extern "C"
// trampolines so ctypes can drive the four C++-linkage launchers of
// hc_trifocal_shim.cpp with the reference's argument lists.  A real
// integration links MAGMA-HIP instead of this file.
#include "magmaHC-kernels.hpp"

struct magma_queue {
    hipStream_t stream;
};
hipStream_t magma_queue_get_hip_stream(magma_queue_t queue) { return queue->stream; }

typedef magmaFloatComplex mfc;

extern "C" {
void *shim_queue_create(void *stream) { return new magma_queue{static_cast<hipStream_t>(stream)}; }
void shim_queue_destroy(void *q) { delete static_cast<magma_queue *>(q); }

double shim_trunpaths(void *q, int n, int ms, int mc, int inc, mfc **ssa, mfc **tra, mfc *sp, mfc *tp, mfc *dp,
                      int *unified, bool *conv, bool *inf) {
    return kernel_GPUHC_trifocal_2op1p_30x30_PH_CodeOpt_TrunPaths(static_cast<magma_queue_t>(q), n, ms, mc, inc, ssa,
                                                                  tra, sp, tp, dp, unified, conv, inf, nullptr);
}
double shim_trunpaths_volta(void *q, int n, int ms, int mc, int inc, mfc **ssa, mfc **tra, mfc *sp, mfc *tp, mfc *dp,
                            int *hx, int *ht, bool *conv, bool *inf) {
    return kernel_GPUHC_trifocal_2op1p_30x30_PH_CodeOpt_TrunPaths_Volta(static_cast<magma_queue_t>(q), n, ms, mc, inc,
                                                                        ssa, tra, sp, tp, dp, hx, ht, conv, inf,
                                                                        nullptr);
}
double shim_ph_codeopt(void *q, int n, int ms, int mc, int inc, mfc **ssa, mfc **tra, mfc *sp, mfc *tp, mfc *dp,
                       int *unified, bool *conv, bool *inf) {
    return kernel_GPUHC_trifocal_2op1p_30x30_PH_CodeOpt(static_cast<magma_queue_t>(q), n, ms, mc, inc, ssa, tra, sp,
                                                        tp, dp, unified, conv, inf, nullptr);
}
double shim_ph_codeopt_volta(void *q, int n, int ms, int mc, int inc, mfc **ssa, mfc **tra, mfc *sp, mfc *tp,
                             mfc *dp, int *hx, int *ht, bool *conv, bool *inf) {
    return kernel_GPUHC_trifocal_2op1p_30x30_PH_CodeOpt_Volta(static_cast<magma_queue_t>(q), n, ms, mc, inc, ssa, tra,
                                                              sp, tp, dp, hx, ht, conv, inf, nullptr);
}
double shim_ph(void *q, int n, int ms, int mc, int inc, mfc **ssa, mfc **tra, mfc *sp, mfc *tp, mfc *dp, int *hx,
               int *ht, bool *conv, bool *inf) {
    return kernel_GPUHC_trifocal_2op1p_30x30_PH(static_cast<magma_queue_t>(q), n, ms, mc, inc, ssa, tra, sp, tp, dp, hx,
                                                ht, conv, inf, nullptr);
}
double shim_trunransac(void *q, int n, int e, int ms, int mc, int inc, mfc **ssa, mfc **tra, mfc *sp, mfc *tp,
                       mfc *dp, int *unified, float *edgels, float *K, bool *conv, bool *inf, bool *found,
                       int *batch_index) {
    return kernel_GPUHC_trifocal_2op1p_30x30_PH_CodeOpt_TrunPaths_TrunRANSAC(
        static_cast<magma_queue_t>(q), n, e, ms, mc, inc, ssa, tra, sp, tp, dp, unified, edgels, K, conv, inf, nullptr,
        found, batch_index);
}
double shim_trunransac_volta(void *q, int n, int e, int ms, int mc, int inc, mfc **ssa, mfc **tra, mfc *sp, mfc *tp,
                             mfc *dp, int *hx, int *ht, float *edgels, float *K, bool *conv, bool *inf, bool *found,
                             int *batch_index) {
    return kernel_GPUHC_trifocal_2op1p_30x30_PH_CodeOpt_TrunPaths_TrunRANSAC_Volta(
        static_cast<magma_queue_t>(q), n, e, ms, mc, inc, ssa, tra, sp, tp, dp, hx, ht, edgels, K, conv, inf, nullptr,
        found, batch_index);
}
}
