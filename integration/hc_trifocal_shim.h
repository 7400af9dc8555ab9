// hc_trifocal_shim.h -- the two calls a reference-side GPU_HC_Solver adds when
// it links the drop-in shim (hc_trifocal_shim.cpp) instead of the CUDA
// launchers.  They have no counterpart in the reference (its launchers need no
// workspace); INTEGRATION.md §1 shows where GPU_HC_Solver calls them.
#pragma once

#include "hc_trifocal.h"
#include "magma_v2.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Allocates, synchronously, everything the launchers need on this queue's
   stream for launches of up to max_samples samples at GPUHC_Max_Steps =
   max_steps: the workspace at its time-slicing size
   (hc_trifocal_workspace_size_for_steps) and the unified-index buffer of the
   Volta variants.  Called from GPU_HC_Solver::Allocate_Arrays
   (GPU_HC_Solver.cpp:137-184) so the launchers never allocate or synchronise.
   A later launch that needs more falls back to growing the workspace on the
   hot path (it synchronises the stream) and prints one warning. */
hcStatus hc_trifocal_shim_reserve(magma_queue_t queue, int max_samples, int max_steps);

/* Synchronises the queue's stream and returns the device-side status of the
   last launch on it (hc_trifocal_workspace_status: HC_ERROR_DEVICE means a
   time-sliced path could not be handed over and its outputs are not final).
   GPU_HC_Solver calls it after its own synchronisation point
   (GPU_HC_Solver.cpp:444-446). */
hcStatus hc_trifocal_shim_status(magma_queue_t queue);

/* Bookkeeping of the queue's stream: workspace bytes held and how many
   launches had to grow it on the hot path (0 after a sufficient reserve). */
hcStatus hc_trifocal_shim_info(magma_queue_t queue, size_t *workspace_bytes, int *hot_path_grows);

#ifdef __cplusplus
}
#endif
