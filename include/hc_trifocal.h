/*
 * hc_trifocal.h -- the drop-in C-ABI boundary of the MI355X-native GPU-HC path
 * tracker for the trifocal_2op1p_30x30 minimal problem.
 *
 * Replaces the four host launchers of the reference
 *   magmaHC/gpu-kernels/magmaHC-kernels.hpp:24-105
 *     kernel_GPUHC_trifocal_2op1p_30x30_PH_CodeOpt_TrunPaths[_Volta]            (:24-61)
 *     kernel_GPUHC_trifocal_2op1p_30x30_PH_CodeOpt_TrunPaths_TrunRANSAC[_Volta] (:63-105)
 * implemented at
 *   magmaHC/gpu-kernels/kernel_GPUHC_trifocal_2op1p_30x30_PH_CodeOpt_TrunPaths.cu:292-386
 *   magmaHC/gpu-kernels/kernel_GPUHC_trifocal_2op1p_30x30_PH_CodeOpt_TrunPaths_TrunRANSAC.cu:329-455
 * and called from GPU_HC_Solver::Solve_by_GPU_HC (magmaHC/GPU_HC_Solver.cpp:390-436).
 *
 * Rules of the boundary:
 *   - plain pointers and sizes, no MAGMA / torch types; hcComplex is
 *     layout-compatible with magmaFloatComplex / cuFloatComplex / float2;
 *   - every buffer is allocated and freed by the caller; the entry points never
 *     allocate, copy to/from the host or synchronise (hipGraph-capturable);
 *   - work is enqueued on the caller's stream on the CURRENT device, which is
 *     never changed; re-entrant across devices/streams;
 *   - errors are returned as hcStatus, never exit();
 *   - result index space is the reference's: batch id b = sample*312 + track.
 */
#ifndef HC_TRIFOCAL_H
#define HC_TRIFOCAL_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HC_NUM_VARS      30   /* Num_Of_Vars   (gpuhc_settings.yaml:17)  */
#define HC_NUM_PARAMS    33   /* Num_Of_Params (gpuhc_settings.yaml:18)  */
#define HC_NUM_TRACKS    312  /* Num_Of_Tracks (gpuhc_settings.yaml:19)  */
#define HC_UNIFIED_INDEX_SIZE 38880 /* 36000 dH/dx + 2880 dH/dt ints (Data_Reader.cpp:167-189) */

typedef struct { float re, im; } hcComplex;         /* == magmaFloatComplex */
typedef void *hcStream;                             /* == hipStream_t       */

typedef enum {
    HC_SUCCESS = 0,
    HC_ERROR_INVALID_VALUE = 1,   /* bad size / null required pointer            */
    HC_ERROR_WORKSPACE = 2,       /* workspace missing or too small               */
    HC_ERROR_LAUNCH = 3,          /* hipLaunchKernel / hipMemsetAsync failed      */
    HC_ERROR_DEVICE = 4,          /* no device / unsupported device (not gfx950)  */
    HC_ERROR_TABLE = 5            /* index table invalid or beyond the kernels' compaction */
} hcStatus;

/* Optional per-path counters (one per batch id).  steps = RK4 predictor
   executions, corrections = corrector iterations; inliers = abort-mode
   reprojection inlier counts of the hypothesis scoring (0 otherwise). */
typedef struct {
    int32_t steps;
    int32_t corrections;
    int32_t inliers21;
    int32_t inliers31;
} hcPathStats;

/* Tracker tuning knobs (GPUHC_* keys of gpuhc_settings.yaml:12-14). */
typedef struct {
    int max_steps;          /* GPUHC_Max_Steps                        (80) */
    int max_corrections;    /* GPUHC_Max_Correction_Steps             (3)  */
    int delta_t_inc_steps;  /* GPUHC_Num_Of_Steps_to_Increase_Delta_t (4)  */
} hcTrackSettings;

/* Arguments of one tracking launch over sub_ransac_iters samples (one GPU's share).
 * Layouts (reference GPU_HC_Solver.cpp:137-184,335-362):
 *   start_sols    312 x 31 complex, ld 31 (x[30] = 1)
 *   tracks        (312*N) x 31 complex, ld 31, in/out; initialised by the caller
 *                 to the start solutions (Feed_Start_Sols_for_Intermediate_Homotopy);
 *                 entries 0..29 of each track are written, entry 30 is not
 *   start_params  34 complex (p[33] = 1)
 *   target/diff   34 complex per sample, contiguous
 *   unified_index 38880 int32: dHdx_indx.txt || dHdt_indx.txt (the reference's
 *                 d_unified_dHdx_dHdt_Index)
 *   converge/infinity  one byte per batch id (bool layout)
 * Alternatively start_sols_array / track_array may point to device arrays of
 * 312 / 312*N per-track pointers (the reference's magma_cset_pointer arrays);
 * when non-NULL they take precedence over the base pointers. */
typedef struct {
    int sub_ransac_iters;                 /* N samples on this device            */
    hcTrackSettings settings;
    const hcComplex *start_sols;          /* d_startSols base                    */
    const hcComplex *const *start_sols_array; /* optional d_startSols_array      */
    hcComplex *tracks;                    /* d_Track base                        */
    hcComplex *const *track_array;        /* optional d_Track_array              */
    const hcComplex *start_params;        /* d_startParams                       */
    const hcComplex *target_params;       /* d_targetParams                      */
    const hcComplex *diff_params;         /* d_diffParams                        */
    const int32_t *unified_index;         /* d_unified_dHdx_dHdt_Index           */
    uint8_t *converge;                    /* d_is_GPU_HC_Sol_Converge            */
    uint8_t *infinity;                    /* d_is_GPU_HC_Sol_Infinity            */
    hcPathStats *stats;                   /* optional, 312*N entries             */
} hcTrackArgs;

/* Extra arguments of the early-abort ("TrunRANSAC") launch. */
typedef struct {
    int num_triplet_edgels;               /* Num_Of_Triplet_Edgels               */
    const float *triplet_edge_locations;  /* E x 6 floats (x1 y1 x2 y2 x3 y3)     */
    const float *intrinsic_matrix;        /* 9 floats, row-major K               */
    uint8_t *found_trifocal_sols;         /* 1 byte flag (caller zeroes it)      */
    int32_t *trifocal_sols_batch_index;   /* 312*N ints (caller sets -1)         */
    /* 0 (default, the reference's semantics, ..._TrunRANSAC.cu:148-152): the
       flag only gates a path's start; paths already in flight when a good
       hypothesis is found run to completion and write their results.
       1: paths in flight also stop at their next step boundary and report
       like a skipped path (track untouched, converge = 0) -- a faster kernel
       exit, same time to the first good pose. */
    int inflight_stop;
    /* Optional (NULL: none): a 4-byte flag shared by every process of a
       multi-GPU run (hc_shared_flag_create on one rank, hc_shared_flag_open on
       the others).  The launch sets it (system scope) when it finds a good
       hypothesis and checks it, besides found_trifocal_sols, before it starts
       each path -- and with inflight_stop at every step boundary -- so every GPU
       stops within a path of any GPU's find instead of at its next launch.
       The reference keeps one flag per GPU (GPU_HC_Solver.cpp:308-333). */
    uint32_t *peer_found;
} hcAbortArgs;

/* Workspace: holds the compacted index tables, the path work queue and the
   device timestamps.  Size does not depend on N.  Caller allocates (device
   memory, 256-B aligned). */
size_t hc_trifocal_workspace_size(void);

/* Workspace size that also enables time slicing for launches of up to
   sub_ransac_iters samples at GPUHC_Max_Steps = 80: 33 KB + (256 + 8 x 28)
   bytes per path more (a suspended path's 256-byte state block and the resume
   ring, one entry per suspension plus 4096 spare entries).  With it, a path that has run a
   slice of steps while other paths wait is suspended at a step boundary and
   resumed after the new paths (same results bit for bit; every path starts
   early, so a launch no longer ends with long paths that were dequeued late).
   Tracking launches only (not abort mode), and only while the step counters
   fit the state block (GPUHC_Max_Steps < 16000, GPUHC_Max_Correction_Steps x
   (GPUHC_Max_Steps + 2) < 65536, GPUHC_Num_Of_Steps_to_Increase_Delta_t <
   16384).  A smaller workspace of at least hc_trifocal_workspace_size() runs
   without slicing.  No initialisation is needed: the first launch on a
   workspace builds its tables and clears its ring; later launches with the
   same index table reuse the tables (an index-table hash is checked). */
size_t hc_trifocal_workspace_size_for(int sub_ransac_iters);

/* The same for a given GPUHC_Max_Steps (hc_trifocal_workspace_size_for assumes
   the reference default, 80): the suspended-path ring holds one entry per
   suspension, at most (max_steps + 1) / 3 per path.  A workspace sized for a
   smaller max_steps than a launch uses runs that launch without slicing. */
size_t hc_trifocal_workspace_size_for_steps(int sub_ransac_iters, int max_steps);

/* GPU-HC tracking of 312*N paths (replaces ..._TrunPaths and ..._TrunPaths_Volta). */
hcStatus hc_trifocal_2op1p_30x30_track(const hcTrackArgs *args, void *workspace,
                                       size_t workspace_bytes, hcStream stream);

/* GPU-HC tracking with on-device RANSAC hypothesis scoring and early abort
   (replaces ..._TrunPaths_TrunRANSAC and ..._TrunRANSAC_Volta). */
hcStatus hc_trifocal_2op1p_30x30_track_abort(const hcTrackArgs *args, const hcAbortArgs *abort_args,
                                             void *workspace, size_t workspace_bytes,
                                             hcStream stream);

/* The cross-process early-stop flag of hcAbortArgs::peer_found.  It lives in
   the creating process's device memory, allocated uncached
   (hipExtMallocWithFlags(hipDeviceMallocUncached): coherent across devices
   while kernels run; fine-grained, then plain hipMalloc, if the device cannot
   export those with hipIpcGetMemHandle); the 64-byte handle travels to the
   other processes (e.g. a torch.distributed broadcast), which map it with
   hc_shared_flag_open (hipIpcOpenMemHandle, peer access over xGMI).  create
   zeroes it; reset zeroes it on a stream before a new run (the caller orders
   the reset before any rank's launch); close(flag, opened = 1 for a handle
   opened here, 0 for the creator's).  hc_shared_flag_memory_kind(flag) of a
   flag created in this process: 2 uncached, 1 fine-grained, 0 plain
   (coarse-grained: another device's find may then be seen only at the next
   synchronisation), -1 not created here. */
typedef struct { unsigned char reserved[64]; } hcIpcHandle;   /* == hipIpcMemHandle_t */
hcStatus hc_shared_flag_create(uint32_t **flag, hcIpcHandle *handle);
int hc_shared_flag_memory_kind(const uint32_t *flag);
hcStatus hc_shared_flag_open(const hcIpcHandle *handle, uint32_t **flag);
hcStatus hc_shared_flag_reset(uint32_t *flag, hcStream stream);
hcStatus hc_shared_flag_close(uint32_t *flag, int opened);

/* GPU-HC tracking WITHOUT the depth-sign path truncation: every path runs
   until it converges, diverges or reaches the step limit.  Replaces the
   archived ablation launchers kernel_GPUHC_trifocal_2op1p_30x30_PH_CodeOpt and
   ..._PH_CodeOpt_Volta (arxived_GPU_code/gpu-kernels/magmaHC-kernels.hpp:61-96),
   whose kernel is ..._TrunPaths without ..._TrunPaths.cu:148-155 (the archived
   kernel files differ in exactly those lines).  Same arguments and outputs as
   hc_trifocal_2op1p_30x30_track. */
hcStatus hc_trifocal_2op1p_30x30_track_ph_codeopt(const hcTrackArgs *args, void *workspace,
                                                  size_t workspace_bytes, hcStream stream);

/* The archived ..._PH kernel (direct parameter homotopy, no code
   optimisation): PH_CodeOpt with the explicit Runge-Kutta helpers of
   magmaHC/dev-get-new-data.cuh:37-71 instead of the loopy RK, i.e. the stage
   sums s += ((k*dt)*gc*1.0)/6 and /3 (a division, where the loopy RK multiplies
   by the rounded 1/6 and 1/3) and x += k*((h/2 or h)*gc), gc = MAGMA_C_ONE.
   Replaces kernel_GPUHC_trifocal_2op1p_30x30_PH
   (arxived_GPU_code/gpu-kernels/magmaHC-kernels.hpp:42-59), which takes
   separate dH/dx and dH/dt tables; here the unified table as everywhere. */
hcStatus hc_trifocal_2op1p_30x30_track_ph(const hcTrackArgs *args, void *workspace,
                                          size_t workspace_bytes, hcStream stream);

/* Device-side outcome of the last launch on this workspace:
     HC_SUCCESS;
     HC_ERROR_TABLE  -- the index table does not fit the kernels' compaction
                        (the tracker then left every output untouched): an
                        index or coefficient out of range, dH/dx entries that
                        do not bin-pack into the 32 lanes' entry slots of
                        8, 5, 3, 3, 1, 1 terms (or a row of more than 6
                        entries), or a dH/dt | H row of more than 13 terms
                        whose partner row (lane ^ 16) has more than 10
                        (Evaluations).  Any dH/dx structure
                        that compacts is tracked: trifocal_2op1p_30x30's own
                        (or one within it) by the LU specialised to it,
                        any other (e.g. the same system with its equations
                        permuted) by the structure-agnostic LU -- both
                        kernels are enqueued and the table decides on the
                        device which one runs;
     HC_ERROR_DEVICE -- time slicing only: a suspended path could not be handed
                        over (the ring overflowed: more than 4096 re-pushes of
                        abandoned tickets in one launch; or a ring entry
                        outside the launch's paths); that path's converge /
                        infinity / stats / track entry are not final.  The
                        control block's ring_fail words hold the ticket, the
                        entry seen, tail and head for diagnosis.  (A consumer
                        that waits too long for a ring entry abandons the
                        ticket and its pusher pushes the path again: a paused
                        wave delays a path, it never loses it.)
   Blocking read -- call after synchronising. */
hcStatus hc_trifocal_workspace_status(const void *workspace);

/* Device timestamps of the last launch on this workspace, in seconds since the
   launch started: [0] = first good hypothesis found (abort mode, <0 if none).
   The device clock rate is queried (hipDeviceAttributeWallClockRate).
   Reads the workspace with a blocking copy -- call after synchronising. */
hcStatus hc_trifocal_read_timings(const void *workspace, double *first_found_seconds);

/* Raw device clock of the last launch on this workspace (s_memrealtime, a
   constant-rate counter shared by every launch on the device; *tick_hz = its
   rate): start = first workgroup of the tracker began, found = first good
   hypothesis (0 if none).  Lets a caller that splits its samples into several
   launches (one workspace each) measure time-to-first-good-pose across them. */
hcStatus hc_trifocal_read_timestamps(const void *workspace, uint64_t *start_ticks, uint64_t *found_ticks,
                                     double *tick_hz);

/* ---- component entry points (batched building blocks, also used by tests) ---- */

/* Batched 30x30 complex solve with the tracker's LU (partial pivoting on
   |re|+|im|, dev-cgesv-batched-small.cuh:38-107 semantics): A row-major n x 30 x 30,
   b n x 30, x n x 30. */
hcStatus hc_cgesv_30x30_batched(int n, const hcComplex *A, const hcComplex *b, hcComplex *x,
                                hcStream stream);

/* Batched evaluation of dH/dx (row-major 30x30), dH/dt and H at (x, p) with
   the compacted tables built from unified_index (gpu-idx-evals/dev-eval-indxing-
   trifocal_2op1p_30x30_LimUnroll_L2Cache.cuh:40-148).
   x: n x 31, p: n x 34, d: n x 34.  Uses the workspace for the tables. */
hcStatus hc_trifocal_eval_batched(int n, const int32_t *unified_index, const hcComplex *x,
                                  const hcComplex *p, const hcComplex *d, hcComplex *Hx,
                                  hcComplex *Ht, hcComplex *H, void *workspace,
                                  size_t workspace_bytes, hcStream stream);

/* hipGetErrorString of the last HIP error seen by an entry point of this thread
   (meaningful after an HC_ERROR_LAUNCH / HC_ERROR_DEVICE return). */
const char *hc_last_error_string(void);

/* Library / kernel identification (for logs and the bench JSON). */
const char *hc_trifocal_version(void);

/* Layout version of the structs of this header.  A caller compares
   hc_trifocal_abi_version() with the HC_TRIFOCAL_ABI_VERSION it was built
   against before its first launch (the Python binding and the reference-named
   shim do): a library of another version reads the argument structs
   differently (version 2 appended hcAbortArgs::peer_found). */
#define HC_TRIFOCAL_ABI_VERSION 2
int hc_trifocal_abi_version(void);

/* Test hook, declared here until ABI version 1's callers have moved to
   include/hc_trifocal_testing.h (where it is documented); still exported. */
void hc_trifocal_set_ring_test(int delay_ticks)
    __attribute__((deprecated("a test hook: include hc_trifocal_testing.h")));

#ifdef __cplusplus
}
#endif
#endif /* HC_TRIFOCAL_H */
