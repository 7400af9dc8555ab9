/*
 * magma_v2.h -- TEST STAND-IN, types only (this repository's own; not MAGMA).
 *
 * Declares just what integration/hc_trifocal_shim.cpp and the reference's
 * launcher header (magmaHC/gpu-kernels/magmaHC-kernels.hpp:24-105) use, with
 * MAGMA 2.5.4's layouts, so the shim compiles and links in this repository
 * (tests/test_shim.py).  In a real integration the include path points at
 * MAGMA-HIP's own magma_v2.h instead and this directory is not used.
 */
#ifndef HC_MAGMA_V2_STANDIN_H
#define HC_MAGMA_V2_STANDIN_H

#include <hip/hip_runtime.h>

typedef double real_Double_t;                               /* magma_types.h */
typedef struct { float x, y; } magmaFloatComplex;           /* == hipFloatComplex / cuFloatComplex layout */
typedef struct magma_queue *magma_queue_t;                  /* opaque queue handle */

/* MAGMA-HIP accessor of a queue's stream (magma_v2.h); the test harness defines it. */
hipStream_t magma_queue_get_hip_stream(magma_queue_t queue);

#endif
