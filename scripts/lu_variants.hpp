// LU lab variants (development tool): candidates for the tracker LU, each
// bit-identical to lu_solve3s by construction; selected by lab_variant<V>.
#pragma once
#include "../trifocal_pose_estimation_using_improved_gpuhc_amd/csrc/hc_lu9.hpp"
namespace hc {
template <int V>
__device__ __forceinline__ cf lab_variant(cf (&rA)[NV], cf rB, int lane, uint32_t pat, LUBuf &L) {
    if constexpr (V == 1) return lu_solve3(rA, rB, lane, L);
    else return lu_solve9<V - 1000>(rA, rB, lane, pat, L);
}
}  // namespace hc
#define LU_LAB_RUNS run<4096>(d, reps, &ref, o); run<12288>(d, reps, &ref, o); run<4096>(d, reps, &ref, o); run<12288>(d, reps, &ref, o);
