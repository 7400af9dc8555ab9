// hc_slot.hpp -- the path slot of the two-paths-per-wave tracker.
//
// The 64 lanes of a wave are two independent "path slots" (half-waves): lane
// l belongs to slot h = l >> 5 and owns equation row r = l & 31 (r < 30) of
// that slot's path.  Both slots execute the same instruction stream -- one
// predictor / corrector stage per iteration: p(t) + dH/dx + dH/dt|H + LU --
// while each slot runs its own stage machine (its own t, step size, stage,
// path id), the reference's per-block state machine
// (kernel_GPUHC_trifocal_2op1p_30x30_PH_CodeOpt_TrunPaths.cu:138-280) with
// the branches turned into per-half predicates.
#pragma once

#include "hc_device.hpp"

namespace hc {

// uniform state of a path slot, parked in LDS while a stage runs
struct SlotState {
    float t0, t_step, dt, h2, scale;
    int s, stepidx, coef, succ, nsteps, ncorr, b, smp, ph, flags;
    int pad;
    // the (t, sample) the slot's prefix tables were built for (hc_eval.hpp
    // build_prefixes): they are rebuilt only when p(t) changes
    float pre_t;
    int pre_smp;
};
// Capacities of the per-slot prefix tables (hc_eval.hpp): the distinct
// (coef, a, b) triples of the dH/dx and H terms (93 in this problem,
// padding term included) and the distinct (a, b) pairs of the dH/dt terms (38).
constexpr int TP_CAP = 96, QP_CAP = 40;
// dH/dx entries in the slot (hc_kernels.hip k_prep_tables packs them; the
// problem has 170): ENT_CAP - 1 is the structural zero, written once per launch.
constexpr int ENT_CAP = 172;
// per path-slot LDS block
struct alignas(16) SlotLDS {
    cf x[32];        // current track (x[30] = 1)
    cf xl[32];       // last successful track
    cf sols[32];     // RK accumulator
    cf ent[ENT_CAP]; // dH/dx entries, packed (k_prep_tables); p(t) and the diff params are staged
                     // in its first 68 entries while the prefixes are built.  The sparse LU
                     // overwrites ent[0 .. LU_SCRATCH_CF) with its store windows (hc_lu.hpp): after
                     // a solve only the structural zero at ENT_CAP - 1 is intact
    cf lu[32];       // the LU's pivot-row buffer (hc_lu.hpp LUBuf)
    cf tp[TP_CAP];   // prefix table T: (c * p[a]) * p[b] per (c, a, b) triple (dH/dx and H terms)
    cf qp[QP_CAP];   // prefix table Q: d[a] * p[b] + d[b] * p[a] per (a, b) pair (dH/dt terms)
    SlotState st;
    char bank_pad[40];   // slot stride = 16 mod 256 B: the slots of one wave (same offsets,
                         // different bases) land on different LDS banks
};
static_assert(sizeof(SlotLDS) % 256 == 16, "SlotLDS stride must shift the LDS banks by 4 per slot");
static_assert(sizeof(SlotLDS) <= 3600, "5 workgroups per CU: 8 slots + the workgroup's tables in 32 KB");

}  // namespace hc
