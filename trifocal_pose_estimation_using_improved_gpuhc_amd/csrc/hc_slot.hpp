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
};
// per path-slot LDS block
struct alignas(16) SlotLDS {
    cf x[32];        // current track (x[30] = 1)
    cf xl[32];       // last successful track
    cf sols[32];     // RK accumulator
    cf p[NPP];       // p(t)
    cf tgt[NPP];     // target params
    cf dif[NPP];     // diff params
    cf ent[NV * 7];  // dH/dx entries of row r at [r*7 + slot], slot 6 = 0 (kept through the LU)
    cf lu[32];       // the LU's pivot-row buffer (hc_lu.hpp LUBuf)
    SlotState st;
    char bank_pad[16];   // slot stride = 16 mod 256 B: the slots of one wave (same offsets,
                         // different bases) land on different LDS banks
};
static_assert(sizeof(SlotLDS) % 256 == 16, "SlotLDS stride must shift the LDS banks by 4 per slot");

}  // namespace hc
