// hc_kernels.hip -- MI355X (gfx950) GPU-HC tracker kernels + the C-ABI of
// include/hc_trifocal.h.
//
// Replaces magmaHC/gpu-kernels/kernel_GPUHC_trifocal_2op1p_30x30_PH_CodeOpt_TrunPaths[_TrunRANSAC][_Volta].cu
// (the four CUDA/MAGMA kernels + launchers, magmaHC-kernels.hpp:24-105).
//
// Design: a persistent grid of 256-thread workgroups.  Each
// wavefront tracks two homotopy paths at a time, one per 32-lane half (lane
// r < 30 of a half owns Jacobian row r, RHS r and x_r in VGPRs).  A half
// whose path ends dequeues the next path id b = sample*312 + track from a
// device work queue (one agent-scope atomicAdd per path), so no slot idles
// while work remains.  One loop iteration runs one predictor or corrector
// "stage" for both halves: p(t) (LDS) + dH/dt|H + dH/dx from the compacted
// index tables + the register LU.  Early abort (TrunRANSAC) scores converged
// paths on the device and raises an agent-scope flag.
#include "hc_device.hpp"
#include "hc_lu.hpp"
#include "../../include/hc_trifocal.h"
#include "../../include/hc_trifocal_testing.h"

#include <atomic>
#include <climits>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <utility>

namespace hc {

thread_local hipError_t g_last_hip_error = hipSuccess;   // shared with hc_pose.hip (hc_last_error_string)
static inline hcStatus launch_status(hcStatus on_fail) {
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) { g_last_hip_error = e; return on_fail; }
    return HC_SUCCESS;
}

// Longest-processing-time-first dequeue order (scripts/make_track_order.py):
// queue position q -> track c_track_order[q / N], sample q % N.  Results are
// per batch id, so the order only changes when a path runs, not what it computes.
__constant__ int c_track_order[NTRK] = {
#include "hc_track_order.inc"
};
__device__ __forceinline__ int path_of_queue_pos(int q, int num_paths, int ordered) {
    if (!ordered) return q;
    const int n = num_paths / NTRK;          // samples in this launch
    const int rank = q / n;
    return (q - rank * n) * NTRK + c_track_order[rank];
}

constexpr int PRIO_TENTHS = 10;   // issue-priority levels over the queue (k_track)
constexpr int WG_THREADS = 256;
constexpr int WAVES_PER_WG = WG_THREADS / WAVE;

// The caller-owned workspace (hc_trifocal_workspace_size()).
struct Workspace {
    // control block, zeroed by k_prep_tables every launch (first 64 bytes)
    unsigned queue;          // path work queue
    unsigned status;         // HC_ERROR_TABLE if the index table does not fit the compaction
    unsigned found;          // device-side "good hypothesis found" flag
    unsigned pad0;
    unsigned long long t_start;   // s_memrealtime when the first workgroup started (abort mode)
    unsigned long long t_found;   // s_memrealtime of the first good hypothesis
    unsigned ring_fail[4];   // time slicing: ticket, tag seen, tail, head of a ring entry that never came (diagnostics)
    unsigned abandoned;      // time slicing: ring tickets abandoned by their consumers (re-pushed; diagnostics)
    unsigned pad1[3];
    // written by k_prep_tables
    EvalTables tab;
};
static_assert(offsetof(Workspace, tab) == 64, "control block is 64 bytes");

// Time slicing.  A path that has run slice_q steps while other
// work waits is suspended at its step boundary: x and its step-control scalars
// go to the path's 256-B suspend block (two full cache lines, one store per
// half), the path id to a FIFO ring.  While new paths remain, the suspending
// half takes one (an unpaired push); after that it swaps with the oldest
// suspended path (a paired push + pop, i.e. round robin).  A half whose path
// ends takes a new path, else the oldest suspended one.  Every path thus starts
// early and the end of a launch is made of short remainders instead of whole
// late-dequeued long paths.  Bit-exact: at a step boundary x == x_last == the
// RK accumulator, and this is the whole vector state.
//
// Ring protocol (no CAS loops): tickets from atomicAdd on head / tail; avail
// counts published entries not yet claimed by unpaired pops (a semaphore:
// decrement, undo if it was empty and retry while the undo leaves it
// positive, so concurrent failures cannot hide an entry).  A paired pop needs
// no claim: its own push precedes it.  A claimed entry may still be in the
// pusher's hands (ticket taken, entry not yet written), hence the short wait
// on its tag.  An entry's tag hashes the launch epoch with its ticket, so the
// ring needs no clearing between launches (only once, when a workspace is
// first used or its ring grows: k_prep_tables).
//
// Suspend block of path b (32 x 8 B): words 0..29 = x, word 30 = (t0, dt),
// word 31 = (stepidx | nsteps << 16, ncorr | succ << 16 | flags << 30); the
// launcher enables slicing only where these fields fit (slice_fits).
constexpr int SUSP_WORDS = 32;
// Steps per time slice: SLICE_Q while at most one suspended path per path slot
// waits (the launch's end, where the rotation's granularity sets the tail;
// profiles/r2n_ab_slice*.jsonl, r3d_ab_lu_slicing.jsonl), SLICE_QBIG while
// more wait (round 3: as fair a rotation with fewer hand-overs, 239 vs 339 MB
// of HBM traffic per config-2 launch at the same launch time;
// profiles/r3g_ab_quantum.jsonl, r3h_ab_quantum.jsonl).
constexpr int SLICE_Q = 3;
constexpr int SLICE_QBIG = 8;
__host__ __device__ constexpr bool slice_fits(int max_steps, int max_corr, int inc_steps) {
    return max_steps >= 0 && max_steps < 16000 && inc_steps >= 0 && inc_steps < 16384 && max_corr >= 0 &&
           (long long)max_corr * (max_steps + 2) < 65536;
}
// Ring: one entry per ticket, never reused within a launch.  A path is
// suspended only after running SLICE_Q steps since it (re)started and runs at
// most max_steps + 1 steps, so a launch pushes at most
// paths * ((max_steps + 1) / SLICE_Q) entries.  (A reused slot is not safe: a
// wave can be paused for hundreds of ms between taking a ticket and reading
// its entry while the rest of its kernel runs on -- seen when another stream's
// first launch created its hardware queue -- and a slot reused meanwhile would
// lose the suspended path; profiles/r2zb_stress*.jsonl.)
// RING_SLACK more entries absorb the re-pushes of abandoned tickets (below).
constexpr unsigned long long RING_SLACK = 4096ull;
__host__ __device__ constexpr unsigned long long ring_entries(long long paths, int max_steps) {
    return (unsigned long long)paths * (unsigned long long)((max_steps + 1) / (SLICE_Q > 0 ? SLICE_Q : 1) + 1) +
           RING_SLACK;
}
// How long a consumer waits for a claimed entry whose pusher holds the ticket
// but has not written it yet before it abandons the ticket (s_memrealtime
// ticks, 100 MHz: 1 ms).  Abandoning loses nothing: the pusher sees the mark
// when it writes and pushes the path again on a new ticket (ring_push).
constexpr unsigned long long RING_ABANDON_TICKS = 100000ull;
// Every sliced launch's ring entry is written once by one atomic exchange,
// either by its pusher (the tagged path id) or by a consumer that gave up
// waiting (the abandon mark: the tag with bit 0 cleared, never a published tag)
__device__ __forceinline__ unsigned long long ring_abandon_mark(unsigned tag) {
    return ((unsigned long long)(tag & ~1u) << 32) | 0xFFFFFFFFull;
}
// (tests, KArgs::ring_test: consumers abandon after an eighth of the pushers' delay)
__device__ __forceinline__ unsigned long long ring_wait_ticks(int ring_test) {
    return ring_test > 0 ? (unsigned long long)(ring_test / 8) : RING_ABANDON_TICKS;
}

struct KArgs {
    int num_paths;
    int ordered;        // dequeue track-major in c_track_order (abort mode off)
    int truncate;       // depth-sign path truncation (..._TrunPaths.cu:148-155); 0 = PH_CodeOpt
    int explicit_rk;    // archived ..._PH: explicit RK helpers (dev-get-new-data.cuh:37-71)
    int max_steps, max_corr, inc_steps;
    const cf *start_sols;
    const cf *const *start_sols_array;
    cf *tracks;
    cf *const *track_array;
    const cf *start_params;
    const cf *target_params;
    const cf *diff_params;
    uint8_t *conv;
    uint8_t *inf;
    hcPathStats *stats;
    Workspace *ws;
    // abort mode
    int num_edgels;
    int inflight_stop;  // paths in flight stop at their next step boundary once a pose is found
    const float *edgels;
    const float *K;
    uint8_t *found_flag;
    unsigned *peer_found;           // cross-process flag of a multi-GPU run (hcAbortArgs::peer_found), or null
    int32_t *batch_index;
    // time slicing (slice_q > 0; tracking without abort only)
    int slice_q;
    int ring_test;                  // tests only (hc_trifocal_set_ring_test): pusher delay in ticks, else 0
    unsigned ring_cap;
    unsigned *rq;                   // ring counters, one 256-B line each: [0] head, [64] tail, [128] avail, [192] meta
    unsigned long long *susp;       // suspend blocks, SUSP_WORDS per path id
    unsigned long long *ring;       // ring_tag(epoch, ticket) << 32 | path id
};
// rq layout: counters zeroed by k_prep_tables every launch; meta: the launch
// epoch, a magic word and the ring entries already cleared (persist)
constexpr int RQ_HEAD = 0, RQ_TAIL = 64, RQ_AVAIL = 128, RQ_EPOCH = 192, RQ_MAGIC = 193, RQ_CLEARED = 194,
              RQ_DLO = 195, RQ_DHI = 196,
              RQ_WORDS = 256;
constexpr unsigned RQ_MAGIC_VALUE = 0x48435432u;   // "HCT2" (the ring-first layout of round 4)
// tag of ticket t's entry in launch `epoch` (never 0, so a cleared entry never
// matches; distinct epochs give distinct tags for the same ticket)
__device__ __forceinline__ unsigned ring_tag(unsigned epoch, unsigned t) {
    return ((epoch * 0x9E3779B1u) ^ (t * 0x85EBCA6Bu)) | 1u;
}

__device__ __forceinline__ unsigned ld_rlx(const unsigned *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// The hand-over data of a suspended path (suspend block, ring entries) is
// written and read with agent-scope relaxed atomics: global_store/load with
// sc1, which write through to, and read from, the device-coherent level, so a
// block needs no cache-wide release / acquire fence (a release fence at agent
// scope is an L2 writeback on this chip).  Ordering, DESIGN.md §3:
//  * writer: block stores, then drain_stores() -- s_waitcnt vmcnt(0), which
//    returns only once every earlier store is acknowledged, written as an asm
//    statement with a "memory" clobber so the compiler cannot move a memory
//    access across it -- then the ring entry store (and, unpaired, the avail
//    increment), so an entry becomes visible only after its block;
//  * reader: the entry is loaded and its tag checked before the block's
//    address (path id) is known, and its loads are issued after that wait.
__device__ __forceinline__ void st_u64_h(unsigned long long *p, unsigned long long v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long ld_u64_h(const unsigned long long *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long pack2(unsigned lo, unsigned hi) {
    return (unsigned long long)lo | ((unsigned long long)hi << 32);
}
__device__ __forceinline__ void st_cf_rlx(cf *p, cf v) {
    st_u64_h(reinterpret_cast<unsigned long long *>(p), pack2(__float_as_uint(v.x), __float_as_uint(v.y)));
}
__device__ __forceinline__ cf ld_cf_rlx(const cf *p) {
    const unsigned long long u = ld_u64_h(reinterpret_cast<const unsigned long long *>(p));
    return cmk(__uint_as_float((unsigned)u), __uint_as_float((unsigned)(u >> 32)));
}
__device__ __forceinline__ int ld_i_rlx(const int *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void drain_stores() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// (pointers and sizes by value: a KArgs reference would put the kernel
// arguments in scratch memory)
__device__ __forceinline__ unsigned long long xchg_u64(unsigned long long *p, unsigned long long v) {
    return __hip_atomic_exchange(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Publishes suspended path b (its block already written and drained).  A
// pusher that finds its ticket abandoned -- it was paused between taking the
// ticket and writing the entry for longer than the consumer waits -- pushes
// again on a new ticket, paired or unpaired as before.  Accounting: every
// live entry is matched by one pop, either a claim on avail (unpaired
// entries publish one) or the paired pop its pusher makes next; an abandoned
// ticket takes one pop with it, and its consumer restores the balance
// (ring_pop gives its claim back; ring_pop_paired publishes its own paired
// push as claimable).  test_delay (tests only): every 16th ticket waits that
// many ticks before its exchange, so that its consumer abandons it.
__device__ __forceinline__ void ring_push(unsigned *rq, unsigned long long *ring, unsigned cap, unsigned epoch, int b,
                                          bool unpaired, Workspace *ws, int test_delay) {
    for (;;) {
        const unsigned t = atomicAdd(&rq[RQ_TAIL], 1u);
        if (t >= cap) {   // more re-pushes than RING_SLACK (the path is lost: reported)
            atomicMax(&ws->status, (unsigned)HC_ERROR_DEVICE);
            return;
        }
        if (__builtin_expect(test_delay > 0, 0) && (t & 15u) == 7u) {
            const unsigned long long w0 = __builtin_amdgcn_s_memrealtime();
            while (__builtin_amdgcn_s_memrealtime() - w0 < (unsigned long long)test_delay) __builtin_amdgcn_s_sleep(8);
        }
        const unsigned tag = ring_tag(epoch, t);
        const unsigned long long old = xchg_u64(&ring[t], ((unsigned long long)tag << 32) | (unsigned)b);
        if (__builtin_expect(old != ring_abandon_mark(tag), 1)) break;
    }
    if (unpaired) atomicAdd(&rq[RQ_AVAIL], 1u);
}
// The entry of ticket h: its pusher took ticket h before (head never passes
// tail), so it is written or about to be.  A pusher paused mid-push is waited
// for up to wait_ticks; then the ticket is abandoned (-2): one exchange writes
// the abandon mark, and if the pusher's entry arrived just before it, the
// exchange returns it and the path is taken after all.  Otherwise the pusher
// will see the mark and push again (ring_push), so no path is lost.  A path
// id outside the launch cannot come from the protocol: reported, -1.
__device__ __forceinline__ int ring_take(unsigned long long *ring, unsigned cap, unsigned epoch, Workspace *ws,
                                         unsigned h, const unsigned *rq, int num_paths, unsigned long long wait_ticks) {
    if (h >= cap) {
        atomicMax(&ws->status, (unsigned)HC_ERROR_DEVICE);
        return -1;
    }
    const unsigned tag = ring_tag(epoch, h);
    unsigned long long e = ld_u64_h(&ring[h]);
    if ((unsigned)(e >> 32) != tag) {
        const unsigned long long w0 = __builtin_amdgcn_s_memrealtime();
        for (;;) {
            __builtin_amdgcn_s_sleep(8);
            e = ld_u64_h(&ring[h]);
            if ((unsigned)(e >> 32) == tag) break;
            if (__builtin_amdgcn_s_memrealtime() - w0 > wait_ticks) {
                e = xchg_u64(&ring[h], ring_abandon_mark(tag));
                if ((unsigned)(e >> 32) == tag) break;
                atomicAdd(&ws->abandoned, 1u);
                return -2;
            }
        }
    }
    if ((unsigned)e < (unsigned)num_paths) return (int)(unsigned)e;
    if (atomicMax(&ws->status, (unsigned)HC_ERROR_DEVICE) == 0u) {
        // diagnostics: ticket, entry seen, tail, head
        ws->ring_fail[0] = h;
        ws->ring_fail[1] = (unsigned)e;
        ws->ring_fail[2] = ld_rlx(&rq[RQ_TAIL]);
        ws->ring_fail[3] = ld_rlx(&rq[RQ_HEAD]);
    }
    return -1;
}
// oldest suspended path id, or -1 if there is none
__device__ __forceinline__ int ring_pop(unsigned *rq, unsigned long long *ring, unsigned cap, unsigned epoch,
                                        Workspace *ws, int num_paths, unsigned long long wait_ticks) {
    int *avail = reinterpret_cast<int *>(&rq[RQ_AVAIL]);
    // after 16 abandoned tickets this pop gives up (-1: the half
    // idles); nothing is lost, the abandoned paths' pushers push them again
    // and keep popping while entries remain
    for (int tries = 0; tries < 16;) {
        if (ld_i_rlx(avail) <= 0) return -1;
        if (atomicSub(avail, 1) > 0) {
            const int b = ring_take(ring, cap, epoch, ws, atomicAdd(&rq[RQ_HEAD], 1u), rq, num_paths, wait_ticks);
            if (b != -2) return b;
            atomicAdd(avail, 1);   // abandoned: the claim goes back (its entry is still to be popped)
            tries++;
            continue;
        }
        if (atomicAdd(avail, 1) + 1 <= 0) return -1;
    }
    return -1;
}
// the swap's pop, right after its own push (no claim).  If its ticket is
// abandoned, the swap's own push has lost the pop that matched it: it is
// published as claimable (avail), and the half looks for a path with an
// unpaired pop
__device__ __forceinline__ int ring_pop_paired(unsigned *rq, unsigned long long *ring, unsigned cap, unsigned epoch,
                                               Workspace *ws, int num_paths, unsigned long long wait_ticks) {
    const int b = ring_take(ring, cap, epoch, ws, atomicAdd(&rq[RQ_HEAD], 1u), rq, num_paths, wait_ticks);
    if (b != -2) return b;
    atomicAdd(&rq[RQ_AVAIL], 1u);
    return ring_pop(rq, ring, cap, epoch, ws, num_paths, wait_ticks);
}

// ---------------------------------------------------------------- table prep
// Compacts the reference's padded unified index (38880 ints: dH/dx at
// ((c*8+j)*5+part)*30 + r, dH/dt at 36000 + (j*6+part)*30 + r; Data_Reader.cpp
// :167-189, ..._LimUnroll_L2Cache.cuh:57-148) into EvalTables.  Lane r < 30
// of the first wave = equation row r.  Every index and coefficient is
// validated; a table that does not fit sets HC_ERROR_TABLE and the tracker
// leaves its outputs untouched.  The tables persist in the workspace: a launch
// whose index table hashes to the one they were built from (all 256 threads
// hash it, ~10 KB each) skips the compaction.
//
// Also the per-launch reset of the time-slicing counters (rq != nullptr): head,
// tail and avail zeroed, the ring epoch bumped; ring entries not cleared yet
// (a workspace's first sliced launch, or a larger ring than before) are zeroed
// once (hash tags never match a zero entry).
constexpr unsigned TAB_MAGIC = 0x48435442u;   // "HCTB"
__device__ __forceinline__ unsigned long long mix64(unsigned long long z) {   // splitmix64 finaliser
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
struct PrepArgs {
    const int32_t *U;
    Workspace *ws;
    const uint8_t *found_in;     // abort mode: the (cross-rank reduced) found flag, else null
    const unsigned *peer_found;  // abort mode: the cross-process flag, or null
    unsigned *rq;                // time slicing, else null
    unsigned long long *ring;
    unsigned ring_cap;
    unsigned susp_entry0, susp_entry1;   // the suspend blocks' span in ring-entry units (from the ring's start)
};
constexpr int PREP_THREADS = 256;
__global__ void __launch_bounds__(PREP_THREADS) k_prep_tables(PrepArgs pa) {
    const int32_t *__restrict__ U = pa.U;
    Workspace *ws = pa.ws;
    EvalTables *T = &ws->tab;
    __shared__ int s_len[32];
    __shared__ int s_bad;
    __shared__ int s_nostruct;   // the dH/dx structure is not within the tracker LU's
    __shared__ unsigned long long s_h[PREP_THREADS];
    __shared__ unsigned s_cleared, s_dlo, s_dhi;
    __shared__ int s_valid;
    const int tid = threadIdx.x;
    {
        // the table's hash (a sum, so any load order gives it): 16-B loads when
        // the caller's table is 16-B aligned (the per-launch check took 40 us
        // with one int per load, a fifth of the launch overhead; round 6)
        unsigned long long h = 0;
        if (((uintptr_t)U & 15u) == 0u) {
            const int4 *U4 = reinterpret_cast<const int4 *>(U);
            static_assert((HX_SIZE + HT_SIZE) % 4 == 0, "whole int4 words");
#pragma unroll 4
            for (int i = tid; i < (HX_SIZE + HT_SIZE) / 4; i += PREP_THREADS) {
                const int4 v = U4[i];
                const unsigned long long b = (unsigned long long)(4 * i) << 32;
                h += mix64(b | (unsigned)v.x) + mix64((b + (1ull << 32)) | (unsigned)v.y) +
                     mix64((b + (2ull << 32)) | (unsigned)v.z) + mix64((b + (3ull << 32)) | (unsigned)v.w);
            }
        } else {
#pragma unroll 8
            for (int i = tid; i < HX_SIZE + HT_SIZE; i += PREP_THREADS)
                h += mix64(((unsigned long long)i << 32) | (unsigned)U[i]);
        }
        s_h[tid] = h;
    }
    if (tid == 0) {
        // the launch's control block (queue, status, flag, timestamps, diagnostics)
        unsigned *cb = reinterpret_cast<unsigned *>(ws);
        for (int q = 0; q < 16; q++) cb[q] = 0u;
        s_bad = 0;
        s_nostruct = 0;
        if (pa.found_in) {
            const bool peer = pa.peer_found &&
                              __hip_atomic_load(pa.peer_found, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u;
            ws->found = (pa.found_in[0] || peer) ? 1u : 0u;
        }
        const bool known = pa.rq && pa.rq[RQ_MAGIC] == RQ_MAGIC_VALUE;
        s_cleared = known ? pa.rq[RQ_CLEARED] : 0u;
        s_dlo = known ? pa.rq[RQ_DLO] : 0u;
        s_dhi = known ? pa.rq[RQ_DHI] : 0u;
    }
    __syncthreads();
    for (int w = PREP_THREADS / 2; w > 0; w >>= 1) {
        if (tid < w) s_h[tid] += s_h[tid + w];
        __syncthreads();
    }
    const unsigned long long src_hash = s_h[0];
    if (pa.rq) {
        // entries never cleared, and cleared entries an earlier launch's
        // suspend blocks overwrote (the dirty range), inside this launch's ring
        for (unsigned e = s_cleared + tid; e < pa.ring_cap; e += PREP_THREADS) pa.ring[e] = 0ull;
        const unsigned dhi = min(s_dhi, min(s_cleared, pa.ring_cap));
        for (unsigned e = s_dlo + tid; e < dhi; e += PREP_THREADS) pa.ring[e] = 0ull;
    }
    if (tid == 0) s_valid = (T->magic == TAB_MAGIC && T->src_hash == src_hash && T->status == 0) ? 1 : 0;
    __syncthreads();
    if (pa.rq && tid == 0) {
        unsigned *rq = pa.rq;
        rq[RQ_HEAD] = 0u;
        rq[RQ_TAIL] = 0u;
        rq[RQ_AVAIL] = 0u;
        const unsigned e = (rq[RQ_MAGIC] == RQ_MAGIC_VALUE) ? rq[RQ_EPOCH] + 1u : 1u;
        rq[RQ_EPOCH] = e ? e : 1u;
        // this launch's suspend blocks start right after its ring: the cleared
        // entries they may overwrite join the dirty range (one interval that
        // covers every such range not re-zeroed yet)
        const unsigned cleared = max(s_cleared, pa.ring_cap);
        unsigned lo = max(s_dlo, pa.ring_cap), hi = s_dhi;                 // what this launch did not re-zero
        const unsigned s0 = pa.susp_entry0, s1 = min(cleared, pa.susp_entry1);   // this launch's blocks
        if (s0 < s1) {
            const bool had = lo < hi;
            lo = had ? min(lo, s0) : s0;
            hi = had ? max(hi, s1) : s1;
        }
        if (hi > cleared) hi = cleared;
        if (lo >= hi) lo = hi = 0u;
        rq[RQ_CLEARED] = cleared;
        rq[RQ_DLO] = lo;
        rq[RQ_DHI] = hi;
        rq[RQ_MAGIC] = RQ_MAGIC_VALUE;
    }
    if (s_valid) return;   // tables built from this index table already
    const int r = tid;
    // dH/dx: entries bin-packed over the 32 lanes (hc_eval.hpp).  A: terms per
    // entry (rows in parallel); B: one thread places the entries, largest first,
    // each in the smallest-capacity slot class with a free lane (ties: lower
    // row, then lower column), numbering the entries 0..169 in placement order
    // (their place in the slot's packed entry block), and lists the distinct
    // prefix triples (c, a, b) of the dH/dx and H terms and pairs (a, b) of the
    // dH/dt terms (padding first: (0, 33, 33) and (33, 33)); C: rows write their
    // terms' words; D: the prefix build jobs.
    __shared__ uint8_t s_cnt[NV][NV];
    __shared__ int s_htn[32];             // dH/dt | H terms of row r (0 for lanes 30, 31)
    __shared__ uint8_t s_place[NV][NV];   // lane << 3 | slot, 0xFF: structural zero
    __shared__ uint16_t s_eoff[NV][NV];   // SlotLDS byte offset of entry (row, column)
    __shared__ uint32_t s_dst[HX_NSLOT / 2][32];
    __shared__ uint32_t s_tri[TP_CAP];    // (uint8)c | a << 8 | b << 16
    __shared__ uint32_t s_pair[QP_CAP];   // a | b << 8
    __shared__ int s_ntri, s_npair;
    __shared__ uint32_t s_th[256], s_ph[128];   // hash sets of the prefix keys (+ 1)
    // slot capacities and starts as locals (a runtime index into the
    // namespace-scope constexpr table does not reach device memory)
    int cap[HX_NSLOT], start[HX_NSLOT];
    for (int s2 = 0, acc2 = 0; s2 < HX_NSLOT; s2++) {
        cap[s2] = HX_GCAP[0] * (s2 == 0) + HX_GCAP[1] * (s2 == 1) + HX_GCAP[2] * (s2 == 2) +
                  HX_GCAP[3] * (s2 == 3) + HX_GCAP[4] * (s2 == 4) + HX_GCAP[5] * (s2 == 5);
        start[s2] = acc2;
        acc2 += cap[s2];
    }
    const int32_t *D = U + HX_SIZE;
    if (r < NV)
        for (int c = 0; c < NV; c++) {
            int n = 0;
            for (int j = 0; j < HX_TERMS; j++)
                if (U[(c * HX_TERMS + j) * HX_PARTS * NV + r] != 0) n++;
            s_cnt[r][c] = (uint8_t)n;
            s_place[r][c] = 0xFFu;
            s_eoff[r][c] = (uint16_t)SLOT_OFF_ENTZERO;
        }
    // the distinct prefix keys of all terms, collected by every thread into LDS
    // hash sets (open addressing, atomicCAS; key + 1, 0 = empty); a term outside
    // the index ranges is left out here and rejected in C
    for (int h = tid; h < 256; h += PREP_THREADS) s_th[h] = 0u;
    for (int h = tid; h < 128; h += PREP_THREADS) s_ph[h] = 0u;
    __syncthreads();
    {
        auto hins = [&](uint32_t *tab, uint32_t mask, uint32_t key) {
            uint32_t h = (key * 2654435761u) >> 20 & mask;
            for (uint32_t probe = 0; probe <= mask; probe++) {
                const uint32_t old = atomicCAS(&tab[h], 0u, key + 1u);
                if (old == 0u || old == key + 1u) return;
                h = (h + 1u) & mask;
            }
            s_bad = 1;   // more distinct keys than the set holds
        };
        for (int i = tid; i < HX_SIZE / HX_PARTS; i += PREP_THREADS) {   // (column, term, row) of dH/dx
            const int base = (i / NV) * HX_PARTS * NV + i % NV;
            const int co = U[base];
            if (co == 0) continue;
            const int a = U[base + NV], b = U[base + 2 * NV];
            if (co >= -128 && co <= 127 && a >= 0 && a < NPP && b >= 0 && b < NPP)
                hins(s_th, 255u, ((uint32_t)co & 0xFFu) | (uint32_t)a << 8 | (uint32_t)b << 16);
        }
        for (int i = tid; i < HT_SIZE / HT_PARTS; i += PREP_THREADS) {
            const int base = (i / NV) * HT_PARTS * NV + i % NV;
            const int co = D[base];
            if (co == 0) continue;
            const int a = D[base + NV], b = D[base + 2 * NV];
            if (co >= -128 && co <= 127 && a >= 0 && a < NPP && b >= 0 && b < NPP) {
                hins(s_th, 255u, ((uint32_t)co & 0xFFu) | (uint32_t)a << 8 | (uint32_t)b << 16);
                hins(s_ph, 127u, (uint32_t)a | (uint32_t)b << 8);
            }
        }
    }
    if (r < 32) {
        // padding words first (other lanes' rows overwrite them in C): tp[0] = 0 on unit operands
        const uint32_t x30p = (uint32_t)(SLOT_OFF_X + 8 * 30);
        for (int k2 = 0; k2 < HX_SLOT_CAP; k2++) T->hx[k2 * 32 + r] = (uint32_t)SLOT_OFF_TP | x30p << 16 | x30p << 24;
        int n = 0;
        if (r < NV)
            for (int j = 0; j < HT_TERMS; j++)
                if (D[j * HT_PARTS * NV + r] != 0) n++;
        s_htn[r] = n;
    }
    __syncthreads();
    if (tid == 0) {
        int used[HX_NSLOT], order[HX_NSLOT];
        for (int s2 = 0; s2 < HX_NSLOT; s2++) { used[s2] = 0; order[s2] = s2; }
        for (int i = 1; i < HX_NSLOT; i++)   // slot classes by capacity, smallest first (stable)
            for (int j2 = i; j2 > 0 && cap[order[j2 - 1]] > cap[order[j2]]; j2--) {
                const int t2 = order[j2]; order[j2] = order[j2 - 1]; order[j2 - 1] = t2;
            }
        for (int q = 0; q < 32; q++)
            for (int w2 = 0; w2 < HX_NSLOT / 2; w2++)
                s_dst[w2][q] = (uint32_t)SLOT_OFF_HXDUMMY | ((uint32_t)SLOT_OFF_HXDUMMY << 16);
        int ne[NV], nent = 0;
        for (int q = 0; q < NV; q++) ne[q] = 0;
        for (int n = HX_TERMS; n >= 1; n--)
            for (int row = 0; row < NV; row++)
                for (int c = 0; c < NV; c++) {
                    if (s_cnt[row][c] != n) continue;
                    int sl = -1;
                    for (int i = 0; i < HX_NSLOT && sl < 0; i++)
                        if (cap[order[i]] >= n && used[order[i]] < 32) sl = order[i];
                    if (sl < 0 || ne[row] >= 6 || nent >= ENT_CAP - 1) { s_bad = 1; continue; }
                    const int ln = used[sl]++;
                    ne[row]++;
                    s_place[row][c] = (uint8_t)(ln << 3 | sl);
                    const uint32_t off = (uint32_t)(SLOT_OFF_ENT + 8 * nent++);
                    s_eoff[row][c] = (uint16_t)off;
                    const int hi = (sl & 1) * 16;
                    s_dst[sl >> 1][ln] = (s_dst[sl >> 1][ln] & ~(0xFFFFu << hi)) | (off << hi);
                }
        // the distinct prefixes, from the hash sets below: (0, 33, 33) and (33, 33)
        // first (the padding words point at slot 0), the others in key order
        int nt = 1, np = 1;
        const uint32_t pad_t = 33u << 8 | 33u << 16, pad_p = 33u | 33u << 8;
        s_tri[0] = pad_t;
        s_pair[0] = pad_p;
        for (int h = 0; h < 256; h++) {
            const uint32_t k = s_th[h] - 1u;
            if (s_th[h] == 0u || k == pad_t) continue;
            if (nt < TP_CAP) s_tri[nt++] = k; else s_bad = 1;
        }
        for (int h = 0; h < 128; h++) {
            const uint32_t k = s_ph[h] - 1u;
            if (s_ph[h] == 0u || k == pad_p) continue;
            if (np < QP_CAP) s_pair[np++] = k; else s_bad = 1;
        }
        for (int i = 2; i < nt; i++)
            for (int j2 = i; j2 > 1 && s_tri[j2 - 1] > s_tri[j2]; j2--) {
                const uint32_t t2 = s_tri[j2]; s_tri[j2] = s_tri[j2 - 1]; s_tri[j2 - 1] = t2;
            }
        for (int i = 2; i < np; i++)
            for (int j2 = i; j2 > 1 && s_pair[j2 - 1] > s_pair[j2]; j2--) {
                const uint32_t t2 = s_pair[j2]; s_pair[j2] = s_pair[j2 - 1]; s_pair[j2 - 1] = t2;
            }
        s_ntri = nt;
        s_npair = np;
    }
    __syncthreads();
    // slot of a key: 0 for the padding key, else binary search in the sorted rest
    auto find = [](const uint32_t *tab, int n, uint32_t key) -> int {
        if (key == tab[0]) return 0;
        int lo = 1, hi = n;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (tab[mid] < key) lo = mid + 1; else hi = mid;
        }
        return lo < n && tab[lo] == key ? lo : 0;
    };
    auto tp_off = [&](int co, int a, int b) -> uint32_t {
        return (uint32_t)(SLOT_OFF_TP +
                          8 * find(s_tri, s_ntri, ((uint32_t)co & 0xFFu) | (uint32_t)a << 8 | (uint32_t)b << 16));
    };
    auto qp_off = [&](int a, int b) -> uint32_t {
        return (uint32_t)(SLOT_OFF_QP + 8 * find(s_pair, s_npair, (uint32_t)a | (uint32_t)b << 8));
    };
    const uint32_t x30 = (uint32_t)(SLOT_OFF_X + 8 * 30);
    if (r < 32) {
        bool bad = false;
        // gather map and structural pattern of row r (padding lanes: zeros)
        uint32_t pat = 0;
        for (int q = 0; q < GM_WORDS; q++) {
            uint32_t v = 0;
            for (int k2 = 0; k2 < 2; k2++) {
                const int c = 2 * q + k2;
                const uint32_t off = r < NV ? s_eoff[r][c] : (uint32_t)SLOT_OFF_ENTZERO;
                v |= off << (16 * k2);
                if (off != (uint32_t)SLOT_OFF_ENTZERO) pat |= 1u << c;
            }
            T->gm[q][r] = v;
        }
        T->pat[r] = pat;
        // the tracker's LU skips the column groups this problem's structure
        // can never fill (hc_lu.hpp LU_STRUCT_PAT); the evaluations take any
        // structure, the tracker only one within it
        if (r < NV && (pat & ~LU_STRUCT_PAT[r]) != 0u) atomicOr(&s_nostruct, 1);
        for (int q = 0; q < HX_NSLOT / 2; q++) T->hxd[q][r] = s_dst[q][r];
        if (r < NV)
            for (int c = 0; c < NV; c++) {
                if (s_place[r][c] == 0xFFu) continue;
                const int ln = s_place[r][c] >> 3, sl = s_place[r][c] & 7;
                int pos = start[sl];
                for (int j = 0; j < HX_TERMS; j++) {
                    const int base = (c * HX_TERMS + j) * HX_PARTS * NV + r;
                    const int co = U[base], a = U[base + NV], b = U[base + 2 * NV], u = U[base + 3 * NV],
                              v = U[base + 4 * NV];
                    if (co == 0) continue;
                    bad |= co < -128 || co > 127 || a < 0 || a >= NPP || b < 0 || b >= NPP || u < 0 || u > NV ||
                           v < 0 || v > NV;
                    if (!bad)
                        T->hx[pos * 32 + ln] = tp_off(co, a, b) | (uint32_t)(SLOT_OFF_X + 8 * u) << 16 |
                                               (uint32_t)(SLOT_OFF_X + 8 * v) << 24;
                    pos++;
                }
            }
        s_len[r] = HX_SLOT_CAP;
        // dH/dt | H (hc_eval.hpp eval_rhs): own terms at positions 0..12; a row
        // of more than 13 terms (an owner) puts its terms 14.. in its light
        // words 13.. (for x[w]) and in its helper's (lane ^ 16) words 10..; the
        // helper's own terms must end before 10 and it needs no help itself
        const int n = s_htn[r];
        const int need_o = max(0, n - HT_FULL);
        const int need_h = max(0, s_htn[r ^ 16] - HT_FULL);
        if (need_o > 0 && s_htn[r ^ 16] > HT_HELP_FIRST) bad = true;
        if (need_h > 0 && n > HT_HELP_FIRST) bad = true;
        const uint2 pad_ht = make_uint2((uint32_t)SLOT_OFF_TP | (uint32_t)SLOT_OFF_QP << 16,
                                        x30 | x30 << 8 | x30 << 16);   // tp[0], qp[0] with coef 0
        int k = 0;
        if (r < NV) {
            for (int j = 0; j < HT_TERMS; j++) {
                const int base = j * HT_PARTS * NV + r;
                const int co = D[base], a = D[base + NV], b = D[base + 2 * NV], u = D[base + 3 * NV],
                          v = D[base + 4 * NV], x3 = D[base + 5 * NV];
                if (co == 0) continue;
                bad |= co < -128 || co > 127 || a < 0 || a >= NPP || b < 0 || b >= NPP || u < 0 || u > NV ||
                       v < 0 || v > NV || x3 < 0 || x3 > NV;
                if (!bad) {
                    const uint2 tw = make_uint2(tp_off(co, a, b) | qp_off(a, b) << 16,
                                                (uint32_t)(SLOT_OFF_X + 8 * u) | ((uint32_t)(SLOT_OFF_X + 8 * v) << 8) |
                                                    ((uint32_t)(SLOT_OFF_X + 8 * x3) << 16) |
                                                    (((uint32_t)co & 0xFFu) << 24));
                    T->ht[k * 32 + r] = tw;   // k < 13: a full term; k >= 13: the light word (x[w])
                    if (k >= HT_FULL) T->ht[(HT_HELP_FIRST + k - HT_FULL) * 32 + (r ^ 16)] = tw;
                }
                k++;
            }
        }
        for (int q = k; q < HT_TERMS; q++)
            if (!(q >= HT_HELP_FIRST && q < HT_HELP_FIRST + need_h)) T->ht[q * 32 + r] = pad_ht;
        if (bad) atomicOr(&s_bad, 1);
    }
    // E: bank-aware places of the (c, a, b) prefixes.  A ds_read_b64 of tp[]
    // serves 32 lanes a cycle when their indices differ mod 32 (or coincide);
    // the words of C read tp at 21 dH/dx and 13 rhs positions, and the sorted
    // numbering above costs ~64 cycles where 34 are the minimum.  Prefixes that
    // share a read position (conflict graph, s_adj) go to different residues:
    // the padding prefix first (tp[0]), then by degree, each to the residue
    // with the fewest conflicts and a free place (3 per residue, ties: fewer
    // used, then the lower residue); C's words are renumbered after it.
    // Places only: the values and their operations stay the same (bit-exact).
    __shared__ uint32_t s_adj[TP_CAP][3];
    __shared__ uint8_t s_pidx[HX_SLOT_CAP + HT_FULL][32];
    __shared__ uint8_t s_tslot[TP_CAP], s_tinv[TP_CAP], s_order[TP_CAP];
    __shared__ int s_deg[TP_CAP];
    for (int i = tid; i < TP_CAP * 3; i += PREP_THREADS) (&s_adj[0][0])[i] = 0u;
    for (int i = tid; i < TP_CAP; i += PREP_THREADS) { s_tinv[i] = 0xFFu; s_tslot[i] = 0u; }
    __syncthreads();
    const int ntri = s_ntri;
    auto tp_index = [&](uint32_t w) -> uint32_t {   // sorted index of a word's tp offset (TP_CAP: none)
        const uint32_t o = w & 0xFFFFu;
        const uint32_t i = (o - (uint32_t)SLOT_OFF_TP) / 8u;
        return o >= (uint32_t)SLOT_OFF_TP && i < (uint32_t)ntri ? i : (uint32_t)TP_CAP;
    };
    for (int i = tid; i < (HX_SLOT_CAP + HT_FULL) * 32; i += PREP_THREADS) {
        const int p = i >> 5, l = i & 31;
        const uint32_t w = p < HX_SLOT_CAP ? T->hx[p * 32 + l] : T->ht[(p - HX_SLOT_CAP) * 32 + l].x;
        s_pidx[p][l] = (uint8_t)min(tp_index(w), (uint32_t)0xFFu);
    }
    __syncthreads();
    for (int i = tid; i < (HX_SLOT_CAP + HT_FULL) * 32; i += PREP_THREADS) {
        const int p = i >> 5, l = i & 31;
        const uint32_t t = s_pidx[p][l];
        if (t >= (uint32_t)ntri) continue;
        for (int l2 = 0; l2 < 32; l2++) {
            const uint32_t u = s_pidx[p][l2];
            if (u != t && u < (uint32_t)ntri) atomicOr(&s_adj[t][u >> 5], 1u << (u & 31));
        }
    }
    __syncthreads();
    if (tid < ntri)
        s_deg[tid] = tid == 0 ? (1 << 20) : __popc(s_adj[tid][0]) + __popc(s_adj[tid][1]) + __popc(s_adj[tid][2]);
    __syncthreads();
    if (tid < ntri) {   // rank by degree, descending (ties: lower index first)
        int rk = 0;
        const int d = s_deg[tid];
        for (int u = 0; u < ntri; u++) rk += (s_deg[u] > d || (s_deg[u] == d && u < tid)) ? 1 : 0;
        s_order[rk] = (uint8_t)tid;
    }
    __syncthreads();
    if (tid < 64) {   // wave 0, lane c < 32: residue c (its members and fill)
        uint32_t m0 = 0u, m1 = 0u, m2 = 0u;
        int fill = 0;
        for (int k2 = 0; k2 < ntri; k2++) {
            const int t = s_order[k2];
            const int conf = __popc(s_adj[t][0] & m0) + __popc(s_adj[t][1] & m1) + __popc(s_adj[t][2] & m2);
            int key = (tid < 32 && fill < 3) ? ((conf * 4 + fill) << 5 | tid) : 0x7FFFFFFF;
            for (int s2 = 32; s2 > 0; s2 >>= 1) key = min(key, __shfl_xor(key, s2, 64));
            if (tid == (key & 31)) {
                const int slot = tid + 32 * fill++;
                s_tslot[t] = (uint8_t)slot;
                s_tinv[slot] = (uint8_t)t;
                if (t < 32) m0 |= 1u << t; else if (t < 64) m1 |= 1u << (t - 32); else m2 |= 1u << (t - 64);
            }
        }
    }
    __syncthreads();
    for (int i = tid; i < HX_SLOT_CAP * 32; i += PREP_THREADS) {
        const uint32_t w = T->hx[i], t = tp_index(w);
        if (t < (uint32_t)TP_CAP) T->hx[i] = (w & ~0xFFFFu) | (uint32_t)(SLOT_OFF_TP + 8 * s_tslot[t]);
    }
    for (int i = tid; i < HT_TERMS * 32; i += PREP_THREADS) {
        const uint32_t w = T->ht[i].x, t = tp_index(w);
        if (t < (uint32_t)TP_CAP) T->ht[i].x = (w & ~0xFFFFu) | (uint32_t)(SLOT_OFF_TP + 8 * s_tslot[t]);
    }
    if (r < 32) {
        // prefix build jobs of lane r (hc_eval.hpp build_prefixes): tp place i
        // holds prefix s_tinv[i], qp place i pair i
        const uint32_t p33 = (uint32_t)(SLOT_OFF_STG + 8 * 33);
        for (int q = 0; q < PRE_ROUNDS; q++) {
            const bool tpr = q < PRE_TP_ROUNDS;
            const int i = (tpr ? q : q - PRE_TP_ROUNDS) * 32 + r;
            uint2 job = make_uint2(p33 | p33 << 16, (uint32_t)SLOT_OFF_HXDUMMY);
            if (tpr && i < TP_CAP && s_tinv[i] != 0xFFu) {
                const uint32_t key = s_tri[s_tinv[i]];
                const uint32_t a = (key >> 8) & 0xFFu, b = key >> 16;
                job = make_uint2((uint32_t)(SLOT_OFF_STG + 8 * a) | (uint32_t)(SLOT_OFF_STG + 8 * b) << 16,
                                 (uint32_t)(SLOT_OFF_TP + 8 * i) | (key & 0xFFu) << 16);
            } else if (!tpr && i < s_npair) {
                const uint32_t a = s_pair[i] & 0xFFu, b = s_pair[i] >> 8;
                job = make_uint2((uint32_t)(SLOT_OFF_STG + 8 * a) | (uint32_t)(SLOT_OFF_STG + 8 * b) << 16,
                                 (uint32_t)(SLOT_OFF_QP + 8 * i));
            }
            T->pre[q][r] = job;
        }
    }
    __syncthreads();
    if (r == 0) {
        // eval_rhs masks: help term q of the helpers (no accumulation), light
        // term q of the owners
        for (int q = 0; q < 4; q++) {
            uint32_t am = 0xFFFFFFFFu, lm = 0u;
            for (int l = 0; l < 32; l++)
                if (s_htn[l] - HT_FULL > q) { am &= ~(1u << (l ^ 16)); lm |= 1u << l; }
            T->ht_acc_mask[q] = am;
            T->ht_light_mask[q] = lm;
        }
        int mx = 0;
        for (int q = 0; q < 32; q++) mx = max(mx, s_len[q]);
        T->hx_len = mx;
        T->status = s_bad ? HC_ERROR_TABLE : 0;
        T->lu_struct = s_nostruct ? 0u : 1u;
        T->src_hash = src_hash;
        T->magic = TAB_MAGIC;
        if (s_bad) ws->status = HC_ERROR_TABLE;
    }
}

// ---------------------------------------------------------------- tracker
// Phases of a path slot (one per half-wave):
enum : int { PH_DEQ = 0, PH_BEGIN = 1, PH_STAGE = 2, PH_FINISH = 3, PH_IDLE = 4 };

// Abort-mode scoring of one half's converged path (dev-trifocal_2op1p-eval.cuh:
// 28-250, 32 lanes per path): inlier counts of views 2 and 3 over all triplet
// edgels.
template <int VIEW>   // 0: view 2 (edgel columns 2, 3), 1: view 3 (columns 4, 5)
__device__ __forceinline__ int score_view(const float *R, float da, float db, float dc, const float *edgels,
                                          int num_edgels, float fx, float fy, float cx, float cy, int r) {
    int c = 0;
    for (int e = r; e < num_edgels; e += 32) {
        const float *g = edgels + (size_t)e * 6;
        const float g0 = g[0], g1 = g[1], gu = g[2 + 2 * VIEW], gv = g[3 + 2 * VIEW];
        const float num = dc * (R[2] * gu + R[5] * gv + R[8]) - (R[2] * da + R[5] * db + R[8] * dc);
        const float den = 1.0f - (R[6] * g0 + R[7] * g1 + R[8]) * (R[2] * gu + R[5] * gv + R[8]);
        const float v2 = num * (R[6] * g0 + R[7] * g1 + R[8]) + den * dc;
        const float v0 = (num * (R[0] * g0 + R[1] * g1 + R[2]) + den * da) / v2;
        const float v1 = (num * (R[3] * g0 + R[4] * g1 + R[5]) + den * db) / v2;
        const float ex = (v0 * fx + cx) - (gu * fx + cx);
        const float ey = (v1 * fy + cy) - (gv * fy + cy);
        c += (__builtin_sqrtf(ex * ex + ey * ey) < 2.0f) ? 1 : 0;
    }
    return c;
}
// The two views are scored in separate passes, each from its own evaluation
// of the hypothesis (12 live values instead of 24): the abort kernel's register
// allocation is otherwise set by this cold path.
__device__ __forceinline__ int2 score_half(const cf *sx, const float *edgels, int num_edgels,
                                           const float *K, int r) {
    const float fx = K[0], fy = K[4], cx = K[3] /* eval quirk, SURVEY Appendix C.4 */, cy = K[5];
    int c21, c31;
    {
        Hyp hy;
        make_hypothesis(sx, hy);
        c21 = score_view<0>(hy.R, hy.T[0], hy.T[1], hy.T[2], edgels, num_edgels, fx, fy, cx, cy, r);
    }
    {
        const cf *sx2 = sx;
        asm volatile("" : "+v"(sx2));   // a second evaluation, not the first one kept live
        Hyp hy;
        make_hypothesis(sx2, hy);
        c31 = score_view<1>(hy.R + 9, hy.T[3], hy.T[4], hy.T[5], edgels, num_edgels, fx, fy, cx, cy, r);
    }
    return make_int2(half_sum_i(c21), half_sum_i(c31));
}

#ifdef HC_DIAG_TIMES
// diagnostic build: [0] first wave start, [1] last wave exit (s_memrealtime),
// [2] summed wave lifetimes, [3] waves
__device__ unsigned long long g_diag_span[4] = {~0ull, 0ull, 0ull, 0ull};
#ifdef HC_DIAG_UTIL
// diagnostic build (with HC_DIAG_TIMES): per 10.24-us bin of s_memrealtime
// (modulo 8192 bins = 84 ms), the path-stages and the wave-stages started
// (64 copies of each bin, picked by workgroup, so the atomics do not serialise)
constexpr int UTIL_BINS = 8192, UTIL_COPIES = 64;
__device__ unsigned long long g_diag_util[UTIL_COPIES][UTIL_BINS][2];
#endif
#endif
#ifdef HC_DIAG_PHASES
// diagnostic build: per-phase shader cycles summed over waves (k_track):
// [0] slot phases, [1] park + p(t), [2] dH/dx, [3] dH/dt | H, [5] LU,
// [6] stage update, [7] wave lifetime, [8] waves
__device__ unsigned long long g_diag_phase[13];
#endif

// kernel_GPUHC_trifocal_pose_PH_CodeOpt_TrunPaths (..._TrunPaths.cu:45-290) and,
// with ABORT, ..._TrunPaths_TrunRANSAC (..._TrunRANSAC.cu:45-327).
// MINW: waves per SIMD the register allocation targets.  GTAB: the term tables
// are read from the workspace (global, L1/L2-resident) instead of being staged
// in LDS, which leaves 27.6 KB LDS per workgroup (5 workgroups per CU).
// ARCH: the archived ablation semantics (KArgs::truncate / explicit_rk read at
// run time); a separate instantiation so the headline kernel carries neither
// switch and the two show up under their own names in a kernel trace.
// LUS: the LU's column groups classed by this problem's dH/dx structure
// (hc_lu.hpp LU_STRUCT_PAT / LU_BOUND: never-fillable groups untested,
// always-live groups unconditional, narrowed pivot search).  Every launch
// enqueues both instantiations; k_prep_tables decides on the device which one
// tracks (EvalTables::lu_struct) and the other returns at once, so a table of
// any structure the reference kernel takes (e.g. the same system with its
// equations permuted) tracks, through the structure-agnostic LU.
typedef uint32_t T_hxd_t[HX_NSLOT / 2][32];
template <bool ABORT, int MINW, bool GTAB, bool ARCH = false, bool LUS = true>
__global__ void __launch_bounds__(WG_THREADS, MINW) k_track(KArgs a) {
    // LU (hc_lu.hpp): the abort kernel's time to the first pose is a lone
    // path's latency, so it runs the latency mode (one LDS round trip per pivot
    // step, in batches of HC_LU_LATB_COLS columns); the tracking kernel the
    // throughput mode (profiles/r6x_ab_track_latency_lu.jsonl: the latency mode
    // is 9 % slower per config-2 launch there)
    constexpr int LUCH = LU_CHUNK;
    constexpr int LULAT = ABORT ? HC_LU_LATB_COLS : 0;
#include "hc_track_body.inc"
}

// Tracking launches that fill at most half of the path slots: the SIMDs are
// short of waves, a path's latency sets the launch time, and the latency-mode
// LU is faster (profiles/r6y_ab_small_launch.jsonl: 1-8 samples -16..-19 %,
// 16 samples -5 %, 24 equal, 100 +9 %).  The same body as k_track.  Such a
// launch needs few waves, so the registers go to 3 waves/SIMD: no spills and
// 16 columns per LU batch (profiles/r7g_ab_small_occupancy.jsonl: a further
// -5 % at 1-4 samples, -4..-7 % at 8-16; 6144 path slots)
#ifndef HC_SMALL_MINW
#define HC_SMALL_MINW 3
#endif
#ifndef HC_SMALL_LAT
#define HC_SMALL_LAT 16
#endif
template <bool LUS>
__global__ void __launch_bounds__(WG_THREADS, HC_SMALL_MINW) k_track_small(KArgs a) {
    constexpr bool ABORT = false, GTAB = true, ARCH = false;
    constexpr int LUCH = LU_CHUNK;
    constexpr int LULAT = HC_SMALL_LAT;
#include "hc_track_body.inc"
}

// ---------------------------------------------------------------- components
// The tracker's building blocks alone, from HBM operands (component ABI entry
// points; parity tests of dev-cgesv-batched-small.cuh and the index evals).

// LU: two systems per wave; a row's structural pattern is its non-zero entries
__global__ void __launch_bounds__(WG_THREADS) k_cgesv(int n, const cf *__restrict__ A, const cf *__restrict__ B,
                                                      cf *__restrict__ X) {
    __shared__ LUBuf s_lu[2 * WAVES_PER_WG];
    __shared__ __attribute__((aligned(16))) cf s_scr[2 * WAVES_PER_WG][LU_SCRATCH_CF];
    const int lane = lane_id();
    const int r = lane & 31;
    const int sys = (blockIdx.x * WAVES_PER_WG + threadIdx.x / WAVE) * 2 + (lane >> 5);
    const bool ok = sys < n && r < NV;
    cf rA[NV];
    uint32_t pat = 0;
#pragma unroll
    for (int c = 0; c < NV; c++) {
        rA[c] = ok ? A[((size_t)sys * NV + r) * NV + c] : cmk(0.0f, 0.0f);
        if (rA[c].x != 0.0f || rA[c].y != 0.0f) pat |= 1u << c;   // NaN counts as non-zero
    }
    const cf rB = ok ? B[(size_t)sys * NV + r] : cmk(0.0f, 0.0f);
    LUBuf &LB = s_lu[(threadIdx.x / WAVE) * 2 + (lane >> 5)];
    cf *scr = s_scr[(threadIdx.x / WAVE) * 2 + (lane >> 5)];
    bool redo;
    cf x = lu_solve<false>(rA, rB, lane, pat, LB, scr, redo, __ballot(sys < n));
    if (__builtin_expect(redo, 0)) {   // solved again densely from the original system
#pragma unroll
        for (int c = 0; c < NV; c++) rA[c] = ok ? A[((size_t)sys * NV + r) * NV + c] : cmk(0.0f, 0.0f);
        x = lu_solve<true>(rA, rB, lane, pat, LB, scr, redo);
    }
    if (ok) X[(size_t)sys * NV + r] = x;
}


// dH/dx, dH/dt, H at n points: one point per half-wave
__global__ void __launch_bounds__(WG_THREADS) k_eval(int n, const Workspace *ws, const cf *__restrict__ X,
                                                     const cf *__restrict__ P, const cf *__restrict__ D,
                                                     cf *__restrict__ HX, cf *__restrict__ HT, cf *__restrict__ H) {
    __shared__ uint32_t s_hx[HX_SLOT_CAP * 32];
    __shared__ uint2 s_ht[HT_TERMS * 32];
    __shared__ uint32_t s_hxd[HX_NSLOT / 2 * 32];
    __shared__ SlotLDS s_slot[2 * WAVES_PER_WG];
    const EvalTables *T = &ws->tab;
    if (ws->status != 0u) return;
    for (int i = threadIdx.x; i < HX_SLOT_CAP * 32; i += WG_THREADS) s_hx[i] = T->hx[i];   // padded table
    for (int i = threadIdx.x; i < HT_TERMS * 32; i += WG_THREADS) s_ht[i] = T->ht[i];
    for (int i = threadIdx.x; i < HX_NSLOT / 2 * 32; i += WG_THREADS) s_hxd[i] = (&T->hxd[0][0])[i];
    {
        float *z = reinterpret_cast<float *>(s_slot);
        for (int i = threadIdx.x; i < (int)(sizeof(s_slot) / 4); i += WG_THREADS) z[i] = 0.0f;
    }
    __syncthreads();
    const int lane = lane_id();
    const int r = lane & 31;
    const int sys = (blockIdx.x * WAVES_PER_WG + threadIdx.x / WAVE) * 2 + (lane >> 5);
    SlotLDS &S = s_slot[(threadIdx.x / WAVE) * 2 + (lane >> 5)];
    const bool ok = sys < n;
    if (ok && r < 31) S.x[r] = X[(size_t)sys * 31 + r];
    if (ok) {   // the point's p and d, staged for the prefix tables
        S.ent[r] = P[(size_t)sys * NPP + r];
        S.ent[NPP + r] = D[(size_t)sys * NPP + r];
        if (r < NPP - 32) {
            S.ent[r + 32] = P[(size_t)sys * NPP + r + 32];
            S.ent[NPP + r + 32] = D[(size_t)sys * NPP + r + 32];
        }
    }
    __shared__ uint32_t s_gm[GM_WORDS][32];
    if (threadIdx.x < 32)
        for (int q = 0; q < GM_WORDS; q++) s_gm[q][threadIdx.x] = T->gm[q][threadIdx.x];
    __syncthreads();
    build_prefix_rounds(S, r, &T->pre[0][0]);
    cf rA[NV];
    eval_hx(rA, s_hx, s_hxd, &s_gm[0][0], S, r);
    const cf ht = eval_rhs<RHS_HT>(s_ht, S, r, true, rhs_masks(T));
    const cf h = eval_rhs<RHS_H>(s_ht, S, r, false, rhs_masks(T));
    if (ok && r < NV) {
#pragma unroll
        for (int c = 0; c < NV; c++) HX[((size_t)sys * NV + r) * NV + c] = rA[c];
        HT[(size_t)sys * NV + r] = ht;
        H[(size_t)sys * NV + r] = h;
    }
}

// Epilogue of a sliced launch: once the tracker has drained, every
// pushed ring entry has been taken (head == tail) and every unpaired push
// claimed (avail == 0).  Otherwise a suspended path was never resumed and its
// outputs are stale: HC_ERROR_DEVICE (hc_trifocal_workspace_status), with
// (~0, avail, tail, head) in ring_fail.  One thread, stream-ordered after k_track.
__global__ void __launch_bounds__(64) k_ring_check(Workspace *ws, const unsigned *rq) {
    if (threadIdx.x != 0) return;
    const unsigned head = ld_rlx(&rq[RQ_HEAD]), tail = ld_rlx(&rq[RQ_TAIL]), avail = ld_rlx(&rq[RQ_AVAIL]);
    if ((head != tail || avail != 0u) && atomicMax(&ws->status, (unsigned)HC_ERROR_DEVICE) == 0u) {
        ws->ring_fail[0] = 0xFFFFFFFFu;
        ws->ring_fail[1] = avail;
        ws->ring_fail[2] = tail;
        ws->ring_fail[3] = head;
    }
}

// ---------------------------------------------------------------- host side
static size_t ws_bytes_needed() { return (sizeof(Workspace) + 255) & ~(size_t)255; }
// + the time-slicing area of a launch of `paths` paths: the ring counters, the
// ring, then a suspend block per path.  The ring starts at a fixed offset, so
// a workspace reused for launches of other sizes keeps its entry i at one
// address (RQ_CLEARED counts entries from there); the suspend blocks follow
// this launch's ring (256-B aligned) and may overwrite cleared entries past
// it: k_prep_tables keeps that span as the dirty range (RQ_DLO, RQ_DHI) and
// re-zeroes it when a later launch's ring covers it.
static size_t ring_bytes(unsigned long long cap) { return ((size_t)cap * sizeof(unsigned long long) + 255) & ~(size_t)255; }
static size_t ws_bytes_for(long long paths, int max_steps) {
    if (paths < 0) paths = 0;
    if (max_steps < 0) max_steps = 0;
    return ws_bytes_needed() + RQ_WORDS * sizeof(unsigned) + ring_bytes(ring_entries(paths, max_steps)) +
           (size_t)paths * SUSP_WORDS * sizeof(unsigned long long);
}
// tests only (hc_trifocal_set_ring_test, include/hc_trifocal_testing.h): pusher
// delay of every 16th ring ticket; read by every launch of every thread
static std::atomic<int> g_ring_test{0};
// tests only (hc_trifocal_set_small_launch): -1 never the small-launch
// kernels, 0 by size, 1 always (tracking launches)
static std::atomic<int> g_small_launch{0};

// Persistent grid: resident workgroups (occupancy API, cached per device and
// kernel) x CUs, capped by the work.  resident_wgs(k) = grid_for(INT_MAX, k).
static int grid_for(int waves_needed, const void *kernel) {
    static std::mutex mu;
    static std::map<std::pair<int, const void *>, std::pair<int, int>> cache;   // -> (CUs, workgroups per CU)
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return -1;
    int cus = 0, per_cu = 0;
    {
        std::lock_guard<std::mutex> g(mu);
        auto it = cache.find({dev, kernel});
        if (it == cache.end()) {
            if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return -1;
            if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, WG_THREADS, 0) != hipSuccess) per_cu = 1;
            if (per_cu < 1) per_cu = 1;
            it = cache.emplace(std::make_pair(dev, kernel), std::make_pair(cus, per_cu)).first;
        }
        cus = it->second.first;
        per_cu = it->second.second;
    }
    const int want = waves_needed / WAVES_PER_WG + (waves_needed % WAVES_PER_WG != 0);
    const int cap = cus * per_cu;
    return want < cap ? want : cap;
}
static int resident_wgs(const void *kernel) { return grid_for(INT_MAX, kernel); }

static hcStatus launch_track(const hcTrackArgs *t, const hcAbortArgs *ab, void *workspace, size_t wsb,
                             hcStream stream, bool abort_mode, bool truncate = true, bool explicit_rk = false) {
    if (!t || t->sub_ransac_iters < 0) return HC_ERROR_INVALID_VALUE;
    if (!workspace || wsb < ws_bytes_needed()) return HC_ERROR_WORKSPACE;
    if (t->sub_ransac_iters == 0) return HC_SUCCESS;
    if ((!t->start_sols && !t->start_sols_array) || (!t->tracks && !t->track_array) || !t->start_params ||
        !t->target_params || !t->diff_params || !t->unified_index || !t->converge || !t->infinity)
        return HC_ERROR_INVALID_VALUE;
    if (t->settings.max_steps < 0 || t->settings.max_corrections < 0 || t->settings.delta_t_inc_steps < 0)
        return HC_ERROR_INVALID_VALUE;
    if (abort_mode && (!ab || ab->num_triplet_edgels <= 0 || !ab->triplet_edge_locations || !ab->intrinsic_matrix ||
                       !ab->found_trifocal_sols || !ab->trifocal_sols_batch_index))
        return HC_ERROR_INVALID_VALUE;
    const long long paths = (long long)t->sub_ransac_iters * NTRK;
    if (paths > 0x7FFFFFFFll) return HC_ERROR_INVALID_VALUE;
    hipStream_t s = (hipStream_t)stream;
    Workspace *ws = (Workspace *)workspace;
    (void)hipGetLastError();  // errors of earlier, unrelated calls are not ours
    KArgs k{};
    k.num_paths = (int)paths;
    // abort mode dequeues sample-major, so whole hypotheses finish as early as possible
    k.ordered = abort_mode ? 0 : 1;
    k.truncate = truncate ? 1 : 0;
    k.explicit_rk = explicit_rk ? 1 : 0;
    k.max_steps = t->settings.max_steps;
    k.max_corr = t->settings.max_corrections;
    k.inc_steps = t->settings.delta_t_inc_steps;
    k.start_sols = (const cf *)t->start_sols;
    k.start_sols_array = (const cf *const *)t->start_sols_array;
    k.tracks = (cf *)t->tracks;
    k.track_array = (cf *const *)t->track_array;
    k.start_params = (const cf *)t->start_params;
    k.target_params = (const cf *)t->target_params;
    k.diff_params = (const cf *)t->diff_params;
    k.conv = t->converge;
    k.inf = t->infinity;
    k.stats = t->stats;
    k.ws = ws;
    // time slicing when the workspace has room for it (hc_trifocal_workspace_size_for) and
    // the step counters fit the suspend block
    // (the suspend blocks' span in ring-entry units, PrepArgs::susp_entry1, is a
    // 32-bit word: slicing only where it fits)
    const size_t susp_end = ring_bytes(ring_entries(paths, t->settings.max_steps)) / 8 + (size_t)paths * SUSP_WORDS;
    if (!abort_mode && SLICE_Q > 0 && wsb >= ws_bytes_for(paths, t->settings.max_steps) &&
        ring_entries(paths, t->settings.max_steps) < 0xFFFFFF00ull && susp_end < (size_t)UINT_MAX &&
        slice_fits(t->settings.max_steps, t->settings.max_corrections, t->settings.delta_t_inc_steps)) {
        char *base = (char *)workspace + ws_bytes_needed();
        k.ring_cap = (unsigned)ring_entries(paths, t->settings.max_steps);
        k.rq = (unsigned *)base;
        k.ring = (unsigned long long *)(base + RQ_WORDS * sizeof(unsigned));
        k.susp = (unsigned long long *)(base + RQ_WORDS * sizeof(unsigned) + ring_bytes(k.ring_cap));
        k.slice_q = SLICE_Q;
        k.ring_test = g_ring_test.load(std::memory_order_relaxed);
    }
    // control block reset, compacted tables (skipped when cached), ring reset
    PrepArgs pa{t->unified_index, ws, abort_mode ? ab->found_trifocal_sols : nullptr,
                abort_mode ? ab->peer_found : nullptr, k.rq, k.ring, k.ring_cap,
                k.rq ? (unsigned)(ring_bytes(k.ring_cap) / 8) : 0u,
                k.rq ? (unsigned)susp_end : 0u};
    hipLaunchKernelGGL(k_prep_tables, dim3(1), dim3(PREP_THREADS), 0, s, pa);
    if (launch_status(HC_ERROR_LAUNCH) != HC_SUCCESS) return HC_ERROR_LAUNCH;
    // term tables read from the workspace (L1/L2).  Tracking: 96 VGPRs, 31 KB
    // LDS per workgroup -> 5 waves/SIMD.  Abort mode: 4 waves/SIMD (the scoring
    // path needs the registers); its tables moved out of the LDS in round 5,
    // where the other waves' LDS traffic was delaying the earliest hypotheses
    // (time to the first pose -2.8 %, profiles/r5q_ttfp_probe.jsonl)
    const bool archived = !truncate || explicit_rk;
    if (abort_mode && archived) return HC_ERROR_INVALID_VALUE;
#ifndef HC_ABORT_GTAB
#define HC_ABORT_GTAB true
#endif
#ifndef HC_ABORT_MINW
#define HC_ABORT_MINW 4
#endif
    const void *kern = abort_mode ? (const void *)k_track<true, HC_ABORT_MINW, HC_ABORT_GTAB>
                       : archived ? (const void *)k_track<false, 5, true, true>
                                  : (const void *)k_track<false, 5, true>;
    // the structure-agnostic twin, enqueued after it: exactly one of the two
    // tracks (EvalTables::lu_struct), the other returns at its first load
    const void *kern_any = abort_mode ? (const void *)k_track<true, HC_ABORT_MINW, HC_ABORT_GTAB, false, false>
                           : archived ? (const void *)k_track<false, 5, true, true, false>
                                      : (const void *)k_track<false, 5, true, false, false>;
#ifndef HC_SMALL_LAUNCH
#define HC_SMALL_LAUNCH 1
#endif
    const int small_mode = g_small_launch.load(std::memory_order_relaxed);
    if (HC_SMALL_LAUNCH && !abort_mode && !archived && small_mode >= 0) {
        // at most half of the throughput kernel's path slots filled, and every
        // path in a slot of the small kernel at once (or forced by the testing
        // hook): the latency-mode instantiations
        const long long slots = 2ll * WAVES_PER_WG * resident_wgs(kern);   // two paths per wave
        const long long small_slots = 2ll * WAVES_PER_WG * resident_wgs((const void *)k_track_small<true>);
        if (small_mode > 0 || (slots > 0 && 2 * paths <= slots && paths <= small_slots)) {
            kern = (const void *)k_track_small<true>;
            kern_any = (const void *)k_track_small<false>;
        }
    }
    const int grid = grid_for((int)((paths + 1) / 2), kern);
    const int grid_any = grid_for((int)((paths + 1) / 2), kern_any);
    if (grid <= 0 || grid_any <= 0) return HC_ERROR_DEVICE;
    if (abort_mode) {
        k.num_edgels = ab->num_triplet_edgels;
        k.inflight_stop = ab->inflight_stop ? 1 : 0;
        k.peer_found = ab->peer_found;
        k.edgels = ab->triplet_edge_locations;
        k.K = ab->intrinsic_matrix;
        k.found_flag = ab->found_trifocal_sols;
        k.batch_index = ab->trifocal_sols_batch_index;
    }
    void *kargs[] = {&k};
    g_last_hip_error = hipLaunchKernel(kern, dim3(grid), dim3(WG_THREADS), kargs, 0, s);
    if (g_last_hip_error != hipSuccess) return HC_ERROR_LAUNCH;
    if (launch_status(HC_ERROR_LAUNCH) != HC_SUCCESS) return HC_ERROR_LAUNCH;
    g_last_hip_error = hipLaunchKernel(kern_any, dim3(grid_any), dim3(WG_THREADS), kargs, 0, s);
    if (g_last_hip_error != hipSuccess) return HC_ERROR_LAUNCH;
    if (launch_status(HC_ERROR_LAUNCH) != HC_SUCCESS) return HC_ERROR_LAUNCH;
    if (k.rq) {   // a suspended path that was never resumed is reported, not left stale
        hipLaunchKernelGGL(k_ring_check, dim3(1), dim3(64), 0, s, ws, (const unsigned *)k.rq);
        return launch_status(HC_ERROR_LAUNCH);
    }
    return HC_SUCCESS;
}

static hcStatus read_control(const void *workspace, Workspace &h) {
    if (hipMemcpy(&h, workspace, 64, hipMemcpyDeviceToHost) != hipSuccess) return HC_ERROR_DEVICE;
    return HC_SUCCESS;
}

// rate of the s_memrealtime counter (hipDeviceAttributeWallClockRate, kHz)
static double wall_clock_hz() {
    int dev = 0, khz = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess ||
        khz <= 0)
        return 100.0e6;   // gfx9: constant 100 MHz
    return (double)khz * 1.0e3;
}

}  // namespace hc

extern "C" {
#ifdef HC_DIAG_PHASES
int hc_diag_phases(unsigned long long *out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(hc::g_diag_phase), sizeof(unsigned long long) * 13) != hipSuccess) return -1;
    if (reset) {
        static const unsigned long long z[13] = {0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(hc::g_diag_phase), z, sizeof(z)) != hipSuccess) return -1;
    }
    return 0;
}
#endif

#ifdef HC_DIAG_LUWORK
int hc_diag_luwork(unsigned long long *out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(hc::g_diag_luwork), sizeof(unsigned long long) * hc::DIAG_LUWORK_WORDS) !=
        hipSuccess)
        return -1;
    if (reset) {
        static const unsigned long long z[hc::DIAG_LUWORK_WORDS] = {0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(hc::g_diag_luwork), z, sizeof(z)) != hipSuccess) return -1;
    }
    return 0;
}
#endif

#ifdef HC_DIAG_LIVE
int hc_diag_live(unsigned long long *out, int reset) {
    constexpr size_t n = sizeof(unsigned long long) * hc::NV * (hc::LIVE_SOLVES + 1);
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(hc::g_diag_live), n) != hipSuccess) return -1;
    if (reset) {
        static const unsigned long long z[hc::NV * (hc::LIVE_SOLVES + 1)] = {0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(hc::g_diag_live), z, n) != hipSuccess) return -1;
    }
    return 0;
}
#endif

size_t hc_trifocal_workspace_size(void) { return hc::ws_bytes_needed(); }

size_t hc_trifocal_workspace_size_for(int sub_ransac_iters) {
    return hc_trifocal_workspace_size_for_steps(sub_ransac_iters, 80);
}

size_t hc_trifocal_workspace_size_for_steps(int sub_ransac_iters, int max_steps) {
    return hc::ws_bytes_for(sub_ransac_iters > 0 ? (long long)sub_ransac_iters * hc::NTRK : 0, max_steps);
}

hcStatus hc_trifocal_2op1p_30x30_track(const hcTrackArgs *args, void *workspace, size_t workspace_bytes,
                                       hcStream stream) {
    return hc::launch_track(args, nullptr, workspace, workspace_bytes, stream, false);
}

hcStatus hc_trifocal_2op1p_30x30_track_abort(const hcTrackArgs *args, const hcAbortArgs *abort_args,
                                             void *workspace, size_t workspace_bytes, hcStream stream) {
    return hc::launch_track(args, abort_args, workspace, workspace_bytes, stream, true);
}

hcStatus hc_trifocal_2op1p_30x30_track_ph_codeopt(const hcTrackArgs *args, void *workspace, size_t workspace_bytes,
                                                  hcStream stream) {
    return hc::launch_track(args, nullptr, workspace, workspace_bytes, stream, false, false);
}

hcStatus hc_trifocal_2op1p_30x30_track_ph(const hcTrackArgs *args, void *workspace, size_t workspace_bytes,
                                          hcStream stream) {
    return hc::launch_track(args, nullptr, workspace, workspace_bytes, stream, false, false, true);
}

hcStatus hc_trifocal_workspace_status(const void *workspace) {
    if (!workspace) return HC_ERROR_INVALID_VALUE;
    hc::Workspace h;
    const hcStatus st = hc::read_control(workspace, h);
    if (st != HC_SUCCESS) return st;
    if (h.status == 0u) return HC_SUCCESS;
    return h.status == (unsigned)HC_ERROR_TABLE ? HC_ERROR_TABLE : HC_ERROR_DEVICE;
}

hcStatus hc_trifocal_read_timings(const void *workspace, double *first_found_seconds) {
    if (!workspace || !first_found_seconds) return HC_ERROR_INVALID_VALUE;
    hc::Workspace h;
    const hcStatus st = hc::read_control(workspace, h);
    if (st != HC_SUCCESS) return st;
    *first_found_seconds = (h.t_found && h.t_start) ? (double)(long long)(h.t_found - h.t_start) / hc::wall_clock_hz() : -1.0;
    return HC_SUCCESS;
}

hcStatus hc_trifocal_read_timestamps(const void *workspace, uint64_t *start_ticks, uint64_t *found_ticks,
                                     double *tick_hz) {
    if (!workspace || !start_ticks || !found_ticks || !tick_hz) return HC_ERROR_INVALID_VALUE;
    hc::Workspace h;
    const hcStatus st = hc::read_control(workspace, h);
    if (st != HC_SUCCESS) return st;
    *start_ticks = h.t_start;
    *found_ticks = h.t_found;
    *tick_hz = hc::wall_clock_hz();
    return HC_SUCCESS;
}

hcStatus hc_cgesv_30x30_batched(int n, const hcComplex *A, const hcComplex *b, hcComplex *x, hcStream stream) {
    if (n < 0 || (n > 0 && (!A || !b || !x))) return HC_ERROR_INVALID_VALUE;
    if (n == 0) return HC_SUCCESS;
    (void)hipGetLastError();
    const int per = 2 * hc::WAVES_PER_WG;
    hipLaunchKernelGGL(hc::k_cgesv, dim3((n + per - 1) / per), dim3(hc::WG_THREADS), 0, (hipStream_t)stream, n,
                       (const hc::cf *)A, (const hc::cf *)b, (hc::cf *)x);
    return hc::launch_status(HC_ERROR_LAUNCH);
}

hcStatus hc_trifocal_eval_batched(int n, const int32_t *unified_index, const hcComplex *x, const hcComplex *p,
                                  const hcComplex *d, hcComplex *Hx, hcComplex *Ht, hcComplex *H, void *workspace,
                                  size_t workspace_bytes, hcStream stream) {
    if (n < 0 || !unified_index || (n > 0 && (!x || !p || !d || !Hx || !Ht || !H))) return HC_ERROR_INVALID_VALUE;
    if (!workspace || workspace_bytes < hc::ws_bytes_needed()) return HC_ERROR_WORKSPACE;
    if (n == 0) return HC_SUCCESS;
    hipStream_t s = (hipStream_t)stream;
    hc::Workspace *ws = (hc::Workspace *)workspace;
    (void)hipGetLastError();
    hc::PrepArgs pa{unified_index, ws, nullptr, nullptr, nullptr, nullptr, 0u, 0u, 0u};
    hipLaunchKernelGGL(hc::k_prep_tables, dim3(1), dim3(hc::PREP_THREADS), 0, s, pa);
    if (hc::launch_status(HC_ERROR_LAUNCH) != HC_SUCCESS) return HC_ERROR_LAUNCH;
    const int per = 2 * hc::WAVES_PER_WG;
    hipLaunchKernelGGL(hc::k_eval, dim3((n + per - 1) / per), dim3(hc::WG_THREADS), 0, s, n, ws,
                       (const hc::cf *)x, (const hc::cf *)p, (const hc::cf *)d, (hc::cf *)Hx, (hc::cf *)Ht,
                       (hc::cf *)H);
    return hc::launch_status(HC_ERROR_LAUNCH);
}

const char *hc_last_error_string(void) { return hipGetErrorString(hc::g_last_hip_error); }

static_assert(sizeof(hcIpcHandle) == sizeof(hipIpcMemHandle_t), "hcIpcHandle mirrors hipIpcMemHandle_t");

namespace hc {
// memory kind of each flag this process created (hc_shared_flag_memory_kind)
static std::mutex g_flag_mu;
static std::map<const void *, int> g_flag_kind;
}  // namespace hc

// The flag is polled by running kernels of other devices (system-scope loads
// and stores over xGMI), so it is allocated where HIP specifies cross-agent
// coherence while kernels run: uncached device memory first (every access
// goes to the owner's memory), fine-grained memory next, plain
// (coarse-grained, coherent only at synchronisation points) as the last
// resort -- each only if it can be exported with hipIpcGetMemHandle.
hcStatus hc_shared_flag_create(uint32_t **flag, hcIpcHandle *handle) {
    if (!flag || !handle) return HC_ERROR_INVALID_VALUE;
    static const unsigned kinds[3] = {hipDeviceMallocUncached, hipDeviceMallocFinegrained, hipDeviceMallocDefault};
    hipError_t last = hipSuccess;
    for (int k = 0; k < 3; k++) {
        void *p = nullptr;
        last = (kinds[k] == hipDeviceMallocDefault) ? hipMalloc(&p, 256) : hipExtMallocWithFlags(&p, 256, kinds[k]);
        if (last != hipSuccess) { (void)hipGetLastError(); continue; }
        hipIpcMemHandle_t h;
        if ((last = hipMemset(p, 0, 256)) != hipSuccess || (last = hipDeviceSynchronize()) != hipSuccess ||
            (last = hipIpcGetMemHandle(&h, p)) != hipSuccess) {
            (void)hipGetLastError();
            (void)hipFree(p);
            continue;
        }
        memcpy(handle, &h, sizeof(h));
        *flag = (uint32_t *)p;
        std::lock_guard<std::mutex> g(hc::g_flag_mu);
        hc::g_flag_kind[p] = 2 - k;
        return HC_SUCCESS;
    }
    hc::g_last_hip_error = last;
    return HC_ERROR_DEVICE;
}

int hc_shared_flag_memory_kind(const uint32_t *flag) {
    std::lock_guard<std::mutex> g(hc::g_flag_mu);
    const auto it = hc::g_flag_kind.find(flag);
    return it == hc::g_flag_kind.end() ? -1 : it->second;
}

hcStatus hc_shared_flag_open(const hcIpcHandle *handle, uint32_t **flag) {
    if (!flag || !handle) return HC_ERROR_INVALID_VALUE;
    hipIpcMemHandle_t h;
    memcpy(&h, handle, sizeof(h));
    void *p = nullptr;
    if ((hc::g_last_hip_error = hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess)) != hipSuccess)
        return HC_ERROR_DEVICE;
    *flag = (uint32_t *)p;
    return HC_SUCCESS;
}

hcStatus hc_shared_flag_reset(uint32_t *flag, hcStream stream) {
    if (!flag) return HC_ERROR_INVALID_VALUE;
    if ((hc::g_last_hip_error = hipMemsetAsync(flag, 0, sizeof(uint32_t), (hipStream_t)stream)) != hipSuccess)
        return HC_ERROR_LAUNCH;
    return HC_SUCCESS;
}

hcStatus hc_shared_flag_close(uint32_t *flag, int opened) {
    if (!flag) return HC_ERROR_INVALID_VALUE;
    if (!opened) {
        std::lock_guard<std::mutex> g(hc::g_flag_mu);
        hc::g_flag_kind.erase(flag);
    }
    hc::g_last_hip_error = opened ? hipIpcCloseMemHandle(flag) : hipFree(flag);
    return hc::g_last_hip_error == hipSuccess ? HC_SUCCESS : HC_ERROR_DEVICE;
}

#ifdef HC_DIAG_TIMES
int hc_diag_span(unsigned long long *out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(hc::g_diag_span), sizeof(unsigned long long) * 4) != hipSuccess) return -1;
    if (reset) {
        static const unsigned long long z[4] = {~0ull, 0ull, 0ull, 0ull};
        if (hipMemcpyToSymbol(HIP_SYMBOL(hc::g_diag_span), z, sizeof(z)) != hipSuccess) return -1;
    }
    return 0;
}
#endif
#ifdef HC_DIAG_UTIL
int hc_diag_util(unsigned long long *out, int reset) {
    const size_t n = sizeof(unsigned long long) * 2 * hc::UTIL_BINS * hc::UTIL_COPIES;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(hc::g_diag_util), n) != hipSuccess) return -1;
    if (reset) {
        void *p = nullptr;
        if (hipGetSymbolAddress(&p, HIP_SYMBOL(hc::g_diag_util)) != hipSuccess || hipMemset(p, 0, n) != hipSuccess) return -1;
    }
    return 0;
}
#endif

int hc_trifocal_abi_version(void) { return HC_TRIFOCAL_ABI_VERSION; }

// tests only (include/hc_trifocal_testing.h): the tracker LU's structural
// patterns and column-group classes (hc_lu.hpp)
unsigned hc_lu_struct_pattern(int row) { return row >= 0 && row < hc::NV ? hc::LU_STRUCT_PAT[row] : 0u; }
unsigned hc_lu_candidates(int step) { return step >= 0 && step < hc::NV ? hc::LU_BOUND.cand[step] : 0u; }
int hc_lu_search_span(int step) { return step >= 0 && step < hc::NV ? hc::lu_search_span(step) : -1; }
int hc_lu_group_class(int step, int group) {
    if (step < 0 || step >= hc::NV - 1 || group < 0 || group >= hc::LuChunks<2>::count(step)) return -1;
    return hc::lu_group_class<2>(step, group);
}

hcStatus hc_trifocal_ring_check_test(void *workspace, size_t workspace_bytes, unsigned head, unsigned tail,
                                     unsigned avail, hcStream stream) {
    if (!workspace || workspace_bytes < hc::ws_bytes_needed() + hc::RQ_WORDS * sizeof(unsigned))
        return HC_ERROR_WORKSPACE;
    hipStream_t s = (hipStream_t)stream;
    unsigned *rq = (unsigned *)((char *)workspace + hc::ws_bytes_needed());
    const unsigned v[3] = {head, tail, avail};
    const int at[3] = {hc::RQ_HEAD, hc::RQ_TAIL, hc::RQ_AVAIL};
    (void)hipGetLastError();
    for (int i = 0; i < 3; i++)
        if ((hc::g_last_hip_error = hipMemcpyAsync(rq + at[i], &v[i], sizeof(unsigned), hipMemcpyHostToDevice, s)) !=
            hipSuccess)
            return HC_ERROR_LAUNCH;
    if ((hc::g_last_hip_error = hipStreamSynchronize(s)) != hipSuccess) return HC_ERROR_DEVICE;
    hipLaunchKernelGGL(hc::k_ring_check, dim3(1), dim3(64), 0, s, (hc::Workspace *)workspace, (const unsigned *)rq);
    return hc::launch_status(HC_ERROR_LAUNCH);
}

void hc_trifocal_set_ring_test(int delay_ticks) {
    hc::g_ring_test.store(delay_ticks > 0 ? (delay_ticks < HC_RING_TEST_MIN_TICKS ? HC_RING_TEST_MIN_TICKS : delay_ticks)
                                          : 0,
                          std::memory_order_relaxed);
}

void hc_trifocal_set_small_launch(int mode) {
    hc::g_small_launch.store(mode < 0 ? -1 : mode > 0 ? 1 : 0, std::memory_order_relaxed);
}

const char *hc_trifocal_version(void) {
    return "hc_trifocal gfx950 v10.7 (2 paths/wave, structurally sparse LDS-broadcast LU with lean pivot steps, "
           "one exec region per pivot step for the eligible rows with the column groups through scratch windows, "
           "column groups by structural class (never-fillable groups untested, always-live groups unconditional), "
           "pivot search narrowed to the candidate rows' DPP group "
           "(abort kernel and tracking launches filling at most half of the path slots -- the latter at 3 waves/SIMD, "
           "16 columns per batch: batched latency mode, one LDS round trip per pivot step, every live-able column "
           "group untested), "
           "structure-agnostic twin kernels for other dH/dx structures, readlane back substitution, pipelined evals over "
           "per-slot prefix tables, 5 waves/SIMD, time slicing at step boundaries with least-attained-service "
           "issue priority)";
}

}  // extern "C"
