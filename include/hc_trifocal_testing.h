/* hc_trifocal_testing.h -- test hooks of libhc_trifocal.so, apart from the
   public ABI (include/hc_trifocal.h) so that no product caller binds them
   (ADVICE r4).  No reference counterpart. */
#ifndef HC_TRIFOCAL_TESTING_H
#define HC_TRIFOCAL_TESTING_H

#include "hc_trifocal.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Every 16th ring ticket of later sliced launches in this process waits
   delay_ticks (device clock ticks, 100 MHz) between its ticket and its entry,
   and consumers abandon a ticket after delay_ticks / 8 instead of 1 ms, so that
   the abandon / re-push hand-over of time slicing runs.  0 (or a negative
   value) restores the default; positive values are raised to at least
   HC_RING_TEST_MIN_TICKS, so that consumers wait a few hundred ticks and a
   stray call cannot make them abandon every ticket.  Read at launch time. */
#define HC_RING_TEST_MIN_TICKS 4096
void hc_trifocal_set_ring_test(int delay_ticks);

/* Which instantiation a tracking launch (hc_trifocal_2op1p_30x30_track) runs:
   0 (the default) the latency-mode kernel when the launch fills at most half
   of the device's path slots, the throughput kernel otherwise; 1 always the
   latency-mode kernel; -1 never.  The results are the same bit for bit; only
   the speed differs.  Read at launch time. */
void hc_trifocal_set_small_launch(int mode);

/* The end-of-launch ring check of a sliced launch (k_ring_check) on ring
   counters set by hand: head, tail and avail are written into the workspace's
   time-slicing area (workspace_bytes must cover the workspace and the ring
   counters), then the check runs on `stream`.  head != tail or avail != 0 --
   a suspended path never resumed -- sets HC_ERROR_DEVICE
   (hc_trifocal_workspace_status) with ring_fail = (~0, avail, tail, head) in
   the control block.  Blocks until the counters are written. */
hcStatus hc_trifocal_ring_check_test(void *workspace, size_t workspace_bytes, unsigned head, unsigned tail,
                                     unsigned avail, hcStream stream);

/* The tracker LU's compiled-in structure (hc_lu.hpp): row `row`'s structural
   pattern of trifocal_2op1p_30x30's dH/dx (bit c: entry (row, c) has terms),
   and the class of column group `group` of pivot step `step` (groups of 2
   after a leading single column when step + 1 is odd): 0 tested, 1 dead (the
   symbolic fill-in bound excludes it), 2 always run; -1 out of range. */
unsigned hc_lu_struct_pattern(int row);
int hc_lu_group_class(int step, int group);
/* The rows that may hold column `step` at that pivot step under the fill-in
   bound (bit r: row r), and the DPP span the tracker's pivot search reduces
   over there: 1 a quad, 2 a half-row, 3 a 16-lane row, 4 the half-wave;
   0 / -1 out of range. */
unsigned hc_lu_candidates(int step);
int hc_lu_search_span(int step);

#ifdef __cplusplus
}
#endif
#endif /* HC_TRIFOCAL_TESTING_H */
