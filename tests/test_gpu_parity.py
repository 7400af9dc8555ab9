"""GPU parity tests: the HIP kernels (through the C-ABI) against the C oracle.

Bar: identical values -- the kernel and the oracle implement the same
op-level spec, so every float must match exactly, treating +0 == -0 and
NaN == NaN; converged / infinity flags and step / correction counts identical.
"""
import contextlib
import ctypes
import os

import numpy as np
import pytest

from conftest import same

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

# Tracking launches run the latency-mode kernel (k_track_small) when they fill
# at most half of the path slots (N <= 16 samples), the throughput kernel
# (k_track) otherwise; the tests below run each size through both
# (hc_trifocal_set_small_launch: 0 by size, 1 always small, -1 never).
KERNEL_BY_SIZE, SMALL_ALWAYS, SMALL_NEVER = 0, 1, -1


@contextlib.contextmanager
def small_launch(L, mode):
    L.hc_trifocal_set_small_launch(mode)
    try:
        yield
    finally:
        L.hc_trifocal_set_small_launch(KERNEL_BY_SIZE)


def _jacobians_from_path(problem, oracle, tgt, dif, n=64, seed=1):
    """Realistic (x, p, d) points: start solutions pushed along t with random noise."""
    rng = np.random.default_rng(seed)
    xs, ps, ds = [], [], []
    for i in range(n):
        k = int(rng.integers(0, 312))
        s = int(rng.integers(0, tgt.shape[0]))
        x = problem.start_sols[k].copy()
        x[:30] += (rng.standard_normal((30, 2)) * 10 ** rng.uniform(-4, -1)).astype(np.float32)
        t = float(np.float32(rng.uniform(0, 1)))
        xs.append(x)
        ps.append(oracle.param_homotopy(t, problem.start_params, tgt[s]))
        ds.append(dif[s])
    return np.stack(xs), np.stack(ps), np.stack(ds)


def test_eval_matches_oracle(problem, oracle, samples100):
    from trifocal_pose_estimation_using_improved_gpuhc_amd.tracker import eval_batched
    tgt, dif, _ = samples100
    X, P, D = _jacobians_from_path(problem, oracle, tgt, dif, n=256)
    HX, HT, H = eval_batched(problem.unified_index, X, P, D)
    for i in range(X.shape[0]):
        A = oracle.eval_hx(problem.dHdx_index, X[i], P[i])
        assert same(HX[i], A).all(), f"dH/dx mismatch at point {i}"
        assert same(HT[i], oracle.eval_ht(problem.dHdt_index, X[i], P[i], D[i])).all(), f"dH/dt mismatch {i}"
        assert same(H[i], oracle.eval_h(problem.dHdt_index, X[i], P[i])).all(), f"H mismatch {i}"


def test_eval_golden_kat(problem):
    from trifocal_pose_estimation_using_improved_gpuhc_amd.tracker import eval_batched
    g = np.load(os.path.join(GOLDEN, "kat_eval.npz"))
    HX, HT, H = eval_batched(problem.unified_index, g["x"][None], g["p"][None], g["d"][None])
    assert same(HX[0], g["Hx"]).all() and same(HT[0], g["Ht"]).all() and same(H[0], g["H"]).all()


def test_cgesv_matches_oracle_on_jacobians(problem, oracle, samples100):
    from trifocal_pose_estimation_using_improved_gpuhc_amd.tracker import cgesv_batched
    tgt, dif, _ = samples100
    X, P, D = _jacobians_from_path(problem, oracle, tgt, dif, n=256, seed=3)
    As = np.stack([oracle.eval_hx(problem.dHdx_index, X[i], P[i]) for i in range(X.shape[0])])
    bs = np.stack([oracle.eval_ht(problem.dHdt_index, X[i], P[i], D[i]) for i in range(X.shape[0])])
    xg = cgesv_batched(As, bs)
    for i in range(As.shape[0]):
        xr = oracle.cgesv_gpu(As[i], bs[i])
        assert same(xg[i], xr).all(), f"LU mismatch on system {i}"


def test_cgesv_edge_cases(oracle):
    """Random dense, exact ties in the pivot column, a zero column (zero pivot)
    and a NaN entry: the kernel follows dev-cgesv-batched-small.cuh semantics."""
    from trifocal_pose_estimation_using_improved_gpuhc_amd.tracker import cgesv_batched
    rng = np.random.default_rng(11)
    n = 64
    A = rng.standard_normal((n, 30, 30, 2)).astype(np.float32)
    b = rng.standard_normal((n, 30, 2)).astype(np.float32)
    A[1, :, 0, :] = 1.0              # every row ties in column 0
    A[2, :, :, :] = np.round(A[2])   # many exact ties throughout
    A[3, :, 5, :] = 0.0              # zero column -> zero pivot at step 5
    A[4, 7, 3, 0] = np.nan           # NaN in the matrix
    A[5, :, :, :] = 0.0              # fully singular
    xg = cgesv_batched(A, b)
    for i in range(n):
        xr = oracle.cgesv_gpu(A[i], b[i])
        assert same(xg[i], xr).all(), f"edge-case LU mismatch on system {i}"
    # well-conditioned systems also solve the linear system
    Ac = A[8:, ..., 0] + 1j * A[8:, ..., 1]
    bc = b[8:, ..., 0] + 1j * b[8:, ..., 1]
    xc = xg[8:, ..., 0] + 1j * xg[8:, ..., 1]
    res = np.abs(np.einsum("nij,nj->ni", Ac, xc) - bc).max(axis=1) / np.abs(bc).max(axis=1)
    assert np.median(res) < 1e-4


def test_cgesv_extreme_scales(problem, oracle, samples100):
    """Every exit of the v9 LU's fast pivot step (hc_lu.hpp): pivots below 2^-90
    and at/above 2^120, entries at/above 2^88 (the whole solve runs dense), an
    infinity, NaN at the pivot position, denormals, and structurally sparse
    tracker Jacobians at those scales -- bit-exact against the oracle."""
    from trifocal_pose_estimation_using_improved_gpuhc_amd.tracker import cgesv_batched
    tgt, dif, _ = samples100
    X, P, D = _jacobians_from_path(problem, oracle, tgt, dif, n=8, seed=5)
    J = np.stack([oracle.eval_hx(problem.dHdx_index, X[i], P[i]) for i in range(8)])
    bJ = np.stack([oracle.eval_ht(problem.dHdt_index, X[i], P[i], D[i]) for i in range(8)])
    rng = np.random.default_rng(12)
    As, bs = [], []
    for scale in (2.0 ** -100, 2.0 ** -60, 2.0 ** 60, 2.0 ** 90, 2.0 ** 121):
        for i in range(4):
            As.append((J[i] * np.float32(scale)).astype(np.float32))
            bs.append(bJ[i])
    A = rng.standard_normal((6, 30, 30, 2)).astype(np.float32)
    A[0, 4, 4, :] = np.float32(2.0 ** -95)        # tiny diagonal, large elsewhere in column
    A[0, :, 4, :] *= np.float32(2.0 ** -100)      # whole column tiny -> tiny pivot
    A[1, 2, 7, 0] = np.inf                        # an infinity
    A[2, :, :, :] = np.diag(np.full(30, np.nan, np.float32))[..., None]   # NaN on the diagonal...
    A[2, :, :, :] += rng.standard_normal((30, 30, 2)).astype(np.float32)  # ...plus finite noise
    A[3, :, :, :] *= np.float32(1e-40)            # denormals
    A[4, 9, 9, :] = np.float32(2.0 ** 125)        # one huge entry
    A[5, :, 0, :] = 0.0
    A[5, 3, 0, :] = np.float32(2.0 ** -126)       # smallest normal as the only pivot candidate
    As.extend(A)
    bs.extend(rng.standard_normal((6, 30, 2)).astype(np.float32))
    As, bs = np.stack(As), np.stack(bs)
    xg = cgesv_batched(As, bs)
    for i in range(As.shape[0]):
        xr = oracle.cgesv_gpu(As[i], bs[i])
        assert same(xg[i], xr).all(), f"extreme-scale LU mismatch on system {i}"


@pytest.mark.parametrize("mode", [KERNEL_BY_SIZE, SMALL_NEVER], ids=["latency_kernel", "throughput_kernel"])
def test_tracker_matches_oracle_small(problem, oracle, samples100, tracker, mode):
    """Full GPU-HC tracking of 2 samples (624 paths) vs the oracle, value for value."""
    tgt, dif, _ = samples100
    N = 2
    with small_launch(tracker.L, mode):
        r = tracker.track(tgt[:N], dif[:N]).host()
    tr, conv, inf, st = oracle.gpuhc_track(problem.start_sols, problem.start_params, tgt[:N], dif[:N],
                                           problem.unified_index)
    assert (r["converge"] == conv).all()
    assert (r["infinity"] == inf).all()
    assert (r["stats"]["steps"] == st["steps"]).all()
    assert (r["stats"]["corrections"] == st["corrections"]).all()
    bad = ~same(r["tracks"][:, :30], tr[:, :30]).all(axis=(1, 2))
    assert not bad.any(), f"{bad.sum()} tracks differ, first {np.nonzero(bad)[0][:5]}"
    # x[30] is never written by the kernel (reference :282 writes tx < 30 only)
    assert (r["tracks"][:, 30, 0] == 1.0).all()


@pytest.mark.parametrize("mode", [KERNEL_BY_SIZE, SMALL_NEVER], ids=["latency_kernel", "throughput_kernel"])
def test_tracker_dense_resolve_matches_oracle(problem, oracle, samples100, tracker, mode):
    """The tracker's dense re-solve (hc_lu.hpp lu_solve<true>, taken when a
    Jacobian entry reaches 2^64 or a pivot leaves the fast-reciprocal range):
    config 2 never takes it (profiles/r3e_lu_work.json), so this run forces it.
    Sample 0 is config 2's, samples 1 and 2 have their target parameters scaled
    by 2^40 and 2^70: their Jacobians pass 2^64 within the first steps (2^70:
    at t = 0.01 already, max |entry| 7.5e36) and most paths run to infinity.
    Because the dequeue is track-major, waves pair a normal path with a scaled
    one, so a normal half is re-solved densely beside a scaled half (the redo is
    wave-uniform) and must come out identical.  Bit-exact against the oracle."""
    tgt, dif, _ = samples100
    T = [tgt[0]]
    for sc in (2.0 ** 40, 2.0 ** 70):
        T.append((tgt[0] * np.float32(sc)).astype(np.float32))
    T = np.stack(T)
    D = (T - problem.start_params[None]).astype(np.float32)   # prepare_target_params' diff
    assert np.array_equal(D[0], dif[0])
    with small_launch(tracker.L, mode):
        r = tracker.track(T, D).host()
    tr, conv, inf, st = oracle.gpuhc_track(problem.start_sols, problem.start_params, T, D, problem.unified_index)
    assert (r["converge"] == conv).all() and (r["infinity"] == inf).all()
    assert (r["stats"]["steps"] == st["steps"]).all()
    assert (r["stats"]["corrections"] == st["corrections"]).all()
    bad = ~same(r["tracks"][:, :30], tr[:, :30]).all(axis=(1, 2))
    assert not bad.any(), f"{bad.sum()} tracks differ, first {np.nonzero(bad)[0][:5]}"
    assert inf[312:].sum() > 600 and conv[:312].sum() > 0   # the scaled samples diverge, sample 0 converges


def test_tracker_dense_resolve_abort_mode(problem, oracle, samples100, tracker):
    """The dense re-solve in the abort kernel (its latency-mode LU with the
    always-live column groups in pairs, then lu_solve<true>): the
    2^40- and 2^70-scaled samples first, so that all 936 paths are dequeued
    before any hypothesis can pass, then config 2's sample 0.  Every tracked
    path equals the oracle's abort-off run bit for bit."""
    tgt, dif, _ = samples100
    T = np.stack([(tgt[0] * np.float32(2.0 ** 40)).astype(np.float32),
                  (tgt[0] * np.float32(2.0 ** 70)).astype(np.float32), tgt[0]])
    D = (T - problem.start_params[None]).astype(np.float32)
    r = tracker.track(T, D, abort=True).host()
    tracker.workspace_status()
    tr, conv, inf, st = oracle.gpuhc_track(problem.start_sols, problem.start_params, T, D, problem.unified_index)
    tracked = r["stats"]["steps"] > 0
    assert tracked[:624].all(), "the scaled samples' paths must all be tracked"
    assert (r["converge"][tracked] == conv[tracked]).all() and (r["infinity"][tracked] == inf[tracked]).all()
    assert (r["stats"]["steps"][tracked] == st["steps"][tracked]).all()
    assert (r["stats"]["corrections"][tracked] == st["corrections"][tracked]).all()
    assert same(r["tracks"][tracked][:, :30], tr[tracked][:, :30]).all()
    assert inf[:624].sum() > 600


@pytest.mark.parametrize("mode", [KERNEL_BY_SIZE, SMALL_ALWAYS], ids=["throughput_kernel", "latency_kernel"])
def test_tracker_matches_golden_N100(problem, samples100, tracker, mode):
    """Config 2 (100 samples, abort off): every flag / count / track hash equals the committed golden run."""
    import sys
    sys.path.insert(0, GOLDEN)
    from make_golden import track_hash
    g = np.load(os.path.join(GOLDEN, "gpuhc_N100_seed0.npz"))
    tgt, dif, _ = samples100
    with small_launch(tracker.L, mode):
        r = tracker.track(tgt, dif).host()
    assert (r["converge"] == g["conv"]).all()
    assert (r["infinity"] == g["inf"]).all()
    assert (r["stats"]["steps"] == g["steps"]).all()
    assert (r["stats"]["corrections"] == g["corrections"]).all()
    h = track_hash(r["tracks"])
    assert (h == g["hash"]).all(), f"{(h != g['hash']).sum()} track hashes differ"
    from trifocal_pose_estimation_using_improved_gpuhc_amd import count_solutions
    assert tuple(g["counts"]) == count_solutions(r["tracks"], r["converge"], r["infinity"])
    # per-path real flags: the input of the prefix pin against the reference's
    # GPU_Sols_Statistics.txt (272 / 5; test_oracle_kat.py)
    real = ((np.abs(r["tracks"][:, :30, 1]).astype(np.float64) <= 1e-4).all(axis=1) & (r["converge"] != 0))
    assert np.array_equal(real.astype(np.uint8), g["real"])
    cc, cr = np.cumsum(r["converge"].astype(np.int64)), np.cumsum(real.astype(np.int64))
    assert (cc[2971:3006] == 272).all() and (cr[2971:3006] == 5).all()


def test_time_slicing_is_bit_exact(problem, samples100, tracker):
    """Time slicing (paths suspended at step boundaries and resumed by any slot,
    hc_trifocal_workspace_size_for) changes when a path runs, never what it
    computes: the config-2 run with and without it agree bit for bit (sign of
    zero and NaN payloads included), and the sliced run did suspend paths."""
    tgt, dif, _ = samples100
    a = tracker.track(tgt, dif, time_slicing=False).host()
    b = tracker.track(tgt, dif, time_slicing=True).host()
    # ring counters after the base workspace (hc_kernels.hip KArgs::rq): [0] head, [64] tail, [128] avail
    off = int(tracker.L.hc_trifocal_workspace_size())
    rq = np.frombuffer(tracker.workspace[off:off + 768].cpu().numpy().tobytes(), np.uint32)
    assert rq[64] > 1000, f"only {rq[64]} suspensions"
    assert rq[0] == rq[64] and rq[128] == 0, "every suspended path was resumed"
    assert (a["converge"] == b["converge"]).all() and (a["infinity"] == b["infinity"]).all()
    assert np.array_equal(a["stats"]["steps"], b["stats"]["steps"])
    assert np.array_equal(a["stats"]["corrections"], b["stats"]["corrections"])
    assert np.array_equal(a["tracks"].view(np.uint32), b["tracks"].view(np.uint32))


def test_time_slicing_concurrent_streams(problem, samples100, tracker):
    """Four sliced launches in flight at once on four streams (own buffers and
    workspaces, the bench's pipelined leg): the suspend / resume hand-over of
    each launch stays inside its own workspace, and every launch equals the
    serial run bit for bit."""
    import torch
    tgt, dif, _ = samples100
    ref = tracker.track(tgt, dif).host()
    dev = tracker.device
    t, d = torch.from_numpy(tgt).to(dev), torch.from_numpy(dif).to(dev)
    streams = [torch.cuda.Stream(dev) for _ in range(4)]
    bufs = [tracker.allocate(tgt.shape[0]) for _ in range(4)]
    wss = [tracker.new_workspace(tgt.shape[0]) for _ in range(4)]
    torch.cuda.synchronize(dev)
    for k in range(4):
        with torch.cuda.stream(streams[k]):
            tracker.reset_tracks(bufs[k])
        tracker.launch(t, d, bufs[k], stream=streams[k], workspace=wss[k])
    torch.cuda.synchronize(dev)
    for k in range(4):
        h = bufs[k].host()
        assert int(tracker.L.hc_trifocal_workspace_status(ctypes.c_void_p(wss[k].data_ptr()))) == 0
        assert (h["converge"] == ref["converge"]).all() and (h["infinity"] == ref["infinity"]).all()
        assert np.array_equal(h["stats"]["steps"], ref["stats"]["steps"])
        assert np.array_equal(h["tracks"].view(np.uint32), ref["tracks"].view(np.uint32))


def test_small_and_large_launches_share_a_workspace(problem, samples100, tracker):
    """One workspace, launches of 100, 8, 100 and 2 samples: the launcher
    alternates between the throughput kernel (k_track) and the latency-mode
    one (k_track_small), which keep the same control block, tables and ring;
    then four 8-sample launches in flight at once on four streams (own
    buffers and workspaces).  Every launch equals the serial run bit for bit."""
    import torch
    tgt, dif, _ = samples100
    ref = tracker.track(tgt, dif, time_slicing=False).host()
    dev = tracker.device
    t, d = torch.from_numpy(tgt).to(dev), torch.from_numpy(dif).to(dev)

    def check(h, n):
        sl = slice(0, n * 312)
        assert (h["converge"] == ref["converge"][sl]).all() and (h["infinity"] == ref["infinity"][sl]).all()
        assert np.array_equal(h["stats"]["steps"], ref["stats"]["steps"][sl])
        assert np.array_equal(h["tracks"].view(np.uint32), ref["tracks"][sl].view(np.uint32))

    ws = tracker.new_workspace(100)
    for n in (100, 8, 100, 2):
        r = tracker.allocate(n)
        tracker.reset_tracks(r)
        tracker.launch(t, d, r, workspace=ws, num_samples=n)
        torch.cuda.synchronize(dev)
        assert int(tracker.L.hc_trifocal_workspace_status(ctypes.c_void_p(ws.data_ptr()))) == 0
        check(r.host(), n)
    streams = [torch.cuda.Stream(dev) for _ in range(4)]
    bufs = [tracker.allocate(8) for _ in range(4)]
    wss = [tracker.new_workspace(8) for _ in range(4)]
    torch.cuda.synchronize(dev)
    for k in range(4):
        with torch.cuda.stream(streams[k]):
            tracker.reset_tracks(bufs[k])
        tracker.launch(t, d, bufs[k], stream=streams[k], workspace=wss[k], num_samples=8)
    torch.cuda.synchronize(dev)
    for k in range(4):
        assert int(tracker.L.hc_trifocal_workspace_status(ctypes.c_void_p(wss[k].data_ptr()))) == 0
        check(bufs[k].host(), 8)


def test_time_slicing_falls_back_when_the_ring_does_not_fit(problem, samples100, tracker):
    """A workspace sized for a smaller GPUHC_Max_Steps than the launch uses
    (hc_trifocal_workspace_size_for_steps) cannot hold one ring entry per
    possible suspension: the launch runs unsliced (ring counters untouched)
    and still equals the serial run bit for bit."""
    import torch
    tgt, dif, _ = samples100
    ref = tracker.track(tgt, dif).host()
    dev = tracker.device
    small = int(tracker.L.hc_trifocal_workspace_size_for_steps(tgt.shape[0], 10))
    assert small < int(tracker.L.hc_trifocal_workspace_size_for_steps(tgt.shape[0], tracker.settings.max_steps))
    ws = torch.zeros(small, dtype=torch.uint8, device=dev)
    r = tracker.allocate(tgt.shape[0])
    tracker.reset_tracks(r)
    tracker.launch(torch.from_numpy(tgt).to(dev), torch.from_numpy(dif).to(dev), r, workspace=ws)
    torch.cuda.synchronize(dev)
    off = int(tracker.L.hc_trifocal_workspace_size())
    rq = np.frombuffer(ws[off:off + 768].cpu().numpy().tobytes(), np.uint32)
    assert rq[64] == 0, "a launch whose ring does not fit must not slice"
    h = r.host()
    assert (h["converge"] == ref["converge"]).all()
    assert np.array_equal(h["tracks"].view(np.uint32), ref["tracks"].view(np.uint32))


def test_time_slicing_workspace_reused_across_launch_sizes(problem, samples100, tracker):
    """One workspace, sliced launches of 100, then 50, then 100 samples: the
    ring sits at a fixed offset, so the 50-sample launch meets only entries
    tagged by an older epoch; its suspend blocks follow its ring and overwrite
    cleared entries, which it records as the dirty range, and the second
    100-sample launch re-zeroes them.  (50 samples: 15 600 paths,
    more than the 10 240 path slots of a full grid, so that launch suspends
    paths too.)  Every launch equals the serial run bit for bit."""
    import torch
    tgt, dif, _ = samples100
    ref = tracker.track(tgt, dif, time_slicing=False).host()
    dev = tracker.device
    t, d = torch.from_numpy(tgt).to(dev), torch.from_numpy(dif).to(dev)
    ws = tracker.new_workspace(100)
    off = int(tracker.L.hc_trifocal_workspace_size())
    for n in (100, 50, 100):
        r = tracker.allocate(n)
        tracker.reset_tracks(r)
        tracker.launch(t, d, r, workspace=ws, num_samples=n)
        torch.cuda.synchronize(dev)
        assert int(tracker.L.hc_trifocal_workspace_status(ctypes.c_void_p(ws.data_ptr()))) == 0
        rq = np.frombuffer(ws[off:off + 1024].cpu().numpy().tobytes(), np.uint32)
        assert rq[64] > 0 and rq[0] == rq[64], "sliced, and every suspended path resumed"
        # RQ_CLEARED: the largest ring so far (one entry per possible suspension + 4096 spare);
        # after the 50-sample launch its suspend blocks lie inside it: the dirty range [195, 196)
        cap = lambda k: k * 312 * ((tracker.settings.max_steps + 1) // 3 + 1) + 4096  # noqa: E731
        assert rq[194] == cap(100)
        if n == 50:
            assert cap(50) <= rq[195] < rq[196] <= cap(100)
        else:
            assert rq[195] == rq[196] == 0
        h = r.host()
        sl = slice(0, n * 312)
        assert (h["converge"] == ref["converge"][sl]).all() and (h["infinity"] == ref["infinity"][sl]).all()
        assert np.array_equal(h["stats"]["steps"], ref["stats"]["steps"][sl])
        assert np.array_equal(h["tracks"].view(np.uint32), ref["tracks"][sl].view(np.uint32))


def test_time_slicing_abandoned_tickets_are_pushed_again(problem, samples100, tracker):
    """A consumer that waits too long for a ring entry abandons the ticket and
    its pusher pushes the path again: no path is lost to a paused wave
    (VERDICT r3 #5).  hc_trifocal_set_ring_test delays every 16th ticket's
    entry by 2 ms and lets consumers abandon after 250 us; the launch abandons
    tickets (control block word 12) and still equals the unsliced run bit for
    bit, with no device error.  (50 samples: more paths than path slots, so
    paths are suspended.)"""
    import torch
    tgt, dif, _ = samples100
    n = 50
    ref = tracker.track(tgt[:n], dif[:n], time_slicing=False).host()
    dev = tracker.device
    ws = tracker.new_workspace(n)
    r = tracker.allocate(n)
    tracker.reset_tracks(r)
    tracker.L.hc_trifocal_set_ring_test(200000)
    try:
        tracker.launch(torch.from_numpy(tgt[:n]).to(dev), torch.from_numpy(dif[:n]).to(dev), r, workspace=ws)
        torch.cuda.synchronize(dev)
    finally:
        tracker.L.hc_trifocal_set_ring_test(0)
    cb = np.frombuffer(ws[:64].cpu().numpy().tobytes(), np.uint32)
    assert int(tracker.L.hc_trifocal_workspace_status(ctypes.c_void_p(ws.data_ptr()))) == 0, cb
    assert cb[12] > 0, "no ticket was abandoned: the test did not reach the re-push"
    h = r.host()
    assert (h["converge"] == ref["converge"]).all() and (h["infinity"] == ref["infinity"]).all()
    assert np.array_equal(h["stats"]["steps"], ref["stats"]["steps"])
    assert np.array_equal(h["tracks"].view(np.uint32), ref["tracks"].view(np.uint32))


def test_tracker_abort_mode(problem, samples100, tracker):
    """Config 3 semantics (abort on): the found hypothesis is one of the passing
    hypotheses of the abort-off run; tracked paths equal the abort-off results;
    skipped paths keep the start solution with conv = 0."""
    import sys
    sys.path.insert(0, GOLDEN)
    from make_golden import track_hash
    g = np.load(os.path.join(GOLDEN, "gpuhc_N100_seed0.npz"))
    passing = set(int(b) for b, s in zip(g["scored_ids"], g["scored"]) if s[0] == 1)
    assert passing, "the golden run must contain a passing hypothesis"
    tgt, dif, _ = samples100
    r = tracker.track(tgt, dif, abort=True).host()
    assert r["found"]
    found_ids = set(int(b) for b in np.nonzero(r["batch_index"] >= 0)[0])
    assert found_ids and found_ids <= passing
    assert all(int(r["batch_index"][b]) == b for b in found_ids)
    st = r["stats"]
    tracked = st["steps"] > 0
    assert (r["converge"][tracked] == g["conv"][tracked]).all()
    assert (track_hash(r["tracks"])[tracked] == g["hash"][tracked]).all()
    skipped = ~tracked
    assert (r["converge"][skipped] == 0).all()
    assert np.array_equal(r["tracks"][skipped][:, :30],
                          np.tile(problem.start_sols[None, :, :30], (100, 1, 1, 1)).reshape(-1, 30, 2)[skipped])
    # inlier counts of scored paths equal the oracle's scoring
    sc = {int(b): s for b, s in zip(g["scored_ids"], g["scored"])}
    for b in np.nonzero(tracked & (r["converge"] == 1))[0]:
        ok, i21, i31 = sc[int(b)]
        if st["inliers21"][b] or st["inliers31"][b] or ok:
            assert (st["inliers21"][b], st["inliers31"][b]) == (i21, i31)
    assert tracker.first_found_seconds() > 0


@pytest.mark.gpu
def test_tracker_abort_chunked(problem, samples100, tracker):
    """The multi-GPU early-stop protocol on one rank: 100 samples in chunks of
    10 launches, one workspace each.  Found ids (made global) are passing
    hypotheses, tracked paths equal the abort-off golden run, and once a chunk
    has found a pose every later chunk skips all of its paths."""
    import sys

    import torch

    from trifocal_pose_estimation_using_improved_gpuhc_amd import sharding
    sys.path.insert(0, GOLDEN)
    from make_golden import track_hash
    g = np.load(os.path.join(GOLDEN, "gpuhc_N100_seed0.npz"))
    passing = set(int(b) for b, s in zip(g["scored_ids"], g["scored"]) if s[0] == 1)
    tgt, dif, _ = samples100
    dev = tracker.device
    t = torch.from_numpy(tgt).to(dev)
    d = torch.from_numpy(dif).to(dev)
    r = tracker.allocate(100, stats=True, abort=True)
    tracker.reset_tracks(r)
    wss = []
    parts = tracker.launch_abort_chunked(t, d, r, chunk_samples=10, workspaces=wss)
    torch.cuda.synchronize(dev)
    h = r.host()
    assert len(parts) == 10 and h["found"]
    found = set()
    for off, n in parts:
        loc = h["batch_index"][off * 312:(off + n) * 312]
        found |= set(int(b) for b in sharding.global_batch_ids(loc, off, 0))
    assert found and found <= passing
    tracked = h["stats"]["steps"] > 0
    assert (h["converge"][tracked] == g["conv"][tracked]).all()
    assert (track_hash(h["tracks"])[tracked] == g["hash"][tracked]).all()
    first_chunk = min(b // 312 for b in found) // 10
    assert not tracked[(first_chunk + 1) * 3120:].any()
    stamps = [tracker.read_timestamps(w)[:2] for w in wss]
    hz = tracker.read_timestamps(wss[0])[2]
    assert sharding.first_found_seconds(stamps, hz) > 0


@pytest.mark.gpu
def test_cli_config2_matches_golden(tmp_path):
    """bin/magmaHC-main (C++ GPU_HC_Solver over the C-ABI) on config 2: the
    solution statistics it writes equal the golden run's counts."""
    import shutil
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cli = os.path.join(root, "trifocal_pose_estimation_using_improved_gpuhc_amd", "bin", "magmaHC-main")
    assert os.path.exists(cli), "CLI not built"
    shutil.copytree(os.path.join(root, "data"), os.path.join(tmp_path, "data"))
    out = subprocess.run([cli, "-p", "trifocal_2op1p_30x30", "-d", str(tmp_path)], capture_output=True, text=True,
                         timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    g = np.load(os.path.join(GOLDEN, "gpuhc_N100_seed0.npz"))
    stats = open(os.path.join(tmp_path, "Output_Write_Files", "GPU_Sols_Statistics.txt")).read().split()
    assert [int(v) for v in stats[:3]] == [int(v) for v in g["counts"]]
    assert float(open(os.path.join(tmp_path, "Output_Write_Files", "GPU_Timings.txt")).read().split()[0]) > 0
    # device pose recovery: the maximal-support pose matches GT_Poses*_000
    pr = open(os.path.join(tmp_path, "Output_Write_Files", "GPU_Pose_Results.txt")).read().split()
    gp = np.load(os.path.join(GOLDEN, "pose_N100_seed0.npz"))
    assert int(pr[0]) == 1 and [int(pr[5]), int(pr[6])] == gp["path"].tolist() and int(pr[7]) == int(gp["num_candidates"])
    assert max(float(v) for v in pr[1:5]) < 1e-3
    # abort mode (config 3 semantics through the CLI)
    out = subprocess.run([cli, "-p", "trifocal_2op1p_30x30", "-d", str(tmp_path), "-n", "1000", "--abort"],
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr


@pytest.mark.gpu
def test_cli_four_rounds(tmp_path):
    """`magmaHC-main -t 4` (TEST_RANSAC_TIMES = 4; cmd/magmaHC-main.cpp:38-48):
    round ti reads Triplet_Edgels_<ti> and GT_Poses*_<ti> and draws its samples
    with srand(ti) (GPU_HC_Solver.cpp:252-306).  Every round writes its timing,
    solution statistics and pose line; every round's counts equal the oracle's
    (tests/golden/cli_rounds_counts.npz)."""
    import shutil
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cli = os.path.join(root, "trifocal_pose_estimation_using_improved_gpuhc_amd", "bin", "magmaHC-main")
    shutil.copytree(os.path.join(root, "data"), os.path.join(tmp_path, "data"))
    out = subprocess.run([cli, "-p", "trifocal_2op1p_30x30", "-d", str(tmp_path), "-t", "4"], capture_output=True,
                         text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    od = os.path.join(tmp_path, "Output_Write_Files")
    ms = [float(v) for v in open(os.path.join(od, "GPU_Timings.txt")).read().split()]
    assert len(ms) == 4 and min(ms) > 0
    stats = [ln.split() for ln in open(os.path.join(od, "GPU_Sols_Statistics.txt")).read().splitlines()]
    assert len(stats) == 4 and all(int(r[0]) > 0 for r in stats)
    g = np.load(os.path.join(GOLDEN, "gpuhc_N100_seed0.npz"))
    assert [int(v) for v in stats[0]] == [int(v) for v in g["counts"]]
    # every round's counts equal the oracle's run of that round's dataset and draw
    rounds = np.load(os.path.join(GOLDEN, "cli_rounds_counts.npz"))["counts"]
    assert [[int(v) for v in r[:3]] for r in stats] == rounds.tolist()
    assert len(open(os.path.join(od, "GPU_Pose_Results.txt")).read().splitlines()) == 4
    assert "Running 4 rounds" in out.stdout


def test_ph_codeopt_matches_oracle_small(problem, oracle, samples100, tracker):
    """The archived ..._PH_CodeOpt semantics (hc_trifocal_2op1p_30x30_track_ph_codeopt:
    no depth-sign truncation) on 2 samples vs the oracle, value for value."""
    tgt, dif, _ = samples100
    N = 2
    r = tracker.track(tgt[:N], dif[:N], truncate=False).host()
    tr, conv, inf, st = oracle.gpuhc_track(problem.start_sols, problem.start_params, tgt[:N], dif[:N],
                                           problem.unified_index, oracle.settings(truncate=False))
    assert (r["converge"] == conv).all() and (r["infinity"] == inf).all()
    assert (r["stats"]["steps"] == st["steps"]).all()
    assert (r["stats"]["corrections"] == st["corrections"]).all()
    assert same(r["tracks"][:, :30], tr[:, :30]).all()


def test_ph_codeopt_matches_golden_N100(problem, samples100, tracker):
    """Config 2 without path truncation: every flag / count / track hash equals the
    oracle's committed run (tests/golden/gpuhc_phcodeopt_N100_seed0.npz)."""
    import sys
    sys.path.insert(0, GOLDEN)
    from make_golden import track_hash
    g = np.load(os.path.join(GOLDEN, "gpuhc_phcodeopt_N100_seed0.npz"))
    tgt, dif, _ = samples100
    r = tracker.track(tgt, dif, truncate=False).host()
    assert (r["converge"] == g["conv"]).all() and (r["infinity"] == g["inf"]).all()
    assert (r["stats"]["steps"] == g["steps"]).all()
    assert (r["stats"]["corrections"] == g["corrections"]).all()
    assert (track_hash(r["tracks"]) == g["hash"]).all()


def test_ph_matches_oracle_small(problem, oracle, samples100, tracker):
    """The archived ..._PH semantics (explicit RK helpers, no truncation;
    hc_trifocal_2op1p_30x30_track_ph) on 2 samples vs the oracle, value for value."""
    tgt, dif, _ = samples100
    N = 2
    r = tracker.track(tgt[:N], dif[:N], truncate=False, explicit_rk=True).host()
    tr, conv, inf, st = oracle.gpuhc_track(problem.start_sols, problem.start_params, tgt[:N], dif[:N],
                                           problem.unified_index, oracle.settings(truncate=False, explicit_rk=True))
    assert (r["converge"] == conv).all() and (r["infinity"] == inf).all()
    assert (r["stats"]["steps"] == st["steps"]).all()
    assert (r["stats"]["corrections"] == st["corrections"]).all()
    assert same(r["tracks"][:, :30], tr[:, :30]).all()


def test_ph_matches_golden_N100(problem, samples100, tracker):
    """Config 2 through the archived ..._PH semantics: every flag / count / track
    hash equals the oracle's committed run (tests/golden/gpuhc_ph_N100_seed0.npz)."""
    import sys
    sys.path.insert(0, GOLDEN)
    from make_golden import track_hash
    g = np.load(os.path.join(GOLDEN, "gpuhc_ph_N100_seed0.npz"))
    tgt, dif, _ = samples100
    r = tracker.track(tgt, dif, truncate=False, explicit_rk=True).host()
    assert (r["converge"] == g["conv"]).all() and (r["infinity"] == g["inf"]).all()
    assert (r["stats"]["steps"] == g["steps"]).all()
    assert (r["stats"]["corrections"] == g["corrections"]).all()
    assert (track_hash(r["tracks"]) == g["hash"]).all()


def _row_permuted(problem, perm):
    """The index tables with the equations (rows) reordered: row r of the new
    system is row perm[r] of the reference's (a valid, equivalent problem)."""
    dx = problem.dHdx_index.reshape(-1, 30)[:, perm].reshape(-1)
    dt = problem.dHdt_index.reshape(-1, 30)[:, perm].reshape(-1)
    return (np.ascontiguousarray(dx, np.int32), np.ascontiguousarray(dt, np.int32),
            np.ascontiguousarray(np.concatenate([dx, dt]), np.int32))


def test_eval_row_permuted_tables_match_oracle(problem, oracle, samples100):
    """The table builder's lane assignments (dH/dx entries bin-packed over the
    32 lanes, the dH/dt | H owner / helper pairs lane ^ 16) for equation orders
    other than the reference's: reversed (the long dH/dt rows land in lanes
    0..11, their helpers in 16..27) and a random order that still pairs every
    long row with a short one."""
    from trifocal_pose_estimation_using_improved_gpuhc_amd.tracker import eval_batched
    tgt, dif, _ = samples100
    X, P, D = _jacobians_from_path(problem, oracle, tgt, dif, n=48, seed=5)
    nt = (problem.dHdt_index.reshape(-1, 30)[::6] != 0).sum(axis=0)   # terms per row (coefficient rows)
    rng = np.random.default_rng(11)
    perms = [np.arange(29, -1, -1)]
    while len(perms) < 2:
        p = rng.permutation(30)
        n = nt[p]
        if all(not (n[r] > 13 and (r ^ 16 >= 30 or n[r ^ 16] > 10)) for r in range(30)):
            perms.append(p)
    for perm in perms:
        dx, dt, U = _row_permuted(problem, perm)
        HX, HT, H = eval_batched(U, X, P, D)
        for i in range(X.shape[0]):
            assert same(HX[i], oracle.eval_hx(dx, X[i], P[i])).all(), f"dH/dx mismatch at point {i}, perm {perm}"
            assert same(HT[i], oracle.eval_ht(dt, X[i], P[i], D[i])).all(), f"dH/dt mismatch {i}, perm {perm}"
            assert same(H[i], oracle.eval_h(dt, X[i], P[i])).all(), f"H mismatch {i}, perm {perm}"


def test_eval_rejects_tables_without_helpers(problem):
    """Two long dH/dt rows paired as lane ^ 16 partners (neither can help the
    other): the table builder rejects the table (HC_ERROR_TABLE) and the
    kernels leave their outputs untouched."""
    import ctypes as C
    import torch
    from trifocal_pose_estimation_using_improved_gpuhc_amd import _abi
    perm = np.arange(30)
    perm[2], perm[19] = 19, 2          # lanes 2 and 18: rows 19 and 18, 16 terms each
    _, _, U = _row_permuted(problem, perm)
    L = _abi.lib()
    dev = torch.device("cuda:0")
    n = 4
    Ut = torch.from_numpy(U).to(dev)
    X = torch.zeros((n, 31, 2), dtype=torch.float32, device=dev)
    P = torch.zeros((n, 34, 2), dtype=torch.float32, device=dev)
    HX = torch.full((n, 30, 30, 2), 7.0, dtype=torch.float32, device=dev)
    HT = torch.full((n, 30, 2), 7.0, dtype=torch.float32, device=dev)
    H = torch.full((n, 30, 2), 7.0, dtype=torch.float32, device=dev)
    wsb = int(L.hc_trifocal_workspace_size())
    ws = torch.zeros(wsb, dtype=torch.uint8, device=dev)
    p = lambda t: C.c_void_p(t.data_ptr())  # noqa: E731
    _abi.check(L.hc_trifocal_eval_batched(n, p(Ut), p(X), p(P), p(P), p(HX), p(HT), p(H), p(ws), wsb,
                                          C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)), "eval")
    torch.cuda.synchronize(dev)
    assert int(L.hc_trifocal_workspace_status(p(ws))) == 5   # HC_ERROR_TABLE
    assert (HX == 7.0).all() and (HT == 7.0).all() and (H == 7.0).all()


def _outside_lu_structure(dx):
    """Rows whose dH/dx structure has an entry outside the specialised LU's
    (hc_lu.hpp LU_STRUCT_PAT, include/hc_trifocal_testing.h)."""
    from trifocal_pose_estimation_using_improved_gpuhc_amd import _abi
    L = _abi.lib()
    coef = dx.reshape(30, 8, 5, 30)[:, :, 0, :]            # [column, term, row]
    pat = [sum(1 << c for c in range(30) if (coef[c, :, r] != 0).any()) for r in range(30)]
    return [r for r in range(30) if pat[r] & ~int(L.hc_lu_struct_pattern(r))]


@pytest.mark.parametrize("mode", [KERNEL_BY_SIZE, SMALL_NEVER], ids=["latency_kernel", "throughput_kernel"])
def test_tracker_row_permuted_structure_matches_oracle(problem, oracle, samples100, ransac0, mode):
    """Any table the reference kernel takes is tracked.  A
    row-permuted system (valid and equivalent) has a dH/dx structure outside
    the one the specialised LU compiles in; k_prep_tables routes it to the
    structure-agnostic instantiation enqueued beside the specialised one.
    Tracking (abort off, the archived PH_CodeOpt semantics, and abort mode)
    of 2 samples equals the oracle on the same permuted tables value for
    value, and the problem's own table still runs the specialised kernel."""
    import dataclasses

    import torch

    from trifocal_pose_estimation_using_improved_gpuhc_amd.tracker import DeviceTracker
    tgt, dif, _ = samples100
    N = 2
    for swap in ((0, 9), (5, 14)):
        perm = np.arange(30)
        perm[swap[0]], perm[swap[1]] = swap[1], swap[0]
        dx, dt, U = _row_permuted(problem, perm)
        assert _outside_lu_structure(dx), f"permutation {swap} stays within the specialised LU's structure"
        tr = DeviceTracker(dataclasses.replace(problem, dHdx_index=dx, dHdt_index=dt), torch.device("cuda:0"))
        tr.set_ransac_data(ransac0)
        for truncate in (True, False):
            with small_launch(tr.L, mode):
                r = tr.track(tgt[:N], dif[:N], truncate=truncate).host()
            tr.workspace_status()
            o_tr, conv, inf, st = oracle.gpuhc_track(problem.start_sols, problem.start_params, tgt[:N], dif[:N], U,
                                                     oracle.settings(truncate=truncate))
            assert (r["converge"] == conv).all() and (r["infinity"] == inf).all(), (swap, truncate)
            assert (r["stats"]["steps"] == st["steps"]).all() and (r["stats"]["corrections"] == st["corrections"]).all()
            bad = ~same(r["tracks"][:, :30], o_tr[:, :30]).all(axis=(1, 2))
            assert not bad.any(), f"{swap} truncate={truncate}: {bad.sum()} tracks differ"
            if truncate:
                ref_conv, ref_tracks = conv, o_tr
        # abort mode: every path it tracked equals the abort-off oracle run
        a = tr.track(tgt[:N], dif[:N], abort=True).host()
        tr.workspace_status()
        tracked = a["stats"]["steps"] > 0
        assert tracked.sum() > 0
        assert (a["converge"][tracked] == ref_conv[tracked]).all()
        assert same(a["tracks"][tracked][:, :30], ref_tracks[tracked][:, :30]).all()
    assert not _outside_lu_structure(problem.dHdx_index)


def test_ring_check_reports_an_undrained_ring(tracker):
    """The end check of a sliced launch (k_ring_check): a ring left
    with head != tail, or with an unclaimed entry (avail != 0), is a suspended
    path that was never resumed: HC_ERROR_DEVICE with ring_fail = (~0, avail,
    tail, head); a drained ring stays silent."""
    import torch
    L = tracker.L
    wsb = int(L.hc_trifocal_workspace_size_for(1))
    hs = ctypes.c_void_p(torch.cuda.current_stream(tracker.device).cuda_stream)
    for head, tail, avail, bad in ((7, 7, 0, False), (9, 7, 0, True), (7, 7, 1, True)):
        ws = torch.zeros(wsb, dtype=torch.uint8, device=tracker.device)
        assert int(L.hc_trifocal_ring_check_test(ctypes.c_void_p(ws.data_ptr()), wsb, head, tail, avail, hs)) == 0
        torch.cuda.synchronize(tracker.device)
        st = int(L.hc_trifocal_workspace_status(ctypes.c_void_p(ws.data_ptr())))
        cb = np.frombuffer(ws[:64].cpu().numpy().tobytes(), np.uint32)
        if bad:
            assert st == 4 and list(cb[8:12]) == [0xFFFFFFFF, avail, tail, head], (st, cb[8:12])
        else:
            assert st == 0 and (cb[8:12] == 0).all()
    small = int(L.hc_trifocal_workspace_size())
    assert int(L.hc_trifocal_ring_check_test(ctypes.c_void_p(ws.data_ptr()), small, 1, 0, 0, hs)) == 2
