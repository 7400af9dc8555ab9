"""Reference-independent solution check (SURVEY.md §8(d) parity gate 2).

A converged real solution x of the target system must make every equation of
H(x, p_target) vanish.  H is evaluated here in FP64 from the reference's own
index table (problems/trifocal_2op1p_30x30/dHdt_indx.txt: term j of equation
r is coef * p[a] * p[b] * x[u] * x[v] * x[w], line j*6 + part, column r;
the same table the reference's eval_Homotopy reads, ..._LimUnroll_L2Cache.cuh
:122-148), independent of the FP32 tracker and of the oracle.

The residual of equation r is reported relative to the size of its terms,
|H_r| / sum_j |term_rj|: the rounding error of an FP32 solution is
proportional to that sum, not to |H_r| (the terms cancel).
"""
import numpy as np

REAL_TOL = 1e-4       # ZERO_IMAG_PART_TOL_FOR_SP (definitions.hpp:25)
RESIDUAL_TOL = 1e-4   # gate: relative FP64 residual of a converged real solution


def relative_residuals(dhdt_index, x, p_target):
    """Per-equation |H_r(x, p)| / sum_j |term_rj| in FP64.
    x: (31, 2) float (x[30] = 1), p_target: (34, 2) float (p[33] = 1)."""
    T = np.asarray(dhdt_index).reshape(16, 6, 30)
    p = np.asarray(p_target, np.float64)
    p = p[:, 0] + 1j * p[:, 1]
    p[33] = 1.0
    xx = np.asarray(x, np.float64)
    xx = xx[:, 0] + 1j * xx[:, 1]
    xx = np.concatenate([xx[:30], [1.0]])
    c = T[:, 0, :].astype(np.float64)
    terms = c * p[T[:, 1, :]] * p[T[:, 2, :]] * xx[T[:, 3, :]] * xx[T[:, 4, :]] * xx[T[:, 5, :]]
    scale = np.abs(terms).sum(axis=0)
    return np.abs(terms.sum(axis=0)) / np.where(scale > 0, scale, 1.0)


def real_converged(tracks, conv):
    """Batch ids of converged paths whose 30 imaginary parts are all within REAL_TOL
    (Evaluations.cpp:145-182)."""
    tr = np.asarray(tracks)
    ids = np.nonzero(np.asarray(conv))[0]
    return np.array([b for b in ids if np.all(np.abs(tr[b, :30, 1]) <= REAL_TOL)], dtype=np.int64)


def max_relative_residual(dhdt_index, tracks, ids, targets):
    """Largest relative residual over the given batch ids (b = sample * 312 + track)."""
    worst = 0.0
    for b in ids:
        worst = max(worst, float(relative_residuals(dhdt_index, tracks[b], targets[b // 312]).max()))
    return worst
