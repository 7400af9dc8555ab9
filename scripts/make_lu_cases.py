#!/usr/bin/env python3
"""Writes scripts/data/lu_cases.bin for scripts/lu_lab.hip (development tool).

NC tracker-like systems from the C oracle: A = dH/dx and b = dH/dt at start
solutions pushed along t with noise (the parity tests' recipe), plus the
structural row patterns of dH/dx (bit c of row r: column c has index terms).
Layout: int32 NC, then NC x (30x30 complex64 A row-major, 30 complex64 b),
then 30 uint32 patterns.
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import oracle as O  # noqa: E402
from trifocal_pose_estimation_using_improved_gpuhc_amd import load_problem, load_ransac_data, prepare_target_params  # noqa

NC = int(sys.argv[1]) if len(sys.argv) > 1 else 64
problem = load_problem()
tgt, dif, _ = prepare_target_params(problem, load_ransac_data(0), 0, 100)
rng = np.random.default_rng(7)
As, bs = [], []
for i in range(NC):
    k = int(rng.integers(0, 312))
    s = int(rng.integers(0, 100))
    x = problem.start_sols[k].copy()
    x[:30] += (rng.standard_normal((30, 2)) * 10 ** rng.uniform(-4, -1)).astype(np.float32)
    t = float(np.float32(rng.uniform(0, 1)))
    p = O.param_homotopy(t, problem.start_params, tgt[s])
    As.append(O.eval_hx(problem.dHdx_index, x, p))
    bs.append(O.eval_ht(problem.dHdt_index, x, p, dif[s]))
T = problem.dHdx_index.reshape(30, 8, 5, 30)          # col, term, part, row
pat = np.zeros(30, np.uint32)
for r in range(30):
    for c in range(30):
        if (T[c, :, 0, r] != 0).any():
            pat[r] |= np.uint32(1 << c)
out = os.path.join(ROOT, "scripts", "data", "lu_cases.bin")
with open(out, "wb") as f:
    np.array([NC], np.int32).tofile(f)
    for A, b in zip(As, bs):
        np.ascontiguousarray(A, np.float32).tofile(f)
        np.ascontiguousarray(b, np.float32).tofile(f)
    pat.tofile(f)
print(out, NC)
