#!/usr/bin/env python3
"""Drives the component kernels on realistic tracker inputs so rocprofv3 PMC
counters (SQ_INSTS_VALU, ...) can be attributed per unit of work (GPU only):

  k_eval   : dH/dx + dH/dt + H at N points (start solutions pushed along t)
  k_cgesv  : the tracker's LU on the dH/dx | dH/dt systems at those points
  k_track  : one config-2 tracking launch (100 samples)

    rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES -- python scripts/valu_breakdown.py
"""
import argparse
import ctypes as C
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from trifocal_pose_estimation_using_improved_gpuhc_amd import _abi, load_problem, load_ransac_data, prepare_target_params  # noqa
from trifocal_pose_estimation_using_improved_gpuhc_amd.tracker import DeviceTracker  # noqa

ap = argparse.ArgumentParser()
ap.add_argument("--points", type=int, default=1 << 16)
args = ap.parse_args()
dev = torch.device("cuda:0")
problem = load_problem()
tgt, dif, _ = prepare_target_params(problem, load_ransac_data(0), 0, 100)
rng = np.random.default_rng(1)
n = args.points
k = rng.integers(0, 312, n)
s = rng.integers(0, 100, n)
X = problem.start_sols[k].copy()
X[:, :30] += (rng.standard_normal((n, 30, 2)) * 10 ** rng.uniform(-4, -1, (n, 1, 1))).astype(np.float32)
t = rng.uniform(0, 1, (n, 1, 1)).astype(np.float32)
sp = problem.start_params[None]
P = (tgt[s] * t + sp * (1 - t)).astype(np.float32)
P[:, 33] = (1.0, 0.0)
D = dif[s]
L = _abi.lib()
U = torch.from_numpy(problem.unified_index).to(dev)
Xt, Pt, Dt = (torch.from_numpy(np.ascontiguousarray(a)).to(dev) for a in (X, P, D))
HX = torch.empty((n, 30, 30, 2), dtype=torch.float32, device=dev)
HT = torch.empty((n, 30, 2), dtype=torch.float32, device=dev)
H = torch.empty((n, 30, 2), dtype=torch.float32, device=dev)
wsb = int(L.hc_trifocal_workspace_size())
ws = torch.zeros(wsb, dtype=torch.uint8, device=dev)
st = C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
p = lambda a: C.c_void_p(a.data_ptr())  # noqa: E731
_abi.check(L.hc_trifocal_eval_batched(n, p(U), p(Xt), p(Pt), p(Dt), p(HX), p(HT), p(H), p(ws), wsb, st), "eval")
Xs = torch.empty_like(HT)
_abi.check(L.hc_cgesv_30x30_batched(n, p(HX), p(HT), p(Xs), st), "cgesv")
tr = DeviceTracker(problem, dev)
r = tr.allocate(100)
tr.reset_tracks(r)
tr.launch(torch.from_numpy(tgt).to(dev), torch.from_numpy(dif).to(dev), r)
torch.cuda.synchronize()
st_h = r.stats.cpu().numpy()
print(f"points {n}; tracker path-stages: predictor {4 * int(st_h[:, 0].sum())}, corrector {int(st_h[:, 1].sum())}")
