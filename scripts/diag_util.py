#!/usr/bin/env python3
"""Throughput timeline of one config-2 launch with time slicing (development
tool, GPU only; build with scripts/build_variant.sh util -DHC_DIAG_TIMES -DHC_DIAG_UTIL).

Per 10.24-us bin the kernel counts the path-stages and wave-stages it starts.
Reported: the launch span, the pairing efficiency (path-stages / 2 x
wave-stages: a wave whose other half is idle runs the stage anyway), and the
path-stage rate in 2 % bins of the span relative to the steady-state rate
(the median of the middle half) -- the slot utilisation of the launch.

    HC_TRIFOCAL_LIB=.../libhc_trifocal_util.so python scripts/diag_util.py OUT.json
"""
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from trifocal_pose_estimation_using_improved_gpuhc_amd import load_problem, load_ransac_data, prepare_target_params  # noqa: E402
from trifocal_pose_estimation_using_improved_gpuhc_amd.tracker import DeviceTracker  # noqa: E402

BINS = 8192
dev = torch.device("cuda:0")
problem = load_problem()
tgt, dif, _ = prepare_target_params(problem, load_ransac_data(0), 0, 100)
tr = DeviceTracker(problem, dev)
L = tr.L
r = tr.allocate(100)
t, d = torch.from_numpy(tgt).to(dev), torch.from_numpy(dif).to(dev)
span = (C.c_ulonglong * 4)()
COPIES = 64
util = (C.c_ulonglong * (2 * BINS * COPIES))()
out = {}
for mode in ("sliced", "unsliced"):
    for i in range(3):
        tr.reset_tracks(r)
        torch.cuda.synchronize(dev)
        assert L.hc_diag_span(span, 1) == 0 and L.hc_diag_util(util, 1) == 0
        tr.launch(t, d, r, time_slicing=(mode == "sliced"))
        torch.cuda.synchronize(dev)
    assert L.hc_diag_span(span, 0) == 0 and L.hc_diag_util(util, 0) == 0
    u = np.frombuffer(util, dtype=np.uint64).reshape(COPIES, BINS, 2).astype(np.int64).sum(axis=0)
    t0, t1 = int(span[0]), int(span[1])
    b0, b1 = t0 >> 10, t1 >> 10
    idx = np.arange(b0, b1 + 1) & (BINS - 1)
    ps, ws = u[idx, 0], u[idx, 1]
    nb = len(idx)
    edges = np.linspace(0, nb, 51).astype(int)
    rate = np.array([ps[a:b].sum() / max(1, b - a) for a, b in zip(edges[:-1], edges[1:])])
    steady = float(np.median(rate[12:38]))
    rel = rate / steady
    out[mode] = {"span_ms": round((t1 - t0) * 1e-5, 3), "path_stages": int(ps.sum()), "wave_stages": int(ws.sum()),
                 "pairing_efficiency": round(float(ps.sum()) / (2 * max(1, ws.sum())), 4),
                 "utilisation_vs_steady": round(float(rel.mean()), 4),
                 "rate_2pct_bins_rel_steady": [round(float(v), 3) for v in rel]}
    # per path (HC_DIAG_TIMES writes the first dequeue and the finish stamp,
    # s_memrealtime low 32 bits, into the stats record): when the paths finish
    # and which ones finish last
    st = r.stats.cpu().numpy().astype(np.int64)
    t_deq = (st[:, 2] - (t0 & 0xFFFFFFFF)) % (1 << 32)
    t_fin = (st[:, 3] - (t0 & 0xFFFFFFFF)) % (1 << 32)
    order = np.argsort(t_fin)
    out[mode]["finish_quantiles_ms"] = {q: round(float(np.percentile(t_fin, q)) * 1e-5, 3) for q in (50, 90, 95, 99, 100)}
    out[mode]["last_paths"] = [{"path": int(b), "steps": int(st[b, 0]), "corrections": int(st[b, 1]),
                                "first_start_ms": round(float(t_deq[b]) * 1e-5, 3),
                                "finish_ms": round(float(t_fin[b]) * 1e-5, 3)} for b in order[-12:]]
    print(json.dumps({k: v for k, v in out[mode].items() if k != "rate_2pct_bins_rel_steady"}), flush=True)
with open(sys.argv[1], "w") as f:
    json.dump(out, f, indent=1)
