#!/usr/bin/env python3
"""Time to the first good pose over repeated config-3 runs (development tool, GPU):
SAMPLES samples (default 1000: config 3; 1: the lone-sample probe, no
contention from other hypotheses), abort on, chunks of 125, dataset K (000)
with srand(0); prints the per-run device times (ms) and their median as one JSON line.

    python scripts/ttfp.py [REPS] [--samples N] [--inflight] [--dataset K]
"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from trifocal_pose_estimation_using_improved_gpuhc_amd import load_problem, load_ransac_data, prepare_target_params, sharding  # noqa
from trifocal_pose_estimation_using_improved_gpuhc_amd.tracker import DeviceTracker  # noqa

argv = sys.argv[1:]
reps = int(argv[0]) if argv and not argv[0].startswith("-") else 10
n = int(argv[argv.index("--samples") + 1]) if "--samples" in argv else 1000
inflight = "--inflight" in argv
ds = int(argv[argv.index("--dataset") + 1]) if "--dataset" in argv else 0
dev = torch.device("cuda:0")
problem = load_problem()
data = load_ransac_data(ds)
t, d, _ = prepare_target_params(problem, data, 0, n)
t, d = torch.from_numpy(t).to(dev), torch.from_numpy(d).to(dev)
tr = DeviceTracker(problem, dev)
tr.set_ransac_data(data)
r = tr.allocate(n, stats=True, abort=True)
wss = []
out = []
for i in range(reps + 1):
    tr.reset_tracks(r)
    torch.cuda.synchronize()
    parts = tr.launch_abort_chunked(t, d, r, 125, wss, inflight_stop=inflight)
    torch.cuda.synchronize()
    hz = tr.read_timestamps(wss[0])[2]
    f = sharding.first_found_seconds([tr.read_timestamps(x)[:2] for x in wss[:len(parts)]], hz)
    if i:
        out.append(round(f * 1e3, 3))
print(json.dumps({"samples": n, "dataset": ds, "inflight_stop": inflight, "ttfp_ms": out, "median": float(np.median(out)),
                  "min": min(out), "max": max(out)}))
