#!/usr/bin/env python3
"""How much of the time to the first good pose is contention (GPU, development
tool): the config-3 abort launch over only the first n samples (one launch, so
fewer co-resident paths compete with sample 0's passing track), for several n;
prints the median / min found time (device clock) per n."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from trifocal_pose_estimation_using_improved_gpuhc_amd import load_problem, load_ransac_data, prepare_target_params, sharding  # noqa
from trifocal_pose_estimation_using_improved_gpuhc_amd.tracker import DeviceTracker  # noqa

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 8
dev = torch.device("cuda:0")
problem = load_problem()
data = load_ransac_data(0)
t, d, _ = prepare_target_params(problem, data, 0, 125)
t, d = torch.from_numpy(t).to(dev), torch.from_numpy(d).to(dev)
tr = DeviceTracker(problem, dev)
tr.set_ransac_data(data)
for n in (1, 2, 8, 32, 125):
    r = tr.allocate(n, stats=True, abort=True)
    wss = []
    out = []
    for i in range(reps + 1):
        tr.reset_tracks(r)
        torch.cuda.synchronize()
        parts = tr.launch_abort_chunked(t[:n], d[:n], r, n, wss)
        torch.cuda.synchronize()
        hz = tr.read_timestamps(wss[0])[2]
        f = sharding.first_found_seconds([tr.read_timestamps(x)[:2] for x in wss[:len(parts)]], hz)
        if i:
            out.append(round(f * 1e3, 3))
    print(json.dumps({"samples": n, "ttfp_ms": out, "median": float(np.median(out)), "min": min(out)}), flush=True)
