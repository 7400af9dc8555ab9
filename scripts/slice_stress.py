#!/usr/bin/env python3
"""Time slicing under concurrency (development tool, GPU only): R rounds of
S sliced config-2 launches in flight at once on S streams (own buffers and
workspaces); per round the wall time, every workspace's status and ring
diagnostics (Workspace::ring_fail: ticket, tag seen, tail, head, wait ticks),
and whether every launch equals the serial run bit for bit.

    python scripts/slice_stress.py OUT.jsonl [S] [R] [--warm-streams]
"""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from trifocal_pose_estimation_using_improved_gpuhc_amd import load_problem, load_ransac_data, prepare_target_params  # noqa: E402
from trifocal_pose_estimation_using_improved_gpuhc_amd.tracker import DeviceTracker  # noqa: E402

out = open(sys.argv[1], "w")
pos = [v for v in sys.argv[2:] if not v.startswith("--")]
NS = int(pos[0]) if len(pos) > 0 else 4
R = int(pos[1]) if len(pos) > 1 else 6
dev = torch.device("cuda:0")
problem = load_problem()
tgt, dif, _ = prepare_target_params(problem, load_ransac_data(0), 0, 100)
tr = DeviceTracker(problem, dev)
ref = tr.track(tgt, dif).host()
t, d = torch.from_numpy(tgt).to(dev), torch.from_numpy(dif).to(dev)
streams = [torch.cuda.Stream(dev) for _ in range(NS)]
bufs = [tr.allocate(100) for _ in range(NS)]
wss = [tr.new_workspace(100) for _ in range(NS)]
if "--warm-streams" in sys.argv:   # a small kernel on every stream first (its hardware queue exists before round 0)
    for st in streams:
        with torch.cuda.stream(st):
            torch.ones(1, device=dev).add_(1)
    torch.cuda.synchronize(dev)
for rnd in range(R):
    for b in bufs:
        b.converge.fill_(7)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for k in range(NS):
        with torch.cuda.stream(streams[k]):
            tr.reset_tracks(bufs[k])
        tr.launch(t, d, bufs[k], stream=streams[k], workspace=wss[k])
    torch.cuda.synchronize(dev)
    ms = (time.perf_counter() - t0) * 1e3
    rec = {"round": rnd, "streams": NS, "wall_ms": round(ms, 2), "launches": []}
    for k in range(NS):
        ctl = np.frombuffer(wss[k][:64].cpu().numpy().tobytes(), np.uint32)
        h = bufs[k].host()
        exact = bool((h["converge"] == ref["converge"]).all() and np.array_equal(h["stats"]["steps"], ref["stats"]["steps"])
                     and np.array_equal(h["tracks"].view(np.uint32), ref["tracks"].view(np.uint32)))
        rec["launches"].append({"status": int(ctl[1]), "ring_fail": [int(v) for v in ctl[8:12]],
                                "wait_ticks": int(ctl[12]), "last_tag": int(ctl[13]), "first_read_ticks": int(ctl[14]),
                                "exact": exact,
                                "unfinished": int((h["converge"] == 7).sum())})
    print(json.dumps(rec), flush=True)
    out.write(json.dumps(rec) + "\n")
out.close()
