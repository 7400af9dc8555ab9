#!/usr/bin/env python3
"""Launch-timeline diagnostic of the tracker (GPU only).

Needs the diagnostic build (HC_DIAG_TIMES: each path's stats carry its
dequeue / finish s_memrealtime stamps, 100 MHz) loaded via HC_TRIFOCAL_LIB.
Tracks config 2 (or --samples N) and prints how busy the path slots were over
the launch: the span, the mean number of busy slots, the time after the queue
ran dry, and the busy-slot curve in 5 % bins of the span.
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from trifocal_pose_estimation_using_improved_gpuhc_amd import load_problem, load_ransac_data, prepare_target_params  # noqa
from trifocal_pose_estimation_using_improved_gpuhc_amd.tracker import DeviceTracker  # noqa


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--samples", type=int, default=100)
    ap.add_argument("--slots", type=int, default=8192, help="path slots of the persistent grid")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    problem = load_problem()
    tgt, dif, _ = prepare_target_params(problem, load_ransac_data(0), 0, args.samples)
    tr = DeviceTracker(problem, dev)
    r = tr.allocate(args.samples)
    tt, dd = torch.from_numpy(tgt).to(dev), torch.from_numpy(dif).to(dev)
    for _ in range(2):
        tr.reset_tracks(r)
        tr.launch(tt, dd, r)
    torch.cuda.synchronize()
    h = r.host()
    st = h["stats"]
    t0 = st["inliers21"].astype(np.int64) & 0xFFFFFFFF
    t1 = st["inliers31"].astype(np.int64) & 0xFFFFFFFF
    base = t0.min()
    t0, t1 = (t0 - base) * 10e-6, (t1 - base) * 10e-6          # ms
    span = float(t1.max())
    dur = t1 - t0
    stages = st["steps"] * 4 + st["corrections"]
    busy_integral = float(dur.sum())
    last_deq = float(t0.max())
    edges = np.linspace(0, span, 21)
    curve = []
    for a, b in zip(edges[:-1], edges[1:]):
        ov = np.clip(np.minimum(t1, b) - np.maximum(t0, a), 0, None).sum() / (b - a)
        curve.append(round(float(ov), 1))
    trk = np.arange(len(dur)) % 312
    per_trk = np.array([dur[trk == k].max() for k in range(312)])
    out = {
        "samples": args.samples, "paths": int(len(dur)), "span_ms": round(span, 3),
        "mean_busy_slots": round(busy_integral / span, 1), "slots": args.slots,
        "slot_utilisation": round(busy_integral / span / args.slots, 4),
        "last_dequeue_ms": round(last_deq, 3), "after_last_dequeue_ms": round(span - last_deq, 3),
        "path_ms": {"mean": round(float(dur.mean()), 3), "p50": round(float(np.median(dur)), 3),
                    "p99": round(float(np.percentile(dur, 99)), 3), "max": round(float(dur.max()), 3)},
        "us_per_stage_mean": round(float((dur / np.maximum(stages, 1)).mean() * 1e3), 2),
        "max_stages": int(stages.max()), "longest_path_stages": int(stages[np.argmax(dur)]),
        "busy_slots_per_5pct": curve,
        "slowest_tracks": [int(k) for k in np.argsort(-per_trk)[:10]],
    }
    print(json.dumps(out))


if __name__ == "__main__":
    main()
