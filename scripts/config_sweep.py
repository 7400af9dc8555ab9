#!/usr/bin/env python3
"""Config 3 / config 5 characterisation (GPU only), JSON on stdout:

  abort_N100   Evaluate_RANSAC_HC_Sols counts (converged, real, infinity --
               the reference's file columns, Evaluations.cpp:145-182) of abort-mode
               runs of 100 samples, in both abort semantics, 3 runs each (which
               paths are skipped depends on scheduling).  Reported next to the
               reference's committed Output_Write_Files/GPU_Sols_Statistics.txt
               (272 5 495, run settings unknown).
  noisy        pose success rate of RANSAC runs on sigma-px noisy synthcurves
               (Triplet_Edgels_000, noise seed 20250215 + trial, samples
               srand(trial)) for samples in {100, 1000} and sigma in {0.5, 1, 2}:
               track + device pose support + GT residuals (Evaluations.cpp:523-543),
               plus the fraction of runs whose best candidate passes the
               reference's 90 % inlier test (dev-trifocal_2op1p-eval.cuh:241-246).
"""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from trifocal_pose_estimation_using_improved_gpuhc_amd import (count_solutions, load_problem, load_ransac_data,  # noqa
                                                               pose, prepare_target_params, synthcurves)
from trifocal_pose_estimation_using_improved_gpuhc_amd.tracker import DeviceTracker  # noqa

TRIALS = int(os.environ.get("SWEEP_TRIALS", "10"))


def main():
    dev = torch.device("cuda:0")
    problem = load_problem()
    data = load_ransac_data(0)
    tr = DeviceTracker(problem, dev)
    tr.set_ransac_data(data)
    out = {"reference_GPU_Sols_Statistics": [272, 5, 495]}
    tgt, dif, _ = prepare_target_params(problem, data, seed=0, num_samples=100)
    for inflight in (0, 1):
        runs = []
        for _ in range(3):
            r = tr.track(tgt, dif, abort=True, inflight_stop=bool(inflight)).host()
            c = count_solutions(r["tracks"], r["converge"], r["infinity"])
            runs.append({"counts": list(c), "paths_tracked": int((r["stats"]["steps"] > 0).sum()),
                         "found_ids": [int(b) for b in np.nonzero(r["batch_index"] >= 0)[0]]})
        out[f"abort_N100_inflight_stop{inflight}"] = runs
    print(json.dumps({k: v for k, v in out.items()}), file=sys.stderr, flush=True)
    noisy = []
    for S in (100, 1000):
        res = tr.allocate(S, stats=True)
        for sigma in (0.5, 1.0, 2.0):
            ok, cands, best90, t_tot = [], [], [], 0.0
            for t in range(TRIALS):
                nd = synthcurves.noisy(data, sigma, synthcurves.DEFAULT_SEED + t)
                ta, da, _ = prepare_target_params(problem, nd, seed=t, num_samples=S)
                tg, df = torch.from_numpy(ta).to(dev), torch.from_numpy(da).to(dev)
                E = torch.from_numpy(np.ascontiguousarray(nd.locations)).to(dev)
                tr.reset_tracks(res)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                tr.launch(tg, df, res)
                inl, sel = pose.pose_support(res.tracks, res.converge, E, tr.K)
                t_tot += time.perf_counter() - t0
                rs, good = pose.residuals(nd, sel)
                ok.append(bool(good))
                cands.append(int(sel["num_candidates"]))
                n_e = nd.locations.shape[0]
                best90.append(bool(sel["num_candidates"] > 0 and sel["inliers21"] >= 0.9 * n_e
                                   and sel["inliers31"] >= 0.9 * n_e))
            noisy.append({"samples": S, "sigma_px": sigma, "trials": TRIALS, "success_rate": float(np.mean(ok)),
                          "median_candidates": int(np.median(cands)), "best_passes_90pct": float(np.mean(best90)),
                          "ms_per_run": round(t_tot / TRIALS * 1e3, 3)})
            print(json.dumps(noisy[-1]), file=sys.stderr, flush=True)
    out["noisy"] = noisy
    print(json.dumps(out))


if __name__ == "__main__":
    main()
