#!/usr/bin/env python3
"""The tracker on data it was not fitted to (GPU only).

What was fitted on which data: the dequeue order (csrc/hc_track_order.inc) on
the per-track costs of synthcurves datasets 001 and 002; the LU's always-live
column groups (hc_lu.hpp LU_ALWAYS) on the group liveness of 000/001/002; every
time-to-first-pose figure before round 6 on dataset 000.  Datasets 003 (the
CLI's round 3: srand(3)), 010, 050 and 099 were never used for any fitting.

Per case -- a dataset with the reference's samples (srand(ti)), dataset 000
with another srand, dataset 000 with sigma = 1 px noise, the shards of ranks
1..7 of an 8-GPU config-2 run -- one JSON line:
  * the config-2 launch (100 samples x 312 paths): median of 7 launches by HIP
    events, product build; path-stages, and time per path-stage;
  * the rare pivot steps and dense re-solves, from the HC_DIAG_LUWORK build of
    the same sources (a child process, HC_TRIFOCAL_LIB);
  * the device pose support over those tracks and its GT verdict
    (GT_Poses21/31 of the dataset; Evaluations.cpp:523-543 tolerances);
  * (dataset cases, --ttfp-runs > 0) config 3's time to the first good pose:
    1000 samples, abort on, chunks of 125, both abort semantics, median / min /
    max over the runs (the bench's early_abort leg on that dataset).

    python scripts/datasets.py path/to/libhc_trifocal_luwork.so [--ttfp-runs 12] [--no-shards]
"""
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
# (dataset, srand seed, sigma px)
CASES = [(0, 0, None), (1, 0, None), (2, 0, None), (3, 3, None), (10, 0, None), (50, 0, None), (99, 0, None),
         (0, 2, None), (0, 0, 1.0)]
SHARDS8 = range(1, 8)   # ranks 1..7 of an 8-GPU config-2 run (samples 100 g .. 100 g + 99 of the srand(0) draw)
FITTED = {0: "benchmark data (LU_ALWAYS fitted on 000/001/002; track order on 001/002)",
          1: "LU_ALWAYS and track order fitted on it", 2: "LU_ALWAYS and track order fitted on it"}


def ttfp(tr, problem, data, seed, runs, inflight, dev):
    """Config 3 on `data`: per run the device time from the first chunk's start to
    the first good pose (ms), or None when no sample of the 1000 passes."""
    import torch

    from trifocal_pose_estimation_using_improved_gpuhc_amd import prepare_target_params, sharding
    t, d, _ = prepare_target_params(problem, data, seed, 1000)
    t, d = torch.from_numpy(t).to(dev), torch.from_numpy(d).to(dev)
    tr.set_ransac_data(data)
    r = tr.allocate(1000, stats=True, abort=True)
    wss, out = [], []
    for i in range(runs + 1):
        tr.reset_tracks(r)
        torch.cuda.synchronize(dev)
        parts = tr.launch_abort_chunked(t, d, r, 125, wss, inflight_stop=inflight)
        torch.cuda.synchronize(dev)
        hz = tr.read_timestamps(wss[0])[2]
        f = sharding.first_found_seconds([tr.read_timestamps(x)[:2] for x in wss[:len(parts)]], hz)
        if i:   # the first run warms the chunk workspaces
            out.append(round(f * 1e3, 3) if f >= 0 else None)
    ok = [v for v in out if v is not None]
    first = np.nonzero(r.batch_index.cpu().numpy() >= 0)[0]
    return {"median": float(np.median(ok)) if ok else None, "min": min(ok) if ok else None,
            "max": max(ok) if ok else None, "found_runs": len(ok), "runs": len(out),
            "found_batch_ids_last_run": [int(b) for b in first[:4]]}


def main():
    import torch

    from trifocal_pose_estimation_using_improved_gpuhc_amd import (_abi, load_problem, load_ransac_data, pose,
                                                                   prepare_target_params, synthcurves)
    from trifocal_pose_estimation_using_improved_gpuhc_amd.tracker import DeviceTracker
    argv = sys.argv[1:]
    luwork = os.path.abspath(argv[0])
    runs = int(argv[argv.index("--ttfp-runs") + 1]) if "--ttfp-runs" in argv else 12
    dev = torch.device("cuda:0")
    problem = load_problem()
    tr = DeviceTracker(problem, dev)
    r = tr.allocate(100)
    s = torch.cuda.current_stream(dev)
    cases = [(ds, seed, sigma, None) for ds, seed, sigma in CASES]
    if "--no-shards" not in argv:
        cases += [(0, 0, None, g) for g in SHARDS8]
    for ds, seed, sigma, g8 in cases:
        data = load_ransac_data(ds)
        if sigma is not None:
            data = synthcurves.noisy(data, sigma, synthcurves.DEFAULT_SEED)
        if g8 is None:
            tgt, dif, _ = prepare_target_params(problem, data, seed, 100)
        else:
            ta, da, _ = prepare_target_params(problem, data, seed, 800, num_gpus=8)
            tgt, dif = ta[100 * g8:100 * g8 + 100].copy(), da[100 * g8:100 * g8 + 100].copy()
        t, d = torch.from_numpy(tgt).to(dev), torch.from_numpy(dif).to(dev)
        ms = []
        for i in range(8):
            tr.reset_tracks(r)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s)
            tr.launch(t, d, r, stream=s)
            b.record(s)
            torch.cuda.synchronize(dev)
            if i:
                ms.append(a.elapsed_time(b))
        tr.workspace_status()
        st = r.stats.cpu().numpy()
        stages = 4 * int(st[:, 0].sum()) + int(st[:, 1].sum())
        kms = float(np.median(ms))
        E = torch.from_numpy(np.ascontiguousarray(data.locations)).to(dev)
        K = torch.from_numpy(np.ascontiguousarray(data.K)).to(dev)
        _, sel = pose.pose_support(r.tracks, r.converge, E, K)
        res, ok = pose.residuals(data, sel)
        args = [sys.executable, os.path.join(ROOT, "scripts", "lu_work.py"), "--dataset", str(ds), "--seed", str(seed)]
        if sigma is not None:
            args += ["--sigma", str(sigma)]
        if g8 is not None:
            args += ["--shard8", str(g8)]
        p = subprocess.run(args, env=dict(os.environ, HC_TRIFOCAL_LIB=luwork), capture_output=True, text=True,
                           timeout=300)
        lw = json.loads(p.stdout.strip().splitlines()[-1]) if p.returncode == 0 else {"error": p.stderr[-500:]}
        line = {
            "dataset": f"{ds:03d}", "srand": seed, "sigma_px": sigma, "shard_of_8": g8,
            "fitted_on": FITTED.get(ds, "never used for fitting") if (seed, sigma, g8) == (0, None, None) or ds != 0
            else "never used for fitting (dataset 000, other samples)",
            "kernel_ms": round(kms, 4), "paths_per_s": round(31200 / (kms / 1e3), 1),
            "path_stages": stages, "us_per_path_stage_x_slots": round(kms * 1e3 / max(1, stages), 6),
            "converged": int(r.converge.sum().item()),
            "rare_steps_per_wave_solve": lw.get("rare_steps_per_wave_solve"),
            "solves_rerun_densely": lw.get("solves_rerun_densely"),
            "live_groups_per_wave_solve": lw.get("live_groups_per_wave_solve"),
            "executed_fraction": lw.get("executed_fraction"),
            "pose": {"gt_match": bool(ok), "gt_match_acos_clamped": pose.success_clamped(data, sel, res),
                     "candidates": sel["num_candidates"],
                     "residuals": [round(float(v), 6) for v in res]},
            "build_id": _abi.build_id(),
            "measured_at": time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime())}
        if runs > 0 and g8 is None and sigma is None:
            line["ttfp_config3_ms"] = {"reference_semantics": ttfp(tr, problem, data, seed, runs, False, dev),
                                       "inflight_stop": ttfp(tr, problem, data, seed, runs, True, dev)}
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
