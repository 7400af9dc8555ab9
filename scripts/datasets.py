#!/usr/bin/env python3
"""The config-2 launch off its training data (GPU only).

The dequeue order (csrc/hc_track_order.inc) was fitted on the per-track costs
of synthcurves datasets 001 and 002, and the inline tie steps / slot classes on
this problem's Jacobians.  For each case -- datasets 000 (the benchmark's),
001, 002 with the reference's srand(0) samples, dataset 000 with srand(1) and
srand(2) (samples never used for any fitting), dataset 000 with sigma = 1 px
noise, and the shards of ranks 1..7 of an 8-GPU config-2 run -- this times the config-2 launch (100 samples x 312 paths, median of 7
launches by HIP events, product build) and counts, with the HC_DIAG_LUWORK
build of the same sources (a child process, HC_TRIFOCAL_LIB), the rare pivot
steps and the dense re-solves.  One JSON line per case.

    python scripts/datasets.py path/to/libhc_trifocal_luwork.so
"""
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
CASES = [(0, 0, None), (1, 0, None), (2, 0, None), (0, 1, None), (0, 2, None), (0, 0, 1.0)]
SHARDS8 = range(1, 8)   # ranks 1..7 of an 8-GPU config-2 run (samples 100 g .. 100 g + 99 of the srand(0) draw)


def main():
    import torch

    from trifocal_pose_estimation_using_improved_gpuhc_amd import (_abi, load_problem, load_ransac_data,
                                                                   prepare_target_params, synthcurves)
    from trifocal_pose_estimation_using_improved_gpuhc_amd.tracker import DeviceTracker
    luwork = os.path.abspath(sys.argv[1])
    dev = torch.device("cuda:0")
    problem = load_problem()
    tr = DeviceTracker(problem, dev)
    r = tr.allocate(100)
    s = torch.cuda.current_stream(dev)
    cases = [(ds, seed, sigma, None) for ds, seed, sigma in CASES] + [(0, 0, None, g) for g in SHARDS8]
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
        args = [sys.executable, os.path.join(ROOT, "scripts", "lu_work.py"), "--dataset", str(ds), "--seed", str(seed)]
        if sigma is not None:
            args += ["--sigma", str(sigma)]
        if g8 is not None:
            args += ["--shard8", str(g8)]
        p = subprocess.run(args, env=dict(os.environ, HC_TRIFOCAL_LIB=luwork), capture_output=True, text=True,
                           timeout=300)
        lw = json.loads(p.stdout.strip().splitlines()[-1]) if p.returncode == 0 else {"error": p.stderr[-500:]}
        print(json.dumps({
            "dataset": f"{ds:03d}", "srand": seed, "sigma_px": sigma,
            "shard_of_8": g8,
            "fitted_on": ("track order fitted on 001/002" if ds in (1, 2) and sigma is None and seed == 0 else
                          "benchmark data (track order from 001/002)" if (ds, seed, sigma, g8) == (0, 0, None, None)
                          else "never used for fitting"),
            "kernel_ms": round(kms, 4), "paths_per_s": round(31200 / (kms / 1e3), 1),
            "path_stages": stages, "us_per_path_stage_x_slots": round(kms * 1e3 / max(1, stages), 6),
            "converged": int(r.converge.sum().item()),
            "rare_steps_per_wave_solve": lw.get("rare_steps_per_wave_solve"),
            "solves_rerun_densely": lw.get("solves_rerun_densely"),
            "live_groups_per_wave_solve": lw.get("live_groups_per_wave_solve"),
            "executed_fraction": lw.get("executed_fraction"),
            "build_id": _abi.build_id(),
            "measured_at": time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime())}), flush=True)


if __name__ == "__main__":
    main()
