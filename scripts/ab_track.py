#!/usr/bin/env python3
"""A/B timing of tracker library builds (development tool, GPU only).

    python scripts/ab_track.py NAME=path/to/lib.so [NAME=...] [--rounds 2] [--samples 100] [--sizes 2,8,32]

Runs each build in its own process (HC_TRIFOCAL_LIB), rounds interleaved
(A B A B ...): config-2 launches timed with HIP events on the launch stream
(median of 7), single-sample lone-launch latency, and a bit-exactness check of
every flag / step count / track hash against the committed golden run
(tests/golden/gpuhc_N100_seed0.npz).  One JSON line per build and round.
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(samples, sizes=()):
    sys.path.insert(0, ROOT)
    import numpy as np
    import torch

    def track_hash(tracks):   # the golden fixture's per-path hash (tests/golden/make_golden.py)
        a = np.ascontiguousarray(tracks[:, :30, :], np.float32).copy()
        a[a == 0] = 0.0
        a[np.isnan(a)] = np.float32(np.nan)
        w = a.reshape(a.shape[0], -1).view(np.uint32).astype(np.uint64)
        h = np.zeros(a.shape[0], np.uint64)
        with np.errstate(over="ignore"):
            for k in range(w.shape[1]):
                h = (h * np.uint64(1099511628211)) ^ w[:, k]
        return h
    from trifocal_pose_estimation_using_improved_gpuhc_amd import load_problem, load_ransac_data, prepare_target_params
    from trifocal_pose_estimation_using_improved_gpuhc_amd.tracker import DeviceTracker
    dev = torch.device("cuda:0")
    problem = load_problem()
    tgt, dif, _ = prepare_target_params(problem, load_ransac_data(0), 0, max(100, samples))
    tr = DeviceTracker(problem, dev)
    out = {}
    for n, reps in ((samples, 7), (1, 5)) + tuple((k, 5) for k in sizes):
        r = tr.allocate(n)
        t, d = torch.from_numpy(tgt[:n]).to(dev), torch.from_numpy(dif[:n]).to(dev)
        s = torch.cuda.current_stream(dev)
        ms = []
        for i in range(reps + 1):
            tr.reset_tracks(r)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s)
            tr.launch(t, d, r, stream=s)
            b.record(s)
            torch.cuda.synchronize(dev)
            if i:
                ms.append(a.elapsed_time(b))
        out[f"ms_{n}"] = round(float(np.median(ms)), 4)
        if n == 100:
            g = np.load(os.path.join(ROOT, "tests", "golden", "gpuhc_N100_seed0.npz"))
            h = r.host()
            out["exact"] = bool((h["converge"] == g["conv"]).all() and (h["stats"]["steps"] == g["steps"]).all()
                                and (h["stats"]["corrections"] == g["corrections"]).all()
                                and (track_hash(h["tracks"]) == g["hash"]).all())
    print(json.dumps(out))


def main():
    args = [a for a in sys.argv[1:] if "=" in a]
    rounds = int(sys.argv[sys.argv.index("--rounds") + 1]) if "--rounds" in sys.argv else 2
    samples = int(sys.argv[sys.argv.index("--samples") + 1]) if "--samples" in sys.argv else 100
    sizes = sys.argv[sys.argv.index("--sizes") + 1] if "--sizes" in sys.argv else ""
    builds = [a.split("=", 1) for a in args]
    for rnd in range(rounds):
        for name, lib in builds:
            env = dict(os.environ, HC_TRIFOCAL_LIB=os.path.abspath(lib))
            p = subprocess.run([sys.executable, __file__, "--child", str(samples), "--sizes", sizes], env=env, capture_output=True,
                               text=True, timeout=300)
            if p.returncode != 0:
                print(json.dumps({"build": name, "round": rnd, "error": p.stderr[-2000:]}), flush=True)
                sys.exit(1)
            res = json.loads(p.stdout.strip().splitlines()[-1])
            print(json.dumps({"build": name, "round": rnd, **res}), flush=True)


if __name__ == "__main__":
    if "--child" in sys.argv:
        sz = sys.argv[sys.argv.index("--sizes") + 1] if "--sizes" in sys.argv else ""
        child(int(sys.argv[sys.argv.index("--child") + 1]), tuple(int(k) for k in sz.split(",") if k))
    else:
        main()
