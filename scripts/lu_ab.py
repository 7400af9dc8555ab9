#!/usr/bin/env python3
"""A/B of the batched LU component (hc_cgesv_30x30_batched) across library
builds (development tool, GPU only).

    python scripts/lu_ab.py NAME=path/to/lib.so [NAME=...] [--rounds 2] [--points 262144]

Each build runs in its own process (HC_TRIFOCAL_LIB): tracker-like Jacobian
systems (start solutions pushed along t, config-2 parameters, evaluated by the
library's own eval component) are solved and timed with HIP events (median of
7); a hash of the solutions is printed so builds can be compared bit for bit.
One JSON line per build and round.
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(n):
    sys.path.insert(0, ROOT)
    import ctypes as C
    import hashlib

    import numpy as np
    import torch

    from trifocal_pose_estimation_using_improved_gpuhc_amd import _abi, load_problem, load_ransac_data, prepare_target_params
    dev = torch.device("cuda:0")
    problem = load_problem()
    tgt, dif, _ = prepare_target_params(problem, load_ransac_data(0), 0, 100)
    rng = np.random.default_rng(1)
    k = rng.integers(0, 312, n)
    s = rng.integers(0, 100, n)
    X = problem.start_sols[k].copy()
    X[:, :30] += (rng.standard_normal((n, 30, 2)) * 10 ** rng.uniform(-4, -1, (n, 1, 1))).astype(np.float32)
    t = rng.uniform(0, 1, (n, 1, 1)).astype(np.float32)
    P = (tgt[s] * t + problem.start_params[None] * (1 - t)).astype(np.float32)
    P[:, 33] = (1.0, 0.0)
    D = dif[s]
    L = _abi.lib()
    p = lambda a: C.c_void_p(a.data_ptr())  # noqa: E731
    U = torch.from_numpy(problem.unified_index).to(dev)
    Xt, Pt, Dt = (torch.from_numpy(np.ascontiguousarray(a)).to(dev) for a in (X, P, D))
    HX = torch.empty((n, 30, 30, 2), dtype=torch.float32, device=dev)
    HT = torch.empty((n, 30, 2), dtype=torch.float32, device=dev)
    H = torch.empty((n, 30, 2), dtype=torch.float32, device=dev)
    wsb = int(L.hc_trifocal_workspace_size())
    ws = torch.zeros(wsb, dtype=torch.uint8, device=dev)
    st = C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    _abi.check(L.hc_trifocal_eval_batched(n, p(U), p(Xt), p(Pt), p(Dt), p(HX), p(HT), p(H), p(ws), wsb, st), "eval")
    Xs = torch.empty_like(HT)
    ms = []
    for i in range(8):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        _abi.check(L.hc_cgesv_30x30_batched(n, p(HX), p(HT), p(Xs), st), "cgesv")
        b.record()
        torch.cuda.synchronize()
        if i:
            ms.append(a.elapsed_time(b))
    sol = Xs.cpu().numpy()
    sol = np.where(sol == 0, 0.0, sol).astype(np.float32)   # +-0 are one class
    h = hashlib.sha1(np.ascontiguousarray(sol).view(np.uint32).tobytes()).hexdigest()[:16]
    med = float(np.median(ms))
    print(json.dumps({"ms": round(med, 4), "ns_per_solve": round(med * 1e6 / n, 3), "hash": h}))


def main():
    args = [a for a in sys.argv[1:] if "=" in a]
    rounds = int(sys.argv[sys.argv.index("--rounds") + 1]) if "--rounds" in sys.argv else 2
    n = int(sys.argv[sys.argv.index("--points") + 1]) if "--points" in sys.argv else 1 << 18
    for rnd in range(rounds):
        for name, lib in (a.split("=", 1) for a in args):
            env = dict(os.environ, HC_TRIFOCAL_LIB=os.path.abspath(lib))
            pr = subprocess.run([sys.executable, __file__, "--child", str(n)], env=env, capture_output=True,
                                text=True, timeout=300)
            if pr.returncode != 0:
                print(json.dumps({"build": name, "round": rnd, "error": pr.stderr[-2000:]}), flush=True)
                sys.exit(1)
            print(json.dumps({"build": name, "round": rnd, **json.loads(pr.stdout.strip().splitlines()[-1])}),
                  flush=True)


if __name__ == "__main__":
    if "--child" in sys.argv:
        child(int(sys.argv[sys.argv.index("--child") + 1]))
    else:
        main()
