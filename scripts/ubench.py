#!/usr/bin/env python3
"""Component micro-benchmarks of the tracker's building blocks (GPU only).

Times the batched 30x30 LU kernel, the batched evaluation kernel and one
tracking launch, each with HIP events, and prints per-unit costs so the
tracker's time can be attributed (eval vs LU vs control).
"""
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from trifocal_pose_estimation_using_improved_gpuhc_amd import _abi, load_problem, load_ransac_data, prepare_target_params  # noqa
from trifocal_pose_estimation_using_improved_gpuhc_amd.tracker import DeviceTracker  # noqa


def timeit(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    return float(np.median(ts))


def main():
    L = _abi.lib()
    dev = torch.device("cuda:0")
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    out = {}
    n = 1 << 18
    g = torch.Generator(device=dev).manual_seed(0)
    A = torch.randn((n, 30, 30, 2), generator=g, device=dev)
    b = torch.randn((n, 30, 2), generator=g, device=dev)
    x = torch.empty_like(b)
    ms = timeit(lambda: _abi.check(L.hc_cgesv_30x30_batched(n, C.c_void_p(A.data_ptr()), C.c_void_p(b.data_ptr()),
                                                             C.c_void_p(x.data_ptr()), st), "cgesv"))
    out["cgesv_ms"] = ms
    out["cgesv_ns_per_solve"] = ms * 1e6 / n
    problem = load_problem()
    data = load_ransac_data(0)
    tgt, dif, _ = prepare_target_params(problem, data, 0, 100)
    U = torch.from_numpy(problem.unified_index).to(dev)
    X = torch.from_numpy(np.tile(problem.start_sols, (n // 312 + 1, 1, 1))[:n]).to(dev).contiguous()
    P = torch.from_numpy(np.tile(tgt, (n // 100 + 1, 1, 1))[:n]).to(dev).contiguous()
    D = torch.from_numpy(np.tile(dif, (n // 100 + 1, 1, 1))[:n]).to(dev).contiguous()
    HX = torch.empty((n, 30, 30, 2), device=dev)
    HT = torch.empty((n, 30, 2), device=dev)
    H = torch.empty((n, 30, 2), device=dev)
    wsb = int(L.hc_trifocal_workspace_size())
    ws = torch.zeros(wsb, dtype=torch.uint8, device=dev)
    ms = timeit(lambda: _abi.check(L.hc_trifocal_eval_batched(
        n, C.c_void_p(U.data_ptr()), C.c_void_p(X.data_ptr()), C.c_void_p(P.data_ptr()), C.c_void_p(D.data_ptr()),
        C.c_void_p(HX.data_ptr()), C.c_void_p(HT.data_ptr()), C.c_void_p(H.data_ptr()), C.c_void_p(ws.data_ptr()),
        wsb, st), "eval"))
    out["eval_ms"] = ms
    out["eval_ns_per_point"] = ms * 1e6 / n
    tr = DeviceTracker(problem, dev)
    r = tr.allocate(100)
    tt = torch.from_numpy(tgt).to(dev)
    dd = torch.from_numpy(dif).to(dev)

    def run():
        tr.reset_tracks(r)
        tr.launch(tt, dd, r)
    ms = timeit(run)
    h = r.host()
    stages = int(h["stats"]["steps"].sum()) * 4 + int(h["stats"]["corrections"].sum())
    out["track_ms"] = ms
    out["track_stages"] = stages
    out["track_ns_per_stage"] = ms * 1e6 / stages
    # latency: one RANSAC sample (312 paths, < 1 wave per CU) -- the launch lasts
    # as long as its longest path (same stage count for every bit-identical build)
    r1 = tr.allocate(1)
    t1, d1 = tt[:1].contiguous(), dd[:1].contiguous()

    def run1():
        tr.reset_tracks(r1)
        tr.launch(t1, d1, r1)
    ms1 = timeit(run1)
    h1 = r1.host()
    st1 = h1["stats"]["steps"] * 4 + h1["stats"]["corrections"]
    out["track1_ms"] = ms1
    out["track1_max_stages"] = int(st1.max())
    out["track1_us_per_stage"] = ms1 * 1e3 / int(st1.max())
    out["version"] = L.hc_trifocal_version().decode()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
