#!/usr/bin/env python3
"""Per-phase cycle split of the tracker loop (GPU only, development tool).

Needs the HC_DIAG_PHASES build loaded via HC_TRIFOCAL_LIB: every wave sums the
shader cycles (s_memtime) it spends in each phase of a stage iteration.  Prints
the split in cycles per wave-iteration for 1 RANSAC sample (lone waves: the
latency of a stage), for config 2 (100 samples, full occupancy) and for the
abort kernel on 1 sample (abort1: the lone latency that sets the time to the
first pose).
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

NAMES = ["slot_phases", "park_pt", "dHdx", "dHdt_H", "lu_forward", "lu_backward", "stage_update", "lifetime", "waves",
         "lu_search", "lu_bcast", "lu_rcp", "lu_update"]


def main():
    L = _abi.lib()
    fn = L.hc_diag_phases
    fn.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
    dev = torch.device("cuda:0")
    problem = load_problem()
    data = load_ransac_data(0)
    tgt, dif, _ = prepare_target_params(problem, data, 0, 100)
    tr = DeviceTracker(problem, dev)
    tr.set_ransac_data(data)
    out = {}
    for n, abort in ((1, False), (100, False), (1, True)):
        r = tr.allocate(n, abort=abort)
        tt, dd = torch.from_numpy(tgt[:n]).to(dev), torch.from_numpy(dif[:n]).to(dev)
        tr.reset_tracks(r)
        tr.launch(tt, dd, r, abort=abort)
        torch.cuda.synchronize()
        buf = (C.c_ulonglong * 13)()
        fn(buf, 1)
        tr.reset_tracks(r)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        tr.launch(tt, dd, r, abort=abort)
        b.record()
        torch.cuda.synchronize()
        fn(buf, 1)
        v = np.array(list(buf), dtype=np.float64)
        h = r.host()
        stages = int(h["stats"]["steps"].sum()) * 4 + int(h["stats"]["corrections"].sum())
        iters = stages / 2.0   # lower bound on wave-iterations (both halves busy)
        waves = v[8]
        d = {NAMES[i]: round(v[i] / waves, 1) for i in range(8)}
        d["per_stage_pair"] = {NAMES[i]: round(v[i] / iters, 1) for i in list(range(7)) + list(range(9, 13))}
        d["ms"] = a.elapsed_time(b)
        d["waves"] = int(waves)
        d["stages"] = stages
        d["clock_ghz_est"] = round(v[7] / waves / (d["ms"] * 1e6), 3)
        out[f"abort_samples_{n}" if abort else f"samples_{n}"] = d
    print(json.dumps(out))


if __name__ == "__main__":
    main()
