#!/usr/bin/env python3
"""What can any dequeue order gain?  (development tool, GPU only)

    HC_TRIFOCAL_LIB=lib/libhc_trifocal_po.so python scripts/order_bound.py

Needs the round-2 experiment build with -DHC_AB_PATH_ORDER, whose
hc_ab_set_path_order sets an explicit per-path dequeue order.  That hook left
the product tree in round 3; run this against the round-2
sources: git worktree add /tmp/r2 136b029, then scripts/build_variant.sh there.  Times config-2 launches (HIP events, median of 7) under:
  builtin    the product's held-out per-track order
  lpt        the paths' ACTUAL costs from the golden run, longest first
             (clairvoyant; bounds every order)
  long1st    clairvoyant only about which paths run to the step limit
  shortest   the reverse of lpt (worst case)
  natural    sample-major
and checks that every order gives the golden results.
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


def main():
    dev = torch.device("cuda:0")
    problem = load_problem()
    tgt, dif, _ = prepare_target_params(problem, load_ransac_data(0), 0, 100)
    g = np.load(os.path.join(ROOT, "tests", "golden", "gpuhc_N100_seed0.npz"))
    cost = 4 * g["steps"].astype(np.int64) + g["corrections"].astype(np.int64)
    n = cost.size
    L = _abi.lib()
    L.hc_ab_set_path_order.argtypes = [C.c_void_p]
    L.hc_ab_set_path_order.restype = C.c_int
    if "--timeline" in sys.argv:
        L.hc_diag_span.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
    tr = DeviceTracker(problem, dev)
    r = tr.allocate(100)
    t, d = torch.from_numpy(tgt).to(dev), torch.from_numpy(dif).to(dev)
    s = torch.cuda.current_stream(dev)
    long_ = cost >= 450
    orders = {
        "builtin": None,
        "lpt": np.argsort(-cost, kind="stable"),
        "long1st": np.concatenate([np.flatnonzero(long_), np.flatnonzero(~long_)]),
        "shortest": np.argsort(cost, kind="stable"),
        "natural": np.arange(n),
    }
    print(json.dumps({"paths": int(n), "stages": int(cost.sum()), "long": int(long_.sum()),
                      "max_cost": int(cost.max())}), flush=True)
    for rnd in range(2):
        for name, o in orders.items():
            ot = None if o is None else torch.from_numpy(o.astype(np.int32)).to(dev)
            assert L.hc_ab_set_path_order(None if ot is None else C.c_void_p(ot.data_ptr())) == 0
            ms = []
            kspan = (C.c_ulonglong * 4)()
            for i in range(8):
                if "--timeline" in sys.argv:
                    L.hc_diag_span(kspan, 1)      # reset: the last launch's span is read below
                tr.reset_tracks(r)
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(s)
                tr.launch(t, d, r, stream=s)
                b.record(s)
                torch.cuda.synchronize(dev)
                if i:
                    ms.append(a.elapsed_time(b))
            h = r.host()
            exact = bool((h["converge"] == g["conv"]).all() and (h["stats"]["steps"] == g["steps"]).all()
                         and (h["stats"]["corrections"] == g["corrections"]).all())
            res = {"order": name, "round": rnd, "ms": round(float(np.median(ms)), 3),
                   "min_ms": round(float(np.min(ms)), 3), "exact": exact}
            if "--timeline" in sys.argv:   # build with -DHC_DIAG_TIMES: stats carry dequeue/finish stamps
                t0 = h["stats"]["inliers21"].astype(np.int64) & 0xFFFFFFFF
                t1 = h["stats"]["inliers31"].astype(np.int64) & 0xFFFFFFFF
                base = t0.min()
                t0, t1 = (t0 - base) * 10e-6, (t1 - base) * 10e-6          # ms (100 MHz)
                span = float(t1.max())
                res.update(span_ms=round(span, 3), slot_util=round(float((t1 - t0).sum()) / span / 10240, 4),
                           last_dequeue_ms=round(float(t0.max()), 3),
                           finish_ms_q=[round(float(v), 2) for v in np.percentile(t1, [50, 90, 99, 99.9, 100])],
                           finished_in_last_2ms=int((t1 > span - 2.0).sum()))
                L.hc_diag_span(kspan, 0)   # kernel span and summed wave lifetimes (100 MHz)
                ks = (kspan[1] - kspan[0]) * 1e-5
                res.update(kernel_span_ms=round(ks, 3),
                           first_dequeue_after_ms=round(((int(base) - kspan[0]) & 0xFFFFFFFF) * 1e-5, 3),
                           wave_alive_frac=round(kspan[2] / max(1, kspan[3]) * 1e-5 / ks, 4))
            print(json.dumps(res), flush=True)
    L.hc_ab_set_path_order(None)


if __name__ == "__main__":
    main()
