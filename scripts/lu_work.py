#!/usr/bin/env python3
"""Executed LU work of the tracker (GPU only, development tool).

Needs the HC_DIAG_LUWORK build (scripts/build_variant.sh luwork -DHC_DIAG_LUWORK,
loaded through HC_TRIFOCAL_LIB): every LU solve adds the rank-1 update
elements it executes (columns of the executed column groups x lanes of active
path slots below the pivot).  The dense algorithm (the reference's) updates
sum_{I} (29 - I)^2 = 8555 elements per solve; the structurally sparse LU skips
column groups that are zero in both pivot rows of a wave.  Prints the executed
fraction for one config-2 launch; bench.py prices the LU's update FLOPs with it.
Also counts the solves the sparse LU handed to the dense re-solve (round 3).
--scaled: the input of tests/test_gpu_parity.py::test_tracker_dense_resolve_
matches_oracle instead (sample 0 and its target parameters x 2^40 and x 2^70),
to show that test reaches the dense re-solve.
"""
import ctypes as C
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from trifocal_pose_estimation_using_improved_gpuhc_amd import _abi, load_problem, load_ransac_data, prepare_target_params  # noqa
from trifocal_pose_estimation_using_improved_gpuhc_amd.tracker import DeviceTracker  # noqa

DENSE_UPDATE_ELEMENTS = sum((29 - i) ** 2 for i in range(30))   # 8555


def main():
    L = _abi.lib()
    fn = L.hc_diag_luwork
    fn.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
    fn.restype = C.c_int
    out = (C.c_ulonglong * 10)()
    dev = torch.device("cuda:0")
    problem = load_problem()
    argv = sys.argv[1:]
    ds = int(argv[argv.index("--dataset") + 1]) if "--dataset" in argv else 0
    seed = int(argv[argv.index("--seed") + 1]) if "--seed" in argv else 0
    data = load_ransac_data(ds)
    if "--sigma" in argv:   # noisy synthcurves of the dataset (trifocal_..._amd/synthcurves.py)
        from trifocal_pose_estimation_using_improved_gpuhc_amd import synthcurves
        data = synthcurves.noisy(data, float(argv[argv.index("--sigma") + 1]), synthcurves.DEFAULT_SEED)
    if "--shard8" in argv:   # rank g's shard of an 8-GPU config-2 run
        g8 = int(argv[argv.index("--shard8") + 1])
        ta, da, _ = prepare_target_params(problem, data, seed, 800, num_gpus=8)
        tgt, dif = ta[100 * g8:100 * g8 + 100].copy(), da[100 * g8:100 * g8 + 100].copy()
    else:
        tgt, dif, _ = prepare_target_params(problem, data, seed, 100)
    scaled = "--scaled" in argv
    if scaled:
        tgt = np.stack([tgt[0]] + [(tgt[0] * np.float32(s)).astype(np.float32) for s in (2.0 ** 40, 2.0 ** 70)])
        dif = (tgt - problem.start_params[None]).astype(np.float32)
    tr = DeviceTracker(problem, dev)
    r = tr.allocate(tgt.shape[0])
    tr.reset_tracks(r)
    torch.cuda.synchronize()
    if fn(out, 1) != 0:
        raise RuntimeError("hc_diag_luwork failed (a diagnostic build of other sources?)")
    tr.launch(torch.from_numpy(tgt).to(dev), torch.from_numpy(dif).to(dev), r)
    torch.cuda.synchronize()
    if fn(out, 1) != 0:
        raise RuntimeError("hc_diag_luwork failed")
    st = r.stats.cpu().numpy()
    stages = 4 * int(st[:, 0].sum()) + int(st[:, 1].sum())
    elems, solves, dense = int(out[0]), int(out[1]), int(out[2])
    wsolves, groups, rare = int(out[3]), int(out[4]), int(out[5])
    ev = [int(out[6]), int(out[7]), int(out[8])]
    res = {"config": ("sample 0 of config 2 + its target params x 2^40, x 2^70 (one launch)" if scaled
                      else "config 2 (100 samples, abort off), one launch" +
                      ("" if (ds, seed) == (0, 0) and "--sigma" not in argv else
                       f", dataset {ds:03d}, srand({seed})" + (f", sigma {argv[argv.index('--sigma') + 1]} px"
                                                              if "--sigma" in argv else ""))),
           "sparse_solves_completed": solves, "path_stages": stages,
           "solves_rerun_densely": dense,
           "check": "sparse_solves_completed + solves_rerun_densely == path_stages",
           "check_ok": solves + dense == stages,
           "executed_update_elements": elems,
           "executed_update_elements_per_solve": elems / max(1, solves),
           "dense_update_elements_per_solve": DENSE_UPDATE_ELEMENTS,
           "executed_fraction": elems / max(1, solves) / DENSE_UPDATE_ELEMENTS,
           "wave_solves": wsolves,
           "live_groups_per_wave_solve": groups / max(1, wsolves),
           "rare_steps_per_wave_solve": rare / max(1, wsolves),
           "wave_stages": sum(ev),
           "rhs_eval_kinds": {"mixed": ev[0], "dHdt_only": ev[1], "H_only": ev[2]},
           "prefix_rebuilds": int(out[9]),
           "prefix_rebuilds_per_wave_stage": int(out[9]) / max(1, sum(ev)),
           # the product build of the same sources (bench.py prices its LU with this file)
           "build_id": _abi.build_id(_abi.PRODUCT_LIB_PATH),
           "diag_build_id": _abi.build_id(),
           "measured_at": time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime())}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
