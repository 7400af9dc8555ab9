#!/usr/bin/env python3
"""How often each LU column group is live, per pivot step (GPU only, development tool).

Needs the HC_DIAG_LIVE build (scripts/build_variant.sh live -DHC_DIAG_LIVE,
loaded through HC_TRIFOCAL_LIB).  One config-2 launch (or --dataset / --seed);
every eighth workgroup counts, per pivot step I and column group K of the
sparse solve (hc_lu.hpp LuChunks<2>), the wave-solves whose group test found
the group live.  Prints one JSON object: live[I][K] as a fraction of the
sampled wave-solves, and the groups live in at least 0.99 / 0.999 of them.
"""
import ctypes as C
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from trifocal_pose_estimation_using_improved_gpuhc_amd import _abi, load_problem, load_ransac_data, prepare_target_params  # noqa
from trifocal_pose_estimation_using_improved_gpuhc_amd.tracker import DeviceTracker  # noqa

NV, SOLVES = 30, 16


def chunks(i, ch=2):
    """(start, len) of the column groups of step i (LuChunks<2>)."""
    single = 1 if ((i + 1) & 1) and (i + 1 < NV) else 0
    out = [(i + 1, 1)] if single else []
    j = i + 1 + single
    while j < NV:
        out.append((j, min(ch, NV - j)))
        j += ch
    return out


def main():
    L = _abi.lib()
    fn = L.hc_diag_live
    fn.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
    fn.restype = C.c_int
    out = (C.c_ulonglong * (NV * (SOLVES + 1)))()
    argv = sys.argv[1:]
    ds = int(argv[argv.index("--dataset") + 1]) if "--dataset" in argv else 0
    seed = int(argv[argv.index("--seed") + 1]) if "--seed" in argv else 0
    dev = torch.device("cuda:0")
    problem = load_problem()
    tgt, dif, _ = prepare_target_params(problem, load_ransac_data(ds), seed, 100)
    tr = DeviceTracker(problem, dev)
    r = tr.allocate(tgt.shape[0])
    tr.reset_tracks(r)
    torch.cuda.synchronize()
    if fn(out, 1) != 0:
        raise RuntimeError("hc_diag_live failed (not the HC_DIAG_LIVE build?)")
    tr.launch(torch.from_numpy(tgt).to(dev), torch.from_numpy(dif).to(dev), r)
    torch.cuda.synchronize()
    if fn(out, 1) != 0:
        raise RuntimeError("hc_diag_live failed")
    live, ge99, ge999, never = [], [], [], []
    for i in range(NV - 1):
        row = out[i * (SOLVES + 1):(i + 1) * (SOLVES + 1)]
        n = max(1, int(row[SOLVES]))
        fr = [int(row[k]) / n for k in range(len(chunks(i)))]
        live.append([round(f, 5) for f in fr])
        for k, f in enumerate(fr):
            (ge999 if f >= 0.999 else ge99 if f >= 0.99 else never if f == 0.0 else []).append([i, k])
    print(json.dumps({"config": f"config 2, dataset {ds:03d}, srand({seed}), one launch, every 8th workgroup",
                      "sampled_wave_solves": int(out[SOLVES]), "live": live,
                      "groups": sum(len(x) for x in live), "expected_live": round(sum(sum(x) for x in live), 2),
                      "live_ge_0999": ge999, "live_099_0999": ge99, "never_live": never,
                      "diag_build_id": _abi.build_id(),
                      "measured_at": time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime())}))


if __name__ == "__main__":
    main()
