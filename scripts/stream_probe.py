"""Concurrent launches of the sliced vs unsliced tracker on 1/2/4 streams
(config 2 batches, own buffers and workspace per stream): wall ms per batch.
Usage: python scripts/stream_probe.py OUT.jsonl [STREAMS,...]
(run two copies at once to see launches of two processes on one GPU)"""
import json
import sys
import time

import torch

sys.path.insert(0, ".")
from trifocal_pose_estimation_using_improved_gpuhc_amd import load_problem, load_ransac_data, prepare_target_params  # noqa: E402
from trifocal_pose_estimation_using_improved_gpuhc_amd.tracker import DeviceTracker  # noqa: E402

dev = torch.device("cuda:0")
problem = load_problem()
data = load_ransac_data(0)
S = 100
tgt_np, dif_np, _ = prepare_target_params(problem, data, seed=0, num_samples=S, num_gpus=1)
tgt = torch.from_numpy(tgt_np).to(dev)
dif = torch.from_numpy(dif_np).to(dev)
tr = DeviceTracker(problem, dev)
out = open(sys.argv[1], "w")
for sliced in (True, False):
    for ns in (tuple(int(v) for v in sys.argv[2].split(",")) if len(sys.argv) > 2 else (1, 2, 4)):
        streams = [torch.cuda.Stream(dev) for _ in range(ns)]
        bufs = [tr.allocate(S) for _ in range(ns)]
        wss = [tr.new_workspace(S if sliced else 0) for _ in range(ns)]
        K = 8

        def run(n):
            for i in range(n):
                k = i % ns
                with torch.cuda.stream(streams[k]):
                    tr.reset_tracks(bufs[k])
                tr.launch(tgt, dif, bufs[k], stream=streams[k], workspace=wss[k], time_slicing=sliced)
        run(ns)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        run(K)
        torch.cuda.synchronize(dev)
        el = time.perf_counter() - t0
        import ctypes
        st = [int(tr.L.hc_trifocal_workspace_status(ctypes.c_void_p(w.data_ptr()))) for w in wss]
        rec = {"sliced": sliced, "streams": ns, "batches": K, "ms_per_batch": round(el / K * 1e3, 3), "status": st}
        print(json.dumps(rec), flush=True)
        out.write(json.dumps(rec) + "\n")
        del bufs, wss
out.close()
