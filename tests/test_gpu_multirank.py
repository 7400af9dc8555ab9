"""The multi-GPU paths on the one GPU a test box has.

1. Two ranks (torch.distributed, gloo over GPU tensors), both on cuda:0,
   started before anything touches the GPU: each runs the real
   DeviceTracker.launch_abort_chunked on its gpu-major shard (the RCCL code
   path with gloo as the transport) and gather_pose_selection over its device
   pose support.  The 99 samples 1..99 of the seed-0 run are used so that the
   only passing hypothesis of rank 1's shard (sample 51) sits in its first
   chunk and rank 0's shard has none: the flag raised on rank 1 must stop
   rank 0 after its first chunk.  Every tracked path equals the single-rank
   golden run, and the merged pose equals the oracle's selection over the
   union of both ranks' paths.
2. The C++ GPU_HC_Solver multi-device loop (GPU_HC_Solver.cpp:85-88,390-444,
   494-506) with 2 and 3 logical GPUs sharing device 0 (Share_Devices): the
   statistics and the pose equal the one-GPU run.
"""
import os
import shutil
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
GOLDEN = os.path.join(HERE, "golden")
FIRST, TOTAL, CHUNK = 1, 99, 10      # samples 1..99 of the seed-0 run


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(rank, world, port, out_dir):
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from trifocal_pose_estimation_using_improved_gpuhc_amd import (load_problem, load_ransac_data, pose,
                                                                       prepare_target_params, sharding)
        from trifocal_pose_estimation_using_improved_gpuhc_amd.tracker import DeviceTracker
        dev = torch.device("cuda:0")
        problem = load_problem()
        data = load_ransac_data(0)
        tgt, dif, _ = prepare_target_params(problem, data, seed=0, num_samples=FIRST + TOTAL)
        off, cnt = sharding.shard(TOTAL, world, rank)
        t = torch.from_numpy(tgt[FIRST + off:FIRST + off + cnt]).to(dev)
        d = torch.from_numpy(dif[FIRST + off:FIRST + off + cnt]).to(dev)
        tr = DeviceTracker(problem, dev)
        tr.set_ransac_data(data)
        r = tr.allocate(cnt, stats=True, abort=True)
        tr.reset_tracks(r)
        wss = []
        stream = torch.cuda.Stream(dev)
        parts = tr.launch_abort_chunked(t, d, r, CHUNK, wss, stream=stream)
        torch.cuda.synchronize(dev)
        inl = torch.empty((cnt * 312, 2), dtype=torch.int32, device=dev)
        sel = torch.empty(pose.SEL_BYTES, dtype=torch.uint8, device=dev)
        pose.launch_pose_support(r.tracks, r.converge, tr.edgels, tr.K, inl, sel)
        torch.cuda.synchronize(dev)
        merged = sharding.gather_pose_selection(sel, (FIRST + off) * 312)
        h = r.host()
        np.savez(os.path.join(out_dir, f"rank{rank}.npz"), off=off, cnt=cnt, nchunks=len(parts),
                 tracks=h["tracks"], conv=h["converge"], inf=h["infinity"], steps=h["stats"]["steps"],
                 corrections=h["stats"]["corrections"], batch_index=h["batch_index"], found=h["found"],
                 merged=np.array([merged["num_candidates"], merged["path21"], merged["inliers21"],
                                  merged["path31"], merged["inliers31"]], np.int64))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(240)
def test_two_ranks_share_cuda0_abort_and_pose(tmp_path, oracle, ransac0):
    import torch.multiprocessing as mp
    sys.path.insert(0, GOLDEN)
    from make_golden import track_hash
    mp.start_processes(_rank_main, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True, start_method="spawn")
    g = np.load(os.path.join(GOLDEN, "gpuhc_N100_seed0.npz"))
    passing = set(int(b) for b, s in zip(g["scored_ids"], g["scored"]) if s[0] == 1)
    R = [np.load(os.path.join(tmp_path, f"rank{r}.npz")) for r in range(2)]
    assert [int(x["cnt"]) for x in R] == [50, 49] and [int(x["nchunks"]) for x in R] == [5, 5]
    for x in R:
        base = (FIRST + int(x["off"])) * 312          # global batch id of the rank's first path
        n = int(x["cnt"]) * 312
        gl = slice(base, base + n)
        tracked = x["steps"] > 0
        assert (x["conv"][tracked] == g["conv"][gl][tracked]).all()
        assert (x["steps"][tracked] == g["steps"][gl][tracked]).all()
        assert (track_hash(x["tracks"])[tracked] == g["hash"][gl][tracked]).all()
        assert bool(x["found"])                       # the reduced flag reached every rank
        ids = np.nonzero(x["batch_index"] >= 0)[0]
        assert set(int(b) + base for b in ids) <= passing
    r0, r1 = R
    # rank 0 (samples 1..50, no passing hypothesis) tracked its first chunk in full and
    # nothing after it: rank 1's flag from its first chunk (sample 51) stopped it
    t0 = r0["steps"] > 0
    assert t0[:CHUNK * 312].all() and not t0[CHUNK * 312:].any()
    assert len(np.nonzero(r0["batch_index"] >= 0)[0]) == 0
    assert len(np.nonzero(r1["batch_index"] >= 0)[0]) > 0
    assert not (r1["steps"][CHUNK * 312:] > 0).any()
    # merged pose == the oracle's selection over the union of the ranks' paths
    tr = np.concatenate([r0["tracks"], r1["tracks"]])
    cv = np.concatenate([r0["conv"], r1["conv"]])
    _, sel = oracle.pose_support(tr, cv, ransac0.locations, ransac0.K)
    exp = [sel["num_candidates"], sel["path21"] + FIRST * 312, sel["inliers21"], sel["path31"] + FIRST * 312,
           sel["inliers31"]]
    for x in R:
        assert x["merged"].tolist() == exp


def _rank_main_shared_flag(rank, world, port, out_dir):
    """One abort launch per rank over its whole shard (no chunk boundary to
    carry the flag), in-flight stop on, with the cross-process SharedFlag."""
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from trifocal_pose_estimation_using_improved_gpuhc_amd import (load_problem, load_ransac_data,
                                                                       prepare_target_params, sharding)
        from trifocal_pose_estimation_using_improved_gpuhc_amd.tracker import DeviceTracker
        dev = torch.device("cuda:0")
        problem = load_problem()
        data = load_ransac_data(0)
        tgt, dif, _ = prepare_target_params(problem, data, seed=0, num_samples=FIRST + TOTAL)
        off, cnt = sharding.shard(TOTAL, world, rank)
        t = torch.from_numpy(tgt[FIRST + off:FIRST + off + cnt]).to(dev)
        d = torch.from_numpy(dif[FIRST + off:FIRST + off + cnt]).to(dev)
        tr = DeviceTracker(problem, dev)
        tr.set_ransac_data(data)
        r = tr.allocate(cnt, stats=True, abort=True)
        tr.reset_tracks(r)
        flag = sharding.SharedFlag(device=dev)
        assert flag.ptr is not None, flag.error
        stream = torch.cuda.Stream(dev)
        flag.arm(stream)
        wss = []
        parts = tr.launch_abort_chunked(t, d, r, cnt, wss, stream=stream, inflight_stop=True, peer_found=flag)
        torch.cuda.synchronize(dev)
        h = r.host()
        kind = flag.memory_kind
        dist.barrier()
        flag.close()
        np.savez(os.path.join(out_dir, f"rank{rank}.npz"), off=off, cnt=cnt, nchunks=len(parts),
                 tracks=h["tracks"], conv=h["converge"], steps=h["stats"]["steps"],
                 batch_index=h["batch_index"], found=h["found"], kind=str(kind))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(240)
def test_two_ranks_shared_flag_stops_other_rank_mid_launch(tmp_path, oracle, ransac0):
    """The cross-process flag (hcAbortArgs::peer_found, sharding.SharedFlag) on
    two ranks sharing cuda:0, each tracking its whole 49/50-sample shard in ONE
    abort launch: rank 1's first hypothesis (sample 51) passes, and rank 0 --
    which has no passing hypothesis and no chunk boundary to learn of it --
    stops within that launch (fewer than its 15 600 paths completed).  Every
    completed path equals the single-rank golden run, and the merged pose
    equals the oracle's selection over both ranks' paths."""
    import torch.multiprocessing as mp
    sys.path.insert(0, GOLDEN)
    from make_golden import track_hash
    mp.start_processes(_rank_main_shared_flag, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True,
                       start_method="spawn")
    g = np.load(os.path.join(GOLDEN, "gpuhc_N100_seed0.npz"))
    passing = set(int(b) for b, s in zip(g["scored_ids"], g["scored"]) if s[0] == 1)
    R = [np.load(os.path.join(tmp_path, f"rank{r}.npz")) for r in range(2)]
    assert [int(x["nchunks"]) for x in R] == [1, 1]
    for x in R:
        base = (FIRST + int(x["off"])) * 312
        gl = slice(base, base + int(x["cnt"]) * 312)
        done = x["steps"] > 0
        assert (x["conv"][done] == g["conv"][gl][done]).all()
        assert (track_hash(x["tracks"])[done] == g["hash"][gl][done]).all()
        assert (x["conv"][~done] == 0).all()
        ids = np.nonzero(x["batch_index"] >= 0)[0]
        assert set(int(b) + base for b in ids) <= passing
    r0, r1 = R
    # the owner's flag is in memory that is coherent across devices while
    # kernels run (uncached; fine-grained where the device cannot export that)
    assert str(r0["kind"]) in ("uncached", "fine-grained"), str(r0["kind"])
    assert str(r1["kind"]) == "None"
    assert len(np.nonzero(r1["batch_index"] >= 0)[0]) > 0 and bool(r1["found"])
    assert len(np.nonzero(r0["batch_index"] >= 0)[0]) == 0
    assert bool(r0["found"])          # the chunk-boundary reduction still delivers the byte
    n0 = int((r0["steps"] > 0).sum())
    assert n0 < int(r0["cnt"]) * 312, f"rank 0 completed all {n0} paths: the peer flag never stopped it"


@pytest.mark.timeout(300)
@pytest.mark.parametrize("gpus", [2, 3])
def test_cli_logical_gpus_share_device(tmp_path, gpus):
    """magmaHC-main -g N --share-devices: N gpu-major shards, N streams on device 0,
    results stacked: the statistics and the selected pose equal the golden one-GPU run."""
    cli = os.path.join(ROOT, "trifocal_pose_estimation_using_improved_gpuhc_amd", "bin", "magmaHC-main")
    shutil.copytree(os.path.join(ROOT, "data"), os.path.join(tmp_path, "data"))
    out = subprocess.run([cli, "-p", "trifocal_2op1p_30x30", "-d", str(tmp_path), "-g", str(gpus), "--share-devices"],
                         capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stdout + out.stderr
    g = np.load(os.path.join(GOLDEN, "gpuhc_N100_seed0.npz"))
    stats = open(os.path.join(tmp_path, "Output_Write_Files", "GPU_Sols_Statistics.txt")).read().split()
    assert [int(v) for v in stats[:3]] == [int(v) for v in g["counts"]]
    pr = open(os.path.join(tmp_path, "Output_Write_Files", "GPU_Pose_Results.txt")).read().split()
    gp = np.load(os.path.join(GOLDEN, "pose_N100_seed0.npz"))
    assert int(pr[0]) == 1 and [int(pr[5]), int(pr[6])] == gp["path"].tolist()
    assert int(pr[7]) == int(gp["num_candidates"])


@pytest.mark.timeout(300)
def test_cli_abort_across_gpus_share_device(tmp_path):
    """magmaHC-main --abort --abort-across-gpus on 2 logical GPUs sharing device 0:
    the C++ GPU_HC_Solver allocates one found flag for both launches
    (Abort_Across_GPUs, hcAbortArgs::peer_found).  The run finds a pose that
    matches GT, and it tracks no more than the abort-off golden run converges
    (the skipped paths report conv = 0)."""
    cli = os.path.join(ROOT, "trifocal_pose_estimation_using_improved_gpuhc_amd", "bin", "magmaHC-main")
    shutil.copytree(os.path.join(ROOT, "data"), os.path.join(tmp_path, "data"))
    out = subprocess.run([cli, "-p", "trifocal_2op1p_30x30", "-d", str(tmp_path), "-g", "2", "--share-devices",
                          "--abort", "--inflight-stop", "--abort-across-gpus"],
                         capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stdout + out.stderr
    g = np.load(os.path.join(GOLDEN, "gpuhc_N100_seed0.npz"))
    stats = [int(v) for v in open(os.path.join(tmp_path, "Output_Write_Files", "GPU_Sols_Statistics.txt")).read().split()[:2]]
    assert 0 < stats[0] <= int(g["counts"][0]) and stats[1] <= int(g["counts"][1])
    pr = open(os.path.join(tmp_path, "Output_Write_Files", "GPU_Pose_Results.txt")).read().split()
    assert int(pr[0]) == 1
