"""Multi-rank logic on the CPU: gpu-major sample shards and the early-stop
flag protocol (trifocal_pose_estimation_using_improved_gpuhc_amd/sharding.py),
world_size 2 over gloo.  The GPU launch is replaced by a stand-in that marks
the chunks it "tracked" and raises the flag when a chunk holds a passing
sample, exactly as the abort kernel does with the flag it reads at start."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from trifocal_pose_estimation_using_improved_gpuhc_amd import sharding, split_samples


@pytest.mark.parametrize("n,g", [(8000, 8), (100, 1), (1001, 8), (7, 8), (1000, 3), (0, 2)])
def test_shard_matches_reference_split(n, g):
    sub = split_samples(max(n, 1), g) if n else np.zeros(g, int)
    covered = []
    for rank in range(g):
        off, cnt = sharding.shard(n, g, rank)
        assert cnt == sub[rank]
        assert off == int(sub[:rank].sum())
        covered.extend(range(off, off + cnt))
    assert covered == list(range(n))


def test_chunks_cover_the_shard():
    assert sharding.chunks(10, 4) == [(0, 4), (4, 4), (8, 2)]
    assert sharding.chunks(0, 4) == []
    assert sharding.chunks(125, 125) == [(0, 125)]
    with pytest.raises(ValueError):
        sharding.chunks(10, 0)
    with pytest.raises(ValueError):
        sharding.shard(10, 2, 2)


def test_helpers():
    assert sharding.first_found_seconds([(100, 0), (250, 0)], 100.0) == -1.0
    assert sharding.first_found_seconds([(100, 0), (250, 400)], 100.0) == pytest.approx(3.0)
    assert sharding.first_found_seconds([(0, 0)], 1.0) == -1.0
    ids = sharding.global_batch_ids(np.array([-1, 5, -1, 17]), chunk_offset=2, shard_offset=100)
    assert ids.tolist() == [5 + 312 * 102, 17 + 312 * 102]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, total, chunk, passing, out_dir, use_max=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        off, cnt = sharding.shard(total, world, rank)
        flag = torch.zeros(1, dtype=torch.uint8)
        worked = []

        def launch_chunk(k, o, n):
            if flag.item() == 0:                     # the kernel skips every path once the flag is set
                worked.append(k)
                if any(off + o <= s < off + o + n for s in passing):
                    flag.fill_(1)

        nchunks = sharding.run_abort_chunks(launch_chunk, flag, cnt, chunk,
                                            max_count=sharding.max_shard(total, world) if use_max else None)
        np.save(os.path.join(out_dir, f"r{rank}.npy"), np.array([nchunks, int(flag.item())] + worked, np.int64))
    finally:
        dist.destroy_process_group()


def _run(world, total, chunk, passing, tmp_path, use_max=False):
    mp.start_processes(_worker, args=(world, _free_port(), total, chunk, passing, str(tmp_path), use_max),
                       nprocs=world, join=True, start_method="fork")
    return [np.load(os.path.join(tmp_path, f"r{r}.npy")).tolist() for r in range(world)]


def test_early_stop_propagates_across_ranks(tmp_path):
    """2 ranks x 40 samples, chunks of 10: a pass in rank 1's chunk 1 (global
    sample 55) stops rank 0 after its chunk 1 as well."""
    res = _run(2, 80, 10, [55], tmp_path)
    for r in res:
        nchunks, flag, worked = r[0], r[1], r[2:]
        assert nchunks == 4 and flag == 1
        assert worked == [0, 1]


def test_no_pass_tracks_everything(tmp_path):
    res = _run(2, 50, 10, [], tmp_path)
    assert [r[2:] for r in res] == [[0, 1, 2], [0, 1, 2]]
    assert [r[1] for r in res] == [0, 0]


def test_pass_in_first_chunk_of_rank0(tmp_path):
    res = _run(2, 41, 8, [3], tmp_path)            # uneven shards: 21 / 20
    assert [r[0] for r in res] == [3, 3]
    assert [r[2:] for r in res] == [[0], [0]]


@pytest.mark.timeout(120)
def test_uneven_chunk_counts_do_not_hang(tmp_path):
    """17 samples on 2 ranks in chunks of 8: shards 9 / 8 give rank 0 two
    chunks and rank 1 one.  Every rank must make the same number of flag
    reductions (rank 1 pads with one that launches nothing); a pass in rank
    0's last chunk still reaches rank 1."""
    res = _run(2, 17, 8, [], tmp_path)
    assert [r[0] for r in res] == [2, 1]
    assert [r[2:] for r in res] == [[0, 1], [0]]
    res = _run(2, 17, 8, [8], tmp_path)              # global sample 8 = rank 0's second chunk
    assert [r[1] for r in res] == [1, 1]
    assert [r[2:] for r in res] == [[0, 1], [0]]


@pytest.mark.timeout(120)
def test_max_count_agrees_without_a_host_read(tmp_path):
    """With max_count (every rank knows the largest shard, sharding.max_shard)
    the ranks agree on the number of flag reductions without the extra
    all_reduce + host read: same chunks, same stop, no hang on uneven shards."""
    assert sharding.max_shard(17, 2) == 9 and sharding.max_shard(16, 2) == 8 and sharding.max_shard(5, 8) == 1
    res = _run(2, 17, 8, [8], tmp_path, use_max=True)
    assert [r[0] for r in res] == [2, 1] and [r[1] for r in res] == [1, 1]
    assert [r[2:] for r in res] == [[0, 1], [0]]
    res = _run(3, 80, 10, [55], tmp_path, use_max=True)   # shards 27 / 27 / 26, the pass in rank 2's chunk 0
    assert all(r[1] == 1 for r in res)


def _pose_worker(rank, world, port, cuts, out_dir):
    """Each rank selects over its shard with the oracle (standing in for the
    device kernel) and the shards are merged through gather_pose_selection."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import oracle as O
        from test_pose import _fixture_tracks
        from trifocal_pose_estimation_using_improved_gpuhc_amd import _abi, load_ransac_data
        d = load_ransac_data(0)
        g, tr, conv = _fixture_tracks()
        tr[312 * 99 + 7] = tr[int(g["path"][0])]
        conv[312 * 99 + 7] = 1
        a, b = cuts[rank] * 312, cuts[rank + 1] * 312
        _, s = O.pose_support(tr[a:b], conv[a:b], d.locations, d.K)
        st = _abi.hcPoseSelection()
        for k in ("num_candidates", "path21", "inliers21", "path31", "inliers31"):
            setattr(st, k, int(s[k]))
        if s["num_candidates"]:
            st.key21 = (s["inliers21"] << 32) | s["path21"]
            st.key31 = (s["inliers31"] << 32) | s["path31"]
        for k in ("R21", "t21", "R31", "t31"):
            getattr(st, k)[:] = [float(v) for v in s[k]]
        raw = torch.from_numpy(np.frombuffer(bytes(st), np.uint8).copy())
        m = sharding.gather_pose_selection(raw, a)
        np.save(os.path.join(out_dir, f"p{rank}.npy"),
                np.array([m["num_candidates"], m["path21"], m["inliers21"], m["path31"], m["inliers31"]], np.int64))
    finally:
        dist.destroy_process_group()


def test_pose_selection_merges_across_ranks(tmp_path, oracle):
    """world 2 (gloo): merged selection == the oracle's selection over all paths."""
    from test_pose import _fixture_tracks
    from trifocal_pose_estimation_using_improved_gpuhc_amd import load_ransac_data
    d = load_ransac_data(0)
    g, tr, conv = _fixture_tracks()
    tr[312 * 99 + 7] = tr[int(g["path"][0])]
    conv[312 * 99 + 7] = 1
    full = oracle.pose_support(tr, conv, d.locations, d.K)[1]
    cuts = [0, 68, 100]
    mp.start_processes(_pose_worker, args=(2, _free_port(), cuts, str(tmp_path)), nprocs=2, join=True,
                       start_method="fork")
    exp = [full["num_candidates"], full["path21"], full["inliers21"], full["path31"], full["inliers31"]]
    for r in range(2):
        assert np.load(os.path.join(tmp_path, f"p{r}.npy")).tolist() == exp
