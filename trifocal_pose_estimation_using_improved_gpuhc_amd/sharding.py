"""Multi-GPU sharding of RANSAC samples and the early-stop ("good pose found") flag.

One process per GPU (torch.distributed; backend "nccl" == RCCL on ROCm).  RANSAC
samples are independent, so each rank tracks its own contiguous gpu-major shard
-- the reference's split (magmaHC/GPU_HC_Solver.cpp:85-88, 263-265) -- and the
data path needs no collective.  RCCL carries only:

  * the early-stop flag in abort mode: a rank's samples run in chunks; after
    every chunk launch a 1-byte all_reduce(MAX) of the rank's found flag is
    enqueued on the same stream, and the next chunk's table-prep kernel copies
    the reduced flag into the workspace, so every rank skips its remaining
    paths once any rank has found a passing hypothesis.  Nothing synchronises
    with the host between chunks (stream order does it);
  * the maximal-support pose: each rank selects over its own paths on the
    device (hc_trifocal_pose_support); the 136-byte selections are
    all-gathered and merged by key (hc_pose_merge) as if one launch had
    covered every rank's paths (gather_pose_selection);
  * timing (barrier, max / min over ranks) in bench.py.

With a SharedFlag (hcAbortArgs::peer_found) the stop no longer waits for a
chunk boundary: the flag lives in one rank's device memory, every other rank
maps it (hipIpcOpenMemHandle over xGMI), a launch sets it with a system-scope
store when it finds a pose and polls it before every path it starts (with
inflight_stop also at every step boundary).  The chunk-boundary reduction
stays as the fallback and for the found bytes the host reads.

The reference has no cross-GPU early stop: each GPU keeps its own flag
(GPU_HC_Solver.cpp:308-333).  With one rank the protocol reduces to the
reference behaviour.
"""
from __future__ import annotations

from typing import Callable, List, Tuple

import numpy as np


def shard(num_samples: int, world: int, rank: int) -> Tuple[int, int]:
    """(offset, count) of rank's samples: N/G + (g < N%G) each, gpu-major."""
    if world <= 0 or not 0 <= rank < world or num_samples < 0:
        raise ValueError("bad shard request")
    base, extra = divmod(num_samples, world)
    count = base + (1 if rank < extra else 0)
    offset = rank * base + min(rank, extra)
    return offset, count


def chunks(count: int, chunk_samples: int) -> List[Tuple[int, int]]:
    """Split a rank's `count` samples into launches of at most chunk_samples."""
    if chunk_samples <= 0:
        raise ValueError("chunk_samples must be positive")
    return [(o, min(chunk_samples, count - o)) for o in range(0, count, chunk_samples)]


def run_abort_chunks(launch_chunk: Callable[[int, int, int], None], flag, count: int, chunk_samples: int,
                     group=None, stream=None, max_count: int | None = None) -> int:
    """Early-stop protocol over this rank's samples.

    launch_chunk(k, offset, n) enqueues chunk k (samples [offset, offset+n) of
    the shard); the launch reads `flag` when it starts and sets it when a
    passing hypothesis is found.  After each launch the flag is max-reduced
    over all ranks.  Every rank makes the same number of reductions -- the
    largest chunk count over the ranks, so a rank whose shard is a chunk
    shorter (uneven sample counts) pads with reductions that launch nothing
    instead of leaving its peers waiting.  The caller that knows the largest
    shard (max_count: every rank computes shard() of every rank) passes it and
    nothing synchronises with the host; without it one extra all_reduce agrees
    on the count (a host read).  With
    RCCL the reductions and the launches are ordered on `stream` (the launch
    stream; default: the current stream), so nothing synchronises with the
    host between chunks; with gloo they are synchronous.  Returns the number
    of chunks this rank launched (all of its own: a chunk that starts with the
    flag set skips its paths on the device).
    """
    import contextlib

    import torch
    import torch.distributed as dist
    parts = chunks(count, chunk_samples)
    multi = dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1
    on_gpu = getattr(flag, "is_cuda", False)
    ctx = torch.cuda.stream(stream) if (on_gpu and stream is not None) else contextlib.nullcontext()
    with ctx:
        rounds = len(parts)
        if multi and max_count is not None:
            rounds = max(rounds, len(chunks(max_count, chunk_samples)))
        elif multi:
            n = torch.tensor([rounds], dtype=torch.int64, device=flag.device)
            dist.all_reduce(n, op=dist.ReduceOp.MAX, group=group)
            rounds = int(n.item())
        for k in range(rounds):
            if k < len(parts):
                launch_chunk(k, *parts[k])
            if multi:
                dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=group)
    return len(parts)


def max_shard(num_samples: int, world: int) -> int:
    """The largest shard of num_samples over world ranks (rank 0's: the first
    num_samples % world ranks take one extra sample)."""
    return shard(num_samples, world, 0)[1]


def first_found_seconds(stamps: List[Tuple[int, int]], tick_hz: float) -> float:
    """Time from the first chunk's start to the earliest found stamp of this
    rank's chunk workspaces ((start_ticks, found_ticks) per chunk, 0 = none);
    -1 if nothing was found."""
    starts = [s for s, _ in stamps if s]
    found = [f for _, f in stamps if f]
    if not starts or not found:
        return -1.0
    return float(min(found) - min(starts)) / tick_hz


def global_batch_ids(local_batch_index: np.ndarray, chunk_offset: int, shard_offset: int) -> np.ndarray:
    """Batch ids written by a chunk launch (b = sample*312 + track within the
    launch, reference layout) -> ids in the whole RANSAC run."""
    ids = np.asarray(local_batch_index)
    ids = ids[ids >= 0]
    return ids + 312 * (chunk_offset + shard_offset)


def gather_pose_selection(selection, path_offset: int, group=None, quirks: bool = False) -> dict:
    """All-gathers every rank's raw hcPoseSelection bytes (a uint8 tensor on the
    rank's device, or on the CPU for gloo) and merges them with the ranks'
    first global batch ids.  Returns the merged selection (global batch ids)
    on every rank."""
    import torch
    import torch.distributed as dist

    from . import pose
    multi = dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1
    if not multi:
        return pose.merge([selection], [path_offset], quirks)
    world = dist.get_world_size(group)
    sel = selection.reshape(-1)[:pose.SEL_BYTES].contiguous()
    parts = [torch.empty_like(sel) for _ in range(world)]
    dist.all_gather(parts, sel, group=group)
    off = torch.tensor([path_offset], dtype=torch.int64, device=sel.device)
    offs = [torch.empty_like(off) for _ in range(world)]
    dist.all_gather(offs, off, group=group)
    return pose.merge([p.cpu().numpy() for p in parts], [int(o.item()) for o in offs], quirks)


class SharedFlag:
    """The cross-process early-stop flag of a multi-GPU abort run
    (hcAbortArgs::peer_found; include/hc_trifocal.h hc_shared_flag_*).

    Rank `owner` of `group` allocates it in its device memory; the 64-byte IPC
    handle is broadcast over torch.distributed (a CPU tensor for gloo, a device
    tensor for RCCL) and every other rank maps it with hipIpcOpenMemHandle.
    Construction is collective.  If any rank cannot create or map it, every
    rank gets .ptr = None (the chunk-boundary reduction alone then stops the
    run) and .error says why."""

    def __init__(self, group=None, owner: int = 0, device=None):
        import ctypes as C

        import torch
        import torch.distributed as dist

        from . import _abi
        self._L = _abi.lib()
        self.ptr = None
        self.opened = False
        self.error = None
        rank = dist.get_rank(group)
        src = dist.get_global_rank(group, owner) if group is not None else owner
        on_gpu = dist.get_backend(group) == "nccl"
        dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        handle = _abi.hcIpcHandle()
        p = C.c_void_p()
        ok = 1
        if rank == owner:
            st = self._L.hc_shared_flag_create(C.byref(p), C.byref(handle))
            if st != 0:
                ok, self.error = 0, f"hc_shared_flag_create: {_abi.HC_STATUS.get(st, st)}"
        buf = torch.tensor(list(bytes(handle.reserved)), dtype=torch.uint8, device=dev if on_gpu else "cpu")
        dist.broadcast(buf, src=src, group=group)
        if rank != owner:
            C.memmove(handle.reserved, bytes(buf.cpu().tolist()), 64)
            st = self._L.hc_shared_flag_open(C.byref(handle), C.byref(p))
            if st != 0:
                ok, self.error = 0, f"hc_shared_flag_open: {_abi.HC_STATUS.get(st, st)} " \
                                    f"({self._L.hc_last_error_string().decode(errors='replace')})"
            else:
                self.opened = True
        agree = torch.tensor([ok], dtype=torch.int32, device=dev if on_gpu else "cpu")
        dist.all_reduce(agree, op=dist.ReduceOp.MIN, group=group)
        if int(agree.item()) == 1:
            self.ptr = p.value
        elif p.value:
            self._L.hc_shared_flag_close(C.c_void_p(p.value), 1 if self.opened else 0)
            self.error = self.error or "another rank could not map the flag"
        self._group = group
        self._owner = owner
        self._rank = rank

    def arm(self, stream=None) -> None:
        """Zeroes the flag before a run.  Every rank first drains its device
        (a launch of the previous run still queued on a non-owner rank could
        otherwise set the flag after the reset), then the owner resets and
        synchronises, and a barrier on both sides orders the reset after every
        rank's previous launches and before any rank's next one."""
        import ctypes as C

        import torch
        import torch.distributed as dist
        if self.ptr is None:
            return
        s = stream if stream is not None else torch.cuda.current_stream()
        torch.cuda.synchronize(s.device)
        dist.barrier(group=self._group)
        if self._rank == self._owner:
            st = self._L.hc_shared_flag_reset(C.c_void_p(self.ptr), C.c_void_p(s.cuda_stream))
            if st != 0:
                raise RuntimeError(f"hc_shared_flag_reset failed: {st}")
            s.synchronize()
        dist.barrier(group=self._group)

    @property
    def memory_kind(self):
        """The owner's allocation (include/hc_trifocal.h hc_shared_flag_memory_kind):
        'uncached', 'fine-grained', 'coarse-grained', or None on a mapping rank."""
        import ctypes as C
        if self.ptr is None or self._rank != self._owner:
            return None
        k = self._L.hc_shared_flag_memory_kind(C.c_void_p(self.ptr))
        return {2: "uncached", 1: "fine-grained", 0: "coarse-grained"}.get(k)

    def close(self) -> None:
        """Collective: the mapping ranks unmap before the owner frees."""
        import ctypes as C

        import torch.distributed as dist
        if self.ptr is None:
            return
        if self.opened:
            self._L.hc_shared_flag_close(C.c_void_p(self.ptr), 1)
        dist.barrier(group=self._group)
        if not self.opened:
            self._L.hc_shared_flag_close(C.c_void_p(self.ptr), 0)
        self.ptr = None
