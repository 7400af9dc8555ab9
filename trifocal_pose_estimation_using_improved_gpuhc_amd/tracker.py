"""Device-side driver of the HIP tracker (one GPU / one process).

torch is used only as plumbing: device allocations, the HIP stream and events.
All compute runs in the native kernels behind include/hc_trifocal.h.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np
import torch

from . import _abi
from .problem import Problem, RansacData

PATH_STATS_DTYPE = np.dtype([("steps", "<i4"), ("corrections", "<i4"), ("inliers21", "<i4"), ("inliers31", "<i4")])


def _ptr(t: torch.Tensor | None):
    return None if t is None else C.c_void_p(t.data_ptr())


def _require_gpu(device) -> torch.device:
    dev = torch.device(device)
    if dev.type != "cuda" or not torch.cuda.is_available():
        raise _abi.HCError("the GPU-HC tracker needs a ROCm GPU (no CPU fallback exists)")
    return dev


@dataclass
class TrackResult:
    tracks: torch.Tensor          # (312N, 31, 2) float32 on device
    converge: torch.Tensor        # (312N,) uint8
    infinity: torch.Tensor        # (312N,) uint8
    stats: torch.Tensor | None    # (312N, 4) int32 [steps, corrections, inliers21, inliers31]
    found: torch.Tensor | None = None         # abort mode: (1,) uint8
    batch_index: torch.Tensor | None = None   # abort mode: (312N,) int32

    def host(self):
        out = dict(tracks=self.tracks.cpu().numpy(), converge=self.converge.cpu().numpy(),
                   infinity=self.infinity.cpu().numpy())
        if self.stats is not None:
            out["stats"] = self.stats.cpu().numpy().view(PATH_STATS_DTYPE).reshape(-1)
        if self.found is not None:
            out["found"] = bool(self.found.cpu().item())
            out["batch_index"] = self.batch_index.cpu().numpy()
        return out


class DeviceTracker:
    """Holds the problem constants on one device and launches tracking runs.

    Mirrors what GPU_HC_Solver keeps per GPU (magmaHC/GPU_HC_Solver.cpp:137-184):
    start solutions, start parameters, the unified dH/dx||dH/dt index table.
    """

    def __init__(self, problem: Problem, device="cuda:0", max_steps=None, max_corrections=None,
                 delta_t_inc_steps=None):
        self.device = _require_gpu(device)
        self.L = _abi.lib()
        s = problem.settings
        self.settings = _abi.hcTrackSettings(
            int(max_steps if max_steps is not None else s.get("GPUHC_Max_Steps", 80)),
            int(max_corrections if max_corrections is not None else s.get("GPUHC_Max_Correction_Steps", 3)),
            int(delta_t_inc_steps if delta_t_inc_steps is not None else
                s.get("GPUHC_Num_Of_Steps_to_Increase_Delta_t", 4)))
        dev = self.device
        self.start_sols = torch.from_numpy(problem.start_sols).to(dev)
        self.start_params = torch.from_numpy(problem.start_params).to(dev)
        self.unified = torch.from_numpy(problem.unified_index).to(dev)
        self.ws_bytes = int(self.L.hc_trifocal_workspace_size())
        self.workspace = torch.zeros(self.ws_bytes, dtype=torch.uint8, device=dev)
        self.edgels = None
        self.K = None

    def set_ransac_data(self, data: RansacData):
        self.edgels = torch.from_numpy(np.ascontiguousarray(data.locations)).to(self.device)
        self.K = torch.from_numpy(np.ascontiguousarray(data.K)).to(self.device)

    def allocate(self, num_samples: int, stats: bool = True, abort: bool = False) -> TrackResult:
        n = num_samples * 312
        dev = self.device
        r = TrackResult(
            tracks=torch.empty((n, 31, 2), dtype=torch.float32, device=dev),
            converge=torch.empty(n, dtype=torch.uint8, device=dev),
            infinity=torch.empty(n, dtype=torch.uint8, device=dev),
            stats=torch.empty((n, 4), dtype=torch.int32, device=dev) if stats else None)
        if abort:
            r.found = torch.zeros(1, dtype=torch.uint8, device=dev)
            r.batch_index = torch.full((n,), -1, dtype=torch.int32, device=dev)
        return r

    def reset_tracks(self, r: TrackResult):
        """Feed_Start_Sols_for_Intermediate_Homotopy: every sample starts at the start solutions."""
        n = r.tracks.shape[0] // 312
        r.tracks.view(n, 312, 31, 2).copy_(self.start_sols.unsqueeze(0).expand(n, -1, -1, -1))
        if r.found is not None:
            r.found.zero_()
            r.batch_index.fill_(-1)

    def launch(self, target: torch.Tensor, diff: torch.Tensor, r: TrackResult, abort: bool = False,
               stream: torch.cuda.Stream | None = None, workspace: torch.Tensor | None = None,
               sample_offset: int = 0, num_samples: int | None = None, inflight_stop: bool = False,
               truncate: bool = True, explicit_rk: bool = False, time_slicing: bool = True,
               peer_found=None) -> None:
        """Enqueue one tracking run on `stream` (no synchronisation).

        Samples [sample_offset, sample_offset + num_samples) of `target`/`diff`
        are tracked into the matching rows of `r` (defaults: all of them); the
        launch's batch ids (abort-mode batch_index values) are local to it.
        inflight_stop (abort mode): paths in flight also stop once a pose is
        found (hcAbortArgs::inflight_stop; default: the reference's semantics,
        they run to completion).  truncate=False: no depth-sign path
        truncation (the archived ..._PH_CodeOpt kernel, hc_trifocal_2op1p_30x30_track_ph_codeopt);
        with explicit_rk=True as well, the archived ..._PH kernel (hc_trifocal_2op1p_30x30_track_ph).
        peer_found (abort mode): a sharding.SharedFlag of a multi-GPU run
        (hcAbortArgs::peer_found): set here on a find, polled before each path.
        time_slicing (tracking launches): suspend and resume paths at step
        boundaries so every path starts early (hc_trifocal_workspace_size_for;
        bit-identical results).  The default workspace grows to the size that
        enables it; a caller's workspace enables it if it is large enough."""
        if num_samples is None:
            num_samples = target.shape[0] - sample_offset
        if num_samples < 0 or sample_offset < 0 or sample_offset + num_samples > target.shape[0] or \
                (sample_offset + num_samples) * 312 > r.tracks.shape[0]:
            raise _abi.HCError("sample range outside the buffers")
        p0, p1 = sample_offset * 312, (sample_offset + num_samples) * 312
        if workspace is None and not abort and time_slicing:
            need = int(self.L.hc_trifocal_workspace_size_for_steps(num_samples, self.settings.max_steps))
            if self.workspace.numel() < need:
                # grown rarely (the first sliced launch of a size): the old
                # workspace may still be in use by a launch on any stream, and
                # the new one is zero-filled on the current stream, which need
                # not be `stream` -- synchronise on both sides of the swap
                torch.cuda.synchronize(self.device)
                self.workspace = torch.zeros(need, dtype=torch.uint8, device=self.device)
                torch.cuda.synchronize(self.device)
        ws_t = workspace if workspace is not None else self.workspace
        if ws_t.numel() < self.ws_bytes:
            raise _abi.HCError("workspace too small")
        wsb = ws_t.numel() if (time_slicing and not abort) else self.ws_bytes
        a = _abi.hcTrackArgs()
        a.sub_ransac_iters = num_samples
        a.settings = self.settings
        a.start_sols = self.start_sols.data_ptr()
        a.start_sols_array = None
        a.tracks = r.tracks[p0:p1].data_ptr()
        a.track_array = None
        a.start_params = self.start_params.data_ptr()
        a.target_params = target[sample_offset:].data_ptr()
        a.diff_params = diff[sample_offset:].data_ptr()
        a.unified_index = self.unified.data_ptr()
        a.converge = r.converge[p0:p1].data_ptr()
        a.infinity = r.infinity[p0:p1].data_ptr()
        a.stats = r.stats[p0:p1].data_ptr() if r.stats is not None else None
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        hs = C.c_void_p(s.cuda_stream)
        ws = C.c_void_p(ws_t.data_ptr())
        if abort and not truncate:
            raise _abi.HCError("abort mode always truncates paths (..._TrunRANSAC.cu)")
        if explicit_rk and truncate:
            raise _abi.HCError("the archived ..._PH kernel has no path truncation: pass truncate=False")
        if abort:
            if self.edgels is None:
                raise _abi.HCError("abort mode needs set_ransac_data() first")
            ab = _abi.hcAbortArgs()
            ab.num_triplet_edgels = self.edgels.shape[0]
            ab.triplet_edge_locations = self.edgels.data_ptr()
            ab.intrinsic_matrix = self.K.data_ptr()
            ab.found_trifocal_sols = r.found.data_ptr()
            ab.trifocal_sols_batch_index = r.batch_index[p0:p1].data_ptr()
            ab.inflight_stop = 1 if inflight_stop else 0
            ab.peer_found = None if peer_found is None else peer_found.ptr
            _abi.check(self.L.hc_trifocal_2op1p_30x30_track_abort(C.byref(a), C.byref(ab), ws, wsb, hs),
                       "hc_trifocal_2op1p_30x30_track_abort")
        elif explicit_rk:
            _abi.check(self.L.hc_trifocal_2op1p_30x30_track_ph(C.byref(a), ws, wsb, hs),
                       "hc_trifocal_2op1p_30x30_track_ph")
        elif not truncate:
            _abi.check(self.L.hc_trifocal_2op1p_30x30_track_ph_codeopt(C.byref(a), ws, wsb, hs),
                       "hc_trifocal_2op1p_30x30_track_ph_codeopt")
        else:
            _abi.check(self.L.hc_trifocal_2op1p_30x30_track(C.byref(a), ws, wsb, hs),
                       "hc_trifocal_2op1p_30x30_track")

    def new_workspace(self, num_samples: int = 0) -> torch.Tensor:
        """A workspace; with num_samples > 0, large enough for time slicing of
        tracking launches of up to that many samples."""
        n = (int(self.L.hc_trifocal_workspace_size_for_steps(num_samples, self.settings.max_steps))
             if num_samples > 0 else self.ws_bytes)
        return torch.zeros(n, dtype=torch.uint8, device=self.device)

    def launch_abort_chunked(self, target: torch.Tensor, diff: torch.Tensor, r: TrackResult, chunk_samples: int,
                             workspaces: list, group=None, stream: torch.cuda.Stream | None = None,
                             inflight_stop: bool = False, peer_found=None, max_count: int | None = None) -> list:
        """Abort-mode run of all of target's samples in chunks, with the
        cross-rank early-stop flag (sharding.run_abort_chunks): the launches
        and the flag reductions share one stream.  workspaces: one per chunk
        (grown as needed).  peer_found: a sharding.SharedFlag, so the launches
        also stop on another rank's find within a path (not only at the next
        chunk boundary).  max_count: the largest shard over the ranks
        (sharding.max_shard), so the chunk count needs no host-side agreement.
        Returns the (offset, count) chunks."""
        from . import sharding
        parts = sharding.chunks(target.shape[0], chunk_samples)
        while len(workspaces) < len(parts):
            workspaces.append(self.new_workspace())
        s = stream if stream is not None else torch.cuda.current_stream(self.device)

        def one(k, off, n):
            self.launch(target, diff, r, abort=True, stream=s, workspace=workspaces[k], sample_offset=off,
                        num_samples=n, inflight_stop=inflight_stop, peer_found=peer_found)
        sharding.run_abort_chunks(one, r.found, target.shape[0], chunk_samples, group=group, stream=s,
                                  max_count=max_count)
        return parts

    def workspace_status(self, workspace: torch.Tensor | None = None) -> None:
        """Raises HCError if the last launch on workspace failed on the device:
        HC_ERROR_TABLE (the index table does not fit the compaction; outputs
        untouched) or HC_ERROR_DEVICE (time slicing: a suspended path's ring
        entry never came or the ring overflowed; the lost path's outputs are
        not written; diagnostics in the control block's ring_fail words)."""
        ws = workspace if workspace is not None else self.workspace
        _abi.check(self.L.hc_trifocal_workspace_status(C.c_void_p(ws.data_ptr())), "hc_trifocal_workspace_status")

    def read_timestamps(self, workspace: torch.Tensor | None = None):
        """(start_ticks, found_ticks, tick_hz) of the last launch on workspace."""
        a, b, hz = C.c_uint64(0), C.c_uint64(0), C.c_double(0.0)
        ws = workspace if workspace is not None else self.workspace
        _abi.check(self.L.hc_trifocal_read_timestamps(C.c_void_p(ws.data_ptr()), C.byref(a), C.byref(b), C.byref(hz)),
                   "hc_trifocal_read_timestamps")
        return a.value, b.value, hz.value

    def track(self, target: np.ndarray, diff: np.ndarray, abort: bool = False, stats: bool = True,
              inflight_stop: bool = False, truncate: bool = True, explicit_rk: bool = False,
              time_slicing: bool = True) -> TrackResult:
        """Synchronous convenience wrapper: H2D params, reset tracks, launch, sync, status check."""
        tgt = torch.from_numpy(np.ascontiguousarray(target, np.float32)).to(self.device)
        dif = torch.from_numpy(np.ascontiguousarray(diff, np.float32)).to(self.device)
        r = self.allocate(tgt.shape[0], stats=stats, abort=abort)
        self.reset_tracks(r)
        self.launch(tgt, dif, r, abort=abort, inflight_stop=inflight_stop, truncate=truncate, explicit_rk=explicit_rk,
                    time_slicing=time_slicing)
        torch.cuda.synchronize(self.device)
        self.workspace_status()
        return r

    def first_found_seconds(self) -> float:
        v = C.c_double(0.0)
        _abi.check(self.L.hc_trifocal_read_timings(C.c_void_p(self.workspace.data_ptr()), C.byref(v)),
                   "hc_trifocal_read_timings")
        return v.value


def cgesv_batched(A: np.ndarray, b: np.ndarray, device="cuda:0") -> np.ndarray:
    """Batched tracker-LU solve of n 30x30 complex systems (A row-major (n,30,30,2))."""
    dev = _require_gpu(device)
    L = _abi.lib()
    At = torch.from_numpy(np.ascontiguousarray(A, np.float32)).to(dev)
    bt = torch.from_numpy(np.ascontiguousarray(b, np.float32)).to(dev)
    xt = torch.empty_like(bt)
    n = At.shape[0]
    _abi.check(L.hc_cgesv_30x30_batched(n, _ptr(At), _ptr(bt), _ptr(xt),
                                        C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)),
               "hc_cgesv_30x30_batched")
    torch.cuda.synchronize(dev)
    return xt.cpu().numpy()


def eval_batched(unified: np.ndarray, x: np.ndarray, p: np.ndarray, d: np.ndarray, device="cuda:0"):
    """Batched dH/dx, dH/dt, H at (x, p) with the tracker's compacted tables."""
    dev = _require_gpu(device)
    L = _abi.lib()
    n = x.shape[0]
    U = torch.from_numpy(np.ascontiguousarray(unified, np.int32)).to(dev)
    X = torch.from_numpy(np.ascontiguousarray(x, np.float32)).to(dev)
    P = torch.from_numpy(np.ascontiguousarray(p, np.float32)).to(dev)
    D = torch.from_numpy(np.ascontiguousarray(d, np.float32)).to(dev)
    HX = torch.empty((n, 30, 30, 2), dtype=torch.float32, device=dev)
    HT = torch.empty((n, 30, 2), dtype=torch.float32, device=dev)
    H = torch.empty((n, 30, 2), dtype=torch.float32, device=dev)
    wsb = int(L.hc_trifocal_workspace_size())
    ws = torch.zeros(wsb, dtype=torch.uint8, device=dev)
    _abi.check(L.hc_trifocal_eval_batched(n, _ptr(U), _ptr(X), _ptr(P), _ptr(D), _ptr(HX), _ptr(HT), _ptr(H),
                                          _ptr(ws), wsb, C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)),
               "hc_trifocal_eval_batched")
    torch.cuda.synchronize(dev)
    return HX.cpu().numpy(), HT.cpu().numpy(), H.cpu().numpy()
