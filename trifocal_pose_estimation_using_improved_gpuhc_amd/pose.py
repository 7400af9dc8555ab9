"""Pose recovery, maximal-support selection and GT pose error.

Device side: hc_trifocal_pose_support (include/hc_pose.h, csrc/hc_pose.hip)
replaces the host loops of Evaluations::Transform_GPUHC_Sols_to_Trifocal_Relative_Pose
(magmaHC/Evaluations.cpp:298-358) and get_Solution_with_Maximal_Support
(:382-504).  Host side: hc_pose_merge (per-GPU selections -> one) and
hc_pose_residuals (Measure_Relative_Pose_Error, :523-543).
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch

from . import _abi
from .problem import RansacData

SEL_BYTES = _abi.POSE_SELECTION_BYTES


def _stream_handle(stream, device):
    s = stream if stream is not None else torch.cuda.current_stream(device)
    return C.c_void_p(s.cuda_stream)


def launch_pose_support(tracks: torch.Tensor, converge: torch.Tensor, edgels: torch.Tensor, K: torch.Tensor,
                        inliers: torch.Tensor, selection: torch.Tensor, quirks: bool = False, stream=None) -> None:
    """Enqueue candidate filter + pose + inlier scoring + selection (no sync).
    tracks (n, 31, 2) f32, converge (n,) u8, edgels (E, 6) f32, K (9,) f32 on the
    same device; inliers (n, 2) i32 and selection (SEL_BYTES,) u8 are outputs."""
    n = converge.numel()
    if tracks.shape[0] != n or inliers.numel() < 2 * n or selection.numel() < SEL_BYTES:
        raise _abi.HCError("pose_support: buffer sizes do not match")
    for t in (tracks, converge, edgels, K, inliers, selection):
        if not t.is_cuda or not t.is_contiguous():
            raise _abi.HCError("pose_support: buffers must be contiguous device tensors")
    L = _abi.lib()
    _abi.check(L.hc_trifocal_pose_support(n, C.c_void_p(tracks.data_ptr()), C.c_void_p(converge.data_ptr()),
                                          int(edgels.shape[0]), C.c_void_p(edgels.data_ptr()),
                                          C.c_void_p(K.data_ptr()), _abi.HC_POSE_REFERENCE_QUIRKS if quirks else 0,
                                          C.c_void_p(inliers.data_ptr()), C.c_void_p(selection.data_ptr()),
                                          _stream_handle(stream, tracks.device)),
               "hc_trifocal_pose_support")


def selection_struct(raw: np.ndarray | torch.Tensor) -> _abi.hcPoseSelection:
    b = raw.cpu().numpy() if isinstance(raw, torch.Tensor) else np.asarray(raw)
    return _abi.hcPoseSelection.from_buffer_copy(np.ascontiguousarray(b, np.uint8).tobytes()[:SEL_BYTES])


def selection_dict(s: _abi.hcPoseSelection) -> dict:
    return dict(num_candidates=s.num_candidates, path21=s.path21, inliers21=s.inliers21, path31=s.path31,
                inliers31=s.inliers31, key21=s.key21, key31=s.key31,
                R21=np.array(s.R21[:], np.float32), t21=np.array(s.t21[:], np.float32),
                R31=np.array(s.R31[:], np.float32), t31=np.array(s.t31[:], np.float32))


def pose_support(tracks: torch.Tensor, converge: torch.Tensor, data_edgels: torch.Tensor, K: torch.Tensor,
                 quirks: bool = False):
    """Synchronous wrapper: returns (inliers (n, 2) numpy, selection dict)."""
    dev = tracks.device
    n = converge.numel()
    inl = torch.empty((n, 2), dtype=torch.int32, device=dev)
    sel = torch.empty(SEL_BYTES, dtype=torch.uint8, device=dev)
    launch_pose_support(tracks, converge, data_edgels, K, inl, sel, quirks)
    torch.cuda.synchronize(dev)
    return inl.cpu().numpy(), selection_dict(selection_struct(sel))


def merge(parts: list, path_offsets: list, quirks: bool = False) -> dict:
    """hc_pose_merge: per-GPU selections (raw bytes or structs) with their first
    batch ids -> one selection with global batch ids."""
    n = len(parts)
    arr = (_abi.hcPoseSelection * max(1, n))()
    for i, p in enumerate(parts):
        arr[i] = p if isinstance(p, _abi.hcPoseSelection) else selection_struct(p)
    offs = np.ascontiguousarray(path_offsets, np.int32)
    out = _abi.hcPoseSelection()
    _abi.lib().hc_pose_merge(n, C.cast(arr, C.c_void_p), C.c_void_p(offs.ctypes.data),
                             _abi.HC_POSE_REFERENCE_QUIRKS if quirks else 0, C.byref(out))
    return selection_dict(out)


def residuals(data: RansacData, sel: dict):
    """Measure_Relative_Pose_Error: ([rot21, rot31, transl21, transl31], success)."""
    out = np.zeros(4, np.float32)
    a = [np.ascontiguousarray(v, np.float32) for v in (data.pose21, data.pose31, sel["R21"], sel["t21"],
                                                        sel["R31"], sel["t31"])]
    ok = _abi.lib().hc_pose_residuals(*[C.c_void_p(v.ctypes.data) for v in a], C.c_void_p(out.ctypes.data))
    return out, bool(ok)


def success_clamped(data: RansacData, sel: dict, out: np.ndarray) -> bool:
    """The GT verdict with the rotation residual's acos argument clamped to
    [-1, 1].  The reference (Evaluations.cpp:360-374) does not clamp: an exact
    rotation whose float trace rounds above 3 gives acos(> 1) = NaN, and the
    pose counts as a failure.  Reported beside the reference verdict, never
    instead of it."""
    rot = []
    for gt, R in ((data.pose21, sel["R21"]), (data.pose31, sel["R31"])):
        G = np.asarray(gt, np.float64)[:9].reshape(3, 3)
        M = G.T @ np.asarray(R, np.float64).reshape(3, 3)
        rot.append(float(np.arccos(np.clip(0.5 * (np.trace(M) - 1.0), -1.0, 1.0))))
    return bool(rot[0] < 0.1 and rot[1] < 0.1 and float(out[2]) < 0.1 and float(out[3]) < 0.1)
