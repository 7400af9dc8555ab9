"""TEST INFRASTRUCTURE ONLY -- ctypes loader for the C oracle (oracle/hc_oracle.c).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module, and only as the checker / CPU baseline.  The product path lives in
trifocal_pose_estimation_using_improved_gpuhc_amd/ and never imports oracle/.

Parity status: pinned by reference-data KATs (H(start)=0, Hx = FD(H)), numpy
LU, and the reference's committed CPU-HC counts, reproduced EXACTLY
(11098 / 521 / 6577) by the restatement built like the reference CPU build and
solving through OpenBLAS 0.3.23 (tests/test_oracle_kat.py, tests/cpuhc_pin.py);
the reference sources are never built or run here (SURVEY.md §8c denial,
binding).  See DESIGN.md §5.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "libhc_oracle.so")

NV, NPP, NT = 30, 34, 312
HX_SIZE, HT_SIZE = 36000, 2880


class Settings(C.Structure):
    _fields_ = [("max_steps", C.c_int), ("max_corrections", C.c_int),
                ("inc_steps", C.c_int), ("num_threads", C.c_int), ("no_truncation", C.c_int),
                ("explicit_rk", C.c_int)]


PATH_STATS_DTYPE = np.dtype([("steps", "<i4"), ("corrections", "<i4"),
                             ("inliers21", "<i4"), ("inliers31", "<i4")])

_lib = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        _lib = C.CDLL(LIB_PATH)
        _lib.orc_cpuhc_track.restype = C.c_double
    return _lib


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


def settings(max_steps=80, max_corrections=3, inc_steps=4, threads=0, truncate=True, explicit_rk=False) -> Settings:
    """explicit_rk=True, truncate=False: the archived ..._PH kernel's semantics."""
    return Settings(max_steps, max_corrections, inc_steps, threads, 0 if truncate else 1, 1 if explicit_rk else 0)


# ----------------------------------------------------------------- readers
def read_problem(problem_dir: str):
    L = lib()
    ss = np.zeros((NT, NV + 1, 2), np.float32)
    sp = np.zeros((NPP, 2), np.float32)
    dhdx = np.zeros(HX_SIZE, np.int32)
    dhdt = np.zeros(HT_SIZE, np.int32)
    assert L.orc_read_start_sols(os.path.join(problem_dir, "start_sols.txt").encode(), _p(ss)) == NT * NV
    assert L.orc_read_start_params(os.path.join(problem_dir, "start_params.txt").encode(), _p(sp)) == 33
    assert L.orc_read_ints(os.path.join(problem_dir, "dHdx_indx.txt").encode(), _p(dhdx), HX_SIZE) == HX_SIZE
    assert L.orc_read_ints(os.path.join(problem_dir, "dHdt_indx.txt").encode(), _p(dhdt), HT_SIZE) == HT_SIZE
    return ss, sp, dhdx, dhdt


def read_edgels(file: str):
    L = lib()
    n = L.orc_count_triplet_edgels(file.encode())
    loc = np.zeros((n, 6), np.float32)
    tan = np.zeros((n, 6), np.float32)
    assert L.orc_read_triplet_edgels(file.encode(), _p(loc), _p(tan), n) == n
    return loc, tan


def read_floats(file: str, n: int):
    out = np.zeros(n, np.float32)
    assert lib().orc_read_floats(file.encode(), _p(out), n) == n
    return out


# ----------------------------------------------------------------- samples
def prepare_target_params(seed, sub_iters, loc, tan, start_params):
    sub = np.ascontiguousarray(sub_iters, dtype=np.int32)
    N = int(sub.sum())
    tgt = np.zeros((N, NPP, 2), np.float32)
    dif = np.zeros((N, NPP, 2), np.float32)
    picked = np.zeros((N, 3), np.int32)
    lib().orc_prepare_target_params(C.c_uint(seed), C.c_int(len(sub)), _p(sub), _p(loc), _p(tan),
                                    C.c_int(loc.shape[0]), _p(start_params), _p(tgt), _p(dif), _p(picked))
    return tgt, dif, picked


# ----------------------------------------------------------------- evals
def param_homotopy(t, sp, tp):
    p = np.zeros((NPP, 2), np.float32)
    lib().orc_param_homotopy_gpu(C.c_float(t), _p(sp), _p(tp), _p(p))
    return p


def eval_hx(dhdx, x, p):
    A = np.zeros((NV, NV, 2), np.float32)
    lib().orc_eval_hx(_p(dhdx), _p(np.ascontiguousarray(x, np.float32)), _p(p), _p(A))
    return A


def eval_ht(dhdt, x, p, d):
    b = np.zeros((NV, 2), np.float32)
    lib().orc_eval_ht(_p(dhdt), _p(np.ascontiguousarray(x, np.float32)), _p(p), _p(d), _p(b))
    return b


def eval_h(dhdt, x, p):
    b = np.zeros((NV, 2), np.float32)
    lib().orc_eval_h(_p(dhdt), _p(np.ascontiguousarray(x, np.float32)), _p(p), _p(b))
    return b


def cgesv_gpu(A, b):
    A = np.ascontiguousarray(A, np.float32).copy()
    b = np.ascontiguousarray(b, np.float32)
    x = np.zeros((NV, 2), np.float32)
    lib().orc_cgesv_gpu(_p(A), _p(b), _p(x))
    return x


def cgesv_lapack(A_rowmajor, b):
    A = np.ascontiguousarray(np.transpose(A_rowmajor, (1, 0, 2)), np.float32).copy()  # col-major
    B = np.ascontiguousarray(b, np.float32).copy()
    info = lib().orc_cgesv_lapack(_p(A), _p(B))
    return B, info


# ----------------------------------------------------------------- trackers
def _tracks_init(start_sols, N):
    return np.ascontiguousarray(np.tile(start_sols[None], (N, 1, 1, 1)).reshape(N * NT, NV + 1, 2))


def gpuhc_track(start_sols, start_params, tgt, dif, unified, s: Settings | None = None):
    """GPU-HC semantics for all 312*N paths. Returns (tracks, conv, inf, stats)."""
    s = s or settings()
    N = tgt.shape[0]
    tracks = _tracks_init(start_sols, N)
    conv = np.zeros(N * NT, np.uint8)
    inf = np.zeros(N * NT, np.uint8)
    stats = np.zeros(N * NT, PATH_STATS_DTYPE)
    lib().orc_gpuhc_track(C.byref(s), C.c_int(N), _p(start_sols), _p(start_params), _p(tgt), _p(dif),
                          _p(unified), _p(tracks), _p(conv), _p(inf), _p(stats))
    return tracks, conv, inf, stats


def gpuhc_track_subset(path_ids, start_sols, start_params, tgt, dif, unified, s: Settings | None = None):
    s = s or settings()
    N = tgt.shape[0]
    ids = np.ascontiguousarray(path_ids, np.int32)
    tracks = _tracks_init(start_sols, N)
    conv = np.zeros(N * NT, np.uint8)
    inf = np.zeros(N * NT, np.uint8)
    stats = np.zeros(N * NT, PATH_STATS_DTYPE)
    lib().orc_gpuhc_track_subset(C.byref(s), C.c_int(len(ids)), _p(ids), _p(start_sols), _p(start_params),
                                 _p(tgt), _p(dif), _p(unified), _p(tracks), _p(conv), _p(inf), _p(stats))
    return tracks, conv, inf, stats


def cpuhc_track(start_sols, start_params, tgt, dif, dhdx, dhdt, s: Settings | None = None):
    """CPU-HC semantics. Returns (tracks, conv, inf, stats, seconds)."""
    s = s or settings()
    N = tgt.shape[0]
    tracks = _tracks_init(start_sols, N)
    conv = np.zeros(N * NT, np.uint8)
    inf = np.zeros(N * NT, np.uint8)
    stats = np.zeros(N * NT, PATH_STATS_DTYPE)
    secs = lib().orc_cpuhc_track(C.byref(s), C.c_int(N), _p(start_sols), _p(start_params), _p(tgt), _p(dif),
                                 _p(dhdx), _p(dhdt), _p(tracks), _p(conv), _p(inf), _p(stats))
    return tracks, conv, inf, stats, secs


def score_hypothesis(x, loc, K):
    in21 = C.c_int(0)
    in31 = C.c_int(0)
    ok = lib().orc_score_hypothesis(_p(np.ascontiguousarray(x, np.float32)), C.c_int(loc.shape[0]),
                                    _p(np.ascontiguousarray(loc, np.float32)),
                                    _p(np.ascontiguousarray(K, np.float32)), C.byref(in21), C.byref(in31))
    return bool(ok), in21.value, in31.value


def count_solutions(tracks, conv, inf):
    out = np.zeros(3, np.int32)
    N = conv.shape[0] // NT
    lib().orc_count_solutions(C.c_int(N), _p(np.ascontiguousarray(tracks, np.float32)), _p(conv), _p(inf), _p(out))
    return tuple(int(v) for v in out)


# ----------------------------------------------------------------- pose recovery (§8 f1)
class PoseSelection(C.Structure):
    """== orc_pose_selection == hcPoseSelection (include/hc_pose.h)."""
    _fields_ = [("num_candidates", C.c_int32), ("path21", C.c_int32), ("inliers21", C.c_int32),
                ("path31", C.c_int32), ("inliers31", C.c_int32), ("pad", C.c_int32),
                ("key21", C.c_uint64), ("key31", C.c_uint64),
                ("R21", C.c_float * 9), ("t21", C.c_float * 3), ("R31", C.c_float * 9), ("t31", C.c_float * 3)]


def selection_dict(s) -> dict:
    return dict(num_candidates=s.num_candidates, path21=s.path21, inliers21=s.inliers21, path31=s.path31,
                inliers31=s.inliers31, R21=np.array(s.R21[:], np.float32), t21=np.array(s.t21[:], np.float32),
                R31=np.array(s.R31[:], np.float32), t31=np.array(s.t31[:], np.float32))


def pose_support(tracks, conv, loc, K, quirks=False):
    """Evaluations.cpp:298-504 restated: returns (inliers (312N, 2) int32, selection dict)."""
    tr = np.ascontiguousarray(tracks, np.float32)
    cv = np.ascontiguousarray(conv, np.uint8)
    n = cv.shape[0]
    inl = np.zeros((n, 2), np.int32)
    sel = PoseSelection()
    lib().orc_pose_support(C.c_int(n), _p(tr), _p(cv), C.c_int(loc.shape[0]),
                           _p(np.ascontiguousarray(loc, np.float32)), _p(np.ascontiguousarray(K, np.float32)),
                           C.c_int(1 if quirks else 0), _p(inl), C.byref(sel))
    return inl, selection_dict(sel)


def pose_residuals(gt21, gt31, sel: dict):
    """Measure_Relative_Pose_Error: ([rot21, rot31, transl21, transl31], success)."""
    s = PoseSelection()
    for k in ("R21", "t21", "R31", "t31"):
        getattr(s, k)[:] = [float(v) for v in sel[k]]
    out = np.zeros(4, np.float32)
    ok = lib().orc_pose_residuals(_p(np.ascontiguousarray(gt21, np.float32)),
                                  _p(np.ascontiguousarray(gt31, np.float32)), C.byref(s), _p(out))
    return out, bool(ok)


def add_pixel_noise(loc, K, sigma_px, seed):
    out = np.zeros_like(np.ascontiguousarray(loc, np.float32))
    lib().orc_add_pixel_noise(C.c_int(loc.shape[0]), _p(np.ascontiguousarray(loc, np.float32)),
                              _p(np.ascontiguousarray(K, np.float32)), C.c_double(sigma_px), C.c_uint64(seed), _p(out))
    return out
