"""Problem / RANSAC data of trifocal_2op1p_30x30 (reference Data_Reader formats).

Everything is parsed by the native host layer (include/hc_host.h) so Python and
the C++ GPU_HC_Solver read bit-identical floats.  Paths follow the reference
layout: <root>/problems/<problem>/... and <root>/RANSAC_Data/<problem>/<dataset>/...
(the repository keeps both under data/).
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass

import numpy as np

from . import _abi

PROBLEM = "trifocal_2op1p_30x30"
REPO_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DATA_ROOT = os.path.join(REPO_ROOT, "data")


def _p(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


def read_settings(path: str) -> dict:
    """Flat `key: value` YAML reader for gpuhc_settings.yaml (yaml-cpp replacement)."""
    out = {}
    with open(path) as f:
        for line in f:
            line = line.split("#", 1)[0].strip()
            if not line or line.startswith("%") or ":" not in line:
                continue
            k, v = line.split(":", 1)
            v = v.strip()
            if v.lower() in ("true", "false"):
                out[k.strip()] = v.lower() == "true"
            else:
                try:
                    out[k.strip()] = int(v)
                except ValueError:
                    try:
                        out[k.strip()] = float(v)
                    except ValueError:
                        out[k.strip()] = v
    return out


@dataclass
class Problem:
    start_sols: np.ndarray      # (312, 31, 2) float32, x[30] = 1
    start_params: np.ndarray    # (34, 2) float32, p[33] = 1
    dHdx_index: np.ndarray      # (36000,) int32
    dHdt_index: np.ndarray      # (2880,) int32
    settings: dict

    @property
    def unified_index(self) -> np.ndarray:
        return np.ascontiguousarray(np.concatenate([self.dHdx_index, self.dHdt_index]).astype(np.int32))


@dataclass
class RansacData:
    locations: np.ndarray       # (E, 6) float32: x1 y1 x2 y2 x3 y3 (metric)
    tangents: np.ndarray        # (E, 6) float32
    K: np.ndarray               # (9,) float32 row-major intrinsics
    pose21: np.ndarray          # (12,) float32: R row-major then t
    pose31: np.ndarray


def problem_dir(root: str = DATA_ROOT, problem: str = PROBLEM) -> str:
    return os.path.join(root, "problems", problem)


def load_problem(root: str = DATA_ROOT, problem: str = PROBLEM) -> Problem:
    L = _abi.lib()
    d = problem_dir(root, problem)
    ss = np.zeros((312, 31, 2), np.float32)
    sp = np.zeros((34, 2), np.float32)
    dx = np.zeros(36000, np.int32)
    dt = np.zeros(2880, np.int32)
    if L.hc_read_start_sols(os.path.join(d, "start_sols.txt").encode(), _p(ss)) != 312 * 30:
        raise _abi.HCError("start solutions not loaded")
    if L.hc_read_start_params(os.path.join(d, "start_params.txt").encode(), _p(sp)) != 33:
        raise _abi.HCError("start parameters not loaded")
    if L.hc_read_int_table(os.path.join(d, "dHdx_indx.txt").encode(), _p(dx), dx.size) != dx.size:
        raise _abi.HCError("dH/dx evaluation indices not loaded")
    if L.hc_read_int_table(os.path.join(d, "dHdt_indx.txt").encode(), _p(dt), dt.size) != dt.size:
        raise _abi.HCError("dH/dt evaluation indices not loaded")
    return Problem(ss, sp, dx, dt, read_settings(os.path.join(d, "gpuhc_settings.yaml")))


def ransac_dir(root: str = DATA_ROOT, problem: str = PROBLEM, dataset: str = "Synthetic") -> str:
    return os.path.join(root, "RANSAC_Data", problem, dataset)


def load_ransac_data(index: int = 0, root: str = DATA_ROOT, problem: str = PROBLEM,
                     dataset: str = "Synthetic") -> RansacData:
    L = _abi.lib()
    d = ransac_dir(root, problem, dataset)
    f = os.path.join(d, "Triplet_Edgels", f"Triplet_Edgels_{index:03d}.txt").encode()
    E = L.hc_count_triplet_edgels(f)
    if E <= 0:
        raise _abi.HCError(f"no triplet edgels in {f!r}")
    loc = np.zeros((E, 6), np.float32)
    tan = np.zeros((E, 6), np.float32)
    if L.hc_read_triplet_edgels(f, _p(loc), _p(tan), E) != E:
        raise _abi.HCError("triplet edgels not loaded")
    K = np.zeros(9, np.float32)
    if L.hc_read_float_table(os.path.join(d, "Intrinsic_Matrix.txt").encode(), _p(K), 9) != 9:
        raise _abi.HCError("intrinsic matrix not loaded")
    poses = []
    for v in ("21", "31"):
        P = np.zeros(12, np.float32)
        L.hc_read_float_table(os.path.join(d, f"GT_Poses{v}", f"GT_Poses{v}_{index:03d}.txt").encode(), _p(P), 12)
        poses.append(P)
    return RansacData(loc, tan, K, poses[0], poses[1])


def split_samples(num_samples: int, num_gpus: int) -> np.ndarray:
    sub = np.zeros(num_gpus, np.int32)
    _abi.lib().hc_split_samples(C.c_int(num_samples), C.c_int(num_gpus), _p(sub))
    return sub


def prepare_target_params(problem: Problem, data: RansacData, seed: int, num_samples: int,
                          num_gpus: int = 1):
    """Reference Prepare_Target_Params: returns (target, diff, picked) for all
    num_samples samples in gpu-major order (sample k is independent of num_gpus)."""
    sub = split_samples(num_samples, num_gpus)
    tgt = np.zeros((num_samples, 34, 2), np.float32)
    dif = np.zeros((num_samples, 34, 2), np.float32)
    picked = np.zeros((num_samples, 3), np.int32)
    _abi.lib().hc_prepare_target_params(C.c_uint(seed), C.c_int(num_gpus), _p(sub), _p(data.locations),
                                        _p(data.tangents), C.c_int(data.locations.shape[0]),
                                        _p(problem.start_params), _p(tgt), _p(dif), _p(picked))
    return tgt, dif, picked


def count_solutions(tracks: np.ndarray, conv: np.ndarray, inf: np.ndarray):
    """(converged, real, infinity) like Evaluations::Evaluate_RANSAC_HC_Sols."""
    out = np.zeros(3, np.int32)
    tr = np.ascontiguousarray(tracks, np.float32)
    n = conv.shape[0] // 312
    _abi.lib().hc_count_solutions(C.c_int(n), _p(tr), _p(np.ascontiguousarray(conv, np.uint8)),
                                  _p(np.ascontiguousarray(inf, np.uint8)), _p(out))
    return tuple(int(v) for v in out)
