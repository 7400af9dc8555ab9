"""Noisy synthcurves datasets (BASELINE.json config 5).

The reference ships noiseless synthetic triplet edgels only
(RANSAC_Data/trifocal_2op1p_30x30/Synthetic/**).  This module perturbs every
point of every view by N(0, sigma^2) pixels with the native generator
(hc_add_pixel_noise: std::mt19937_64 + std::normal_distribution<double>) and
writes datasets in the reference layout (Data_Reader.cpp:191-338):

    <root>/RANSAC_Data/<problem>/<name>/Triplet_Edgels/Triplet_Edgels_XXX.txt
                                       /GT_Poses21/GT_Poses21_XXX.txt, GT_Poses31/...
                                       /Intrinsic_Matrix.txt
so `load_ransac_data(index, dataset=name)` and `magmaHC-main -s <name>` read them.
"""
from __future__ import annotations

import ctypes as C
import os
import shutil

import numpy as np

from . import _abi
from .problem import DATA_ROOT, PROBLEM, RansacData, load_ransac_data, ransac_dir

DEFAULT_SEED = 20250215


def add_pixel_noise(locations: np.ndarray, K: np.ndarray, sigma_px: float, seed: int = DEFAULT_SEED) -> np.ndarray:
    loc = np.ascontiguousarray(locations, np.float32)
    Kc = np.ascontiguousarray(K, np.float32)
    out = np.empty_like(loc)
    _abi.lib().hc_add_pixel_noise(loc.shape[0], C.c_void_p(loc.ctypes.data), C.c_void_p(Kc.ctypes.data),
                                  float(sigma_px), int(seed) & 0xFFFFFFFFFFFFFFFF, C.c_void_p(out.ctypes.data))
    return out


def noisy(data: RansacData, sigma_px: float, seed: int = DEFAULT_SEED) -> RansacData:
    """A copy of `data` whose point locations carry sigma_px pixel noise (tangents, K, GT unchanged)."""
    return RansacData(add_pixel_noise(data.locations, data.K, sigma_px, seed), data.tangents.copy(), data.K.copy(),
                      data.pose21.copy(), data.pose31.copy())


def write_triplet_edgels(path: str, locations: np.ndarray, tangents: np.ndarray) -> None:
    loc = np.ascontiguousarray(locations, np.float32)
    tan = np.ascontiguousarray(tangents, np.float32)
    if _abi.lib().hc_write_triplet_edgels(path.encode(), loc.shape[0], C.c_void_p(loc.ctypes.data),
                                          C.c_void_p(tan.ctypes.data)) != loc.shape[0]:
        raise _abi.HCError(f"cannot write {path}")


def make_noisy_dataset(sigma_px: float, indices=(0,), name: str | None = None, out_root: str = DATA_ROOT,
                       src_root: str = DATA_ROOT, problem: str = PROBLEM, seed: int = DEFAULT_SEED) -> str:
    """Writes a noisy copy of the Synthetic dataset for the given indices; the
    noise seed of index i is seed + i.  Returns the dataset directory."""
    name = name or f"Synthetic_noise{sigma_px:g}px"
    dst = ransac_dir(out_root, problem, name)
    src = ransac_dir(src_root, problem)
    for sub in ("Triplet_Edgels", "GT_Poses21", "GT_Poses31"):
        os.makedirs(os.path.join(dst, sub), exist_ok=True)
    shutil.copyfile(os.path.join(src, "Intrinsic_Matrix.txt"), os.path.join(dst, "Intrinsic_Matrix.txt"))
    for i in indices:
        d = load_ransac_data(i, src_root, problem)
        write_triplet_edgels(os.path.join(dst, "Triplet_Edgels", f"Triplet_Edgels_{i:03d}.txt"),
                             add_pixel_noise(d.locations, d.K, sigma_px, seed + i), d.tangents)
        for v in ("21", "31"):
            shutil.copyfile(os.path.join(src, f"GT_Poses{v}", f"GT_Poses{v}_{i:03d}.txt"),
                            os.path.join(dst, f"GT_Poses{v}", f"GT_Poses{v}_{i:03d}.txt"))
    return dst
