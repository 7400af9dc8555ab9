"""MI355X-native GPU homotopy-continuation path tracker for trifocal_2op1p_30x30.

Product path: HIP kernels for gfx950 behind the C-ABI in include/hc_trifocal.h
(lib/libhc_trifocal.so), driven from C++ (GPU_HC_Solver, magmaHC-main) or from
Python through ctypes (this package).  See DESIGN.md.
"""
from . import _abi
from .problem import (PROBLEM, Problem, RansacData, count_solutions, load_problem, load_ransac_data,
                      prepare_target_params, read_settings, split_samples)

__all__ = ["_abi", "PROBLEM", "Problem", "RansacData", "count_solutions", "load_problem", "load_ransac_data",
           "prepare_target_params", "read_settings", "split_samples"]
