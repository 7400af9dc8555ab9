"""ctypes binding of the C-ABI in include/hc_trifocal.h and include/hc_host.h.

The native library (lib/libhc_trifocal.so, HIP for gfx950) is the product: this
module only marshals pointers.  It raises if the library is missing -- there is
no CPU fallback anywhere in the product path.
"""
from __future__ import annotations

import ctypes as C
import os

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
# HC_TRIFOCAL_LIB: an alternative build of the same library (A/B experiments,
# scripts/build_variant.sh)
LIB_PATH = os.environ.get("HC_TRIFOCAL_LIB") or os.path.join(PKG_DIR, "lib", "libhc_trifocal.so")

# include/hc_trifocal.h HC_TRIFOCAL_ABI_VERSION: the struct layouts below
ABI_VERSION = 2

NUM_VARS, NUM_PARAMS, NUM_TRACKS = 30, 33, 312
NPP = NUM_PARAMS + 1
UNIFIED_INDEX_SIZE = 38880

HC_STATUS = {0: "HC_SUCCESS", 1: "HC_ERROR_INVALID_VALUE", 2: "HC_ERROR_WORKSPACE", 3: "HC_ERROR_LAUNCH",
             4: "HC_ERROR_DEVICE", 5: "HC_ERROR_TABLE"}


class HCError(RuntimeError):
    pass


class hcTrackSettings(C.Structure):
    _fields_ = [("max_steps", C.c_int), ("max_corrections", C.c_int), ("delta_t_inc_steps", C.c_int)]


class hcTrackArgs(C.Structure):
    _fields_ = [("sub_ransac_iters", C.c_int),
                ("settings", hcTrackSettings),
                ("start_sols", C.c_void_p),
                ("start_sols_array", C.c_void_p),
                ("tracks", C.c_void_p),
                ("track_array", C.c_void_p),
                ("start_params", C.c_void_p),
                ("target_params", C.c_void_p),
                ("diff_params", C.c_void_p),
                ("unified_index", C.c_void_p),
                ("converge", C.c_void_p),
                ("infinity", C.c_void_p),
                ("stats", C.c_void_p)]


class hcPoseSelection(C.Structure):
    """include/hc_pose.h"""
    _fields_ = [("num_candidates", C.c_int32), ("path21", C.c_int32), ("inliers21", C.c_int32),
                ("path31", C.c_int32), ("inliers31", C.c_int32), ("pad", C.c_int32),
                ("key21", C.c_uint64), ("key31", C.c_uint64),
                ("R21", C.c_float * 9), ("t21", C.c_float * 3), ("R31", C.c_float * 9), ("t31", C.c_float * 3)]


POSE_SELECTION_BYTES = C.sizeof(hcPoseSelection)
HC_POSE_REFERENCE_QUIRKS = 1


class hcAbortArgs(C.Structure):
    _fields_ = [("num_triplet_edgels", C.c_int),
                ("triplet_edge_locations", C.c_void_p),
                ("intrinsic_matrix", C.c_void_p),
                ("found_trifocal_sols", C.c_void_p),
                ("trifocal_sols_batch_index", C.c_void_p),
                ("inflight_stop", C.c_int),
                ("peer_found", C.c_void_p)]


class hcIpcHandle(C.Structure):
    _fields_ = [("reserved", C.c_ubyte * 64)]


_lib = None


def lib() -> C.CDLL:
    """Load the native library (raises HCError if it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise HCError(f"native library missing: {LIB_PATH} (run `python -c 'import __graft_entry__ as g; g.build()'`)")
        # torch is the process' HIP runtime owner (device memory, streams):
        # load it first so libhc_trifocal.so binds to the same libamdhip64.so.7
        # instead of pulling a second HIP/HSA runtime from /opt/rocm.
        import torch  # noqa: F401
        L = C.CDLL(LIB_PATH)
        L.hc_trifocal_abi_version.restype = C.c_int
        if L.hc_trifocal_abi_version() != ABI_VERSION:
            raise HCError(f"{LIB_PATH}: ABI {L.hc_trifocal_abi_version()}, this binding expects {ABI_VERSION}")
        L.hc_trifocal_set_ring_test.restype = None
        L.hc_trifocal_set_ring_test.argtypes = [C.c_int]
        if hasattr(L, "hc_trifocal_set_small_launch"):   # (test hook, round 6)
            L.hc_trifocal_set_small_launch.restype = None
            L.hc_trifocal_set_small_launch.argtypes = [C.c_int]
        if hasattr(L, "hc_trifocal_ring_check_test"):   # (test hook, round 6)
            L.hc_trifocal_ring_check_test.restype = C.c_int
            L.hc_trifocal_ring_check_test.argtypes = [C.c_void_p, C.c_size_t, C.c_uint, C.c_uint, C.c_uint, C.c_void_p]
        if hasattr(L, "hc_lu_group_class"):   # (test hooks; absent from builds before round 5's LU classes)
            L.hc_lu_struct_pattern.restype = C.c_uint
            L.hc_lu_struct_pattern.argtypes = [C.c_int]
            L.hc_lu_group_class.restype = C.c_int
            L.hc_lu_group_class.argtypes = [C.c_int, C.c_int]
        if hasattr(L, "hc_lu_search_span"):
            L.hc_lu_candidates.restype = C.c_uint
            L.hc_lu_candidates.argtypes = [C.c_int]
            L.hc_lu_search_span.restype = C.c_int
            L.hc_lu_search_span.argtypes = [C.c_int]
        L.hc_trifocal_workspace_size.restype = C.c_size_t
        L.hc_trifocal_workspace_size_for.restype = C.c_size_t
        L.hc_trifocal_workspace_size_for.argtypes = [C.c_int]
        L.hc_trifocal_workspace_size_for_steps.restype = C.c_size_t
        L.hc_trifocal_workspace_size_for_steps.argtypes = [C.c_int, C.c_int]
        L.hc_trifocal_version.restype = C.c_char_p
        L.hc_last_error_string.restype = C.c_char_p
        for fn in ("hc_trifocal_2op1p_30x30_track", "hc_trifocal_2op1p_30x30_track_abort",
                   "hc_trifocal_2op1p_30x30_track_ph_codeopt", "hc_trifocal_2op1p_30x30_track_ph",
                   "hc_trifocal_workspace_status", "hc_trifocal_read_timings", "hc_trifocal_read_timestamps", "hc_cgesv_30x30_batched", "hc_trifocal_eval_batched"):
            getattr(L, fn).restype = C.c_int
        L.hc_trifocal_2op1p_30x30_track.argtypes = [C.POINTER(hcTrackArgs), C.c_void_p, C.c_size_t, C.c_void_p]
        L.hc_trifocal_2op1p_30x30_track_ph_codeopt.argtypes = [C.POINTER(hcTrackArgs), C.c_void_p, C.c_size_t,
                                                               C.c_void_p]
        L.hc_trifocal_2op1p_30x30_track_ph.argtypes = [C.POINTER(hcTrackArgs), C.c_void_p, C.c_size_t, C.c_void_p]
        L.hc_trifocal_2op1p_30x30_track_abort.argtypes = [C.POINTER(hcTrackArgs), C.POINTER(hcAbortArgs),
                                                          C.c_void_p, C.c_size_t, C.c_void_p]
        L.hc_trifocal_read_timings.argtypes = [C.c_void_p, C.POINTER(C.c_double)]
        L.hc_trifocal_workspace_status.argtypes = [C.c_void_p]
        L.hc_trifocal_read_timestamps.restype = C.c_int
        L.hc_trifocal_read_timestamps.argtypes = [C.c_void_p, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64),
                                                  C.POINTER(C.c_double)]
        L.hc_cgesv_30x30_batched.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
        L.hc_trifocal_eval_batched.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                               C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t,
                                               C.c_void_p]
        L.hc_trifocal_pose_support.restype = C.c_int
        L.hc_trifocal_pose_support.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p,
                                               C.c_int, C.c_void_p, C.c_void_p, C.c_void_p]
        L.hc_pose_merge.restype = None
        L.hc_pose_merge.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_int, C.POINTER(hcPoseSelection)]
        L.hc_pose_residuals.restype = C.c_int
        L.hc_pose_residuals.argtypes = [C.c_void_p] * 6 + [C.c_void_p]
        L.hc_add_pixel_noise.restype = None
        L.hc_add_pixel_noise.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_double, C.c_uint64, C.c_void_p]
        L.hc_write_triplet_edgels.restype = C.c_int
        L.hc_write_triplet_edgels.argtypes = [C.c_char_p, C.c_int, C.c_void_p, C.c_void_p]
        L.hc_write_converged_sols.restype = C.c_int
        L.hc_write_converged_sols.argtypes = [C.c_char_p, C.c_int, C.c_void_p, C.c_void_p]
        L.hc_prepare_target_params.argtypes = [C.c_uint, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int,
                                               C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
        for fn in ("hc_read_start_sols", "hc_read_start_params", "hc_read_int_table", "hc_read_float_table",
                   "hc_count_triplet_edgels", "hc_read_triplet_edgels"):
            getattr(L, fn).restype = C.c_int
        # (bound only where present: A/B runs load earlier builds through HC_TRIFOCAL_LIB;
        # the product library exports them, tests/test_abi_host.py)
        if hasattr(L, "hc_shared_flag_create"):
            for fn in ("hc_shared_flag_create", "hc_shared_flag_open", "hc_shared_flag_reset", "hc_shared_flag_close"):
                getattr(L, fn).restype = C.c_int
            L.hc_shared_flag_create.argtypes = [C.POINTER(C.c_void_p), C.POINTER(hcIpcHandle)]
            L.hc_shared_flag_open.argtypes = [C.POINTER(hcIpcHandle), C.POINTER(C.c_void_p)]
            L.hc_shared_flag_reset.argtypes = [C.c_void_p, C.c_void_p]
            L.hc_shared_flag_close.argtypes = [C.c_void_p, C.c_int]
            L.hc_shared_flag_memory_kind.restype = C.c_int
            L.hc_shared_flag_memory_kind.argtypes = [C.c_void_p]
        _lib = L
    return _lib


def check(status: int, what: str) -> None:
    if status != 0:
        detail = lib().hc_last_error_string().decode(errors="replace")
        raise HCError(f"{what} failed: {HC_STATUS.get(status, status)} ({detail})")


# Exported symbols that include/*.h declare (tests check the library exports all of them).
DECLARED_SYMBOLS = (
    "hc_trifocal_workspace_size", "hc_trifocal_workspace_size_for", "hc_trifocal_workspace_size_for_steps", "hc_trifocal_2op1p_30x30_track", "hc_trifocal_2op1p_30x30_track_abort",
    "hc_trifocal_2op1p_30x30_track_ph_codeopt", "hc_trifocal_2op1p_30x30_track_ph",
    "hc_trifocal_workspace_status", "hc_trifocal_read_timings", "hc_trifocal_read_timestamps", "hc_cgesv_30x30_batched", "hc_trifocal_eval_batched", "hc_trifocal_version",
    "hc_last_error_string", "hc_trifocal_abi_version", "hc_trifocal_set_ring_test",
    "hc_trifocal_ring_check_test", "hc_trifocal_set_small_launch",
    "hc_lu_struct_pattern", "hc_lu_group_class", "hc_lu_candidates", "hc_lu_search_span",
    "hc_shared_flag_create", "hc_shared_flag_open", "hc_shared_flag_reset", "hc_shared_flag_close",
    "hc_shared_flag_memory_kind",
    "hc_read_start_sols", "hc_read_start_params", "hc_read_int_table", "hc_read_float_table",
    "hc_count_triplet_edgels", "hc_read_triplet_edgels", "hc_split_samples", "hc_prepare_target_params",
    "hc_count_solutions",
    "hc_trifocal_pose_support", "hc_pose_merge", "hc_pose_residuals", "hc_write_converged_sols",
    "hc_add_pixel_noise", "hc_write_triplet_edgels",
)


def _fatbin_digest(path: str) -> str | None:
    """sha256 of the .hip_fatbin section of an ELF shared library: the gfx950
    code objects of every kernel, independent of the host code around them."""
    import hashlib
    import struct
    with open(path, "rb") as fh:
        elf = fh.read()
    if elf[:4] != b"\x7fELF" or elf[4] != 2:
        return None
    shoff, = struct.unpack_from("<Q", elf, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", elf, 0x3A)
    def sec(i):
        name, _typ, _flags, _addr, off, size = struct.unpack_from("<IIQQQQ", elf, shoff + i * shentsize)
        return name, off, size
    _, stroff, _ = sec(shstrndx)
    for i in range(shnum):
        name, off, size = sec(i)
        end = elf.index(b"\0", stroff + name)
        if elf[stroff + name:end] == b".hip_fatbin":
            return hashlib.sha256(elf[off:off + size]).hexdigest()
    return None


def build_id(path: str | None = None) -> str:
    """Identifies the kernels a profile or bench line measured: the library's
    version tag and the first 12 hex digits of the sha256 of its device code
    (.hip_fatbin).  Profiles under profiles/ carry it and bench.py takes its
    PMC / LU-work sources only from profiles of the loaded build."""
    import re
    path = path or LIB_PATH
    with open(path, "rb") as fh:
        m = re.search(rb"hc_trifocal gfx950 (v[0-9.]+)", fh.read())
    ver = m.group(1).decode() if m else "v?"
    d = _fatbin_digest(path)
    return f"{ver}+{d[:12] if d else 'nofatbin'}"


PRODUCT_LIB_PATH = os.path.join(PKG_DIR, "lib", "libhc_trifocal.so")
