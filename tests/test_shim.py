"""The drop-in launcher shim (integration/hc_trifocal_shim.cpp).

CPU: the shim compiles against the reference's launcher signatures
(integration/magmaHC-kernels.hpp restating magmaHC-kernels.hpp:24-105, with a
types-only MAGMA stand-in) and exports the four C++-linkage launchers (plus the two archived ..._PH_CodeOpt
ablation launchers) with exactly those parameter lists.

GPU: each of the four launchers, called with the reference's argument lists
(pointer arrays d_startSols_array / d_Track_array as GPU_HC_Solver.cpp:352-353
builds them, bool flags, separate dH/dx / dH/dt tables for the Volta variants),
produces exactly what hc_trifocal_2op1p_30x30_track(_abort) produces.
"""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHIM = os.path.join(ROOT, "integration", "build", "libhc_shim_test.so")

SIGNATURES = {
    "kernel_GPUHC_trifocal_2op1p_30x30_PH_CodeOpt_TrunPaths":
        "(magma_queue*, int, int, int, int, magmaFloatComplex**, magmaFloatComplex**, magmaFloatComplex*, "
        "magmaFloatComplex*, magmaFloatComplex*, int*, bool*, bool*, magmaFloatComplex*)",
    "kernel_GPUHC_trifocal_2op1p_30x30_PH_CodeOpt_TrunPaths_Volta":
        "(magma_queue*, int, int, int, int, magmaFloatComplex**, magmaFloatComplex**, magmaFloatComplex*, "
        "magmaFloatComplex*, magmaFloatComplex*, int*, int*, bool*, bool*, magmaFloatComplex*)",
    "kernel_GPUHC_trifocal_2op1p_30x30_PH_CodeOpt_TrunPaths_TrunRANSAC":
        "(magma_queue*, int, int, int, int, int, magmaFloatComplex**, magmaFloatComplex**, magmaFloatComplex*, "
        "magmaFloatComplex*, magmaFloatComplex*, int*, float*, float*, bool*, bool*, magmaFloatComplex*, bool*, int*)",
    "kernel_GPUHC_trifocal_2op1p_30x30_PH_CodeOpt_TrunPaths_TrunRANSAC_Volta":
        "(magma_queue*, int, int, int, int, int, magmaFloatComplex**, magmaFloatComplex**, magmaFloatComplex*, "
        "magmaFloatComplex*, magmaFloatComplex*, int*, int*, float*, float*, bool*, bool*, magmaFloatComplex*, "
        "bool*, int*)",
    # archived ablation launchers (arxived_GPU_code/gpu-kernels/magmaHC-kernels.hpp:61-96)
    "kernel_GPUHC_trifocal_2op1p_30x30_PH_CodeOpt":
        "(magma_queue*, int, int, int, int, magmaFloatComplex**, magmaFloatComplex**, magmaFloatComplex*, "
        "magmaFloatComplex*, magmaFloatComplex*, int*, bool*, bool*, magmaFloatComplex*)",
    "kernel_GPUHC_trifocal_2op1p_30x30_PH_CodeOpt_Volta":
        "(magma_queue*, int, int, int, int, magmaFloatComplex**, magmaFloatComplex**, magmaFloatComplex*, "
        "magmaFloatComplex*, magmaFloatComplex*, int*, int*, bool*, bool*, magmaFloatComplex*)",
    "kernel_GPUHC_trifocal_2op1p_30x30_PH":
        "(magma_queue*, int, int, int, int, magmaFloatComplex**, magmaFloatComplex**, magmaFloatComplex*, "
        "magmaFloatComplex*, magmaFloatComplex*, int*, int*, bool*, bool*, magmaFloatComplex*)",
}


def test_shim_exports_reference_signatures():
    assert os.path.exists(SHIM), "integration shim not built (__graft_entry__.build())"
    out = subprocess.run(["nm", "-DC", SHIM], capture_output=True, text=True, check=True).stdout
    exported = {line.split(" T ", 1)[1].strip() for line in out.splitlines() if " T " in line}
    for name, sig in SIGNATURES.items():
        assert name + sig in exported, f"{name}{sig} not exported"


def test_shim_exports_reserve_and_status():
    """The two calls GPU_HC_Solver adds (integration/hc_trifocal_shim.h): C linkage."""
    assert os.path.exists(SHIM), "integration shim not built (__graft_entry__.build())"
    out = subprocess.run(["nm", "-D", SHIM], capture_output=True, text=True, check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    for name in ("hc_trifocal_shim_reserve", "hc_trifocal_shim_status", "hc_trifocal_shim_info"):
        assert name in exported, name


def _lib():
    from trifocal_pose_estimation_using_improved_gpuhc_amd import _abi
    _abi.lib()                      # the shim binds to the already loaded libhc_trifocal.so
    L = C.CDLL(SHIM)
    L.shim_queue_create.restype = C.c_void_p
    L.shim_queue_create.argtypes = [C.c_void_p]
    L.shim_queue_destroy.argtypes = [C.c_void_p]
    L.hc_trifocal_shim_reserve.argtypes = [C.c_void_p, C.c_int, C.c_int]
    L.hc_trifocal_shim_status.argtypes = [C.c_void_p]
    L.hc_trifocal_shim_info.argtypes = [C.c_void_p, C.POINTER(C.c_size_t), C.POINTER(C.c_int)]
    for f in ("shim_trunpaths", "shim_trunpaths_volta", "shim_trunransac", "shim_trunransac_volta",
              "shim_ph_codeopt", "shim_ph_codeopt_volta", "shim_ph"):
        getattr(L, f).restype = C.c_double
    return L


@pytest.mark.gpu
@pytest.mark.parametrize("abort,truncate,volta,N", [
    (a, t, v, 3) for (a, t) in [(False, True), (True, True), (False, False)] for v in (False, True)] + [
    (False, True, False, 100)])   # enough paths for time slicing: suspended x goes through the pointer arrays
def test_shim_launchers_match_abi(problem, samples100, tracker, ransac0, abort, truncate, volta, N):
    """truncate=False: the archived ..._PH_CodeOpt[_Volta] launchers against
    hc_trifocal_2op1p_30x30_track_ph_codeopt."""
    import torch
    L = _lib()
    dev = tracker.device
    tgt, dif, _ = samples100
    ref = tracker.track(tgt[:N], dif[:N], abort=abort, truncate=truncate).host()
    # the reference's device layout (GPU_HC_Solver.cpp:137-184,335-362): start sols and
    # tracks as 31-complex columns, addressed through per-track pointer arrays
    ss = torch.from_numpy(problem.start_sols).to(dev)
    tracks = ss.unsqueeze(0).expand(N, -1, -1, -1).reshape(N * 312, 31, 2).contiguous()
    ssa = torch.tensor([ss.data_ptr() + k * 31 * 8 for k in range(312)], dtype=torch.int64, device=dev)
    tra = torch.tensor([tracks.data_ptr() + b * 31 * 8 for b in range(312 * N)], dtype=torch.int64, device=dev)
    sp = torch.from_numpy(problem.start_params).to(dev)
    tp = torch.from_numpy(np.ascontiguousarray(tgt[:N])).to(dev)
    dp = torch.from_numpy(np.ascontiguousarray(dif[:N])).to(dev)
    U = torch.from_numpy(problem.unified_index).to(dev)
    hx = torch.from_numpy(np.ascontiguousarray(problem.dHdx_index.reshape(-1))).to(dev)
    ht = torch.from_numpy(np.ascontiguousarray(problem.dHdt_index.reshape(-1))).to(dev)
    conv = torch.zeros(312 * N, dtype=torch.bool, device=dev)
    inf = torch.zeros(312 * N, dtype=torch.bool, device=dev)
    found = torch.zeros(1, dtype=torch.bool, device=dev)
    bidx = torch.full((312 * N,), -1, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev)
    q = L.shim_queue_create(C.c_void_p(stream.cuda_stream))
    p = lambda t: C.c_void_p(t.data_ptr())  # noqa: E731
    s = tracker.settings
    common = [C.c_int(s.max_steps), C.c_int(s.max_corrections), C.c_int(s.delta_t_inc_steps), p(ssa), p(tra), p(sp),
              p(tp), p(dp)]
    tables = [p(hx), p(ht)] if volta else [p(U)]
    if abort:
        E = tracker.edgels
        fn = L.shim_trunransac_volta if volta else L.shim_trunransac
        rv = fn(C.c_void_p(q), C.c_int(N), C.c_int(E.shape[0]), *common, *tables, p(E), p(tracker.K), p(conv), p(inf),
                p(found), p(bidx))
    elif truncate:
        fn = L.shim_trunpaths_volta if volta else L.shim_trunpaths
        rv = fn(C.c_void_p(q), C.c_int(N), *common, *tables, p(conv), p(inf))
    else:
        fn = L.shim_ph_codeopt_volta if volta else L.shim_ph_codeopt
        rv = fn(C.c_void_p(q), C.c_int(N), *common, *tables, p(conv), p(inf))
    torch.cuda.synchronize(dev)
    L.shim_queue_destroy(C.c_void_p(q))
    assert rv == 0.0
    got_conv = conv.cpu().numpy().astype(np.uint8)
    got_tr = tracks.cpu().numpy()
    if not abort:
        assert (got_conv == ref["converge"]).all() and (inf.cpu().numpy().astype(np.uint8) == ref["infinity"]).all()
        assert np.array_equal(got_tr[:, :30], ref["tracks"][:, :30], equal_nan=True)
    else:
        # which paths get skipped depends on scheduling; every path the shim tracked
        # equals the abort-off result and found ids are the direct ABI's passing set
        full = tracker.track(tgt[:N], dif[:N]).host()
        assert bool(found.item())
        ids = np.nonzero(bidx.cpu().numpy() >= 0)[0]
        assert len(ids) and (full["converge"][ids] == 1).all()
        moved = ~np.all(got_tr[:, :30] == np.tile(problem.start_sols[None, :, :30], (N, 1, 1, 1)).reshape(-1, 30, 2),
                        axis=(1, 2))
        assert np.array_equal(got_tr[moved, :30], full["tracks"][moved, :30], equal_nan=True)
        assert (got_conv[moved] == full["converge"][moved]).all()


@pytest.mark.gpu
def test_shim_ph_launcher_matches_abi(problem, samples100, tracker):
    """The archived ..._PH launcher (separate dH/dx, dH/dt tables) against
    hc_trifocal_2op1p_30x30_track_ph."""
    import torch
    L = _lib()
    dev = tracker.device
    N = 2
    tgt, dif, _ = samples100
    ref = tracker.track(tgt[:N], dif[:N], truncate=False, explicit_rk=True).host()
    ss = torch.from_numpy(problem.start_sols).to(dev)
    tracks = ss.unsqueeze(0).expand(N, -1, -1, -1).reshape(N * 312, 31, 2).contiguous()
    ssa = torch.tensor([ss.data_ptr() + k * 31 * 8 for k in range(312)], dtype=torch.int64, device=dev)
    tra = torch.tensor([tracks.data_ptr() + b * 31 * 8 for b in range(312 * N)], dtype=torch.int64, device=dev)
    sp = torch.from_numpy(problem.start_params).to(dev)
    tp = torch.from_numpy(np.ascontiguousarray(tgt[:N])).to(dev)
    dp = torch.from_numpy(np.ascontiguousarray(dif[:N])).to(dev)
    hx = torch.from_numpy(np.ascontiguousarray(problem.dHdx_index.reshape(-1))).to(dev)
    ht = torch.from_numpy(np.ascontiguousarray(problem.dHdt_index.reshape(-1))).to(dev)
    conv = torch.zeros(312 * N, dtype=torch.bool, device=dev)
    inf = torch.zeros(312 * N, dtype=torch.bool, device=dev)
    q = L.shim_queue_create(C.c_void_p(torch.cuda.current_stream(dev).cuda_stream))
    p = lambda t: C.c_void_p(t.data_ptr())  # noqa: E731
    s = tracker.settings
    rv = L.shim_ph(C.c_void_p(q), C.c_int(N), C.c_int(s.max_steps), C.c_int(s.max_corrections),
                   C.c_int(s.delta_t_inc_steps), p(ssa), p(tra), p(sp), p(tp), p(dp), p(hx), p(ht), p(conv), p(inf))
    torch.cuda.synchronize(dev)
    L.shim_queue_destroy(C.c_void_p(q))
    assert rv == 0.0
    assert (conv.cpu().numpy().astype(np.uint8) == ref["converge"]).all()
    assert (inf.cpu().numpy().astype(np.uint8) == ref["infinity"]).all()
    assert np.array_equal(tracks.cpu().numpy()[:, :30], ref["tracks"][:, :30], equal_nan=True)


@pytest.mark.gpu
def test_shim_reserved_stream_never_allocates(problem, samples100, tracker):
    """hc_trifocal_shim_reserve (called from GPU_HC_Solver::Allocate_Arrays)
    sizes the stream's workspace for time slicing up front: launches of up to
    that many samples (plain and Volta) then never allocate on the launch path,
    hc_trifocal_shim_status reports success after the launch, and the results
    equal the ABI's.  A launch on a stream that was not reserved still works
    (the lazy fallback) and is counted."""
    import torch
    L = _lib()
    dev = tracker.device
    N = 100
    tgt, dif, _ = samples100
    ref = tracker.track(tgt[:N], dif[:N]).host()
    stream = torch.cuda.Stream(dev)
    q = L.shim_queue_create(C.c_void_p(stream.cuda_stream))
    s = tracker.settings
    assert L.hc_trifocal_shim_reserve(C.c_void_p(q), N, s.max_steps) == 0
    wsb, grows = C.c_size_t(0), C.c_int(-1)
    assert L.hc_trifocal_shim_info(C.c_void_p(q), C.byref(wsb), C.byref(grows)) == 0
    reserved = wsb.value
    assert reserved == int(tracker.L.hc_trifocal_workspace_size_for_steps(N, s.max_steps)) and grows.value == 0
    ss = torch.from_numpy(problem.start_sols).to(dev)
    ssa = torch.tensor([ss.data_ptr() + k * 31 * 8 for k in range(312)], dtype=torch.int64, device=dev)
    sp = torch.from_numpy(problem.start_params).to(dev)
    tp = torch.from_numpy(np.ascontiguousarray(tgt[:N])).to(dev)
    dp = torch.from_numpy(np.ascontiguousarray(dif[:N])).to(dev)
    U = torch.from_numpy(problem.unified_index).to(dev)
    hx = torch.from_numpy(np.ascontiguousarray(problem.dHdx_index.reshape(-1))).to(dev)
    ht = torch.from_numpy(np.ascontiguousarray(problem.dHdt_index.reshape(-1))).to(dev)
    p = lambda t: C.c_void_p(t.data_ptr())  # noqa: E731
    torch.cuda.synchronize(dev)
    for volta, n in ((False, N), (True, N), (False, 7)):
        tracks = ss.unsqueeze(0).expand(n, -1, -1, -1).reshape(n * 312, 31, 2).contiguous()
        tra = torch.tensor([tracks.data_ptr() + b * 31 * 8 for b in range(312 * n)], dtype=torch.int64, device=dev)
        conv = torch.zeros(312 * n, dtype=torch.bool, device=dev)
        inf = torch.zeros(312 * n, dtype=torch.bool, device=dev)
        torch.cuda.synchronize(dev)
        common = [C.c_int(s.max_steps), C.c_int(s.max_corrections), C.c_int(s.delta_t_inc_steps), p(ssa), p(tra),
                  p(sp), p(tp), p(dp)]
        if volta:
            L.shim_trunpaths_volta(C.c_void_p(q), C.c_int(n), *common, p(hx), p(ht), p(conv), p(inf))
        else:
            L.shim_trunpaths(C.c_void_p(q), C.c_int(n), *common, p(U), p(conv), p(inf))
        assert L.hc_trifocal_shim_status(C.c_void_p(q)) == 0
        assert (conv.cpu().numpy().astype(np.uint8) == ref["converge"][:312 * n]).all()
        assert np.array_equal(tracks.cpu().numpy()[:, :30], ref["tracks"][:312 * n, :30], equal_nan=True)
    assert L.hc_trifocal_shim_info(C.c_void_p(q), C.byref(wsb), C.byref(grows)) == 0
    assert grows.value == 0 and wsb.value == reserved
    L.shim_queue_destroy(C.c_void_p(q))
