"""CPU tests of the C-ABI boundary and the native host data layer.

* the library exports exactly the entry points include/*.h declare;
* argument validation returns the documented hcStatus codes without touching
  a device (no compute call is made here);
* the host layer (readers, RANSAC sample generation, sample split, solution
  counting -- include/hc_host.h) agrees bit for bit with the oracle's
  independent C restatement of Data_Reader.cpp / GPU_HC_Solver.cpp:252-306 /
  Evaluations.cpp:145-182.
"""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import ROOT

INCLUDE = os.path.join(ROOT, "include")


def _declared_c_functions(header):
    """Function names declared in a C header (outside comments)."""
    src = open(os.path.join(INCLUDE, header)).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    src = re.sub(r"//[^\n]*", "", src)
    names = re.findall(r"^[A-Za-z_][\w\s\*]*?\b(hc_\w+)\s*\(", src, flags=re.M)
    return set(names)


def _all_declared():
    """Every function the public headers declare (include/*.h)."""
    names = set()
    for h in sorted(os.listdir(INCLUDE)):
        if h.endswith(".h"):
            names |= _declared_c_functions(h)
    return names


def test_headers_declare_the_bound_symbols():
    from trifocal_pose_estimation_using_improved_gpuhc_amd import _abi
    declared = _all_declared()
    assert declared == set(_abi.DECLARED_SYMBOLS)


def test_library_exports_every_declared_symbol():
    from trifocal_pose_estimation_using_improved_gpuhc_amd import _abi
    out = subprocess.run(["nm", "-D", "--defined-only", _abi.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    exported = {ln.split()[-1] for ln in out.splitlines() if ln.strip()}
    declared = _all_declared()
    missing = declared - exported
    assert not missing, f"declared but not exported: {sorted(missing)}"
    L = _abi.lib()
    for name in declared:
        assert getattr(L, name) is not None


def test_workspace_size_and_version():
    from trifocal_pose_estimation_using_improved_gpuhc_amd import _abi
    L = _abi.lib()
    ws = int(L.hc_trifocal_workspace_size())
    assert 64 <= ws < (1 << 20)
    assert ws % 256 == 0
    assert b"gfx950" in L.hc_trifocal_version()


def test_abi_version_and_build_id():
    """The binding refuses a library of another struct layout; the build id
    names the library's device code (bench.py selects its profiles by it)."""
    from trifocal_pose_estimation_using_improved_gpuhc_amd import _abi
    L = _abi.lib()
    assert L.hc_trifocal_abi_version() == _abi.ABI_VERSION == 2
    hdr = open(os.path.join(ROOT, "include", "hc_trifocal.h")).read()
    assert "#define HC_TRIFOCAL_ABI_VERSION 2" in hdr
    bid = _abi.build_id()
    assert bid.startswith("v") and "+" in bid and len(bid.split("+")[1]) == 12
    assert bid == _abi.build_id(_abi.PRODUCT_LIB_PATH)


def test_workspace_size_for_time_slicing():
    """hc_trifocal_workspace_size_for(N): the base workspace + the time-slicing
    area: ring counters (1 KB), a 256-B suspend block per path and an 8-B ring
    entry per possible suspension -- at most (max_steps + 1) / 3 per path,
    never reused within a launch (+1 per path, + 4096 spare entries for the
    re-pushes of abandoned tickets).  The plain form assumes max_steps = 80."""
    from trifocal_pose_estimation_using_improved_gpuhc_amd import _abi
    L = _abi.lib()
    base = int(L.hc_trifocal_workspace_size())
    s0, s1, s100 = (int(L.hc_trifocal_workspace_size_for(n)) for n in (0, 1, 100))
    assert base < s0 <= s1 < s100
    assert s100 % 256 == 0
    per_path = 256 + 8 * (81 // 3 + 1)
    assert per_path * 312 * 100 + 8 * 4096 <= s100 - base <= per_path * 312 * 100 + 8 * 4096 + 2048
    assert int(L.hc_trifocal_workspace_size_for(-5)) == s0
    assert int(L.hc_trifocal_workspace_size_for_steps(100, 80)) == s100
    s200 = int(L.hc_trifocal_workspace_size_for_steps(100, 200))
    assert s200 - s100 >= 8 * 312 * 100 * (201 // 3 - 81 // 3)


def test_invalid_arguments_are_rejected_before_any_device_work():
    from trifocal_pose_estimation_using_improved_gpuhc_amd import _abi
    L = _abi.lib()
    ws = int(L.hc_trifocal_workspace_size())
    dummy = C.c_void_p(0x1000)          # never dereferenced: validation fails first
    a = _abi.hcTrackArgs()
    a.sub_ransac_iters = 1
    a.settings = _abi.hcTrackSettings(80, 3, 4)
    # null args / null workspace
    assert L.hc_trifocal_2op1p_30x30_track(None, dummy, ws, None) == 1
    assert L.hc_trifocal_2op1p_30x30_track(C.byref(a), None, ws, None) == 2
    assert L.hc_trifocal_2op1p_30x30_track(C.byref(a), dummy, ws - 1, None) == 2
    # required device pointers missing
    assert L.hc_trifocal_2op1p_30x30_track(C.byref(a), dummy, ws, None) == 1
    # negative sizes / settings
    a.sub_ransac_iters = -1
    assert L.hc_trifocal_2op1p_30x30_track(C.byref(a), dummy, ws, None) == 1
    a.sub_ransac_iters = 1
    for f in ("start_sols", "tracks", "start_params", "target_params", "diff_params", "unified_index",
              "converge", "infinity"):
        setattr(a, f, 0x1000)
    a.settings = _abi.hcTrackSettings(-1, 3, 4)
    assert L.hc_trifocal_2op1p_30x30_track(C.byref(a), dummy, ws, None) == 1
    a.settings = _abi.hcTrackSettings(80, 3, 4)
    # too many paths for the int32 batch index of the reference interface
    a.sub_ransac_iters = (1 << 31) // 312 + 1
    assert L.hc_trifocal_2op1p_30x30_track(C.byref(a), dummy, ws, None) == 1
    # abort mode needs its RANSAC arrays
    a.sub_ransac_iters = 1
    ab = _abi.hcAbortArgs()
    assert L.hc_trifocal_2op1p_30x30_track_abort(C.byref(a), None, dummy, ws, None) == 1
    assert L.hc_trifocal_2op1p_30x30_track_abort(C.byref(a), C.byref(ab), dummy, ws, None) == 1
    # zero samples is a no-op success (reference: empty grid)
    a.sub_ransac_iters = 0
    assert L.hc_trifocal_2op1p_30x30_track(C.byref(a), dummy, ws, None) == 0
    # component entry points
    assert L.hc_cgesv_30x30_batched(-1, None, None, None, None) == 1
    assert L.hc_cgesv_30x30_batched(4, None, None, None, None) == 1
    assert L.hc_cgesv_30x30_batched(0, None, None, None, None) == 0
    assert L.hc_trifocal_eval_batched(4, None, None, None, None, None, None, None, dummy, ws, None) == 1
    u = C.c_void_p(0x2000)
    assert L.hc_trifocal_eval_batched(0, u, None, None, None, None, None, None, None, 0, None) == 2
    d = C.c_double(0)
    assert L.hc_trifocal_read_timings(None, C.byref(d)) == 1


def test_host_readers_match_oracle(problem, oracle):
    from trifocal_pose_estimation_using_improved_gpuhc_amd.problem import problem_dir
    ss, sp, dhdx, dhdt = oracle.read_problem(problem_dir())
    assert np.array_equal(problem.start_sols.view(np.uint32), ss.view(np.uint32))
    assert np.array_equal(problem.start_params.view(np.uint32), sp.view(np.uint32))
    assert np.array_equal(problem.dHdx_index, dhdx)
    assert np.array_equal(problem.dHdt_index, dhdt)
    assert np.all(problem.start_sols[:, 30] == np.array([1.0, 0.0], np.float32))
    assert np.all(problem.start_params[33] == np.array([1.0, 0.0], np.float32))


@pytest.mark.parametrize("index", [0, 1, 2])
def test_edgel_reader_matches_oracle(oracle, index):
    from trifocal_pose_estimation_using_improved_gpuhc_amd import load_ransac_data
    from trifocal_pose_estimation_using_improved_gpuhc_amd.problem import ransac_dir
    d = load_ransac_data(index)
    loc, tan = oracle.read_edgels(os.path.join(ransac_dir(), "Triplet_Edgels", f"Triplet_Edgels_{index:03d}.txt"))
    assert np.array_equal(d.locations.view(np.uint32), loc.view(np.uint32))
    assert np.array_equal(d.tangents.view(np.uint32), tan.view(np.uint32))
    K = oracle.read_floats(os.path.join(ransac_dir(), "Intrinsic_Matrix.txt"), 9)
    assert np.array_equal(d.K, K)
    # GT poses: R row-major (orthonormal) then t
    for P in (d.pose21, d.pose31):
        R = P[:9].reshape(3, 3).astype(np.float64)
        assert np.abs(R @ R.T - np.eye(3)).max() < 1e-5


@pytest.mark.parametrize("n,g", [(100, 1), (8000, 8), (1001, 8), (7, 8), (1000, 3)])
def test_split_samples_rule(n, g):
    from trifocal_pose_estimation_using_improved_gpuhc_amd import split_samples
    sub = split_samples(n, g)
    ref = np.array([n // g + (1 if k < n % g else 0) for k in range(g)])   # GPU_HC_Solver.cpp:85-88
    assert np.array_equal(sub, ref)
    assert sub.sum() == n


@pytest.mark.parametrize("n,g,seed", [(100, 1, 0), (37, 4, 0), (64, 8, 7)])
def test_prepare_target_params_matches_oracle(problem, ransac0, oracle, n, g, seed):
    from trifocal_pose_estimation_using_improved_gpuhc_amd import prepare_target_params, split_samples
    tgt, dif, picked = prepare_target_params(problem, ransac0, seed=seed, num_samples=n, num_gpus=g)
    t2, d2, p2 = oracle.prepare_target_params(seed, split_samples(n, g), ransac0.locations, ransac0.tangents,
                                              problem.start_params)
    assert np.array_equal(picked, p2)
    assert np.array_equal(tgt.view(np.uint32), t2.view(np.uint32))
    assert np.array_equal(dif.view(np.uint32), d2.view(np.uint32))
    # reference draw rule: i0 != i1 and i1 != i2 (i0 == i2 allowed), indices in range
    assert np.all(picked[:, 0] != picked[:, 1]) and np.all(picked[:, 1] != picked[:, 2])
    assert picked.min() >= 0 and picked.max() < ransac0.locations.shape[0]
    # params 30..33 are the constants of GPU_HC_Solver.cpp:290-296
    assert np.array_equal(tgt[:, 30:34, 0], np.tile([1.0, 0.5, 1.0, 1.0], (n, 1)).astype(np.float32))


def test_sample_k_is_independent_of_gpu_count(problem, ransac0):
    """gpu-major order: sharding over G GPUs reproduces the same sample sequence."""
    from trifocal_pose_estimation_using_improved_gpuhc_amd import prepare_target_params
    t1, _, p1 = prepare_target_params(problem, ransac0, seed=0, num_samples=64, num_gpus=1)
    t8, _, p8 = prepare_target_params(problem, ransac0, seed=0, num_samples=64, num_gpus=8)
    assert np.array_equal(p1, p8) and np.array_equal(t1, t8)


def test_count_solutions_matches_oracle(oracle):
    from trifocal_pose_estimation_using_improved_gpuhc_amd import count_solutions
    rng = np.random.default_rng(5)
    n = 3
    tracks = rng.standard_normal((312 * n, 31, 2)).astype(np.float32)
    tracks[::3, :30, 1] = 0.0               # a third are real
    tracks[1::7, 4, 1] = 5e-5               # within the 1e-4 imaginary tolerance
    conv = (rng.random(312 * n) < 0.4).astype(np.uint8)
    inf = ((rng.random(312 * n) < 0.2) & (conv == 0)).astype(np.uint8)
    assert count_solutions(tracks, conv, inf) == tuple(oracle.count_solutions(tracks, conv, inf))
    assert count_solutions(tracks, np.zeros_like(conv), np.zeros_like(inf)) == (0, 0, 0)


def test_write_converged_sols_layout(tmp_path):
    """hc_write_converged_sols == Evaluations::Write_Converged_Sols byte layout
    (Evaluations.cpp:120-143): header per sample, global batch id, 30 re/im lines
    printed with std::setprecision(20) (== printf %.20g of the float)."""
    import ctypes as C

    from trifocal_pose_estimation_using_improved_gpuhc_amd import _abi
    rng = np.random.default_rng(3)
    N = 2
    tr = rng.standard_normal((312 * N, 31, 2)).astype(np.float32)
    tr[5, 3, 0] = 0.0
    tr[7, 4, 1] = -0.0
    tr[9, 1, 0] = 1e-30
    conv = (rng.random(312 * N) < 0.1).astype(np.uint8)
    f = str(tmp_path / "sols.txt")
    n = _abi.lib().hc_write_converged_sols(f.encode(), C.c_int(N), C.c_void_p(tr.ctypes.data),
                                           C.c_void_p(conv.ctypes.data))
    assert n == int(conv.sum())
    exp = []
    for ri in range(N):
        exp.append(f"-------------------- RANSAC Iteration {ri + 1} --------------------\n\n")
        for bs in range(312):
            b = ri * 312 + bs
            if conv[b]:
                exp.append(f"{b}\n")
                for v in range(30):
                    exp.append(f"{float(tr[b, v, 0]):.20g}\t{float(tr[b, v, 1]):.20g}\n")
                exp.append("\n")
        exp.append("\n")
    assert open(f).read() == "".join(exp)
