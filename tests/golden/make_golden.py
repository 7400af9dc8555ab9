"""Generates the committed golden fixtures from the C oracle (oracle/hc_oracle.c).

Inputs are the reference's own data files (copied unmodified under data/); the
outputs pin the oracle so later rounds (and the GPU box, which has no
/root/reference) check against fixed vectors:

  samples_seed0.npz     Prepare_Target_Params(srand(0)) for 100 samples: picked edgel ids + target/diff
  gpuhc_N100_seed0.npz  GPU-HC semantics, 100 samples: conv/inf/steps/corrections per path,
                        a 64-bit hash of every final track, full tracks of samples 0..1,
                        hypothesis-scoring results of every converged path
  cpuhc_seed0.npz       CPU-HC semantics: counts for 100 samples + flags/hashes of samples 0..1
  kat_eval.npz          one evaluation point: x, p, d -> dH/dx, dH/dt, H and the LU solve
  pose_N100_seed0.npz   pose recovery / maximal support over the GPU-HC tracks of
                        the 100 samples: the candidate paths' tracks, their inlier counts, the
                        selected path / inliers / pose per view and its GT residuals
  gpuhc_noisy1px_N100.npz  config 5 inputs: Triplet_Edgels_000 with sigma = 1 px noise
                        (noise seed 20250215, the bench's first trial), samples srand(0), 100
                        samples: per-path flags / counts / hashes, the scoring of every
                        converged path, and the maximal-support selection with its GT residuals
  gpuhc_ds{010,050,099}_N100_seed0.npz  config 2 on held-out synthcurves datasets (round 6):
                        flags / counts / hashes, scoring, the maximal-support pose vs that dataset's GT
  cli_rounds_counts.npz the solution counts of `magmaHC-main -t 4`'s rounds 0..3 (dataset ti, srand(ti))

Run:  python tests/golden/make_golden.py [--only pose|noisy|heldout_golden|cli_rounds|...]   (takes ~1-2 min on 8 cores)
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import oracle as O  # noqa: E402

DATA = os.path.join(ROOT, "data")
PROB = os.path.join(DATA, "problems", "trifocal_2op1p_30x30")
RANS = os.path.join(DATA, "RANSAC_Data", "trifocal_2op1p_30x30", "Synthetic")


def track_hash(tracks):
    """Per-path 64-bit polynomial hash of x[0..29] with +0/-0 and NaN canonicalised."""
    a = np.ascontiguousarray(tracks[:, :30, :], np.float32).copy()
    a[a == 0] = 0.0
    a[np.isnan(a)] = np.float32(np.nan)
    w = a.reshape(a.shape[0], -1).view(np.uint32).astype(np.uint64)
    h = np.zeros(a.shape[0], np.uint64)
    P = np.uint64(1099511628211)
    with np.errstate(over="ignore"):
        for k in range(w.shape[1]):
            h = (h * P) ^ w[:, k]
    return h


def pose_fixture(tr, conv, loc, K):
    gt21 = O.read_floats(os.path.join(RANS, "GT_Poses21", "GT_Poses21_000.txt"), 12)
    gt31 = O.read_floats(os.path.join(RANS, "GT_Poses31", "GT_Poses31_000.txt"), 12)
    inl, sel = O.pose_support(tr, conv, loc, K)
    ids = np.nonzero(inl[:, 0] >= 0)[0].astype(np.int32)
    res, ok = O.pose_residuals(gt21, gt31, sel)
    np.savez_compressed(os.path.join(HERE, "pose_N100_seed0.npz"), cand_ids=ids, cand_tracks=tr[ids],
                        cand_inliers=inl[ids], num_candidates=np.int32(sel["num_candidates"]),
                        path=np.array([sel["path21"], sel["path31"]], np.int32),
                        inliers=np.array([sel["inliers21"], sel["inliers31"]], np.int32),
                        R21=sel["R21"], t21=sel["t21"], R31=sel["R31"], t31=sel["t31"], residuals=res,
                        success=np.bool_(ok))
    print("pose: candidates", sel["num_candidates"], "paths", sel["path21"], sel["path31"], "residuals", res, ok)


NOISE_SEED = 20250215   # synthcurves.DEFAULT_SEED


def noisy_fixture(ss, sp, U, loc, tan, K):
    gt21 = O.read_floats(os.path.join(RANS, "GT_Poses21", "GT_Poses21_000.txt"), 12)
    gt31 = O.read_floats(os.path.join(RANS, "GT_Poses31", "GT_Poses31_000.txt"), 12)
    nloc = O.add_pixel_noise(loc, K, 1.0, NOISE_SEED)
    tgt, dif, picked = O.prepare_target_params(0, [100], nloc, tan, sp)
    tr, conv, inf, st = O.gpuhc_track(ss, sp, tgt, dif, U)
    conv_ids = np.nonzero(conv)[0]
    scores = np.array([O.score_hypothesis(tr[b], nloc, K) for b in conv_ids], dtype=np.int64).reshape(-1, 3)
    inl, sel = O.pose_support(tr, conv, nloc, K)
    res, ok = O.pose_residuals(gt21, gt31, sel)
    np.savez_compressed(os.path.join(HERE, "gpuhc_noisy1px_N100.npz"),
                        target=tgt, diff=dif, picked=picked,
                        conv=conv, inf=inf, steps=st["steps"].astype(np.int16),
                        corrections=st["corrections"].astype(np.int16), hash=track_hash(tr),
                        tracks_s01=tr[:624], counts=np.array(O.count_solutions(tr, conv, inf)),
                        scored_ids=conv_ids.astype(np.int32), scored=scores.astype(np.int32),
                        cand_inliers=inl[inl[:, 0] >= 0], num_candidates=np.int32(sel["num_candidates"]),
                        path=np.array([sel["path21"], sel["path31"]], np.int32),
                        inliers=np.array([sel["inliers21"], sel["inliers31"]], np.int32),
                        residuals=res, success=np.bool_(ok))
    print("noisy 1px: counts", O.count_solutions(tr, conv, inf), "passing", int(scores[:, 0].sum()) if len(scores) else 0,
          "candidates", sel["num_candidates"], "paths", sel["path21"], sel["path31"], "residuals", res, ok)


def heldout_fixture(ss, sp, U):
    """Per-path tracking cost (4 * RK4 steps + corrections, GPU-HC semantics) on
    the two synthcurves datasets the benchmark does NOT use (Triplet_Edgels_001,
    _002; srand(0), 100 samples each): the input of scripts/make_track_order.py,
    so the tracker's dequeue order is not fitted on the benchmark workload."""
    costs = []
    for ds in ("001", "002"):
        loc, tan = O.read_edgels(os.path.join(RANS, "Triplet_Edgels", f"Triplet_Edgels_{ds}.txt"))
        tgt, dif, _ = O.prepare_target_params(0, [100], loc, tan, sp)
        _, _, _, st = O.gpuhc_track(ss, sp, tgt, dif, U)
        costs.append((4 * st["steps"].astype(np.int32) + st["corrections"].astype(np.int32)).reshape(100, 312))
    np.savez_compressed(os.path.join(HERE, "track_cost_heldout.npz"), cost=np.concatenate(costs).astype(np.int16),
                        datasets=np.array(["001", "002"]))
    print("held-out track costs", np.concatenate(costs).shape)


HELDOUT_DATASETS = ("010", "050", "099")


def heldout_golden(ss, sp, U, K):
    """Config 2 on synthcurves datasets no tuning ever saw:
    Triplet_Edgels_010 / _050 / _099 with the reference's srand(0) samples,
    100 samples each: per-path flags / counts / hashes (and the full tracks of
    samples 0..1), the scoring of every converged path, and the maximal-support
    pose with its GT residuals against GT_Poses21/31 of the same dataset."""
    for ds in HELDOUT_DATASETS:
        loc, tan = O.read_edgels(os.path.join(RANS, "Triplet_Edgels", f"Triplet_Edgels_{ds}.txt"))
        gt21 = O.read_floats(os.path.join(RANS, "GT_Poses21", f"GT_Poses21_{ds}.txt"), 12)
        gt31 = O.read_floats(os.path.join(RANS, "GT_Poses31", f"GT_Poses31_{ds}.txt"), 12)
        tgt, dif, picked = O.prepare_target_params(0, [100], loc, tan, sp)
        tr, conv, inf, st = O.gpuhc_track(ss, sp, tgt, dif, U)
        conv_ids = np.nonzero(conv)[0]
        scores = np.array([O.score_hypothesis(tr[b], loc, K) for b in conv_ids], dtype=np.int64).reshape(-1, 3)
        inl, sel = O.pose_support(tr, conv, loc, K)
        res, ok = O.pose_residuals(gt21, gt31, sel)
        np.savez_compressed(os.path.join(HERE, f"gpuhc_ds{ds}_N100_seed0.npz"),
                            target=tgt, diff=dif, picked=picked,
                            conv=conv, inf=inf, steps=st["steps"].astype(np.int16),
                            corrections=st["corrections"].astype(np.int16), hash=track_hash(tr),
                            tracks_s01=tr[:624], counts=np.array(O.count_solutions(tr, conv, inf)),
                            scored_ids=conv_ids.astype(np.int32), scored=scores.astype(np.int32),
                            num_candidates=np.int32(sel["num_candidates"]),
                            path=np.array([sel["path21"], sel["path31"]], np.int32),
                            inliers=np.array([sel["inliers21"], sel["inliers31"]], np.int32),
                            residuals=res, success=np.bool_(ok))
        print(f"dataset {ds}: counts", O.count_solutions(tr, conv, inf), "passing",
              int(scores[:, 0].sum()) if len(scores) else 0, "stages", int(4 * st["steps"].sum() + st["corrections"].sum()),
              "candidates", sel["num_candidates"], "residuals", res, ok)


def cli_rounds_fixture(ss, sp, U):
    """The CLI's rounds ti = 0..3 (`magmaHC-main -t 4`, cmd/magmaHC-main.cpp:38-48):
    round ti reads Triplet_Edgels_<ti> and draws its samples with srand(ti)
    (GPU_HC_Solver.cpp:252-306); 100 samples each: the solution counts the CLI
    writes to GPU_Sols_Statistics.txt, one row per round."""
    counts = []
    for ti in range(4):
        loc, tan = O.read_edgels(os.path.join(RANS, "Triplet_Edgels", f"Triplet_Edgels_{ti:03d}.txt"))
        tgt, dif, _ = O.prepare_target_params(ti, [100], loc, tan, sp)
        tr, conv, inf, _ = O.gpuhc_track(ss, sp, tgt, dif, U)
        counts.append(O.count_solutions(tr, conv, inf))
        print(f"round {ti}: counts", counts[-1])
    np.savez_compressed(os.path.join(HERE, "cli_rounds_counts.npz"), counts=np.array(counts, np.int64))


def ph_codeopt_fixture(ss, sp, U, tgt, dif, explicit_rk=False):
    """Config 2 through the archived ..._PH_CodeOpt semantics (no depth-sign
    truncation; the archived kernel is ..._TrunPaths without :148-155), or with
    explicit_rk the archived ..._PH semantics (explicit RK helpers as well)."""
    tr, conv, inf, st = O.gpuhc_track(ss, sp, tgt, dif, U, O.settings(truncate=False, explicit_rk=explicit_rk))
    name = "gpuhc_ph_N100_seed0.npz" if explicit_rk else "gpuhc_phcodeopt_N100_seed0.npz"
    np.savez_compressed(os.path.join(HERE, name),
                        conv=conv, inf=inf, steps=st["steps"].astype(np.int16),
                        corrections=st["corrections"].astype(np.int16), hash=track_hash(tr),
                        counts=np.array(O.count_solutions(tr, conv, inf)), real=real_flags(tr, conv))
    print("PH" if explicit_rk else "PH_CodeOpt", "counts", O.count_solutions(tr, conv, inf), "stages",
          int(4 * st["steps"].sum() + st["corrections"].sum()))


def real_flags(tracks, conv):
    """Per path: converged and every |Im x_v| <= 1e-4 (Evaluations.cpp:145-182,
    definitions.hpp:25) -- the 'real' column of *_Sols_Statistics per path."""
    im_ok = (np.abs(tracks[:, :30, 1]).astype(np.float64) <= 1e-4).all(axis=1)
    return (im_ok & (conv != 0)).astype(np.uint8)


def add_real_flags(ss, sp, U, tgt, dif):
    """Adds per-path `real` flags to gpuhc_N100_seed0.npz and
    gpuhc_phcodeopt_N100_seed0.npz (fields kept; the re-run must reproduce the
    committed hashes).  Input of the batch-id-prefix pin against the reference's
    committed GPU_Sols_Statistics.txt (tests/test_oracle_kat.py)."""
    for name, s in (("gpuhc_N100_seed0.npz", O.settings()),
                    ("gpuhc_phcodeopt_N100_seed0.npz", O.settings(truncate=False))):
        path = os.path.join(HERE, name)
        old = dict(np.load(path))
        tr, conv, inf, _ = O.gpuhc_track(ss, sp, tgt, dif, U, s)
        assert np.array_equal(track_hash(tr), old["hash"]) and np.array_equal(conv, old["conv"]), name
        old["real"] = real_flags(tr, conv)
        np.savez_compressed(path, **old)
        print(name, "real paths", int(old["real"].sum()), "converged", int(conv.sum()))


def main():
    only = sys.argv[sys.argv.index("--only") + 1] if "--only" in sys.argv else None
    ss, sp, dhdx, dhdt = O.read_problem(PROB)
    U = np.concatenate([dhdx, dhdt]).astype(np.int32)
    loc, tan = O.read_edgels(os.path.join(RANS, "Triplet_Edgels", "Triplet_Edgels_000.txt"))
    K = O.read_floats(os.path.join(RANS, "Intrinsic_Matrix.txt"), 9)
    tgt, dif, picked = O.prepare_target_params(0, [100], loc, tan, sp)
    if only == "real":
        add_real_flags(ss, sp, U, tgt, dif)
        return
    if only in ("phcodeopt", "ph"):
        tgt, dif, _ = O.prepare_target_params(0, [100], loc, tan, sp)
        ph_codeopt_fixture(ss, sp, U, tgt, dif, explicit_rk=only == "ph")
        return
    if only == "heldout":
        heldout_fixture(ss, sp, U)
        return
    if only == "heldout_golden":
        heldout_golden(ss, sp, U, K)
        return
    if only == "cli_rounds":
        cli_rounds_fixture(ss, sp, U)
        return
    if only == "pose":
        tr, conv, inf, st = O.gpuhc_track(ss, sp, tgt, dif, U)
        pose_fixture(tr, conv, loc, K)
        return
    if only in (None, "noisy"):
        noisy_fixture(ss, sp, U, loc, tan, K)
        if only == "noisy":
            return
    np.savez_compressed(os.path.join(HERE, "samples_seed0.npz"), picked=picked, target=tgt, diff=dif)

    tr, conv, inf, st = O.gpuhc_track(ss, sp, tgt, dif, U)
    pose_fixture(tr, conv, loc, K)
    conv_ids = np.nonzero(conv)[0]
    scores = np.array([O.score_hypothesis(tr[b], loc, K) for b in conv_ids], dtype=np.int64).reshape(-1, 3)
    np.savez_compressed(os.path.join(HERE, "gpuhc_N100_seed0.npz"),
                        conv=conv, inf=inf, steps=st["steps"].astype(np.int16),
                        corrections=st["corrections"].astype(np.int16), hash=track_hash(tr),
                        tracks_s01=tr[:624], counts=np.array(O.count_solutions(tr, conv, inf)),
                        scored_ids=conv_ids.astype(np.int32), scored=scores.astype(np.int32),
                        real=real_flags(tr, conv))
    print("gpuhc counts", O.count_solutions(tr, conv, inf), "passing", int(scores[:, 0].sum()))

    trc, cc, ic, stc, secs = O.cpuhc_track(ss, sp, tgt, dif, dhdx, dhdt)
    np.savez_compressed(os.path.join(HERE, "cpuhc_seed0.npz"),
                        counts=np.array(O.count_solutions(trc, cc, ic)), conv_s01=cc[:624], inf_s01=ic[:624],
                        steps_s01=stc["steps"][:624].astype(np.int16), hash_s01=track_hash(trc[:624]))
    print("cpuhc counts", O.count_solutions(trc, cc, ic), f"{secs:.1f}s")

    # one evaluation point inside a path: sample 0, track 5, t = 0.37, x = start sol perturbed
    rng = np.random.default_rng(7)
    x = ss[5].copy()
    x[:30] += (rng.standard_normal((30, 2)) * 1e-2).astype(np.float32)
    p = O.param_homotopy(0.37, sp, tgt[0])
    A = O.eval_hx(dhdx, x, p)
    bt = O.eval_ht(dhdt, x, p, dif[0])
    bh = O.eval_h(dhdt, x, p)
    sol = O.cgesv_gpu(A, bt)
    np.savez_compressed(os.path.join(HERE, "kat_eval.npz"), x=x, p=p, d=dif[0], Hx=A, Ht=bt, H=bh, lu_x=sol)


if __name__ == "__main__":
    main()
