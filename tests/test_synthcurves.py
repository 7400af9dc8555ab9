"""Noisy synthcurves generator: the native generator
(std::mt19937_64 + std::normal_distribution) equals the oracle's restatement of
those standard-library algorithms bit for bit; the written dataset reads back
bit-exactly through the reference-format reader; the noise has the requested
pixel statistics."""
import numpy as np


def test_noise_matches_oracle(oracle, ransac0):
    from trifocal_pose_estimation_using_improved_gpuhc_amd import synthcurves
    for sigma, seed in ((1.0, 20250215), (0.5, 1), (3.0, 2 ** 63 + 5), (0.0, 7)):
        a = synthcurves.add_pixel_noise(ransac0.locations, ransac0.K, sigma, seed)
        b = oracle.add_pixel_noise(ransac0.locations, ransac0.K, sigma, seed)
        assert np.array_equal(a, b), (sigma, seed)
    z = synthcurves.add_pixel_noise(ransac0.locations, ransac0.K, 0.0, 3)
    assert np.abs(z - ransac0.locations).max() < 1e-6   # sigma 0: metric -> pixel -> metric round trip only


def test_noise_statistics(ransac0):
    from trifocal_pose_estimation_using_improved_gpuhc_amd import synthcurves
    a = synthcurves.add_pixel_noise(ransac0.locations, ransac0.K, 1.0)
    K = ransac0.K
    du = (a[:, 0::2] - ransac0.locations[:, 0::2]) * K[0]
    dv = (a[:, 1::2] - ransac0.locations[:, 1::2]) * K[4]
    d = np.concatenate([du.ravel(), dv.ravel()]).astype(np.float64)
    assert abs(d.mean()) < 0.03 and abs(d.std() - 1.0) < 0.03
    b = synthcurves.add_pixel_noise(ransac0.locations, ransac0.K, 1.0, seed=1)
    assert not np.array_equal(a, b)


def test_dataset_round_trip(tmp_path, ransac0):
    from trifocal_pose_estimation_using_improved_gpuhc_amd import load_ransac_data, synthcurves
    d = synthcurves.make_noisy_dataset(1.0, indices=(0, 2), name="Noisy1", out_root=str(tmp_path))
    for i in (0, 2):
        r = load_ransac_data(i, root=str(tmp_path), dataset="Noisy1")
        src = load_ransac_data(i)
        exp = synthcurves.add_pixel_noise(src.locations, src.K, 1.0, synthcurves.DEFAULT_SEED + i)
        assert np.array_equal(r.locations, exp)
        assert np.array_equal(r.tangents, src.tangents)
        assert np.array_equal(r.K, src.K) and np.array_equal(r.pose21, src.pose21)
    assert d.endswith("Noisy1")
