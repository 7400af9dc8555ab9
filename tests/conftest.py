"""Shared fixtures.  `-m gpu` tests need a ROCm GPU and the built HIP library;
everything else runs on the CPU (oracle, host data layer, ABI exports)."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (ROCm GPU) and the HIP library")


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as O
    O.lib()
    return O


@pytest.fixture(scope="session")
def problem():
    from trifocal_pose_estimation_using_improved_gpuhc_amd import load_problem
    return load_problem()


@pytest.fixture(scope="session")
def ransac0():
    from trifocal_pose_estimation_using_improved_gpuhc_amd import load_ransac_data
    return load_ransac_data(0)


@pytest.fixture(scope="session")
def samples100(problem, ransac0):
    from trifocal_pose_estimation_using_improved_gpuhc_amd import prepare_target_params
    return prepare_target_params(problem, ransac0, seed=0, num_samples=100)


@pytest.fixture(scope="session")
def tracker(problem, ransac0):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from trifocal_pose_estimation_using_improved_gpuhc_amd.tracker import DeviceTracker
    t = DeviceTracker(problem, "cuda:0")
    t.set_ransac_data(ransac0)
    return t


def same(a, b):
    """Element-wise equality that treats NaN == NaN and +0 == -0 (the parity bar:
    identical values; only the sign of exact zeros may differ)."""
    a = np.asarray(a)
    b = np.asarray(b)
    return (a == b) | (np.isnan(a) & np.isnan(b))
