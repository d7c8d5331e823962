"""pytest configuration: the `gpu` marker, import paths, shared fixtures."""
import os
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parent.parent
PKG = ROOT / "hand-pose-estimation_amd"
for p in (ROOT, PKG, ROOT / "oracle", ROOT / "tests"):
    if str(p) not in sys.path:
        sys.path.insert(0, str(p))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 GPU (run with -m gpu)")


@pytest.hookimpl(trylast=True)
def pytest_collection_modifyitems(config, items):
    # torch's HIP runtime must initialise before libhpe.so's (tests that hand torch device
    # buffers to the ABI): whenever a selected test is a GPU test, however it was selected.
    # trylast: after pytest's own -m / -k deselection, so a CPU-only run never
    # initialises the HIP runtime
    if any(it.get_closest_marker("gpu") for it in items):
        import torch
        torch.cuda.is_available()


@pytest.fixture(scope="session")
def oracle():
    import oracle_c
    return oracle_c.load()


@pytest.fixture(scope="session")
def np_hand():
    import oracle_np
    import hand_data
    geo, rad = hand_data.geometry_cm()
    return oracle_np.Hand(geo, rad)


@pytest.fixture(scope="session")
def ora_hand(oracle):
    import hand_data
    geo, rad = hand_data.geometry_cm()
    return oracle.hand(geo, rad)
