import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLD = os.path.join(ROOT, "tests", "golden")
DATA = os.path.join(ROOT, "tests", "data")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X); run with -m gpu")


@pytest.fixture(scope="session")
def golden():
    with open(os.path.join(GOLD, "golden.json")) as f:
        meta = json.load(f)
    arr = np.load(os.path.join(GOLD, "golden.npz"), allow_pickle=False)
    return meta, arr


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as O
    O.lib()
    return O


@pytest.fixture(scope="session")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.cuda.set_device(0)
    return torch


@pytest.fixture(scope="session")
def drift_golden():
    with open(os.path.join(GOLD, "drift.json")) as f:
        meta = json.load(f)
    return meta, np.load(os.path.join(GOLD, "drift.npz"), allow_pickle=False)


@pytest.fixture(scope="session")
def drift_inputs(drift_golden, oracle):
    """Golden-case inputs regenerated from their parameters (oracle/drift.py beacon_input)."""
    from oracle import drift as OD
    meta, _ = drift_golden
    return {c["name"]: OD.beacon_input(c["payload"], c["fs"], c["f0"], c["fc"], c["drift_hz_per_s"],
                                       c["esn0_db"], c["seed"]) for c in meta["cases"]}
