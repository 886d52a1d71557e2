import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X); run with -m gpu")
    config.addinivalue_line("markers", "slow: long CPU test")


def golden(name: str):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def golden_npy(name: str) -> np.ndarray:
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def unhex(v):
    if isinstance(v, str):
        return float.fromhex(v)
    return [unhex(x) for x in v]


def bits(a) -> np.ndarray:
    return np.ascontiguousarray(a, dtype=np.float64).view(np.uint64)


def sha(a) -> str:
    import hashlib
    return hashlib.sha256(np.ascontiguousarray(a, dtype=np.float64).tobytes()).hexdigest()


@pytest.fixture(scope="session")
def final_scene():
    g = golden("counter_final.json")
    return np.array(unhex(g["spheres"]))


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle
    oracle.build()
    return oracle


@pytest.fixture
def knobs():
    """Set process-default tuning knobs (rt_context_set_tuning(NULL, ...),
    include/rt.h) for one test: contexts created afterwards and the one-shot
    entries take them; the previous values come back at teardown."""
    import petershirleyraytracer_amd as P
    saved = {}

    def set_(name, value):
        if name not in saved:
            saved[name] = P.get_tuning(name)
        P.set_tuning(name, value)

    yield set_
    for k, v in saved.items():
        P.set_tuning(k, v)


def have_gpu() -> bool:
    try:
        import petershirleyraytracer_amd as P
        return P.device_count() > 0
    except Exception:
        return False
