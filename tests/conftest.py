import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP kernels run)")


def load_npz(name):
    with np.load(os.path.join(GOLDEN, name), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def sub(d, prefix):
    """{'sd/x': a} -> {'x': a} for keys under prefix."""
    n = len(prefix)
    return {k[n:]: v for k, v in d.items() if k.startswith(prefix)}


@pytest.fixture(scope="session")
def f1():
    return load_npz("f1_eval_demo.npz")


@pytest.fixture(scope="session")
def f2():
    return load_npz("f2_train_c2.npz")


@pytest.fixture(scope="session")
def f3():
    return load_npz("f3_train_c1.npz")


@pytest.fixture(scope="session")
def f4():
    return load_npz("f4_ops.npz")


@pytest.fixture(scope="session")
def f5():
    return load_npz("f5_scoring.npz")


@pytest.fixture(scope="session")
def f6():
    return load_npz("f6_hour.npz")


@pytest.fixture(scope="session")
def f7():
    return load_npz("f7_metrics.npz")


@pytest.fixture(scope="session")
def f8():
    return load_npz("f8_negatives.npz")
