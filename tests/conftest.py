import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

Q_MK = 134176769  # PreviousPrime(FirstPrime(27, 4096), 4096)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP engine)")


def gpu_available() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def oracle():
    import pyoracle
    pyoracle.build()
    return pyoracle


def make_case(pyoracle, method, k, n, q, baseG, B, seed, N=2048, Q=Q_MK):
    """Seeded synthetic keys / ciphertexts / accumulators (uniform residues)."""
    orc = pyoracle.Oracle(method, k, n, N, Q, q, baseG)
    evk = pyoracle.fill_uniform(int(np.prod(orc.evk_shape)), Q, seed * 1000 + 1).reshape(orc.evk_shape)
    pkey = pyoracle.fill_uniform(int(np.prod(orc.pkey_shape)), Q, seed * 1000 + 2).reshape(orc.pkey_shape)
    bound = q if method == pyoracle.XZW else 2 * N
    ct = pyoracle.fill_uniform(B * k * n, bound, seed * 1000 + 3).reshape(B, k, n)
    acc = pyoracle.fill_uniform(B * k * N, Q, seed * 1000 + 4).reshape(B, k, N)
    return orc, evk, pkey, ct, acc


@pytest.fixture(scope="session")
def mk_gpu():
    import mkfhe_amd
    return mkfhe_amd
