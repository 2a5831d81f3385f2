"""Test configuration: the `gpu` marker and import paths.

CPU tests (-m "not gpu") cover the oracle against the golden fixtures, the
host logic, multi-rank simulations over gloo, and that the C-ABI libraries
load and export every declared symbol.  GPU tests (-m gpu) are the parity
tests proper: HIP path (through the C ABI) vs the oracle.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "bagua-core_amd"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")


@pytest.fixture(scope="session")
def oracle_c():
    from oracle import oracle_c
    oracle_c.build()
    return oracle_c


@pytest.fixture(scope="session")
def goldens():
    import numpy as np
    path = os.path.join(ROOT, "tests", "golden", "codec_v1.npz")
    with np.load(path, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}
