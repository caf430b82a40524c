"""Test configuration: the `gpu` marker and shared helpers.

`-m "not gpu"` runs on CPU only: the oracle against the reference's golden vectors, host logic,
the C-ABI library loading/exports, ISA checks and multi-rank (gloo) plumbing.
`-m gpu` runs the parity tests proper: the gfx950 engine through the C ABI against the oracle.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (ROOT, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) device")


def golden(name):
    import numpy as np

    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


@pytest.fixture(scope="session")
def oracle():
    import klsh_oracle

    klsh_oracle.build()
    return klsh_oracle


@pytest.fixture(scope="session")
def engine():
    """One gfx950 context for the whole GPU session (fails loudly without the library/device)."""
    from kmerlsh_amd import _native

    eng = _native.Engine(0)
    yield eng
    eng.close()
