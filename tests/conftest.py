import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run with -m gpu on the GPU box)")


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as O

    O.lib()  # builds oracle/libsg_oracle.so with gcc if missing
    return O


@pytest.fixture(scope="session")
def ctx():
    """GPU context; the HIP library must load (no fallback)."""
    import shadow_amd

    shadow_amd.load()
    return shadow_amd.default_context(0)
