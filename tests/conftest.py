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


# Shortest-path kernels the routing tests run on.  The defaults: the per-source LDS search
# (sg_sssp.hip) as the build chooses it (whole tables: phases from 8 rows per CU on, i.e. at C3;
# row blocks: the flagged one-launch plan), its forced bounded-phase form, its forced flagged
# one-launch form (bound rows taken once published),
# the bucketed delta-stepping search (sg_bucket.hip: sparse graphs past the LDS search, forced onto
# every sparse graph here by SG_APSP_BUCKET=1), and the slab relaxation (SG_APSP_LDS=0; dense graphs
# otherwise take the register-resident search of sg_dense.hip).
# The non-default option (landmarks) runs in test_option_kernels, or on the whole matrix with
# SG_TEST_ALL_KERNELS=1.
APSP_KERNELS = ["lds", "lds_bounded", "lds_flagged", "bucket", "slab"]
APSP_OPTIONS = ["lds_landmarks"]
if os.environ.get("SG_TEST_ALL_KERNELS"):
    APSP_KERNELS = APSP_KERNELS + APSP_OPTIONS


def set_apsp_kernel(monkeypatch, name: str) -> str:
    """Select a routing kernel by environment; returns its family ("lds", "bucket" or "slab")."""
    monkeypatch.setenv("SG_APSP_LDS", "0" if name == "slab" else "1")
    if name == "bucket":
        monkeypatch.setenv("SG_APSP_BUCKET", "1")
    else:  # the default choice: the bucketed search only past the LDS search's limit
        monkeypatch.delenv("SG_APSP_BUCKET", raising=False)
    monkeypatch.setenv("SG_SSSP_SEEDS", "2" if name in ("lds_bounded", "lds_landmarks") else "1")
    monkeypatch.setenv("SG_SSSP_LANDMARKS", "8" if name == "lds_landmarks" else "0")
    if name == "lds":  # the default choice (flagged one-launch plan for row blocks, phases for whole tables)
        monkeypatch.delenv("SG_SSSP_FLAGGED", raising=False)
    else:
        monkeypatch.setenv("SG_SSSP_FLAGGED", "1" if name == "lds_flagged" else "0")
    return name if name in ("slab", "bucket") else "lds"
