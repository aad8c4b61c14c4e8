"""The non-default shortest-path option, one representative graph shape each (the default
kernels run the whole routing suite, conftest.APSP_KERNELS): landmark rows splitting the
first phase (SG_SSSP_LANDMARKS).  Bit-exact against the oracle."""
import pytest

from conftest import APSP_OPTIONS, set_apsp_kernel
from test_routing_fuzz_gpu import test_random_graph_shapes as _shape

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("option", APSP_OPTIONS)
@pytest.mark.parametrize("n,avg_deg,directed,frac,seed", [
    (300, 12.0, True, 0.7, 2),
    (700, 4.0, False, 0.45, 3),
    (1000, 1.5, True, 1.0, 7),
])
def test_option_kernels(oracle, ctx, monkeypatch, option, n, avg_deg, directed, frac, seed):
    set_apsp_kernel(monkeypatch, option)
    _shape(oracle, ctx, n, avg_deg, directed, frac, seed)
