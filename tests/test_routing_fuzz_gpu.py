"""Routing-table parity across graph shapes that select different kernel paths:
sparse (64-source batches, one arc segment), dense (> 600 in-arcs per node:
32-source batches with arc segments and the atomic-min flush), directed and
undirected, parallel arcs, used-node subsets.  Bit-exact against the oracle."""
import numpy as np
import pytest

from conftest import APSP_KERNELS, set_apsp_kernel
from shadow_amd import NetworkGraph

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True, params=APSP_KERNELS)
def apsp_kernel(request, monkeypatch):
    """The default shortest-path kernels (conftest.APSP_KERNELS): the per-source LDS search,
    also in its forced bounded-phase form, and the slab relaxation."""
    return set_apsp_kernel(monkeypatch, request.param)


def _random_graph(n, avg_deg, directed, seed):
    rng = np.random.default_rng(seed)
    m = int(n * avg_deg / (1 if directed else 2))
    # a ring (both ways when directed) keeps it connected; self-loops on every node
    ring_s = np.arange(n)
    ring_d = (ring_s + 1) % n
    if directed:
        ring_s, ring_d = np.concatenate([ring_s, ring_d]), np.concatenate([ring_d, ring_s])
    s = rng.integers(0, n, m)
    d = rng.integers(0, n, m)
    keep = s != d
    src = np.concatenate([np.arange(n), ring_s, s[keep]]).astype(np.uint32)
    dst = np.concatenate([np.arange(n), ring_d, d[keep]]).astype(np.uint32)
    lat = rng.integers(1, 200, len(src)).astype(np.uint64) * 1000
    loss = np.where(rng.random(len(src)) < 0.6, 0.0, rng.random(len(src)) * 0.05).astype(np.float32)
    return dict(n=n, src=src, dst=dst, lat=lat, loss=loss, directed=directed)


@pytest.mark.parametrize("n,avg_deg,directed,frac,seed", [
    (50, 3.0, False, 1.0, 1),
    (300, 12.0, True, 0.7, 2),
    (700, 4.0, False, 0.45, 3),
    (700, 100.0, True, 1.0, 4),
    (700, 680.0, False, 0.8, 5),   # dense: B = 32, arc segments
    (700, 690.0, True, 0.6, 6),    # dense, directed
    (1000, 1.5, True, 1.0, 7),     # long paths (many passes)
])
def test_random_graph_shapes(oracle, ctx, n, avg_deg, directed, frac, seed):
    g = _random_graph(n, avg_deg, directed, seed)
    used = np.random.default_rng(seed + 100).permutation(n)[:max(1, int(n * frac))].astype(np.uint32)
    net = NetworkGraph(g["n"], g["src"], g["dst"], g["lat"], g["loss"], g["directed"], ctx=ctx)
    t = net.compute_shortest_paths(used)
    rc, olat, oloss, _ = oracle.shortest_paths(g["n"], g["src"], g["dst"], g["lat"], g["loss"], g["directed"], used,
                                               threads=8)
    assert rc == 0
    assert np.array_equal(t.latency_ns, olat)
    assert np.array_equal(t.packet_loss.view(np.uint32), oloss.view(np.uint32))

