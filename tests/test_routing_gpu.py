"""GPU parity: routing-table build (HIP) vs the CPU oracle, bit-exact.

Latency must match exactly (u64 ns) and loss bit-for-bit (f32), for every
used pair, on the reference's own test graphs, the committed golden vectors,
and seeded random graphs.  Errors must match the reference's error cases.
"""
import json
import os
import re

import numpy as np
import pytest

from conftest import APSP_KERNELS, set_apsp_kernel
from shadow_amd import NetworkGraph, ShadowGpuError, _capi, generate_routing_info, synth

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(autouse=True, params=APSP_KERNELS)
def apsp_kernel(request, monkeypatch):
    """Every routing test runs on the default shortest-path kernels (conftest.APSP_KERNELS):
    the per-source LDS-resident search (sg_sssp.hip, the default up to ~10.9k nodes), also in
    its forced bounded-phase form (seed rows, then rows whose keys start at a seed neighbour's
    bounds: the default from 8 rows per CU on), and the batched-source slab relaxation
    (k_relax_w2, dense and larger graphs)."""
    return set_apsp_kernel(monkeypatch, request.param)


def _dense_once(request):
    """Dense graphs take k_sssp_dense under every LDS setting (lds, lds_bounded, lds_flagged, and
    bucket, which takes sparse graphs only): one of them runs it; the slab fixture runs the slab
    kernel."""
    if request.node.callspec.params["apsp_kernel"] in ("lds_bounded", "lds_flagged", "bucket"):
        pytest.skip("the dense-graph search runs under the lds fixture")


def _graph(g, ctx):
    return NetworkGraph(g["n"], g["src"], g["dst"], g["lat"], g["loss"], g["directed"], ctx=ctx)


def _check(oracle, g, used, ctx, shortest=True, rows=None, poison=False):
    """poison: build into device buffers pre-filled with zeros (latency 0, loss 0), so a row
    that is never written, or a bound taken from one, cannot pass by holding an earlier table."""
    net = _graph(g, ctx)
    if rows is None and poison:
        rows = (0, len(used))
    if rows is None:
        t = net.compute_shortest_paths(used) if shortest else net.get_direct_paths(used)
        lat, loss = t.latency_ns, t.packet_loss
    else:
        import torch

        r0, r1 = rows
        nu = len(used)
        dl = torch.zeros((r1 - r0) * nu, dtype=torch.int64, device="cuda")
        df = torch.zeros((r1 - r0) * nu, dtype=torch.float32, device="cuda")
        net.build_rows_device(used, r0, r1, dl.data_ptr(), df.data_ptr(), shortest)
        lat = dl.cpu().numpy().view(np.uint64).reshape(r1 - r0, nu)
        loss = df.cpu().numpy().reshape(r1 - r0, nu)
    fn = oracle.shortest_paths if shortest else oracle.direct_paths
    kw = dict(rows=rows, threads=8) if shortest else {}
    rc, olat, oloss, _ = fn(g["n"], g["src"], g["dst"], g["lat"], g["loss"], g["directed"], used, **kw)
    assert rc == 0
    assert np.array_equal(lat, olat)
    assert np.array_equal(loss.view(np.uint32), oloss.view(np.uint32))
    return lat, loss


def test_reference_test_shortest_path(ctx):
    """graph/mod.rs:564-651, through the GML parser like the reference test."""
    from test_capi_cpu import THREE

    k = json.load(open(os.path.join(GOLD, "reference_kat.json")))["test_shortest_path"]
    for d in (1, 0):
        graph = NetworkGraph.parse(THREE.format(d=d), ctx=ctx)
        n0, n1, n2 = (graph.node_id_to_index(i) for i in range(3))
        paths = graph.compute_shortest_paths([n0, n1, n2])
        lookup = lambda a, b: paths[(a, b)].latency_ns
        want = k["directed_latency" if d else "undirected_latency"]
        got = [[lookup(a, b) for b in (n0, n1, n2)] for a in (n0, n1, n2)]
        assert got == want
        assert len(paths) == 9


def test_one_gbit_switch(ctx):
    from test_capi_cpu import test_parse_one_gbit_switch  # noqa: F401

    text = 'graph [\n  directed 0\n  node [\n    id 0\n  ]\n  edge [\n    source 0\n    target 0\n    latency "1 ms"\n    packet_loss 0.0\n  ]\n]'
    g = NetworkGraph.parse(text, ctx=ctx)
    for fn in (g.compute_shortest_paths, g.get_direct_paths):
        p = fn([0])[(0, 0)]
        assert p.latency_ns == 1_000_000 and p.packet_loss == 0.0
    r = generate_routing_info(g, {0}, True)
    assert r.path(0, 0).latency_ns == 1_000_000 and r.get_smallest_latency_ns() == 1_000_000


def test_golden_vectors(ctx):
    z = np.load(os.path.join(GOLD, "routing_small.npz"))
    for name in sorted({k.split(".")[0] for k in z.files}):
        g = dict(n=int(z[f"{name}.n"][0]), src=z[f"{name}.src"], dst=z[f"{name}.dst"], lat=z[f"{name}.lat"],
                 loss=z[f"{name}.loss"], directed=bool(z[f"{name}.directed"][0]))
        t = _graph(g, ctx).compute_shortest_paths(z[f"{name}.used"])
        assert np.array_equal(t.latency_ns, z[f"{name}.out_lat"]), name
        assert np.array_equal(t.packet_loss.view(np.uint32), z[f"{name}.out_loss"].view(np.uint32)), name


@pytest.mark.parametrize("directed", [False, True])
@pytest.mark.parametrize("seed", [1, 2])
def test_random_sparse(oracle, ctx, directed, seed):
    g = synth.ring_chords_graph(700, 8.0, seed=seed, directed=directed, parallel=0.05)
    used = np.random.default_rng(seed).permutation(700)[:333].astype(np.uint32)
    _check(oracle, g, used, ctx)


def test_multiple_batch_groups(oracle, ctx, monkeypatch):
    """A tiny slab budget forces several sequential batch groups (and partial XCD groups)."""
    monkeypatch.setenv("SG_APSP_GROUP_MB", "1")
    g = synth.ring_chords_graph(1500, 6.0, seed=13)
    used = np.random.default_rng(13).permutation(1500)[:700].astype(np.uint32)
    _check(oracle, g, used, ctx)


def test_complete_graph(oracle, ctx):
    g = synth.complete_graph(300, seed=3)
    _check(oracle, g, np.arange(300, dtype=np.uint32), ctx)


def test_heavy_loss_ties(oracle, ctx):
    """Many equal-latency paths: the loss tie-break decides (graph/mod.rs:305-313)."""
    g = synth.ring_chords_graph(400, 10.0, seed=9)
    rng = np.random.default_rng(4)
    g["lat"] = (rng.integers(1, 4, len(g["lat"])) * 1000).astype(np.uint64)
    g["loss"] = rng.uniform(0, 0.4, len(g["lat"])).astype(np.float32)
    g["loss"][rng.random(len(g["loss"])) < 0.1] = np.float32(1.0)
    _check(oracle, g, np.arange(400, dtype=np.uint32), ctx)


@pytest.mark.parametrize("directed", [False, True])
@pytest.mark.parametrize("bounds", ["1", "4"])
def test_exact_seeds_with_ties(oracle, ctx, monkeypatch, directed, bounds):
    """Bound rows reached over zero-loss arcs seed exact keys (sg_sssp.hip "Exact seeds"): many
    equal-latency paths, lossy arcs beside zero-loss ones, every node used so the seeds apply."""
    monkeypatch.setenv("SG_SSSP_BOUNDS", bounds)
    g = synth.ring_chords_graph(600, 8.0, seed=21, directed=directed)
    rng = np.random.default_rng(21)
    g["lat"] = (rng.integers(1, 5, len(g["lat"])) * 1000).astype(np.uint64)
    loss = rng.uniform(0, 0.3, len(g["lat"])).astype(np.float32)
    loss[rng.random(len(loss)) < 0.6] = 0
    g["loss"] = loss
    _check(oracle, g, np.arange(600, dtype=np.uint32), ctx)


@pytest.mark.parametrize("persist", ["0", "1"])
def test_lds_persistent_and_per_row_workgroups(oracle, ctx, monkeypatch, persist, apsp_kernel):
    """More rows than CUs: the LDS search's persistent workgroups (the default, rows
    claimed from a counter) and one workgroup per row (SG_SSSP_PERSIST=0) give the same
    table."""
    if apsp_kernel in ("slab", "bucket"):
        pytest.skip("LDS knob")
    monkeypatch.setenv("SG_SSSP_PERSIST", persist)
    g = synth.ring_chords_graph(900, 7.0, seed=31, directed=True)
    _check(oracle, g, np.arange(900, dtype=np.uint32), ctx)


@pytest.mark.parametrize("persist", ["0", "1"])
@pytest.mark.parametrize("spin", ["1", "40"])
def test_lds_give_up_takes_wide_kernel(oracle, ctx, monkeypatch, persist, spin, apsp_kernel):
    """The LDS search's safety valve: with a spin budget of 1 or 40 idle polls (SG_SSSP_SPIN_MAX),
    searches give up; the whole workgroup then leaves the kernel, the row is flagged, and the wide
    kernel redoes it.  The table must still be exact, and a persistent workgroup that gave up must
    not leave state behind for the rows other workgroups go on to claim.  When every persistent
    workgroup has given up, the rows none claimed are flagged too (sg_sssp.hip wave_exit); with
    phases (lds_bounded) a later row takes no bounds from a row that gave up (it was never
    written).  The output buffer starts poisoned with zeros, so neither can pass by accident."""
    if apsp_kernel == "slab":
        pytest.skip("LDS knob")
    monkeypatch.setenv("SG_SSSP_PERSIST", persist)
    monkeypatch.setenv("SG_SSSP_SPIN_MAX", spin)
    g = synth.ring_chords_graph(700, 6.0, seed=33)
    _check(oracle, g, np.arange(700, dtype=np.uint32), ctx, poison=True)


def test_exact_seeds_next_to_wide_rows(oracle, ctx, monkeypatch):
    """Rows past 2^32 ns go to the wide kernel after the phases; a later row bounded by such a row
    must take bounds only from it (its 32-bit row is not final everywhere)."""
    monkeypatch.setenv("SG_SSSP_BOUNDS", "4")
    g = synth.ring_chords_graph(300, 6.0, seed=22, directed=True)
    far = np.isin(g["src"], np.arange(0, 300, 23))  # every out-arc of 13 nodes is 5 s long
    g["lat"][far] = np.uint64(5_000_000_000)
    lat, _ = _check(oracle, g, np.arange(300, dtype=np.uint32), ctx)
    assert lat.max() >= (1 << 32) and np.median(lat) < (1 << 32)


def test_wide_fallback_big_latencies(oracle, ctx):
    """Path latencies beyond 2^32 ns take the u64 kernel; must still be exact."""
    g = synth.ring_chords_graph(150, 4.0, seed=8, lat_lo_us=2_000_000, lat_hi_us=9_000_000)
    lat, _ = _check(oracle, g, np.arange(150, dtype=np.uint32), ctx)
    assert lat.max() >= (1 << 34)


def test_huge_edge_latency(oracle, ctx):
    g = synth.ring_chords_graph(60, 4.0, seed=10)
    g["lat"][70] = np.uint64(1) << np.uint64(62)
    _check(oracle, g, np.arange(60, dtype=np.uint32), ctx)


def test_row_shards_concatenate(oracle, ctx):
    g = synth.ring_chords_graph(500, 6.0, seed=12)
    used = np.arange(0, 500, 2, dtype=np.uint32)
    full, _ = _check(oracle, g, used, ctx)
    parts = [_check(oracle, g, used, ctx, rows=(a, b))[0] for a, b in ((0, 70), (70, 71), (71, 250))]
    assert np.array_equal(np.concatenate(parts), full)


def test_direct_paths(oracle, ctx):
    g = synth.complete_graph(120, seed=5)
    _check(oracle, g, np.random.default_rng(0).permutation(120).astype(np.uint32), ctx, shortest=False)
    gd = synth.complete_graph(40, seed=6)
    # a directed complete graph needs both directions
    gd2 = dict(n=40, src=np.concatenate([gd["src"], gd["dst"][40:]]), dst=np.concatenate([gd["dst"], gd["src"][40:]]),
               lat=np.concatenate([gd["lat"], gd["lat"][40:] + 1]), loss=np.concatenate([gd["loss"], gd["loss"][40:]]),
               directed=True)
    _check(oracle, gd2, np.arange(40, dtype=np.uint32), ctx, shortest=False)


def test_errors_match_reference(oracle, ctx):
    cases = [  # (n, src, dst, directed, used, shortest, code, pair)
        (2, [0, 0], [0, 1], False, [0, 1], True, _capi.SG_ERR_NO_EDGE, (1, 1)),
        (2, [0, 0, 1, 0], [0, 0, 1, 1], False, [0, 1], True, _capi.SG_ERR_MULTI_EDGE, (0, 0)),
        (2, [0, 1, 0], [0, 1, 1], True, [0, 1], True, _capi.SG_ERR_UNREACHABLE, (1, 0)),
        (2, [0, 1], [0, 1], False, [0, 1], False, _capi.SG_ERR_NO_EDGE, (0, 1)),
        (2, [0, 1, 0, 1], [0, 1, 1, 0], False, [0, 1], False, _capi.SG_ERR_MULTI_EDGE, (0, 1)),
    ]
    for n, s, d, directed, used, shortest, code, pair in cases:
        m = len(s)
        net = NetworkGraph(n, s, d, [5] * m, [0.0] * m, directed, ctx=ctx)
        with pytest.raises(ShadowGpuError) as e:
            (net.compute_shortest_paths if shortest else net.get_direct_paths)(used)
        assert e.value.code == code and e.value.pair == pair, (e.value.code, e.value.pair, str(e.value))
    # messages name GML ids like the reference
    text = 'graph [\n  node [\n    id 7\n  ]\n  node [\n    id 9\n  ]\n  edge [\n    source 7\n    target 9\n    latency "1 ms"\n  ]\n  edge [\n    source 7\n    target 7\n    latency "1 ms"\n  ]\n]'
    g = NetworkGraph.parse(text, ctx=ctx)
    with pytest.raises(ShadowGpuError, match="No edge connecting node 9 to 9"):
        g.compute_shortest_paths([0, 1])
    # unused isolated node is fine
    net = NetworkGraph(3, [0, 1, 0, 2], [0, 1, 1, 2], [5] * 4, [0.0] * 4, False, ctx=ctx)
    assert net.compute_shortest_paths([0, 1])[(0, 1)].latency_ns == 5


def test_edge_array_validation(oracle, ctx):
    """sg_net_create's checks of edge arrays (graph/mod.rs:101-107 restated for the array
    boundary): the first bad edge in edge order names the error, whichever rule it breaks;
    the endpoint rule is checked before the upload, loss and latency while it runs."""
    base = dict(n=4, src=[0, 1, 2, 3, 0, 1], dst=[0, 1, 2, 3, 1, 2], lat=[5] * 6, loss=[0.0] * 6)
    cases = [
        (dict(loss=[0.0, 0.0, 1.5, 0.0, 0.0, 0.0], dst=[0, 1, 2, 3, 9, 2]), "range [0,1]"),  # loss at 2 before range at 4
        (dict(dst=[0, 1, 2, 9, 1, 2], lat=[5, 5, 5, 5, 0, 5]), "endpoint out of range"),
        (dict(lat=[5, 5, 5, 5, 0, 5]), "must not be 0"),
        (dict(loss=[0.0, 0.0, 0.0, float("nan"), 0.0, 0.0]), "range [0,1]"),
        (dict(loss=[0.0, -0.5, 0.0, 0.0, 0.0, 0.0]), "range [0,1]"),
    ]
    for over, msg in cases:
        a = dict(base, **over)
        with pytest.raises(ShadowGpuError, match=re.escape(msg)):
            NetworkGraph(a["n"], a["src"], a["dst"], a["lat"], np.array(a["loss"], np.float32), False,
                         ctx=ctx).compute_shortest_paths([0, 1, 2, 3])
        # the context stays usable: a valid graph right after a rejected one
        _check(oracle, {"n": 4, "src": np.array(base["src"], np.uint32), "dst": np.array(base["dst"], np.uint32),
                        "lat": np.array(base["lat"], np.uint64), "loss": np.array(base["loss"], np.float32),
                        "directed": False}, np.array([0, 1, 2], np.uint32), ctx)
    # -0.0 is in [0, 1] (a float compare, as the reference's)
    g = NetworkGraph(2, [0, 1, 0], [0, 1, 1], [5, 5, 5], np.array([0.0, 0.0, -0.0], np.float32), False, ctx=ctx)
    assert g.compute_shortest_paths([0, 1])[(0, 1)].latency_ns == 5


@pytest.mark.parametrize("threads", ["1", "4"])
def test_edge_array_validation_threaded(oracle, ctx, monkeypatch, request, threads):
    """Edge lists of 2^18 edges and more are checked and staged by up to 4 host threads
    (sg_routing.hip build_net): the first bad edge in edge order still names the error when
    bad edges sit in several threads' ranges, and a valid graph builds the oracle's table."""
    if request.node.callspec.params["apsp_kernel"] != "lds":
        pytest.skip("host-side upload: runs once, under the lds fixture")
    monkeypatch.setenv("SG_NET_THREADS", threads)
    rng = np.random.default_rng(11)
    n, m = 1500, 300_001
    src = rng.integers(0, n, m).astype(np.uint32)
    dst = ((src + 1 + rng.integers(0, n - 1, m)) % n).astype(np.uint32)  # no self-loop ...
    src[:n], dst[:n] = np.arange(n), np.arange(n)  # ... but one per node
    lat = rng.integers(1, 300_000_000, m).astype(np.uint64)
    loss = np.where(rng.random(m) < 0.8, 0.0, rng.random(m) * 0.02).astype(np.float32)
    g = {"n": n, "src": src, "dst": dst, "lat": lat, "loss": loss, "directed": False}
    _check(oracle, g, np.arange(0, n, 37, dtype=np.uint32), ctx)
    cases = [  # (edge, field, value) in edge order; the error of the first one is raised
        ([(290_000, "dst", n + 5), (80_000, "loss", 2.0), (150_000, "lat", 0)], "range [0,1]"),
        ([(250_000, "lat", 0), (140_000, "src", n), (299_999, "loss", -1.0)], "endpoint out of range"),
        ([(299_999, "lat", 0), (220_000, "loss", float("nan"))], "range [0,1]"),
        ([(300_000, "lat", 0)], "must not be 0"),
    ]
    for bad, msg in cases:
        a = {k: (v.copy() if isinstance(v, np.ndarray) else v) for k, v in g.items()}
        for e, field, value in bad:
            a[field][e] = value
        with pytest.raises(ShadowGpuError, match=re.escape(msg)):
            _graph(a, ctx).compute_shortest_paths([0, 1])


def test_min_latency_device(ctx):
    import torch

    x = torch.tensor([9, 7, 11, 3 << 40], dtype=torch.int64, device="cuda")
    g = NetworkGraph(1, [0], [0], [1], [0.0], False, ctx=ctx)
    assert g.min_latency_device(x.data_ptr(), 4) == 7
    assert g.min_latency_device(x.data_ptr(), 0) == (1 << 64) - 1


def test_bad_node_lists(ctx):
    """sg_routing_build's node-list check: the first bad entry names the error (an index out
    of range, or a node listed twice), and the context stays usable."""
    g = NetworkGraph(4, [0, 1, 2, 3, 0, 1, 2], [0, 1, 2, 3, 1, 2, 3], [5] * 7, [0.0] * 7, False, ctx=ctx)
    for used, msg in (([0, 9, 0], "node index out of range"), ([0, 1, 0, 9], "duplicate node in node list"),
                      ([3, 2, 1, 0, 3], "duplicate node in node list"), ([4], "node index out of range")):
        with pytest.raises(ShadowGpuError, match=re.escape(msg)):
            g.compute_shortest_paths(np.array(used, np.uint32))
    assert g.compute_shortest_paths([3, 0])[(3, 0)].latency_ns == 15


def test_empty_used(ctx):
    g = NetworkGraph(2, [0, 1], [0, 1], [1, 1], [0.0, 0.0], False, ctx=ctx)
    assert len(g.compute_shortest_paths([])) == 0


@pytest.mark.parametrize("env", [{"SG_APSP_B": "32"}, {"SG_APSP_B": "32", "SG_APSP_NPW": "8"},
                                 {"SG_APSP_B": "32", "SG_APSP_SPL": "1"}, {"SG_APSP_FRONTIER": "0"}, {"SG_APSP_SPL": "1"},
                                 {"SG_APSP_SPL": "1", "SG_APSP_NPW": "16"}, {"SG_APSP_SPL": "1", "SG_APSP_FRONTIER": "0"},
                                 {"SG_APSP_NPW": "8", "SG_APSP_STAGE": "128", "SG_APSP_GROUP": "8"},
                                 {"SG_APSP_NPW": "16", "SG_APSP_STAGE": "128", "SG_APSP_GROUP": "4"},
                                 {"SG_APSP_B": "32", "SG_APSP_SPL": "1", "SG_APSP_NPW": "16"}, {"SG_APSP_PASS_CHUNK": "1"},
                                 {"SG_APSP_OUT_TPB": "1"}, {"SG_APSP_OUT_TPB": "4"},
                                 {"SG_APSP_OUT_TPB": "4", "SG_APSP_B": "32"}, {"SG_APSP_SEG": "3"},
                                 {"SG_APSP_SEG": "4", "SG_APSP_B": "32"}, {"SG_APSP_SEG": "16", "SG_APSP_PASS_CHUNK": "1"}])
def test_kernel_variants_bit_exact(oracle, ctx, monkeypatch, env, apsp_kernel):
    """Every A/B variant of the slab relaxation kernel (slab width, frontier, item size) is exact."""
    if apsp_kernel in ("lds", "bucket"):
        pytest.skip("slab-kernel knobs")
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    g = synth.ring_chords_graph(900, 7.0, seed=21, parallel=0.03)
    used = np.random.default_rng(21).permutation(900)[:612].astype(np.uint32)
    _check(oracle, g, used, ctx)


@pytest.mark.parametrize("nseg", ["2", "5"])
def test_arc_segments_directed_dense(oracle, ctx, monkeypatch, nseg, apsp_kernel, request):
    """Arc segments (atomic-min flush) on a directed, nearly complete graph with
    parallel arcs, used-subset rows (the LDS search: a dense directed graph)."""
    _dense_once(request)
    if apsp_kernel == "lds" and nseg != "2":
        pytest.skip("one LDS run is enough")
    monkeypatch.setenv("SG_APSP_SEG", nseg)
    g = synth.complete_graph(160, seed=11)
    rng = np.random.default_rng(11)
    extra = rng.integers(0, 160, (4000, 2)).astype(np.uint32)
    extra = extra[extra[:, 0] != extra[:, 1]]
    gd = dict(n=160, directed=True,
              src=np.concatenate([g["src"], g["dst"][160:], extra[:, 0]]),
              dst=np.concatenate([g["dst"], g["src"][160:], extra[:, 1]]),
              lat=np.concatenate([g["lat"], g["lat"][160:][::-1], rng.integers(1, 400, len(extra)).astype(np.uint64) * 10**6]),
              loss=np.concatenate([g["loss"], g["loss"][160:][::-1], np.full(len(extra), np.float32(0.01))]))
    used = rng.permutation(160)[:131].astype(np.uint32)
    _check(oracle, gd, used, ctx)


def test_c2_scale_from_gml(oracle, ctx, request):
    """C2: a 1,200-node complete undirected graph (about 720k edges)
    parsed from GML text, every node used.  The full shortest-path table is
    bit-exact against the oracle, and so is the direct-path table
    (use_shortest_path: false)."""
    _dense_once(request)
    g = synth.complete_graph(1200, seed=2)  # dense: the relaxation splits chunks into ~9 arc segments
    net = NetworkGraph.parse(synth.graph_to_gml(g), ctx=ctx)
    assert net.n_nodes == 1200 and len(net.edge_src) == len(g["src"])
    used = np.arange(1200, dtype=np.uint32)
    for fn, ofn in ((net.compute_shortest_paths, oracle.shortest_paths), (net.get_direct_paths, oracle.direct_paths)):
        t = fn(used)
        kw = dict(threads=8) if ofn is oracle.shortest_paths else {}
        rc, olat, oloss, _ = ofn(g["n"], g["src"], g["dst"], g["lat"], g["loss"], False, used, **kw)
        assert rc == 0
        assert np.array_equal(t.latency_ns, olat)
        assert np.array_equal(t.packet_loss.view(np.uint32), oloss.view(np.uint32))


def test_c5_scale_row_samples(oracle, ctx):
    """C5 scale: a 50k-node ring + chords graph, mean degree 8, all
    nodes used.  Row blocks at the start, middle and end of the table, bit-exact
    against the oracle's Dijkstra rows."""
    g = synth.ring_chords_graph(50000, 8.0, seed=5)
    used = np.arange(50000, dtype=np.uint32)
    for rows in ((0, 128), (25000, 25064), (49936, 50000)):
        _check(oracle, g, used, ctx, rows=rows)


@pytest.fixture(scope="module")
def c3_oracle(oracle):
    g = synth.ring_chords_graph(10000, 8.0, seed=1)
    used = np.arange(10000, dtype=np.uint32)
    rc, olat, oloss, _ = oracle.shortest_paths(g["n"], g["src"], g["dst"], g["lat"], g["loss"], False, used,
                                               threads=min(16, os.cpu_count() or 1))
    assert rc == 0
    return g, used, olat, oloss


def test_c3_full_table(c3_oracle, ctx):
    """The headline C3 build (bench.py `value`): the 10k-node ring + chords graph,
    all 10^8 (latency, loss) cells bit-exact against the oracle's Dijkstra."""
    g, used, olat, oloss = c3_oracle
    _check_full(g, used, olat, oloss, ctx)


def test_c3_row_blocks(c3_oracle, ctx, apsp_kernel):
    """The row blocks one rank builds in a sharded C3 build (bench.py at N = 2, 4, 8): their
    own phase plans (3, 2 and no phases by rows per CU, bounds only from rows in the block),
    every cell against the oracle's rows."""
    import torch

    if apsp_kernel == "slab":
        pytest.skip("the slab kernel's row blocks are covered by test_row_shards_concatenate")
    g, used, olat, oloss = c3_oracle
    net = _graph(g, ctx)
    n = len(used)
    for r0, r1 in ((5000, 10000), (2500, 5000), (8750, 10000)):
        dl = torch.empty((r1 - r0) * n, dtype=torch.int64, device="cuda")
        df = torch.empty((r1 - r0) * n, dtype=torch.float32, device="cuda")
        net.build_rows_device(used, r0, r1, dl.data_ptr(), df.data_ptr(), True)
        assert np.array_equal(dl.cpu().numpy().view(np.uint64).reshape(r1 - r0, n), olat[r0:r1]), (r0, r1)
        assert np.array_equal(df.cpu().numpy().view(np.uint32).reshape(r1 - r0, n), oloss[r0:r1].view(np.uint32))


def _check_full(g, used, olat, oloss, ctx):
    import torch

    net = _graph(g, ctx)
    n = len(used)
    dl = torch.empty(n * n, dtype=torch.int64, device="cuda")
    df = torch.empty(n * n, dtype=torch.float32, device="cuda")
    net.build_rows_device(used, 0, n, dl.data_ptr(), df.data_ptr(), True)
    lat = dl.cpu().numpy().view(np.uint64).reshape(n, n)
    bad = np.argwhere(lat != olat)
    assert len(bad) == 0, f"{len(bad)} latency cells differ, first {bad[:3].tolist()}"
    loss = df.cpu().numpy().view(np.uint32).reshape(n, n)
    bad = np.argwhere(loss != oloss.view(np.uint32))
    assert len(bad) == 0, f"{len(bad)} loss cells differ, first {bad[:3].tolist()}"


@pytest.mark.parametrize("delta", ["1", "1000", "3000000", "40000000", "4000000000"])
def test_lds_bucket_widths(oracle, ctx, monkeypatch, delta, apsp_kernel):
    """The LDS search's bucket width changes the relaxation order only: from
    1 ns (Dijkstra-like, many buckets) to 4 s (one bucket, chaotic Bellman-Ford),
    on a tie-heavy lossy graph, directed and undirected."""
    if apsp_kernel in ("slab", "bucket"):
        pytest.skip("LDS knob")
    monkeypatch.setenv("SG_APSP_DELTA", delta)
    for directed in (False, True):
        g = synth.ring_chords_graph(700, 6.0, seed=31, directed=directed, parallel=0.05)
        g["lat"] = (g["lat"] // 10**7 + 1) * 10**7  # coarse latencies: many equal-latency paths
        g["loss"] = np.where(np.arange(len(g["loss"])) % 3 == 0, np.float32(0.05), g["loss"]).astype(np.float32)
        used = np.random.default_rng(31).permutation(700)[:500].astype(np.uint32)
        _check(oracle, g, used, ctx)


@pytest.mark.parametrize("n", [10900, 11200])
def test_lds_size_limit(oracle, ctx, n):
    """Node counts just inside and just past the LDS-resident search's limit (the
    second runs on the bucketed search, or the slab kernel under its fixture): sampled
    rows exact."""
    g = synth.ring_chords_graph(n, 8.0, seed=7)
    used = np.arange(n, dtype=np.uint32)
    for rows in ((0, 64), (n - 64, n)):
        _check(oracle, g, used, ctx, rows=rows)


@pytest.mark.parametrize("block_rows", ["64", "1000", "20000"])
def test_routing_info_fill_c3(c3_oracle, ctx, monkeypatch, block_rows, apsp_kernel, request):
    """sg_routing_info_fill: the whole C3 table straight into the dense host
    RoutingInfo, row blocks copied while the next builds (generate_routing_info,
    sim_config.rs:411-448, in a shuffled used-id order as a HashSet yields them)."""
    if request.node.callspec.params["apsp_kernel"] != "lds" and block_rows != "1000":
        pytest.skip("the block sizes on the default kernel; one run of each other kernel")
    monkeypatch.setenv("SG_RI_BLOCK_ROWS", block_rows)
    g, used, olat, oloss = c3_oracle
    net = _graph(g, ctx)
    order = np.random.default_rng(3).permutation(10000)
    ri = generate_routing_info(net, order.tolist(), True)
    assert ri.pinned
    lat, loss = ri.latency_ns, ri.packet_loss
    assert np.array_equal(lat, olat[np.ix_(order, order)])
    assert np.array_equal(loss.view(np.uint32), oloss.view(np.uint32)[np.ix_(order, order)])
    assert ri.get_smallest_latency_ns() == int(olat.min())
    rng = np.random.default_rng(5)
    for a, b in rng.integers(0, 10000, (200, 2)):
        p = ri.path(int(a), int(b))
        assert p.latency_ns == int(olat[a, b]) and np.float32(p.packet_loss).view(np.uint32) == oloss.view(np.uint32)[a, b]


def test_routing_info_direct_and_errors(oracle, ctx):
    """Direct paths into the host RoutingInfo, and a failing build leaves a usable
    error (the reference's Err from get_edge_weight, graph/mod.rs:256-293)."""
    g = synth.complete_graph(90, seed=4)
    net = _graph(g, ctx)
    ri = generate_routing_info(net, range(90), False)
    rc, olat, oloss, _ = oracle.direct_paths(g["n"], g["src"], g["dst"], g["lat"], g["loss"], False,
                                             np.arange(90, dtype=np.uint32))
    assert rc == 0 and np.array_equal(ri.latency_ns, olat)
    assert ri.get_smallest_latency_ns() == int(olat.min())
    # a row rewritten after the fill: the minimum follows it both ways (per-row minima)
    ri.set_rows(7, np.full((1, 90), 3, np.uint64), oloss[7:8])
    assert ri.get_smallest_latency_ns() == 3
    ri.set_rows(7, olat[7:8], oloss[7:8])
    assert ri.get_smallest_latency_ns() == int(olat.min())
    keep = ~((g["src"] == 5) & (g["dst"] == 5))  # node 5 loses its self-loop
    g2 = dict(g, src=g["src"][keep], dst=g["dst"][keep], lat=g["lat"][keep], loss=g["loss"][keep])
    with pytest.raises(ShadowGpuError) as e:
        generate_routing_info(_graph(g2, ctx), range(90), True)
    assert e.value.code == _capi.SG_ERR_NO_EDGE


@pytest.mark.parametrize("split", ["0", "1", "5", "16"])
def test_dense_row_split(oracle, ctx, monkeypatch, split):
    """The dense search's rounds with few settled rows split each row's arcs over several waves
    (sg_dense.hip, SG_DENSE_SPLIT: never, below 1, 5 and 16 rows): a complete graph with coarse
    latencies (ties decided by loss), all rows and a shuffled used subset, and a directed copy with
    three 700-arc hubs whose rows stay unsorted; bit-exact."""
    monkeypatch.setenv("SG_DENSE_SPLIT", split)
    g = synth.complete_graph(300, seed=21)
    g["lat"] = (g["lat"] // 10**7 + 1) * 10**7
    _check(oracle, g, np.arange(300, dtype=np.uint32), ctx)
    _check(oracle, g, np.random.default_rng(21).permutation(300)[:200].astype(np.uint32), ctx)
    # three nodes with 700 parallel out-arcs each (past the sort's 512-arc LDS array at 300 nodes):
    # their rows stay unsorted and are never cut, split or not
    rng = np.random.default_rng(22)
    hub = np.repeat(np.array([3, 150, 299], dtype=g["src"].dtype), 700)
    tail = rng.integers(0, 300, len(hub)).astype(g["dst"].dtype)
    keep = hub != tail
    hub, tail = hub[keep], tail[keep]
    rv = g["src"] != g["dst"]  # the reverse arcs (self-loops once)
    g2 = dict(g, directed=True, src=np.concatenate([g["src"], g["dst"][rv], hub]),
              dst=np.concatenate([g["dst"], g["src"][rv], tail]),
              lat=np.concatenate([g["lat"], g["lat"][rv], rng.integers(10**6, 4 * 10**8, len(hub)).astype(np.uint64)]),
              loss=np.concatenate([g["loss"], g["loss"][rv],
                                   np.where(rng.random(len(hub)) < 0.5, 0.0, 0.01).astype(np.float32)]))
    _check(oracle, g2, np.arange(300, dtype=np.uint32), ctx)


@pytest.mark.parametrize("env", [{}, {"SG_DENSE_RTN": "0"}, {"SG_DENSE_THREADS": "384"},
                                 {"SG_DENSE_SPEC": "0"}, {"SG_DENSE_SW": "4", "SG_DENSE_G": "4"},
                                 {"SG_DENSE_SW": "16", "SG_DENSE_THREADS": "512", "SG_DENSE_SPEC": "0"},
                                 {"SG_DENSE_LAZY": "0"}, {"SG_DENSE_LAZY": "0", "SG_DENSE_SEED": "0"},
                                 {"SG_DENSE_LAZY": "0", "SG_DENSE_SEED": "1"}, {"SG_DENSE_LAZY": "0", "SG_DENSE_SEED": "64"},
                                 {"SG_DENSE_LAZY": "0", "SG_DENSE_SEED": "150", "SG_DENSE_SEED_SW": "64",
                                  "SG_DENSE_SEED_THREADS": "1024"},
                                 {"SG_DENSE_LAZY": "0", "SG_DENSE_SEED": "16,48", "SG_DENSE_SEED_SW": "16"},
                                 {"SG_DENSE_LAZY": "0", "SG_DENSE_SEED": "8,24,100", "SG_DENSE_SEED_SW": "32",
                                  "SG_DENSE_SW": "8", "SG_DENSE_THREADS": "512"}])
def test_dense_search_forms(oracle, ctx, monkeypatch, env, request):
    """The dense search's forms (sg_dense.hip): the lazy search (the default: rows resumed where
    they stopped, whole chunks or cut at the threshold, 4 to 16 lanes per row, 2 or 4 rows in
    flight, 256, 384 or 512 threads, the atomic's returned key or a settled-bit read) and the T-cut search with seed rows (SG_DENSE_LAZY=0,
    SG_DENSE_SEED: a first launch computes the block's first rows, the second starts every row's
    keys at bounds from its nearest seed row).
    A complete graph with coarse latencies (ties decided by loss) on all rows, a shuffled used
    subset and a row block into a zeroed buffer; the directed copy with unsorted 700-arc hubs
    (relaxed whole; a seed row is the first marked arc, not the lightest); latencies past 2^32 ns
    (saturated rows, finished by the wide kernel); the 1,200-node C2 graph; bit-exact every cell.
    The T-cut search under its defaults (one seed launch of n_cu rows from 2 n_cu rows on: the
    300-node cases run unseeded), no seeds, 1 to 150 seed rows, two and three levels."""
    _dense_once(request)
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    g = synth.complete_graph(300, seed=31)
    g["lat"] = (g["lat"] // 10**7 + 1) * 10**7
    g["loss"] = np.where(np.arange(len(g["loss"])) % 4 == 0, np.float32(0.03), g["loss"]).astype(np.float32)
    _check(oracle, g, np.arange(300, dtype=np.uint32), ctx)
    _check(oracle, g, np.random.default_rng(31).permutation(300)[:290].astype(np.uint32), ctx)
    _check(oracle, g, np.arange(300, dtype=np.uint32), ctx, rows=(7, 300), poison=True)
    rng = np.random.default_rng(32)
    hub = np.repeat(np.array([0, 1, 150, 299], dtype=g["src"].dtype), 700)
    tail = rng.integers(0, 300, len(hub)).astype(g["dst"].dtype)
    keep = hub != tail
    hub, tail = hub[keep], tail[keep]
    rv = g["src"] != g["dst"]
    g2 = dict(g, directed=True, src=np.concatenate([g["src"], g["dst"][rv], hub]),
              dst=np.concatenate([g["dst"], g["src"][rv], tail]),
              lat=np.concatenate([g["lat"], g["lat"][rv], rng.integers(10**6, 4 * 10**8, len(hub)).astype(np.uint64)]),
              loss=np.concatenate([g["loss"], g["loss"][rv],
                                   np.where(rng.random(len(hub)) < 0.5, 0.0, 0.01).astype(np.float32)]))
    _check(oracle, g2, np.arange(300, dtype=np.uint32), ctx)
    g3 = dict(g, lat=(rng.integers(1_000_000, 9_000_000, len(g["lat"])) * 1000).astype(np.uint64))
    lat, _ = _check(oracle, g3, np.arange(300, dtype=np.uint32), ctx)
    assert lat.max() >= (1 << 32)
    _check(oracle, synth.complete_graph(1200, seed=2), np.arange(1200, dtype=np.uint32), ctx)


@pytest.mark.parametrize("env", [{}, {"SG_DENSE_SPEC": "0"}, {"SG_DENSE_SW": "4"}, {"SG_DENSE_SW": "16", "SG_DENSE_THREADS": "512"},
                                 {"SG_DENSE_RTN": "0", "SG_DENSE_THREADS": "384"}])
def test_dense_fuzz(oracle, ctx, monkeypatch, env, request):
    """Random dense graphs through the lazy search's forms: 70-400 nodes, 65-220 arcs per node,
    directed or not, latencies wide (1 ns - 100 ms), coarse (ties decided by loss) or tiny (1-9 ns),
    parallel arcs, a few nodes reached over long arcs only, hubs with more arcs than the sort's LDS
    array (unsorted rows), losses of 0, 1 and in between; every cell bit-exact."""
    _dense_once(request)
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    rng = np.random.default_rng(4242)
    for case in range(8):
        n = int(rng.integers(70, 400))
        deg = float(rng.integers(65, 220))
        directed = bool(case % 2)
        m = int(n * deg / (1 if directed else 2))
        src, dst = rng.integers(0, n, m), rng.integers(0, n, m)
        if case % 4 == 3:  # hubs past the sort's array: 1.5 n arcs each
            hub = rng.choice(n, 3, replace=False)
            src = np.r_[src, np.repeat(hub, int(1.5 * n))]
            dst = np.r_[dst, rng.integers(0, n, 3 * int(1.5 * n))]
        keep = src != dst
        src, dst = src[keep], dst[keep]
        kind = case % 3
        if kind == 0:
            lat = rng.integers(1, 10**8, len(src))
        elif kind == 1:
            lat = rng.integers(1, 6, len(src)) * 10**6
        else:
            lat = rng.integers(1, 10, len(src))
        if case in (2, 5):  # the last 5 nodes reached over long arcs only
            lat = np.where(dst >= n - 5, rng.integers(10**8, 2 * 10**8, len(src)), lat)
        loss = rng.choice(np.array([0.0, 0.0, 0.01, 0.3, 1.0], np.float32), len(src))
        src = np.r_[src, np.arange(n)].astype(np.uint32)  # one self-loop per node
        dst = np.r_[dst, np.arange(n)].astype(np.uint32)
        lat = np.r_[lat, np.full(n, 1000)].astype(np.uint64)
        loss = np.r_[loss, np.zeros(n, np.float32)].astype(np.float32)
        g = dict(n=n, src=src, dst=dst, lat=lat, loss=loss, directed=directed)
        if not directed:
            assert 2 * (len(src) - n) > 64 * n
        else:
            assert len(src) - n > 64 * n
        _check(oracle, g, np.arange(n, dtype=np.uint32), ctx)


def test_dense_at_size_limit(oracle, ctx, request):
    """The dense search at its size limit (DENSE_MAX = 4,096 nodes: 96 KB of LDS per row, one row
    per CU) on a 140-arcs-per-node graph with coarse latencies (ties by loss): the whole table,
    and a row block of a shuffled used subset into a zeroed buffer; bit-exact."""
    _dense_once(request)
    g = synth.ring_chords_graph(4096, 140.0, seed=77)
    g["lat"] = (g["lat"] // 10**6 + 1) * 10**6
    assert len(g["src"]) * 2 > 64 * 4096  # dense: more than 64 arcs per node
    _check(oracle, g, np.arange(4096, dtype=np.uint32), ctx)
    used = np.random.default_rng(77).permutation(4096)[:3000].astype(np.uint32)
    _check(oracle, g, used, ctx, rows=(500, 2600), poison=True)


@pytest.mark.parametrize("case", ["ties", "wide", "parallel_directed", "used_subset", "tiny_wmin",
                                  "far_tiny_wmin"])
def test_dense_graph_cases(oracle, ctx, case, request):
    """Dense graphs (mean out-degree past 64: the register-resident search of sg_dense.hip under
    the LDS fixtures, the slab under `slab`): equal-latency paths decided by loss, latencies past
    2^32 ns (wide rows), parallel arcs in a directed graph, a used-node subset with rows and
    columns in a shuffled order, 1-ns arcs (one-node rounds), and a directed graph with a 1-ns
    smallest arc and latencies spread to 1 ms whose last 40 nodes are reached over 100-200 ms arcs
    only: the lazy search's rounds with every reached key settled and the far nodes not yet reached
    (a relaxation budget that doubles; stepping by w_min took one round per distinct candidate
    value)."""
    _dense_once(request)
    rng = np.random.default_rng(sum(map(ord, case)))
    n = 520
    if case == "parallel_directed":
        g = synth.ring_chords_graph(n, 150.0, seed=5, directed=True, parallel=0.2)
    elif case == "far_tiny_wmin":
        m = 100 * n
        src, dst = rng.integers(0, n, m), rng.integers(0, n, m)
        keep = src != dst
        src, dst = src[keep], dst[keep]
        lat = rng.integers(1, 10**6, len(src)).astype(np.uint64)
        lat[0] = 1
        far = dst >= n - 40  # the last 40 nodes are reached over 100-200 ms arcs only
        lat[far] = rng.integers(10**8, 2 * 10**8, int(far.sum()))
        src = np.concatenate([src, np.arange(n)]).astype(np.uint32)  # + one self-loop each
        dst = np.concatenate([dst, np.arange(n)]).astype(np.uint32)
        lat = np.concatenate([lat, np.full(n, 10**6, np.uint64)])
        loss = np.where(rng.random(len(src)) < 0.5, 0.0, 0.01).astype(np.float32)
        g = dict(n=n, src=src, dst=dst, lat=lat, loss=loss, directed=True)
    else:
        g = synth.ring_chords_graph(n, 180.0, seed=6)
    if case == "ties":
        g["lat"] = (rng.integers(1, 4, len(g["lat"])) * 1000).astype(np.uint64)
        g["loss"] = rng.uniform(0, 0.4, len(g["lat"])).astype(np.float32)
        g["loss"][rng.random(len(g["loss"])) < 0.1] = np.float32(1.0)
    if case == "wide":
        g["lat"] = (rng.integers(1_000_000, 9_000_000, len(g["lat"])) * 1000).astype(np.uint64)
    if case == "tiny_wmin":
        g["lat"] = rng.integers(1, 40, len(g["lat"])).astype(np.uint64)
    used = np.arange(n, dtype=np.uint32)
    if case == "used_subset":
        used = rng.permutation(n)[:333].astype(np.uint32)
    lat, _ = _check(oracle, g, used, ctx)
    if case == "wide":
        assert lat.max() >= (1 << 32)
    if case == "far_tiny_wmin":
        assert lat[: n - 40, n - 40:].min() >= 10**8


@pytest.mark.parametrize("env", [{"SG_BUCKET_DELTA": "4000000000"}, {"SG_BUCKET_DELTA": "4096"},
                                 {"SG_BUCKET_DELTA": "4194304"}, {"SG_BUCKET_RING": "2"},
                                 {"SG_BUCKET_RING": "4", "SG_BUCKET_DELTA": "262144"},
                                 {"SG_BUCKET_HASH": "6"}, {"SG_BUCKET_CHUNKS": "4"},
                                 {"SG_BUCKET_CHUNKS": "6", "SG_BUCKET_RING": "2"},
                                 {"SG_BUCKET_STAGE": "0"}, {"SG_BUCKET_STAGE": "40", "SG_BUCKET_DELTA": "30000000"},
                                 {"SG_BUCKET_THREADS": "1024"}, {"SG_BUCKET_THREADS": "1024", "SG_BUCKET_DELTA": "30000000"},
                                 {"SG_BUCKET_MODE": "queue"}, {"SG_BUCKET_MODE": "queue", "SG_BUCKET_RING": "2"},
                                 {"SG_BUCKET_MODE": "queue", "SG_BUCKET_HASH": "6"}, {"SG_BAND_NPW": "5"},
                                 {"SG_BAND_NPW": "64", "SG_BUCKET_HASH": "7"}, {"SG_BAND_FILTER": "1"},
                                 {"SG_BAND_FILTER": "1", "SG_BUCKET_DELTA": "4096"},
                                 {"SG_BAND_FILTER": "1", "SG_BUCKET_RING": "2"}])
def test_bucket_search_knobs(oracle, ctx, monkeypatch, env, apsp_kernel):
    """The bucketed search (sg_bucket.hip) under its knobs, on a tie-heavy lossy graph (10-ms arc
    latencies), directed and undirected, a used subset: exact bands (k_sssp_band: the default
    10-ms width, 4-us and 4-ms), bands past the smallest arc (k_sssp_bucket: one band for the
    whole row, chaotic relaxation in the hash; 30-ms bands that relax into themselves through the
    queue; the queue kernel forced at 10 ms), 1024-thread workgroups, rings of 2 and 4 slots (most candidates go to the far lists and come
    back by far steps), entries stored straight to the arena (no LDS staging) or overflowing a
    40-entry staging array, and its safety valves -- a 64-slot hash that fills and arenas of 4 and 6
    chunks that run out: the row gives up, the workgroup leaves, and the wide kernel redoes the
    row (the output starts poisoned, so no row passes by holding an earlier table); and the banded
    search's nodes per wave (5: many steps per band; 64 with band splits); and the banded search's
    append filter (SG_BAND_FILTER, off by default: a candidate later than its node's best appended
    bucket is dropped), with 10-ms and 4-us bands (buckets past the filter's 255-bucket window) and
    a 2-slot ring (far lists)."""
    if apsp_kernel != "bucket":
        pytest.skip("bucketed-search knobs")
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    for directed in (False, True):
        g = synth.ring_chords_graph(700, 6.0, seed=41, directed=directed, parallel=0.05)
        g["lat"] = (g["lat"] // 10**7 + 1) * 10**7  # coarse latencies: many equal-latency paths
        g["loss"] = np.where(np.arange(len(g["loss"])) % 3 == 0, np.float32(0.05), g["loss"]).astype(np.float32)
        used = np.random.default_rng(41).permutation(700)[:500].astype(np.uint32)
        _check(oracle, g, used, ctx, poison=True)


def test_band_degree_classes(oracle, ctx, monkeypatch):
    """The banded search on its degree-class numbering (sg_bucket.hip k_band_classes): nodes of
    every out-degree class -- hubs of degree 30-60 (class 16, whose arc offsets are read), nodes
    of degree 1 .. 15, and isolated unused nodes (degree 0) -- directed and undirected, a used
    subset in shuffled order, two graphs interleaved on one context (the numbering is cached per
    graph) and a row block; every cell against the oracle."""
    monkeypatch.setenv("SG_APSP_LDS", "1")
    monkeypatch.setenv("SG_APSP_BUCKET", "1")
    rng = np.random.default_rng(53)
    graphs = []
    for directed in (False, True):
        g = synth.ring_chords_graph(640, 4.0, seed=53 + directed, directed=directed, parallel=0.05)
        n0 = g["n"]
        hubs = rng.choice(n0, 6, replace=False)
        src, dst = [g["src"]], [g["dst"]]
        for h in hubs:
            k = int(rng.integers(30, 61))
            t = rng.choice(n0, k, replace=False)
            t = t[t != h]
            src.append(np.full(len(t), h, dtype=g["src"].dtype))
            dst.append(t.astype(g["dst"].dtype))
        iso = np.arange(n0, n0 + 10, dtype=g["src"].dtype)  # self-loops only: out-degree 0
        src.append(iso)
        dst.append(iso)
        m = sum(len(x) for x in src) - len(g["src"])
        g = dict(g, n=n0 + 10, src=np.concatenate(src), dst=np.concatenate(dst),
                 lat=np.concatenate([g["lat"], rng.integers(10**6, 9 * 10**7, m).astype(np.uint64)]),
                 loss=np.concatenate([g["loss"], np.where(rng.random(m) < 0.5, 0.0, 0.01).astype(np.float32)]))
        graphs.append(g)
    used = rng.permutation(640)[:500].astype(np.uint32)
    for g in graphs + graphs:
        _check(oracle, g, used, ctx)
    _check(oracle, graphs[0], used, ctx, rows=(100, 260), poison=True)


def test_dense_sorted_arcs_per_graph(oracle, ctx):
    """The dense search sorts a graph's arcs once and reuses them on later builds of the same
    graph (the context's workspace remembers whose arcs it holds): rebuilds with other row ranges
    and used sets, interleaved with a second graph on the same context, all bit-exact."""
    import torch

    ga = synth.complete_graph(300, seed=11)
    gb = synth.complete_graph(260, seed=12)
    na, nb = _graph(ga, ctx), _graph(gb, ctx)
    cases = [(na, ga, np.arange(300, dtype=np.uint32), (0, 300)), (nb, gb, np.arange(260, dtype=np.uint32), (0, 260)),
             (na, ga, np.arange(299, -1, -1, dtype=np.uint32)[::2].copy(), (10, 150)),
             (na, ga, np.arange(300, dtype=np.uint32), (200, 300)), (nb, gb, np.arange(260, dtype=np.uint32), (5, 60))]
    for net, g, used, (r0, r1) in cases:
        nu = len(used)
        dl = torch.zeros((r1 - r0) * nu, dtype=torch.int64, device="cuda")
        df = torch.zeros((r1 - r0) * nu, dtype=torch.float32, device="cuda")
        net.build_rows_device(used, r0, r1, dl.data_ptr(), df.data_ptr(), True)
        rc, olat, oloss, _ = oracle.shortest_paths(g["n"], g["src"], g["dst"], g["lat"], g["loss"], g["directed"],
                                                   used, rows=(r0, r1), threads=8)
        assert rc == 0
        assert np.array_equal(dl.cpu().numpy().view(np.uint64).reshape(r1 - r0, nu), olat)
        assert np.array_equal(df.cpu().numpy().reshape(r1 - r0, nu).view(np.uint32), oloss.view(np.uint32))
