"""CPU-only checks of the C ABI library: it loads, exports every declared
symbol, and its host-side GML ingest follows the reference parser."""
import ctypes as C
import os
import re

import numpy as np
import pytest

import shadow_amd
from shadow_amd import NetworkGraph, ShadowGpuError, _capi


def test_library_exports_every_declared_symbol():
    L = shadow_amd.load()  # no GPU call: only dlopen + symbol lookup
    with open(_capi.HEADER_PATH) as f:
        hdr = f.read()
    declared = set(re.findall(r"\b(sg_[a-z0-9_]+)\s*\(", hdr))
    assert declared, "header parse failed"
    assert declared == set(_capi.EXPORTED)
    for name in sorted(declared):
        assert hasattr(L, name), name
    assert L.sg_abi_version() == _capi.SG_ABI_VERSION == 7


def test_missing_library_fails_loudly(tmp_path, monkeypatch):
    monkeypatch.setattr(_capi, "_lib", None)
    with pytest.raises(shadow_amd.ShadowGpuUnavailable):
        _capi.load(str(tmp_path / "nope.so"))
    monkeypatch.setattr(_capi, "_lib", None)
    shadow_amd.load()


THREE = """graph [
  directed {d}
  node [
    id 0
  ]
  node [
    id 1
  ]
  node [
    id 2
  ]
  edge [
    source 0
    target 0
    latency "3333 ns"
  ]
  edge [
    source 1
    target 1
    latency "5555 ns"
  ]
  edge [
    source 2
    target 2
    latency "7777 ns"
  ]
  edge [
    source 0
    target 1
    latency "3 ns"
  ]
  edge [
    source 1
    target 0
    latency "5 ns"
  ]
  edge [
    source 0
    target 2
    latency "7 ns"
  ]
  edge [
    source 2
    target 1
    latency "11 ns"
  ]
]"""


def test_parse_reference_three_node_graph():
    for d in (0, 1):
        g = NetworkGraph.parse(THREE.format(d=d))
        assert g.n_nodes == 3 and g.directed == bool(d)
        assert g.edge_latency_ns.tolist() == [3333, 5555, 7777, 3, 5, 7, 11]
        assert g.edge_packet_loss.tolist() == [0.0] * 7
        assert [g.node_id_to_index(i) for i in range(3)] == [0, 1, 2]


def test_parse_one_gbit_switch():
    text = """graph [
  directed 0
  node [
    id 0
    host_bandwidth_up "1 Gbit"
    host_bandwidth_down "1 Gbit"
  ]
  edge [
    source 0
    target 0
    latency "1 ms"
    packet_loss 0.0
  ]
]"""
    g = NetworkGraph.parse(text)
    assert g.edge_latency_ns.tolist() == [1_000_000] and g.edge_packet_loss.tolist() == [0.0]


def test_nonexistent_id():
    """graph/mod.rs:535-561 test_nonexistent_id."""
    for tid in (2, 3):
        text = f"""graph [
                node [
                  id 1
                ]
                node [
                  id 3
                ]
                edge [
                  source 1
                  target {tid}
                  latency "1 ns"
                ]
            ]"""
        if tid == 3:
            NetworkGraph.parse(text)
        else:
            with pytest.raises(ShadowGpuError) as e:
                NetworkGraph.parse(text)
            assert "doesn't exist" in str(e.value)


def _edge_graph(body):
    return "graph [\n  node [\n    id 0\n  ]\n  edge [\n    source 0\n    target 0\n" + body + "  ]\n]"


@pytest.mark.parametrize("body,ns", [
    ('    latency "5"\n', 5_000_000_000),          # no unit -> seconds (units.rs:227-231)
    ('    latency "7 us"\n', 7_000),
    ('    latency "7 μs"\n', 7_000),
    ('    latency "2 min"\n', 120_000_000_000),
    ('    latency "+3 ms"\n', 3_000_000),
    ('    latency "1 h"\n    jitter "2 ms"\n', 3_600_000_000_000),
])
def test_latency_units(body, ns):
    assert NetworkGraph.parse(_edge_graph(body)).edge_latency_ns.tolist() == [ns]


@pytest.mark.parametrize("body,msg", [
    ('    latency "0 ms"\n', "must not be 0"),
    ('    latency "1.5 ms"\n', "not a valid unit"),
    ('    latency "-1 ms"\n', "not a valid unit"),
    ('    latency "3 fortnights"\n', "not a valid unit"),
    ('    latency 5\n', "not a string"),
    ('    packet_loss 0.1\n', "'latency' was not provided"),
    ('    latency "1 ms"\n    packet_loss 0\n', "not a float"),   # Int tried before Float
    ('    latency "1 ms"\n    packet_loss 1.5\n', "range [0,1]"),
    ('    latency "1 ms"\n    packet_loss -0.5\n', "range [0,1]"),
    ('    latency "99999999999999 h"\n', "outside of the bounds"),
])
def test_edge_errors(body, msg):
    with pytest.raises(ShadowGpuError) as e:
        NetworkGraph.parse(_edge_graph(body))
    assert msg in str(e.value)


def test_loss_is_correctly_rounded_f32():
    for s in ("0.1", "0.25", "1e-3", "0.30000001192092896", ".5", "1.0"):
        g = NetworkGraph.parse(_edge_graph(f'    latency "1 ms"\n    packet_loss {s}\n'))
        assert g.edge_packet_loss[0] == np.float32(float(s))


def test_duplicate_node_id_remaps_to_later_node():
    text = "graph [\n  node [\n    id 4\n  ]\n  node [\n    id 4\n  ]\n]"
    g = NetworkGraph.parse(text)
    assert g.n_nodes == 2 and g.node_id_to_index(4) == 1


def test_parser_structure_errors():
    for text in ("graph [\n  directed 2\n]", "graph [\n  directed 1\n  directed 1\n]",
                 "graph [\n  node [\n    label \"x\"\n  ]\n]", "graph [\n  edge [\n    target 0\n  ]\n]",
                 "grap [\n]", "graph [\n  node [\n    id 0\n    id 1\n  ]\n]"):
        with pytest.raises(ShadowGpuError):
            NetworkGraph.parse(text)


def test_synth_gml_round_trip():
    from shadow_amd import synth

    g = synth.ring_chords_graph(50, 6.0, seed=2, parallel=0.1)
    p = NetworkGraph.parse(synth.graph_to_gml(g))
    assert np.array_equal(p.edge_src, g["src"]) and np.array_equal(p.edge_dst, g["dst"])
    assert np.array_equal(p.edge_latency_ns, g["lat"])
    assert np.array_equal(p.edge_packet_loss.view(np.uint32), g["loss"].view(np.uint32))


def test_ip_assignment_skips_broadcast():
    """graph/mod.rs:653-662 test_increment_address_skip_broadcast."""
    from shadow_amd import IpAssignment, ipv4_to_u32

    a = ipv4_to_u32("11.0.0.254")
    nxt = IpAssignment.increment_address(a)
    assert nxt > a and nxt != ipv4_to_u32("11.0.0.255")
    ipa = IpAssignment()
    ips = [ipa.assign(0) for _ in range(300)]
    assert ips[0] == ipv4_to_u32("11.0.0.1") and all(ip & 0xFF not in (0, 255) for ip in ips)
