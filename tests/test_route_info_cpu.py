"""CPU checks of the host half of the routing boundary (sg_routing_info,
sg_route_info.hip): the dense RoutingInfo answers RoutingInfo::path,
get_smallest_latency_ns and increment_packet_count (graph/mod.rs:434-481) and the
WorkerShared / worker_* lookups (worker.rs:517-555, 651-684) exactly as a
HashMap<(u32, u32), PathProperties> built from the same table would.  The table
comes from the oracle (no GPU); sg_routing_info_fill is the GPU test's job."""
import numpy as np
import pytest

from shadow_amd import IpAssignment, PathProperties, RoutingInfo, ShadowGpuError, synth


def _table(n=40, seed=3):
    from oracle import oracle as O

    g = synth.ring_chords_graph(n, 5.0, seed=seed)
    rc, lat, loss, _ = O.shortest_paths(n, g["src"], g["dst"], g["lat"], g["loss"], False,
                                        np.arange(n, dtype=np.uint32), threads=2)
    assert rc == 0
    return lat, loss


@pytest.mark.parametrize("ids", ["compact", "sparse"])
def test_path_matches_hashmap(ids):
    lat, loss = _table()
    n = lat.shape[0]
    rng = np.random.default_rng(1)
    node_ids = np.arange(100, 100 + n) if ids == "compact" else rng.choice(10**9, n, replace=False)
    ri = RoutingInfo(node_ids, lat, loss)
    ref = {(int(a), int(b)): PathProperties(int(lat[i, j]), np.float32(loss[i, j]))
           for i, a in enumerate(node_ids) for j, b in enumerate(node_ids)}  # the reference's map
    for (a, b), p in ref.items():
        assert ri.path(a, b) == p
        assert np.float32(ri.path(a, b).packet_loss).view(np.uint32) == np.float32(p.packet_loss).view(np.uint32)
    assert ri.path(int(node_ids[0]), 7) is None and ri.path(7, int(node_ids[0])) is None
    assert ri.get_smallest_latency_ns() == min(p.latency_ns for p in ref.values())
    assert np.array_equal(ri.latency_ns, lat) and np.array_equal(ri.packet_loss.view(np.uint32), loss.view(np.uint32))
    assert ri.index(int(node_ids[5])) == 5 and ri.index(7) is None


def test_duplicate_node_id_rejected():
    with pytest.raises(ShadowGpuError):
        RoutingInfo([3, 4, 3])


def test_empty_table_has_no_smallest_latency():
    assert RoutingInfo([]).get_smallest_latency_ns() is None


def test_packet_counters_saturate_and_reject_unknown_pairs():
    lat, loss = _table(6)
    ri = RoutingInfo(range(6), lat, loss)
    for _ in range(3):
        ri.increment_packet_count(1, 2)
    assert ri.packet_count(1, 2) == 3 and ri.packet_count(2, 1) == 0
    with pytest.raises(KeyError):
        ri.increment_packet_count(1, 99)


def test_worker_lookups_follow_ip_assignment():
    """WorkerShared::latency / reliability / is_routable through IpAssignment::get_node."""
    lat, loss = _table(30)
    loss = loss.copy()
    loss[3, 4] = np.float32(0.3)
    node_ids = list(range(500, 530))
    ri = RoutingInfo(node_ids, lat, loss)
    ipa = IpAssignment()
    host_node = [node_ids[h % 30] for h in range(75)] + [999]  # the last host's node has no routing row
    ips = [ipa.assign(nid) for nid in host_node]
    ri.set_addresses(ips, host_node)
    for _ in range(300):
        a, b = np.random.default_rng(_).integers(0, 75, 2)
        i, j = node_ids.index(host_node[a]), node_ids.index(host_node[b])
        assert ri.latency(ips[a], ips[b]) == int(lat[i, j])
        assert ri.reliability(ips[a], ips[b]).view(np.uint32) == np.float32(np.float32(1.0) - loss[i, j]).view(np.uint32)
        assert ri.is_routable(ips[a], ips[b])
    unknown = ips[-1] + 7
    assert not ri.is_routable(ips[0], unknown) and ri.latency(ips[0], unknown) is None
    assert ri.is_routable(ips[0], ips[-1])  # assigned: routable (the graph is connected) ...
    assert ri.latency(ips[0], ips[-1]) is None  # ... but no path row: None
    with pytest.raises(ShadowGpuError):
        ri.set_addresses([ips[0], ips[0]], [500, 501])


def test_sparse_addresses():
    lat, loss = _table(10)
    ri = RoutingInfo(range(10), lat, loss)
    rng = np.random.default_rng(4)
    ips = (rng.permutation(2**20)[:20].astype(np.uint64) * 4001 + 9).astype(np.uint32)
    nodes = [k % 10 for k in range(20)]
    ri.set_addresses(ips, nodes)
    for k in range(20):
        for m in range(20):
            assert ri.latency(int(ips[k]), int(ips[m])) == int(lat[nodes[k], nodes[m]])


def test_wide_latencies_keep_u64():
    """Paths of 2^32 - 1 ns (4.29 s) or more: the cell says SG_CELL_WIDE and the u64 latency
    lives in the side table; every lookup and the decoded rows give it back exactly."""
    lat, loss = _table(12)
    lat = lat.copy()
    lat[2, 5] = (1 << 40) + 3
    lat[7, 7] = (1 << 32) - 1  # exactly the sentinel value: also kept wide
    lat[11, 0] = (1 << 63) + 17
    ri = RoutingInfo(range(12), lat, loss)
    assert np.array_equal(ri.latency_ns, lat) and np.array_equal(ri.packet_loss.view(np.uint32), loss.view(np.uint32))
    assert ri.path(2, 5).latency_ns == (1 << 40) + 3 and ri.path(7, 7).latency_ns == (1 << 32) - 1
    assert ri.cells[2, 5] >> np.uint64(32) == np.uint64(0xFFFFFFFF)
    lr, _ = ri.rows(7, 12)
    assert np.array_equal(lr, lat[7:12])
    ips = [ipv for ipv in range(0x0B000001, 0x0B000001 + 12)]
    ri.set_addresses(ips, list(range(12)))
    assert ri.latency(ips[11], ips[0]) == (1 << 63) + 17
    # rewriting a row drops its old wide entries
    lat2 = lat.copy()
    lat2[2, 5] = 77
    ri.set_rows(2, lat2[2:3], loss[2:3])
    assert ri.path(2, 5).latency_ns == 77 and ri.path(11, 0).latency_ns == (1 << 63) + 17


def test_smallest_latency_needs_every_row():
    """get_smallest_latency_ns is over the whole table (graph/mod.rs:478-480): None until every
    row is set, and recomputed when rows are rewritten with larger values."""
    lat, loss = _table(8)
    ri = RoutingInfo(range(8))
    ri.set_rows(0, lat[:4], loss[:4])
    assert ri.get_smallest_latency_ns() is None
    ri.set_rows(4, lat[4:], loss[4:])
    assert ri.get_smallest_latency_ns() == int(lat.min())
    big = np.full_like(lat, 10**12)
    ri.set_rows(0, big, loss)
    assert ri.get_smallest_latency_ns() == 10**12


def test_smallest_latency_after_many_row_rewrites():
    """A row rewritten hundreds of times (the per-row written flag must not wrap) keeps the
    whole-table minimum current; each rewrite updates its own row's minimum only."""
    lat, loss = _table(6)
    ri = RoutingInfo(range(6), lat, loss)
    for k in range(300):
        row = lat[3:4] + np.uint64(k)
        ri.set_rows(3, row, loss[3:4])
    want = min(int(np.delete(lat, 3, axis=0).min()), int(lat[3].min()) + 299)
    assert ri.get_smallest_latency_ns() == want
    small = np.full_like(lat[1:2], 5)
    ri.set_rows(1, small, loss[1:2])
    assert ri.get_smallest_latency_ns() == 5
    ri.set_rows(1, lat[1:2], loss[1:2])  # back up: the minimum rises again
    assert ri.get_smallest_latency_ns() == want
    wide = np.full_like(lat, 1 << 40)  # every cell wide: the u64 minimum from the side table
    wide[4, 2] = (1 << 40) - 9
    ri.set_rows(0, wide, loss)
    assert ri.get_smallest_latency_ns() == (1 << 40) - 9
