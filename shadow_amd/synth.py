"""Seeded synthetic workloads for parity tests and bench.py.

C2: complete undirected graph, integer-ms latencies U[1,300], self-loops U[1,10] ms,
    loss 0 w.p. 0.8 else U(0, 0.02) as f32.
C3: undirected ring + random chords to mean degree ~8, self-loops, integer-us
    latencies U[1000, 100000] (as ns), loss as C2.
C4: hosts -> node h mod n_nodes, packets src-major, dst uniform != src,
    send_time U[round_start, round_end), payload 0 w.p. 0.2 else 1448.
Host seeds follow Shadow's derivation (sim_config.rs:50-54,221-242).
"""
from __future__ import annotations

import numpy as np

from .graph import IpAssignment, ipv4_to_u32

MASK64 = (1 << 64) - 1


# ---------------------------------------------------------------------------
# Host seeds: HostInfo.seed = first u64 of Xoshiro256++::seed_from_u64(general
# seed) XOR SipHash-1-3(k=0)(hostname || 0xFF)  (CPU setup, not the hot path)
# ---------------------------------------------------------------------------
def _rotl(x, k):
    return ((x << k) | (x >> (64 - k))) & MASK64


def splitmix64_stream(seed: int, n: int):
    st = seed & MASK64
    out = []
    for _ in range(n):
        st = (st + 0x9E3779B97F4A7C15) & MASK64
        z = st
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & MASK64
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & MASK64
        out.append(z ^ (z >> 31))
    return out


def xoshiro_first_u64(seed: int) -> int:
    s0, s1, s2, s3 = splitmix64_stream(seed, 4)
    return (_rotl((s0 + s3) & MASK64, 23) + s0) & MASK64


def siphash13(data: bytes) -> int:
    v0, v1, v2, v3 = 0x736F6D6570736575, 0x646F72616E646F6D, 0x6C7967656E657261, 0x7465646279746573

    def rnd(v0, v1, v2, v3):
        v0 = (v0 + v1) & MASK64; v1 = _rotl(v1, 13); v1 ^= v0; v0 = _rotl(v0, 32)
        v2 = (v2 + v3) & MASK64; v3 = _rotl(v3, 16); v3 ^= v2
        v0 = (v0 + v3) & MASK64; v3 = _rotl(v3, 21); v3 ^= v0
        v2 = (v2 + v1) & MASK64; v1 = _rotl(v1, 17); v1 ^= v2; v2 = _rotl(v2, 32)
        return v0, v1, v2, v3

    n = len(data)
    i = 0
    while i + 8 <= n:
        m = int.from_bytes(data[i:i + 8], "little")
        v3 ^= m
        v0, v1, v2, v3 = rnd(v0, v1, v2, v3)
        v0 ^= m
        i += 8
    b = ((n & 0xFF) << 56) | int.from_bytes(data[i:], "little")
    v3 ^= b
    v0, v1, v2, v3 = rnd(v0, v1, v2, v3)
    v0 ^= b
    v2 ^= 0xFF
    for _ in range(3):
        v0, v1, v2, v3 = rnd(v0, v1, v2, v3)
    return v0 ^ v1 ^ v2 ^ v3


def host_seed(general_seed: int, hostname: str) -> int:
    return xoshiro_first_u64(general_seed) ^ siphash13(hostname.encode() + b"\xff")


def host_seeds(general_seed: int, hostnames) -> np.ndarray:
    r = xoshiro_first_u64(general_seed)
    return np.array([r ^ siphash13(h.encode() + b"\xff") for h in hostnames], dtype=np.uint64)


# ---------------------------------------------------------------------------
# Graphs (edge lists in GML edge order; node index == GML id)
# ---------------------------------------------------------------------------
def _loss(rng: np.random.Generator, m: int, p_zero: float = 0.8, hi: float = 0.02) -> np.ndarray:
    loss = rng.uniform(0.0, hi, m).astype(np.float32)
    loss[rng.random(m) < p_zero] = 0.0
    return loss


def complete_graph(n: int, seed: int = 1):
    """C2: every unordered pair once + one self-loop per node, undirected."""
    rng = np.random.default_rng(seed)
    iu, ju = np.triu_indices(n, 1)
    src = np.concatenate([np.arange(n), iu]).astype(np.uint32)
    dst = np.concatenate([np.arange(n), ju]).astype(np.uint32)
    lat = np.concatenate([rng.integers(1, 11, n), rng.integers(1, 301, len(iu))]).astype(np.uint64) * 1_000_000
    loss = _loss(rng, len(src))
    return dict(n=n, src=src, dst=dst, lat=lat, loss=loss, directed=False)


def ring_chords_graph(n: int, mean_degree: float = 8.0, seed: int = 1, directed: bool = False,
                      lat_lo_us: int = 1000, lat_hi_us: int = 100000, parallel: float = 0.0):
    """C3: ring (connected) + random chords to ~mean_degree, self-loops, optional parallel edges."""
    rng = np.random.default_rng(seed)
    ring_s = np.arange(n)
    ring_d = (ring_s + 1) % n
    n_chords = max(0, int(n * mean_degree / 2) - n)
    cs = rng.integers(0, n, n_chords)
    cd = rng.integers(0, n, n_chords)
    keep = cs != cd
    cs, cd = cs[keep], cd[keep]
    if directed:  # keep strong connectivity with the reverse ring
        ring_s, ring_d = np.concatenate([ring_s, ring_d]), np.concatenate([ring_d, ring_s])
    src = np.concatenate([np.arange(n), ring_s, cs])
    dst = np.concatenate([np.arange(n), ring_d, cd])
    if parallel > 0:
        k = int(len(src) * parallel)
        pick = rng.integers(n, len(src), k)  # duplicate non-self-loop edges
        src, dst = np.concatenate([src, src[pick]]), np.concatenate([dst, dst[pick]])
    m = len(src)
    lat = rng.integers(lat_lo_us, lat_hi_us + 1, m).astype(np.uint64) * 1000
    return dict(n=n, src=src.astype(np.uint32), dst=dst.astype(np.uint32), lat=lat, loss=_loss(rng, m),
                directed=directed)


def graph_to_gml(g, node_ids=None) -> str:
    """GML text with losses as shortest round-trip f32 decimals (no double rounding)."""
    n = g["n"]
    ids = list(range(n)) if node_ids is None else list(node_ids)
    out = ["graph [", f"  directed {1 if g['directed'] else 0}"]
    for i in ids:
        out += ["  node [", f"    id {i}", "  ]"]
    for s, d, l, p in zip(g["src"], g["dst"], g["lat"], g["loss"]):
        out += ["  edge [", f"    source {ids[s]}", f"    target {ids[d]}", f'    latency "{int(l)} ns"',
                f"    packet_loss {repr(float(np.float32(p)))}", "  ]"]
    out.append("]")
    return "\n".join(out) + "\n"


# ---------------------------------------------------------------------------
# Hosts and packets
# ---------------------------------------------------------------------------
def make_hosts(n_hosts: int, n_nodes: int, general_seed: int = 1, exact_seeds: bool = True):
    """Hosts 'host%06d' (HostId = name order) on node h mod n_nodes, IPs from IpAssignment."""
    names = [f"host{h:06d}" for h in range(n_hosts)]
    node = (np.arange(n_hosts) % n_nodes).astype(np.uint32)
    ipa = IpAssignment()
    ips = np.array([ipa.assign(int(node[h])) for h in range(n_hosts)], dtype=np.uint32)
    if exact_seeds:
        seeds = host_seeds(general_seed, names)
    else:  # fast path for very large host counts: seeds are inputs to the kernel either way
        seeds = np.random.default_rng(general_seed).integers(0, 2**63, n_hosts, dtype=np.int64).astype(np.uint64)
    return dict(n=n_hosts, ip=ips, route=node, seed=seeds)


def make_packets(n_packets: int, hosts, round_start: int, round_end: int, seed: int = 1,
                 p_ack: float = 0.2, p_unknown_dst: float = 0.0, hot_dst: int = -1, p_hot: float = 0.0,
                 src_hosts=None):
    """C4 recipe: grouped by ascending source host, send_time ascending within a host.

    src_hosts: restrict senders to these host ids (a rank's own hosts); destinations stay global.
    """
    rng = np.random.default_rng(seed)
    H = hosts["n"]
    if src_hosts is None:
        src = np.sort(rng.integers(0, H, n_packets)).astype(np.uint32)
    else:
        src_hosts = np.sort(np.asarray(src_hosts, dtype=np.uint32))
        src = np.sort(src_hosts[rng.integers(0, len(src_hosts), n_packets)]).astype(np.uint32)
    dst = rng.integers(0, H - 1, n_packets)
    dst = np.where(dst >= src, dst + 1, dst) if H > 1 else np.zeros(n_packets, np.int64)
    if hot_dst >= 0 and p_hot > 0:
        hot = rng.random(n_packets) < p_hot
        dst = np.where(hot & (src != hot_dst), hot_dst, dst)
    dst_ip = hosts["ip"][dst].astype(np.uint32)
    if p_unknown_dst > 0:
        unk = rng.random(n_packets) < p_unknown_dst
        dst_ip = np.where(unk, np.uint32(ipv4_to_u32("10.9.9.9")), dst_ip).astype(np.uint32)
    payload = np.where(rng.random(n_packets) < p_ack, 0, 1448).astype(np.uint32)
    t = rng.integers(round_start, round_end, n_packets).astype(np.uint64)
    # send order within a host is time order: sort by (src, t) stably
    order = np.lexsort((t, src))
    return dict(src=src[order], dst_ip=dst_ip[order], payload=payload[order], send_time=t[order])
