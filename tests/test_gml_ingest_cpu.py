"""GML ingest at scale: the multi-threaded parse
(sg_gml_parse_threads) gives the single-threaded parse's graph and its first
error, whatever the chunking; f32 loss values are correctly rounded; and
xz-compressed graph files load like load_network_graph (graph/mod.rs:483-513)."""
import ctypes
import lzma
import random

import numpy as np
import pytest

from shadow_amd import ShadowGpuError, synth
from shadow_amd.graph import NetworkGraph


def _big_gml(n=12000, seed=3, label_every=0):
    g = synth.ring_chords_graph(n, 8.0, seed=seed, parallel=0.05)
    text = synth.graph_to_gml(g)
    if label_every:
        # labels whose text looks like item boundaries: a chunk guess inside a string
        # must be detected and the parse continued from the true boundary
        fake = '"x\n  node [\n    id 7\n  ]\n  edge [\n"'
        out, k = [], 0
        for line in text.split("\n"):
            out.append(line)
            if line.strip() == "node [":
                k += 1
                if k % label_every == 0:
                    out.append(f"    label {fake}")
        text = "\n".join(out)
    assert n < 10000 or len(text) > 4 << 20  # large enough to be split over threads
    return g, text


def _same(a, b):
    assert a.n_nodes == b.n_nodes and a.directed == b.directed
    for k in ("edge_src", "edge_dst", "edge_latency_ns", "node_ids"):
        assert np.array_equal(getattr(a, k), getattr(b, k)), k
    assert np.array_equal(a.edge_packet_loss.view(np.uint32), b.edge_packet_loss.view(np.uint32))


@pytest.mark.parametrize("threads", [2, 3, 8, 16])
def test_threads_match_single_thread(threads):
    g, text = _big_gml()
    one = NetworkGraph.parse(text, threads=1)
    many = NetworkGraph.parse(text, threads=threads)
    _same(one, many)
    assert np.array_equal(many.edge_src, g["src"]) and np.array_equal(many.edge_latency_ns, g["lat"])
    assert np.array_equal(many.edge_packet_loss.view(np.uint32), g["loss"].view(np.uint32))


def test_chunk_guess_inside_a_string():
    _, text = _big_gml(label_every=3)
    _same(NetworkGraph.parse(text, threads=1), NetworkGraph.parse(text, threads=8))


@pytest.mark.parametrize("where", [0.1, 0.5, 0.93])
def test_first_error_wins_across_chunks(where):
    """Two faults in different chunks: the parse reports the earlier one, as the
    sequential parser does -- syntax errors before node errors before edge errors."""
    _, text = _big_gml()
    lines = text.split("\n")

    def fault(frac, old, new):
        i = int(len(lines) * frac)
        while old not in lines[i]:
            i += 1
        lines[i] = lines[i].replace(old, new)

    fault(where, "latency", "latency_typo")            # edge conversion error (later phase)
    fault(min(where + 0.05, 0.99), "target", "targt")  # syntax-phase error, later in the text
    bad = "\n".join(lines)
    msgs = []
    for th in (1, 8):
        with pytest.raises(ShadowGpuError) as e:
            NetworkGraph.parse(bad, threads=th)
        msgs.append(str(e.value))
    assert msgs[0] == msgs[1] and "'target' doesn't exist" in msgs[0]


def test_missing_endpoint_reported_in_edge_order():
    _, text = _big_gml()
    lines = text.split("\n")
    hits = [i for i, ln in enumerate(lines) if ln.strip().startswith("source ")]
    lines[hits[len(hits) * 3 // 4]] = "    source 99999999"
    lines[hits[len(hits) // 4]] = "    source 88888888"
    bad = "\n".join(lines)
    for th in (1, 8):
        with pytest.raises(ShadowGpuError) as e:
            NetworkGraph.parse(bad, threads=th)
        assert "Edge source 88888888 doesn't exist" in str(e.value)


def test_f32_matches_libc_strtof():
    """The fast path (m * 10^e in f64, then f32 unless on an f32 midpoint) against
    glibc strtof, which rounds correctly, on random and midpoint decimals."""
    libc = ctypes.CDLL(None)
    libc.strtof.restype = ctypes.c_float
    libc.strtof.argtypes = [ctypes.c_char_p, ctypes.c_void_p]
    rng = random.Random(5)
    vals = ["0.0", "1.0", ".5", "0.1", "1e-3", "0.30000001192092896", "1.00000005960464477539062500",
            "1.0000000596046448", "0.999999970197677612304688", "0.000000000000000000001", "1e-39", "1e-45",
            "3.4028235e38", "0.33333334", "0.0000123", "5e-8"]
    for _ in range(3000):
        k = rng.randint(1, 19)
        digits = "".join(rng.choice("0123456789") for _ in range(k))
        vals.append(f"0.{digits}")
        vals.append(f"{rng.randint(0, 9)}.{digits}e-{rng.randint(0, 30)}")
    vals = [v for v in vals if 0.0 <= float(v) <= 1.0]
    body = "".join(f"  edge [\n    source 0\n    target 0\n    latency \"1 ns\"\n    packet_loss {v}\n  ]\n"
                   for v in vals)
    g = NetworkGraph.parse("graph [\n  directed 1\n  node [\n    id 0\n  ]\n" + body + "]")
    want = np.array([libc.strtof(v.encode(), None) for v in vals], np.float32)
    assert np.array_equal(g.edge_packet_loss.view(np.uint32), want.view(np.uint32))


def test_from_file_plain_and_xz(tmp_path):
    g, text = _big_gml(n=2000)
    plain = tmp_path / "g.gml"
    plain.write_text(text)
    xz = tmp_path / "g.gml.xz"
    with lzma.open(xz, "wb", format=lzma.FORMAT_XZ) as f:
        f.write(text.encode())
    a = NetworkGraph.from_file(plain)
    b = NetworkGraph.from_file(xz, compression="xz")
    _same(a, b)
    assert np.array_equal(b.edge_dst, g["dst"])
    with pytest.raises(ShadowGpuError, match="Failed to decompress file"):
        NetworkGraph.from_file(plain, compression="xz")
    # a truncated stream, a missing file, invalid UTF-8 (String::from_utf8 / read_to_string)
    cut = tmp_path / "cut.gml.xz"
    cut.write_bytes(xz.read_bytes()[:-40])
    with pytest.raises(ShadowGpuError, match="Failed to decompress file"):
        NetworkGraph.from_file(cut, compression="xz")
    with pytest.raises(ShadowGpuError, match="Failed to read file"):
        NetworkGraph.from_file(tmp_path / "absent.gml")
    bad = tmp_path / "bad.gml"
    bad.write_bytes(text.encode().replace(b"graph [", b"graph [ \xc0\xaf", 1))
    with pytest.raises(ShadowGpuError, match="UTF-8"):
        NetworkGraph.from_file(bad)
    badxz = tmp_path / "bad.gml.xz"
    with lzma.open(badxz, "wb", format=lzma.FORMAT_XZ) as f:
        f.write(b"graph [ \xed\xa0\x80 ]")  # an encoded surrogate
    with pytest.raises(ShadowGpuError, match="utf-8"):
        NetworkGraph.from_file(badxz, compression="xz")
    # threads: the same graph from the xz file on 1 and 8 threads
    _same(NetworkGraph.from_file(xz, compression="xz", threads=1), NetworkGraph.from_file(xz, compression="xz",
                                                                                           threads=8))


def test_utf8_check_matches_python(tmp_path):
    """sg_gml_load's UTF-8 check accepts exactly what a strict decoder accepts."""
    rng = np.random.default_rng(3)
    cases = [b"\xf4\x90\x80\x80", b"\xf0\x8f\xbf\xbf", b"\xe0\x9f\xbf", b"\xc1\xbf", b"\xef\xbf\xbf",
             b"\xf4\x8f\xbf\xbf", b"\xe2\x82", "\u00e9\u4e2d\U0001f600".encode()]
    cases += [bytes(rng.integers(0x80, 0x100, 3).astype(np.uint8)) for _ in range(200)]
    for k, c in enumerate(cases):
        f = tmp_path / f"u{k}.gml"
        f.write_bytes(b"graph [\n  label \"" + c + b"\"\n  node [\n    id 0\n  ]\n]")
        try:
            c.decode("utf-8")
            ok = True
        except UnicodeDecodeError:
            ok = False
        if ok:
            NetworkGraph.from_file(f)
        else:
            with pytest.raises(ShadowGpuError, match="UTF-8"):
                NetworkGraph.from_file(f)
