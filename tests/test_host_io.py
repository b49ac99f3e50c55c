"""Text formats (load_data.cc:125-184) through the library's parallel
parser/writer, checked against the reference's own dumpCSRToFile /
loadCSRFromFile / loadGraphFromFile (oracle/_ref, built from the reference
sources; those cases skip where it is absent), and the binary sidecar cache
(SURVEY.md §8f rank 3). CPU only."""
from __future__ import annotations

import ctypes
import os
import time

import numpy as np
import pytest

from helpers import REF_SO, ptr


def _prep():
    from spmm_hip import prep
    return prep


@pytest.fixture(scope="module")
def ref():
    if not os.path.exists(REF_SO):
        pytest.skip("oracle/_ref not built (reference sources absent)")
    L = ctypes.CDLL(REF_SO)
    L.ref_dump_csr.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                               ctypes.c_void_p]
    for f in (L.ref_load_csr, L.ref_load_graph):
        f.restype = ctypes.c_int64
        f.argtypes = [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                      ctypes.c_int64]
    return L


def _graph(seed=3, n=20000, nnz=300000):
    return _prep().powerlaw_csr(n, nnz, 1500, 2.3, seed)


def test_our_dump_reads_back_in_the_reference(ref, tmp_path):
    rp, ci = _graph()
    prefix = str(tmp_path / "g")
    _prep().dump_csr(prefix, rp, ci)
    orp, oci = np.zeros(rp.size, np.int32), np.zeros(ci.size, np.int32)
    packed = ref.ref_load_csr(prefix.encode(), ptr(orp), ptr(oci), rp.size, ci.size)
    assert packed >= 0 and (packed >> 32) == rp.size - 1 and (packed & 0xffffffff) == ci.size
    assert np.array_equal(orp, rp) and np.array_equal(oci, ci)


def test_reference_dump_reads_back_here_byte_identical(ref, tmp_path):
    rp, ci = _graph(4)
    a, b = str(tmp_path / "ref"), str(tmp_path / "ours")
    ref.ref_dump_csr(a.encode(), rp.size - 1, ci.size, ptr(rp), ptr(ci))
    _prep().dump_csr(b, rp, ci)
    for suf in ("_indptr.txt", "_indices.txt"):
        assert open(a + suf, "rb").read() == open(b + suf, "rb").read()
    r2, c2 = _prep().load_csr(a)
    assert np.array_equal(r2, rp) and np.array_equal(c2, ci)


def test_edge_list_matches_reference(ref, tmp_path):
    rng = np.random.default_rng(8)
    n, m = 3000, 40000
    src, dst = rng.integers(0, n, m), rng.integers(0, n, m)  # duplicates included
    f = tmp_path / "e.txt"
    f.write_text(f"{n} {m}\n" + "".join(f"{a}\t{b}\n" for a, b in zip(src, dst)))
    rp, ci = _prep().load_graph(str(f))
    orp, oci = np.zeros(n + 1, np.int32), np.zeros(m, np.int32)
    assert ref.ref_load_graph(str(f).encode(), ptr(orp), ptr(oci), n + 1, m) >= 0
    assert np.array_equal(rp, orp) and np.array_equal(ci, oci)


def test_malformed_text_is_rejected(tmp_path):
    prep = _prep()
    p = tmp_path / "bad"
    (tmp_path / "bad_indptr.txt").write_text("3\n0 1 x\n")
    (tmp_path / "bad_indices.txt").write_text("1\n0\n")
    with pytest.raises(OSError):
        prep.load_csr(str(p))
    (tmp_path / "bad_indptr.txt").write_text("4\n0 1 1\n")  # one value short
    with pytest.raises(OSError):
        prep.load_csr(str(p))
    g = tmp_path / "g.txt"
    g.write_text("3 2\n0 1\n5 0\n")  # source out of range
    with pytest.raises(OSError):
        prep.load_graph(str(g))


@pytest.mark.parametrize("with_val", [False, True])
def test_binary_roundtrip_and_corruption(tmp_path, with_val):
    prep = _prep()
    rp, ci = _graph(5)
    v = np.random.default_rng(1).uniform(-1, 1, ci.size).astype(np.float32) if with_val else None
    f = str(tmp_path / "g.csrbin")
    prep.save_csr_bin(f, rp, ci, v)
    r2, c2, v2 = prep.load_csr_bin(f)
    assert np.array_equal(r2, rp) and np.array_equal(c2, ci)
    assert (v2 is None) if v is None else np.array_equal(v2, v)
    raw = bytearray(open(f, "rb").read())
    raw[len(raw) // 2] ^= 0x10  # flip one bit in the payload
    open(f, "wb").write(bytes(raw))
    with pytest.raises(ValueError, match="checksum"):
        prep.load_csr_bin(f)
    open(f, "wb").write(b"not a cache")
    with pytest.raises(OSError):
        prep.load_csr_bin(f)


def test_cached_loader_uses_and_refreshes_the_sidecar(tmp_path):
    prep = _prep()
    rp, ci = _graph(6)
    prefix = str(tmp_path / "g")
    prep.dump_csr(prefix, rp, ci)
    r1, c1 = prep.load_csr_cached(prefix)  # parses text, writes g.csrbin
    assert os.path.exists(prefix + ".csrbin")
    assert np.array_equal(r1, rp) and np.array_equal(c1, ci)
    r2, c2 = prep.load_csr_cached(prefix)  # served from the sidecar
    assert np.array_equal(r2, rp) and np.array_equal(c2, ci)
    # newer text wins over an older sidecar
    time.sleep(0.01)
    rp3, ci3 = _graph(7)
    prep.dump_csr(prefix, rp3, ci3)
    r3, c3 = prep.load_csr_cached(prefix)
    assert np.array_equal(r3, rp3) and np.array_equal(c3, ci3)
    # a corrupt sidecar falls back to the text and is rewritten
    raw = bytearray(open(prefix + ".csrbin", "rb").read())
    raw[-5] ^= 1
    open(prefix + ".csrbin", "wb").write(bytes(raw))
    os.utime(prefix + ".csrbin")
    r4, c4 = prep.load_csr_cached(prefix)
    assert np.array_equal(r4, rp3) and np.array_equal(c4, ci3)
    assert np.array_equal(prep.load_csr_bin(prefix + ".csrbin")[1], ci3)
