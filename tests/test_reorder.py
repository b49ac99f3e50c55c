"""Reorder front-end (include/spmm_reorder.h) against
the reference's own reorder_strategy.cc / getHeatmap / loadPermutation /
analyzeBlockSparseMetrics outputs (tests/golden/ref_reorder.npz, made by
tests/golden/make_golden.py from oracle/_ref) and the oracle's restatement.
Index arrays are compared bit for bit. CPU only."""
from __future__ import annotations

import numpy as np
import pytest

from helpers import load_reorder_golden, oracle_reorder

GRAPHS = ["rand300", "band200", "pl2000", "comm1500"]
KINDS = ["degree", "bfs", "rcm", "permute"]


@pytest.fixture(scope="module")
def rg():
    return load_reorder_golden()


def _prep():
    from spmm_hip import prep
    return prep


@pytest.mark.parametrize("g", GRAPHS)
@pytest.mark.parametrize("kind", KINDS)
def test_oracle_matches_reference(oracle, rg, g, kind):
    rp, ci = rg[f"{g}_rowptr"], rg[f"{g}_colind"]
    orp, oci = oracle_reorder(oracle, kind, rp, ci, rg[f"{g}_perm"])
    assert np.array_equal(orp, rg[f"{g}_{kind}_rowptr"])
    assert np.array_equal(oci, rg[f"{g}_{kind}_colind"])


@pytest.mark.parametrize("g", GRAPHS)
@pytest.mark.parametrize("kind", KINDS)
def test_reorder_bit_exact_vs_reference(rg, g, kind):
    """spmm_reorder_* + spmm_permute_csr reproduce the reference's reordered
    graph exactly (ties in the degree sorts included)."""
    prep = _prep()
    rp, ci = rg[f"{g}_rowptr"], rg[f"{g}_colind"]
    perm = rg[f"{g}_perm"] if kind == "permute" else prep.reorder(rp, ci, kind)
    assert np.array_equal(np.sort(perm), np.arange(rp.size - 1))
    nrp, nci = prep.permute_csr(rp, ci, perm)
    assert np.array_equal(nrp, rg[f"{g}_{kind}_rowptr"])
    assert np.array_equal(nci, rg[f"{g}_{kind}_colind"])


@pytest.mark.parametrize("g", GRAPHS)
@pytest.mark.parametrize("bs", [16, 64])
def test_heatmap_vs_reference(rg, g, bs):
    prep = _prep()
    h = prep.block_heatmap(rg[f"{g}_rowptr"], rg[f"{g}_colind"], bs)
    assert np.array_equal(h.ravel(), rg[f"{g}_heatmap{bs}"])


@pytest.mark.parametrize("g", GRAPHS)
def test_block_metrics_text_vs_reference(rg, g):
    """Same numbers as analyzeBlockSparseMetrics prints (6 significant digits,
    the iostream default), block sizes 2..64."""
    prep = _prep()
    rp, ci = rg[f"{g}_rowptr"], rg[f"{g}_colind"]
    lines = []
    for bs in (2, 4, 8, 16, 32, 64):
        m = prep.block_metrics(rp, ci, bs)
        lines.append(f"blockSize={bs} density={m['density']:.6g} "
                     f"utilization={m['utilization']:.6g} average={m['average']:.6g}")
        assert m["nnzb"] == prep.calculate_nnzb(rp.size - 1, rp, ci, bs)
    assert "\n".join(lines) + "\n" == str(rg[f"{g}_metrics_text"])


def test_permutation_files(rg, tmp_path):
    prep = _prep()
    perm = rg["pl2000_perm"]
    f = str(tmp_path / "p.txt")
    prep.dump_permutation(f, perm)
    assert np.array_equal(prep.load_permutation(f, perm.size), perm)
    bad = tmp_path / "bad.txt"
    bad.write_text("0 1 1\n")
    with pytest.raises(ValueError):
        prep.load_permutation(str(bad), 3)
    with pytest.raises(ValueError):
        prep.load_permutation(str(tmp_path / "missing.txt"), 3)


def test_heatmap_dump_format(tmp_path):
    prep = _prep()
    rp = np.array([0, 2, 3, 3], np.int32)
    ci = np.array([0, 2, 1], np.int32)
    h = prep.block_heatmap(rp, ci, 2)
    assert h.tolist() == [[2, 1], [0, 0]]
    f = tmp_path / "h.txt"
    prep.dump_heatmap(str(f), h)
    assert f.read_text() == "2\n2 1 \n0 0 \n"  # utility.cc:90-100


def test_permute_carries_values_and_rejects_bad_input():
    prep = _prep()
    rp = np.array([0, 2, 3], np.int32)
    ci = np.array([0, 1, 0], np.int32)
    v = np.array([1.0, 2.0, 3.0], np.float32)
    nrp, nci, nv = prep.permute_csr(rp, ci, [1, 0], v)
    assert nrp.tolist() == [0, 1, 3] and nci.tolist() == [1, 0, 1]
    assert nv.tolist() == [3.0, 2.0, 1.0]
    with pytest.raises(ValueError):
        prep.permute_csr(rp, ci, [0, 0])  # not a permutation
    with pytest.raises(ValueError):
        prep.reorder(rp, np.array([0, 1, 5], np.int32), "bfs")  # column out of range
    with pytest.raises(ValueError):
        prep.reorder(rp, ci, "metis")


def test_rcm_recovers_scrambled_communities(rg):
    """The point of the front-end: on a scrambled community graph the
    reordered pattern packs into fewer 16 x 16 blocks."""
    prep = _prep()
    rp, ci = rg["comm1500_rowptr"], rg["comm1500_colind"]
    before = prep.block_metrics(rp, ci, 16)["nnzb"]
    nrp, nci = prep.permute_csr(rp, ci, prep.reorder(rp, ci, "rcm"))
    after = prep.block_metrics(nrp, nci, 16)["nnzb"]
    assert after < 0.75 * before  # 8057 -> 5662 blocks


@pytest.mark.parametrize("seed", [1, 2])
def test_reorder_vs_oracle_on_generated_graphs(oracle, seed):
    """Larger power-law graphs from the library's generator (threaded row
    sorts in play): library == oracle restatement, all methods."""
    prep = _prep()
    rp, ci = prep.powerlaw_csr(30000, 300000, 2000, 2.3, seed)
    for kind in ("degree", "bfs", "rcm"):
        nrp, nci = prep.permute_csr(rp, ci, prep.reorder(rp, ci, kind))
        orp, oci = oracle_reorder(oracle, kind, rp, ci)
        assert np.array_equal(nrp, orp) and np.array_equal(nci, oci), kind
