"""Host preprocessing of the product (libspmm_hip.so, CPU side) against the
reference's own outputs (golden fixtures) and the oracle: bit-exact index
arrays and values. CPU only."""
from __future__ import annotations

import numpy as np
import pytest

from helpers import ptr


def _prep():
    from spmm_hip import prep
    return prep


def test_rng_feeders_match_reference(golden):
    prep = _prep()
    prep.rng_seed(1234)
    assert np.array_equal(prep.random_array(64 * 64), golden["ref"]["dense_64x64"])
    for (m, n, p) in [(64, 80, 0.1), (300, 257, 0.03), (1000, 1200, 0.01)]:
        prep.rng_seed(1234)
        rp, ci, v = prep.random_csr(m, n, p)
        key = f"csr_{m}_{n}_{p}"
        assert np.array_equal(rp, golden["ref"][key + "_rowptr"])
        assert np.array_equal(ci, golden["ref"][key + "_colind"])
        assert np.array_equal(v, golden["ref"][key + "_val"])
    prep.rng_seed(1234)
    rp, ci, v = prep.random_bsr(12, 10, 4, 0.2)
    assert np.array_equal(rp, golden["ref"]["bsr_12_10_4_rowptr"])
    assert np.array_equal(ci, golden["ref"]["bsr_12_10_4_colind"])
    assert np.array_equal(v, golden["ref"]["bsr_12_10_4_val"])


@pytest.mark.parametrize("g", ["rand300", "band200"])
@pytest.mark.parametrize("bs", [2, 4, 16, 32])
def test_csr2bsr_bit_exact_vs_reference(golden, g, bs):
    """Index arrays and block values equal the reference divide_matrix output
    (density -> 0, unit values) and calculateNnzb."""
    prep = _prep()
    r = golden["ref"]
    rp, ci = r[f"{g}_rowptr"], r[f"{g}_colind"]
    n = rp.size - 1
    brp, bci, bval = prep.csr2bsr(n, n, rp, ci, np.ones(ci.size, np.float32), bs, 0)
    assert np.array_equal(brp, r[f"{g}_bs{bs}_all_bsr_rp"])
    assert np.array_equal(bci, r[f"{g}_bs{bs}_all_bsr_ci"])
    assert np.array_equal(bval, r[f"{g}_bs{bs}_all_bsr_val"])
    assert prep.calculate_nnzb(n, rp, ci, bs) == int(r[f"{g}_bs{bs}_nnzb"][0])


@pytest.mark.parametrize("bs", [1, 3, 16, 32])
@pytest.mark.parametrize("direction", [0, 1])
def test_csr2bsr_bsr2csr_vs_oracle(oracle, golden, bs, direction):
    prep = _prep()
    r = golden["ref"]
    rp, ci, v = r["csr_1000_1200_0.01_rowptr"], r["csr_1000_1200_0.01_colind"], \
        r["csr_1000_1200_0.01_val"]
    m, n = 1000, 1200
    brp, bci, bval = prep.csr2bsr(m, n, rp, ci, v, bs, direction)
    mb = (m + bs - 1) // bs
    obrp = np.zeros(mb + 1, np.int32)
    nnzb = oracle.oracle_csr2bsr_nnz(m, bs, ptr(rp), ptr(ci), ptr(obrp))
    obci, obval = np.zeros(nnzb, np.int32), np.zeros(nnzb * bs * bs, np.float32)
    oracle.oracle_csr2bsr(direction, m, bs, ptr(rp), ptr(ci), ptr(v), ptr(obrp), ptr(obci),
                          ptr(obval))
    assert np.array_equal(brp, obrp) and np.array_equal(bci, obci)
    assert np.array_equal(bval, obval)
    nb = (n + bs - 1) // bs
    crp, cci, cv = prep.bsr2csr(mb, nb, brp, bci, bval, bs, direction)
    orp = np.zeros(mb * bs + 1, np.int32)
    oci = np.zeros(nnzb * bs * bs, np.int32)
    ov = np.zeros(nnzb * bs * bs, np.float32)
    oracle.oracle_bsr2csr(direction, mb, bs, ptr(brp), ptr(bci), ptr(bval), ptr(orp), ptr(oci),
                          ptr(ov))
    assert np.array_equal(crp, orp) and np.array_equal(cci, oci) and np.array_equal(cv, ov)
    assert crp[-1] == nnzb * bs * bs  # bsr2csr.cu:177


@pytest.mark.parametrize("g", ["rand300", "band200"])
@pytest.mark.parametrize("bs", [2, 4, 16, 32])
@pytest.mark.parametrize("tag,density", [("all", 1e-9), ("d25", 0.25)])
def test_divide_bit_exact_vs_reference(oracle, golden, g, bs, tag, density):
    """divide_matrix (divide.cu:52-127): BSR part and CSR remainder equal the
    reference's own output on unit values, and the oracle's restatement."""
    from helpers import oracle_divide
    prep = _prep()
    r = golden["ref"]
    rp, ci = r[f"{g}_rowptr"], r[f"{g}_colind"]
    n = rp.size - 1
    ones = np.ones(ci.size, np.float32)
    out = prep.divide(n, rp, ci, ones, bs, density)
    ref = [r[f"{g}_bs{bs}_{tag}_{nm}"] for nm in ("csr_rp", "csr_ci", "bsr_rp", "bsr_ci",
                                                  "bsr_val")]
    crp, cci, cv, brp, bci, bv = out
    for got, want in zip((crp, cci, brp, bci, bv), ref):
        assert np.array_equal(got, want)
    assert np.all(cv == 1.0)
    for got, want in zip(out, oracle_divide(oracle, n, bs, density, rp, ci, ones)):
        assert np.array_equal(got, want)


def test_divide_density_zero_admits_empty_blocks(oracle):
    """divide.cu:91: occupancy 0 >= density 0, so every block is admitted."""
    from helpers import oracle_divide
    prep = _prep()
    rp = np.array([0, 1, 1, 2, 2], np.int32)
    ci = np.array([0, 3], np.int32)
    v = np.array([2.0, 3.0], np.float32)
    crp, cci, cv, brp, bci, bv = prep.divide(4, rp, ci, v, 2, 0.0)
    assert brp.tolist() == [0, 2, 4] and bci.tolist() == [0, 1, 0, 1] and cci.size == 0
    assert bv.reshape(4, 4)[0, 0] == 2.0 and bv.reshape(4, 4)[3, 1] == 3.0
    for got, want in zip((crp, cci, cv, brp, bci, bv), oracle_divide(oracle, 4, 2, 0.0, rp, ci, v)):
        assert np.array_equal(got, want)


def test_csr2bsr_duplicates_are_summed_and_errors():
    prep = _prep()
    rp = np.array([0, 3], np.int32)
    ci = np.array([1, 1, 2], np.int32)
    v = np.array([1.0, 2.0, 4.0], np.float32)
    brp, bci, bval = prep.csr2bsr(1, 4, rp, ci, v, 2, 0)
    assert brp.tolist() == [0, 2] and bci.tolist() == [0, 1]
    assert bval.tolist() == [0, 3, 0, 0, 4, 0, 0, 0]
    with pytest.raises(Exception):
        prep.csr2bsr(1, 2, rp, np.array([0, 1, 9], np.int32), v, 2, 0)  # col out of range


def test_partition_rows_balances_nnz():
    prep = _prep()
    rp, ci = prep.powerlaw_csr(20000, 400000, 3000, 2.3, 3)
    for parts in (1, 2, 3, 8):
        b = prep.partition_rows(rp, parts)
        assert b[0] == 0 and b[-1] == 20000 and np.all(np.diff(b) >= 0)
        cost = [(rp[b[i + 1]] - rp[b[i]]) + (b[i + 1] - b[i]) for i in range(parts)]
        total = rp[-1] + 20000
        # each part within one row's cost of the ideal share
        assert max(cost) <= total / parts + 3001 + 1


def test_powerlaw_generator_properties():
    prep = _prep()
    n, nnz, dmax = 50000, 1000000, 5000
    rp, ci = prep.powerlaw_csr(n, nnz, dmax, 2.3, 1234)
    rp2, ci2 = prep.powerlaw_csr(n, nnz, dmax, 2.3, 1234)
    assert np.array_equal(rp, rp2) and np.array_equal(ci, ci2)  # deterministic
    assert rp[-1] == nnz and ci.size == nnz
    deg = np.diff(rp)
    assert deg.max() >= dmax - 5 and deg.min() >= 0
    assert ci.min() >= 0 and ci.max() < n
    for r in np.random.default_rng(0).choice(n, 200):
        row = ci[rp[r]:rp[r + 1]]
        assert np.all(np.diff(row) > 0)  # sorted, no duplicates


def test_community_generator_properties():
    prep = _prep()
    rp, ci = prep.community_csr(20000, 50.0, 64, 512, 0.9, 5)
    assert rp[0] == 0 and rp[-1] == ci.size and ci.max() < 20000
    deg = np.diff(rp)
    assert 35 < deg.mean() < 55
    # most edges stay near the diagonal (community order)
    r = np.repeat(np.arange(20000), deg)
    assert np.mean(np.abs(ci - r) < 512) > 0.85


def test_text_csr_roundtrip(tmp_path):
    prep = _prep()
    rp, ci = prep.powerlaw_csr(3000, 20000, 300, 2.3, 9)
    prefix = str(tmp_path / "g")
    prep.dump_csr(prefix, rp, ci)
    assert open(prefix + "_indptr.txt").readline().strip() == "3001"  # load_data.cc:131
    rp2, ci2 = prep.load_csr(prefix)
    assert np.array_equal(rp, rp2) and np.array_equal(ci, ci2)


def test_load_graph_edge_list(tmp_path):
    prep = _prep()
    f = tmp_path / "e.txt"
    f.write_text("4 5\n0 3\n0 1\n2 2\n3 0\n0 2\n")
    rp, ci = prep.load_graph(str(f))
    assert rp.tolist() == [0, 3, 3, 4, 5] and ci.tolist() == [1, 2, 3, 2, 0]


@pytest.mark.parametrize("bs,K", [(16, 512), (32, 128)])
def test_hybrid_plan_is_the_model_minimum(bs, K):
    """The planner's threshold minimises its own cost model over every
    threshold, and divide at the returned density yields the reported split."""
    prep = _prep()
    rp, ci = prep.community_csr(6000, 60.0, 64, 512, 0.95, 11)
    n = rp.size - 1
    v = np.ones(ci.size, np.float32)
    plan = prep.hybrid_plan(rp, ci, bs, K)
    crp, cci, cv, brp, bci, bv = prep.divide(n, rp, ci, v, bs, plan["density"])
    assert bci.size == plan["nnzb"] and cci.size == plan["csr_nnz"]
    tb = (4 * (bs * bs + bs * K) + 4) / 7.0e12
    tn = (8 + 4 * K) / 7.5e12

    def cost(T):
        _, c2, _, _, b2, _ = prep.divide(n, rp, ci, v, bs, T / (bs * bs))
        return b2.size * tb + c2.size * tn

    best = min(cost(T) for T in range(1, bs * bs + 2, max(1, bs * bs // 64)))
    assert plan["est_seconds"] <= best * (1 + 1e-9)
    assert abs(plan["est_seconds"] - (bci.size * tb + cci.size * tn)) <= 1e-9 * best
