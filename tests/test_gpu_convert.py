"""Device csr2bsr / bsr2csr (spmm_*_dev) against the host
conversions and the reference's own divide_matrix output: index arrays and
values bit for bit."""
from __future__ import annotations

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def _prep():
    from spmm_hip import prep
    return prep


def _ops():
    from spmm_hip import ops
    return ops


def _dev(*arrs):
    return [torch.from_numpy(np.ascontiguousarray(a)).cuda() for a in arrs]


def _host(*ts):
    return [t.cpu().numpy() for t in ts]


def _graphs():
    prep = _prep()
    rng = np.random.default_rng(3)
    out = {}
    prep.rng_seed(1234)
    rp, ci, v = prep.random_csr(1000, 1200, 0.01)
    out["random"] = (1000, 1200, rp, ci, v)
    rp, ci = prep.community_csr(3000, 30.0, 40, 200, 0.9, 7)
    out["community"] = (3000, 3000, rp, ci, rng.uniform(-1, 1, ci.size).astype(np.float32))
    # duplicates (sorted, repeated columns) and empty rows
    rows = [np.sort(rng.integers(0, 700, rng.integers(0, 12))) for _ in range(513)]
    rows[5] = np.zeros(0, int)
    rows[7] = np.array([3, 3, 3, 64, 64])
    rp = np.concatenate([[0], np.cumsum([len(r) for r in rows])]).astype(np.int32)
    ci = np.concatenate(rows).astype(np.int32)
    out["dups"] = (513, 700, rp, ci, rng.uniform(-1, 1, ci.size).astype(np.float32))
    return out


GRAPHS = _graphs()


@pytest.mark.parametrize("g", list(GRAPHS))
@pytest.mark.parametrize("bs", [1, 2, 3, 4, 16, 32, 64])
@pytest.mark.parametrize("direction", [0, 1])
def test_csr2bsr_dev_equals_host(device, g, bs, direction):
    m, n, rp, ci, v = GRAPHS[g]
    hb = _prep().csr2bsr(m, n, rp, ci, v, bs, direction)
    db = _host(*_ops().csr2bsr(*_dev(rp, ci, v), m=m, n=n, bs=bs, direction=direction))
    for a, b, nm in zip(db, hb, ("rowptr", "colind", "val")):
        assert np.array_equal(a, b), f"{g} bs={bs} dir={direction}: {nm}"
    # and back: bsr2csr on the device equals the host expansion
    mb, nb = (m + bs - 1) // bs, (n + bs - 1) // bs
    hc = _prep().bsr2csr(mb, nb, *hb, bs, direction)
    dc = _host(*_ops().bsr2csr(*_dev(*hb), mb=mb, nb=nb, bs=bs, direction=direction))
    for a, b, nm in zip(dc, hc, ("rowptr", "colind", "val")):
        assert np.array_equal(a, b), f"bsr2csr {g} bs={bs} dir={direction}: {nm}"


@pytest.mark.parametrize("gname", ["rand300", "band200"])
@pytest.mark.parametrize("bs", [2, 4, 16, 32])
def test_csr2bsr_dev_vs_reference_divide(device, golden, gname, bs):
    """The reference's divide_matrix at density -> 0 (unit values) is csr2bsr."""
    r = golden["ref"]
    rp, ci = r[f"{gname}_rowptr"], r[f"{gname}_colind"]
    n = rp.size - 1
    brp, bci, bval = _host(*_ops().csr2bsr(*_dev(rp, ci, np.ones(ci.size, np.float32)), m=n,
                                           n=n, bs=bs))
    assert np.array_equal(brp, r[f"{gname}_bs{bs}_all_bsr_rp"])
    assert np.array_equal(bci, r[f"{gname}_bs{bs}_all_bsr_ci"])
    assert np.array_equal(bval, r[f"{gname}_bs{bs}_all_bsr_val"])


def test_one_based_and_errors(device):
    from spmm_hip._lib import SpmmError
    m, n, rp, ci, v = GRAPHS["community"]
    b0 = _host(*_ops().csr2bsr(*_dev(rp, ci, v), m=m, n=n, bs=8))
    b1 = _host(*_ops().csr2bsr(*_dev(rp + 1, ci + 1, v), m=m, n=n, bs=8, base=1))
    assert np.array_equal(b1[0], b0[0] + 1) and np.array_equal(b1[1], b0[1] + 1)
    assert np.array_equal(b1[2], b0[2])
    bad = ci.copy()
    bad[10] = n + 5
    with pytest.raises(SpmmError):
        _ops().csr2bsr(*_dev(rp, bad, v), m=m, n=n, bs=8)
    with pytest.raises(SpmmError):
        _ops().csr2bsr(*_dev(rp, ci, v), m=m, n=n, bs=65)


def test_products_scale_roundtrip(device):
    """Full BASELINE scale (products stand-in, bs = 16): device csr2bsr equals
    the host conversion; timed for DESIGN.md."""
    import time
    prep = _prep()
    rp, ci = prep.community_csr(2449029, 27.0, 32, 512, 0.97, 1234)
    n = rp.size - 1
    v = np.random.default_rng(2).uniform(-1, 1, ci.size).astype(np.float32)
    drp, dci, dv = _dev(rp, ci, v)
    _ops().csr2bsr(drp, dci, dv, m=n, n=n, bs=16)  # warm-up
    torch.cuda.synchronize()
    t = time.perf_counter()
    out = _ops().csr2bsr(drp, dci, dv, m=n, n=n, bs=16)
    torch.cuda.synchronize()
    t = time.perf_counter() - t
    hb = prep.csr2bsr(n, n, rp, ci, v, 16)
    brp, bci = _host(out[0], out[1])
    assert np.array_equal(brp, hb[0]) and np.array_equal(bci, hb[1])
    assert torch.equal(out[2], torch.from_numpy(hb[2]).cuda())
    print(f"device csr2bsr products bs=16: {t * 1e3:.1f} ms")
