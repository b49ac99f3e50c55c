"""BASELINE.json configs 1, 2 and 4 on the HIP path, each on its own inputs
(SURVEY.md §8d table):

* config 1: the graph spmm.cc's baseline is quoted on — randomCSRMatrix(16384,
  16384, 2^-10) + randomDenseMatrix(16384, 32) from a fresh mt19937_64(1234),
  whose digests tests/golden/ref_config1.json took from the reference's own
  load_data.cc — run through the CSR kernel against the oracle, weighted and
  pattern-only (spmm.cc's unit values);
* config 2: the ogbn-arxiv stand-in (n = 169,343, nnz = 1,166,243), K = 128,
  every element against the f64 oracle;
* config 4: ogbn-products stand-in at K = 256, row-partitioned for 2 / 4 / 8
  ranks on this one device (dist.make_shard, each shard written in place into
  its rows of the contiguous C the exchange fills), bit-identical to the
  whole-matrix run and checked on sampled oracle rows; plus the
  native single-process multi-GPU entry (spmm_csr_f32_multi over
  ncclCommInitAll on this box's one GPU).
"""
from __future__ import annotations

import hashlib
import json
import os

import numpy as np
import pytest

from helpers import TOL_F32, assert_normwise, oracle_csrmm_f64, oracle_csrmm_pieces_f32

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _dev(*arrs):
    return [torch.from_numpy(np.ascontiguousarray(a)).cuda() for a in arrs]


def _sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def test_config1_graph_on_the_gpu(oracle, device):
    from spmm_hip import ops, prep
    d = json.load(open(os.path.join(GOLDEN, "ref_config1.json")))
    prep.rng_seed(1234)
    rp, ci, v = prep.random_csr(d["m"], d["n"], d["p"])
    B = prep.random_dense_matrix(d["m"], d["K"])
    # the inputs are the reference's, bit for bit
    assert ci.size == d["nnz"]
    assert (_sha(rp), _sha(ci), _sha(v), _sha(B)) == (
        d["rowptr_sha256"], d["colind_sha256"], d["val_sha256"], d["B_sha256"])
    drp, dci, dv, dB = _dev(rp, ci, v, B)
    C = ops.gespmm_csrmm(drp, dci, dv, dB)
    ones = torch.ones_like(dv)
    Cp = ops.gespmm_csrmm(drp, dci, ones, dB)  # spmm.cc's pattern-only product
    torch.cuda.synchronize()
    ref, absd = oracle_csrmm_f64(oracle, d["m"], d["K"], rp, ci, v, B, d["K"], 0)
    assert_normwise(C.cpu().numpy(), ref, absd, TOL_F32, "config 1 weighted")
    # spmm.cc csr_spmm (double accumulation, unit values): the oracle restatement
    ip64, ix64 = rp.astype(np.int64), ci.astype(np.int64)
    Bd = B.astype(np.float64)
    out = np.empty((d["m"], d["K"]))
    from helpers import ptr
    oracle.oracle_spmm_cc_csr(d["m"], d["K"], ptr(ip64), ptr(ix64), ptr(Bd), d["K"], ptr(out))
    absp, _ = oracle_csrmm_f64(oracle, d["m"], d["K"], rp, ci, np.ones_like(v), np.abs(B),
                               d["K"], 0)
    assert_normwise(Cp.cpu().numpy(), out, absp, TOL_F32, "config 1 spmm.cc pattern-only")


def test_config2_arxiv_size(oracle, device):
    from spmm_hip import ops, prep
    n, nnz, K = 169343, 1166243, 128
    rp, ci = prep.powerlaw_csr(n, nnz, 13161, 2.3, 1234)
    assert ci.size == nnz
    rng = np.random.default_rng(5)
    v = rng.uniform(-1, 1, nnz).astype(np.float32)
    B = rng.uniform(-1, 1, (n, K)).astype(np.float32)
    drp, dci, dv, dB = _dev(rp, ci, v, B)
    C = ops.gespmm_csrmm(drp, dci, dv, dB)
    C2 = ops.gespmm_csrmm(drp, dci, dv, dB)
    torch.cuda.synchronize()
    assert torch.equal(C, C2), "not deterministic"
    ref, absd = oracle_csrmm_f64(oracle, n, K, rp, ci, v, B, K, 0)
    got = C.cpu().numpy()
    assert_normwise(got, ref, absd, TOL_F32, "arxiv stand-in, every element")
    want = oracle_csrmm_pieces_f32(oracle, n, K, rp, ci, v, B, K, 0).reshape(n, K)
    assert np.array_equal(got, want), "arxiv stand-in: not bit-identical to the piece oracle"


@pytest.fixture(scope="module")
def products_k256():
    from spmm_hip import prep
    n, nnz, K = 2449029, 61859140, 256
    rp, ci = prep.powerlaw_csr(n, nnz, 17481, 2.3, 1234)
    v = np.random.default_rng(2).uniform(-1, 1, nnz).astype(np.float32)
    return rp, ci, v, K


def _sample_rows(rp, n, rng):
    deg = np.diff(rp)
    return np.unique(np.concatenate([rng.choice(n, 1500, replace=False), np.argsort(deg)[-20:]]))


def _oracle_rows(oracle, rp, ci, v, Bh, rows, K):
    deg = np.diff(rp)
    sub_rp = np.concatenate([[0], np.cumsum(deg[rows])]).astype(np.int32)
    sub_ci = np.concatenate([ci[rp[r]:rp[r + 1]] for r in rows]).astype(np.int32)
    sub_v = np.concatenate([v[rp[r]:rp[r + 1]] for r in rows]).astype(np.float32)
    return oracle_csrmm_f64(oracle, rows.size, K, sub_rp, sub_ci, sub_v, Bh, K, 0)


def test_config4_products_k256_row_shards(oracle, device, products_k256):
    from spmm_hip import dist as sdist
    from spmm_hip import ops
    rp, ci, v, K = products_k256
    n = rp.size - 1
    g = torch.Generator(device=device)
    g.manual_seed(1234)
    B = torch.rand((n, K), device=device, generator=g) * 2 - 1
    drp, dci, dv = _dev(rp, ci, v)
    Cw = torch.empty((n, K), device=device)
    ops.csrmm(drp, dci, dv, B, n=K, k=n, ldb=K, C=Cw, ldc=K)
    del drp, dci, dv
    rng = np.random.default_rng(8)
    rows = _sample_rows(rp, n, rng)
    Bh = B.cpu().numpy()
    ref, rabs = _oracle_rows(oracle, rp, ci, v, Bh, rows, K)
    torch.cuda.synchronize()
    assert_normwise(Cw.cpu().numpy()[rows], ref, rabs, TOL_F32, "products K=256 whole matrix")
    for world in (2, 4, 8):
        shards = [sdist.make_shard(rp, ci, v, r, world) for r in range(world)]
        # the contiguous C the exchange fills: rank r's rows written in place
        # by the kernel, at their global rows
        C = torch.full((n, K), float("nan"), device=device)
        for sh in shards:
            srp, sci, sv = _dev(sh.rowptr, sh.colind, sh.val)
            ops.csrmm(srp, sci, sv, B, m=sh.rows, n=K, k=n, ldb=K, C=C[sh.row0:sh.row1], ldc=K)
        torch.cuda.synchronize()
        assert C.shape == Cw.shape
        assert torch.equal(C, Cw), f"world {world}: not bit-identical to the whole matrix"
        assert_normwise(C.cpu().numpy()[rows], ref, rabs, TOL_F32, f"world {world} sampled rows")
        assert [sh.rows for sh in shards] == list(np.diff(shards[0].bounds))


@pytest.mark.parametrize("chunks", [1, 4])
def test_config4_native_multi_entry(oracle, device, products_k256, chunks):
    """spmm_csr_f32_multi (include/spmm_multi.h) over ncclCommInitAll on this
    box's one GPU: the chunks' kernels write straight into the n x K C and
    run the per-chunk event chain of P > 1 (a one-part call has no peer to
    exchange with). Any chunking is bit-identical to the whole-matrix call
    (pieces: the association is the row's). The output is C itself: nothing
    past row n is written."""
    from spmm_hip import ops, prep
    rp, ci, v, K = products_k256
    n = rp.size - 1
    g = torch.Generator(device=device)
    g.manual_seed(77)
    B = torch.rand((n, K), device=device, generator=g) * 2 - 1
    drp, dci, dv = _dev(rp, ci, v)
    Cw = torch.empty((n, K), device=device)
    ops.csrmm(drp, dci, dv, B, n=K, k=n, ldb=K, C=Cw, ldc=K)
    mg = ops.MultiGPU([device.index or 0])
    bounds = prep.partition_rows(rp, 1)
    Cm = torch.full((n + 1, K), float("nan"), device=device)
    mg.set_timing(True)
    mg.csrmm(bounds, [(drp, dci, dv)], [ci.size], [B], [Cm[:n]], m=n, n=K, k=n, ldb=K, ldc=K,
             chunks=chunks)
    mg.synchronize()
    comp, tot = mg.times()
    assert 0 < comp[0] <= tot[0]
    torch.cuda.synchronize()
    assert bool(torch.isnan(Cm[n]).all())
    assert torch.equal(Cm[:n], Cw)
    mg.close()


def test_config4_native_multi_checks_outputs(device):
    """MultiGPU.csrmm refuses a C shorter than m x n (ldc) and a tensor on
    another device before anything is launched (the kernel and the exchange
    would write past a short C)."""
    from spmm_hip import ops
    mg = ops.MultiGPU([device.index or 0])
    rp = torch.tensor([0, 1, 2], dtype=torch.int32, device=device)
    ci = torch.tensor([0, 1], dtype=torch.int32, device=device)
    v = torch.ones(2, device=device)
    B = torch.ones((2, 8), device=device)
    short = torch.empty((1, 8), device=device)  # m x n = 2 x 8 needed
    with pytest.raises(ValueError, match="m x n output"):
        mg.csrmm([0, 2], [(rp, ci, v)], [2], [B], [short], m=2, n=8, k=2, ldb=8, ldc=8,
                 chunks=4)
    with pytest.raises(ValueError, match="HIP device"):
        mg.csrmm([0, 2], [(rp, ci, v)], [2], [B.cpu()], [short], m=2, n=8, k=2, ldb=8, ldc=8)
    ok = torch.empty((2, 8), device=device)
    mg.csrmm([0, 2], [(rp, ci, v)], [2], [B], [ok], m=2, n=8, k=2, ldb=8, ldc=8)
    torch.cuda.synchronize()  # ordered on the current stream: no explicit mg.synchronize()
    assert torch.equal(ok, torch.ones((2, 8), device=device))
    mg.close()


def test_config4_native_multi_orders_against_default_stream(device):
    """MultiGPU.csrmm on torch's legacy default stream (cuda_stream == 0, the
    NULL entry of spmm_multi_set_user_streams): the kernels start after a slow
    producer of B queued there, and a copy of C queued there afterwards sees the
    finished all-gather. No device-wide synchronize between the three: the
    copy to the host waits for the default stream alone."""
    from spmm_hip import ops
    torch.cuda.set_stream(torch.cuda.default_stream(device))
    assert torch.cuda.current_stream(device).cuda_stream == 0
    m, K = 4096, 64
    rp = torch.arange(0, 2 * m + 1, 2, dtype=torch.int32, device=device)  # 2 nnz per row
    ci = (torch.arange(2 * m, dtype=torch.int32, device=device) * 7) % m
    v = torch.ones(2 * m, device=device)
    B = torch.zeros((m, K), device=device)
    C = torch.zeros((m, K), device=device)
    mg = ops.MultiGPU([device.index or 0])
    torch.cuda.synchronize()
    for rep in range(2):  # the ordering holds on every call, not only the first
        torch.cuda._sleep(100_000_000)  # ~40-50 ms of spinning on the default stream
        B.fill_(3.0 + rep)              # the producer of B, behind it
        mg.csrmm([0, m], [(rp, ci, v)], [2 * m], [B], [C], m=m, n=K, k=m, ldb=K, ldc=K,
                 chunks=2)
        got = C[:m].cpu()  # queued on the default stream after the call
        assert bool((got == 2 * (3.0 + rep)).all()), f"call {rep}: C read before the product"
    mg.close()


def test_config4_torch_distributed_world1(tmp_path):
    """bench.py's N > 1 path through RCCL on this one GPU: a fresh child
    process initialises torch.distributed (nccl backend) at world 1 before any
    GPU call, then partitioned_spmm (chunks = 1, bit-identical to the
    whole-matrix kernel) and chunked_spmm with 4 chunks (within the fp32 bar),
    both into the contiguous n x K C, and a max-over-ranks all_reduce."""
    import subprocess
    import sys
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT="29541", RANK="0",
               LOCAL_RANK="0", WORLD_SIZE="1", HSA_ENABLE_IPC_MODE_LEGACY="0")
    child = os.path.join(os.path.dirname(os.path.abspath(__file__)), "dist_world1_child.py")
    r = subprocess.run([sys.executable, "-u", child], env=env, capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    res = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    print(res)
    assert res["backend"] == "nccl" and res["world"] == 1
    assert res["chunks1_bit_identical"]
    assert res["chunks4_within_bar"] and res["chunks4_no_nan"], res
    assert res["chunks4_bit_identical"], res
    assert res["exchange_requests_world1"] == 0 and res["allreduce_max_ok"]
