"""The reference-compatible drivers (spmm-denseblock_amd/bin/*): same CLIs,
same files, same stdout lines. CPU drivers run everywhere; the HIP drivers
are `gpu`-marked and check their result lines on a real device."""
from __future__ import annotations

import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT

BIN = os.path.join(ROOT, "spmm-denseblock_amd", "bin")


def _run(args, cwd, timeout=300, env=None):
    exe = os.path.join(BIN, args[0])
    if not os.path.exists(exe):
        pytest.fail(f"{exe} not built (make -C spmm-denseblock_amd all)")
    r = subprocess.run([exe] + [str(a) for a in args[1:]], cwd=cwd, capture_output=True,
                       text=True, timeout=timeout,
                       env=None if env is None else {**os.environ, **env})
    assert r.returncode == 0, r.stdout + r.stderr
    return r.stdout


def _check_dump(path, rp, ci, B, what):
    """The driver's C (SPMM_DRIVER_DUMP, row-major) against the f64 oracle of
    the same product (unit values, B = the driver's randomDenseMatrix)."""
    from helpers import TOL_F32, assert_normwise, load_oracle, oracle_csrmm_f64
    n, K = rp.size - 1, B.shape[1]
    got = np.fromfile(path, dtype=np.float32).reshape(n, K)
    ref, absd = oracle_csrmm_f64(load_oracle(), n, K, rp, ci, np.ones(ci.size, np.float32),
                                 np.ascontiguousarray(B[:n]), K, 0)
    assert_normwise(got, ref, absd, TOL_F32, what)
    return got


def _edge_list(tmp_path, name, rp, ci):
    os.makedirs(tmp_path / "tmp", exist_ok=True)
    n = rp.size - 1
    rows = np.repeat(np.arange(n), np.diff(rp))
    with open(tmp_path / "tmp" / f"{name}.txt", "w") as f:
        f.write(f"{n} {ci.size}\n")
        f.write("".join(f"{a} {b}\n" for a, b in zip(rows, ci)))


def test_spmm_cpu_small_kat(tmp_path):
    out = _run(["spmm_cpu", 2048, 0.005, 8, 1], tmp_path)
    assert "small csr_spmm: [[4,6,7],[8,17,3]]" in out  # spmm.cc:45-52
    assert "small coo_spmm: [[4,6,7],[8,17,3]]" in out  # spmm.cc:54-61
    line = next(x for x in out.splitlines() if x.startswith("coo GFLOP/s"))
    assert float(line.split("=")[-1]) <= 1e-12  # coo and csr agree


def test_reorder_graph_cli(tmp_path):
    """reorder_graph.cc:26-48: original + rcmk CSR files, metrics, heatmaps;
    the rcmk files equal the library's (and so the reference's) RCM order."""
    from helpers import load_reorder_golden
    from spmm_hip import prep
    g = load_reorder_golden()
    rp, ci = g["comm1500_rowptr"], g["comm1500_colind"]
    _edge_list(tmp_path, "comm", rp, ci)
    out = _run(["reorder_graph", "comm"], tmp_path).splitlines()
    assert out[0] == "dataset=comm" and out[1] == f"n=1500 nnz={ci.size}"
    # the original order's metric lines are exactly the reference's text
    assert "\n".join(out[2:8]) + "\n" == str(g["comm1500_metrics_text"])
    r2, c2 = prep.load_csr(str(tmp_path / "tmp" / "comm_rcmk"))
    assert np.array_equal(r2, g["comm1500_rcm_rowptr"])
    assert np.array_equal(c2, g["comm1500_rcm_colind"])
    r0, c0 = prep.load_csr(str(tmp_path / "tmp" / "comm_original"))
    assert np.array_equal(r0, rp) and np.array_equal(c0, ci)
    heat = (tmp_path / "tmp" / "comm_original_heatmap.txt").read_text().splitlines()
    assert heat[0] == "6" and len(heat) == 7  # ceil(1500 / 256) blocks
    assert sum(int(x) for line in heat[1:] for x in line.split()) == ci.size


def test_rabbit_reorder_cli(tmp_path):
    from helpers import load_reorder_golden
    from spmm_hip import prep
    g = load_reorder_golden()
    rp, ci, perm = g["pl2000_rowptr"], g["pl2000_colind"], g["pl2000_perm"]
    _edge_list(tmp_path, "pl", rp, ci)
    prep.dump_permutation(str(tmp_path / "tmp" / "pl_rabbit.txt"), perm)
    _run(["rabbit_reorder", "pl"], tmp_path)
    r2, c2 = prep.load_csr(str(tmp_path / "tmp" / "pl_rabbit"))
    assert np.array_equal(r2, g["pl2000_permute_rowptr"])
    assert np.array_equal(c2, g["pl2000_permute_colind"])


@pytest.mark.gpu
@pytest.mark.parametrize("impl,tb", [("gespmm", 0), ("cusparseScsrmm", 0),
                                     ("cusparseScsrmm2", 1)])
def test_run_csrmm_cli(tmp_path, impl, tb):
    """run_csrmm.cu:46-171's CLI and lines, and its C checked against the
    oracle (B = randomDenseMatrix(n, dim) from the seeded generator)."""
    from spmm_hip import prep
    rp, ci = prep.powerlaw_csr(20000, 200000, 500, 2.3, 5)
    os.makedirs(tmp_path / "tmp", exist_ok=True)
    prep.dump_csr(str(tmp_path / "tmp" / "pl"), rp, ci)
    dump = str(tmp_path / "C.bin")
    out = _run(["run_csrmm", "pl", 64, impl, tb], tmp_path, env={"SPMM_DRIVER_DUMP": dump})
    assert "n=20000 nnz=200000" in out and "average csrmm cost time" in out
    assert out.rstrip().endswith("end")
    prep.rng_seed(1234)
    B = prep.random_dense_matrix(20000, 64)
    _check_dump(dump, rp, ci, B, f"run_csrmm {impl}")


@pytest.mark.gpu
@pytest.mark.parametrize("chunks", [1, 3])
def test_run_csrmm_multi_gpu_cli(tmp_path, chunks):
    """--gpus 1 (single-process RCCL, ncclCommInitAll over this box's one
    GPU): with one chunk the same kernel on the same rows, so C is
    bit-identical to the single-GPU run; with 3 chunks within the fp32 bar."""
    from spmm_hip import prep
    rp, ci = prep.powerlaw_csr(20000, 200000, 500, 2.3, 5)
    os.makedirs(tmp_path / "tmp", exist_ok=True)
    prep.dump_csr(str(tmp_path / "tmp" / "pl"), rp, ci)
    one, multi = str(tmp_path / "C1.bin"), str(tmp_path / "Cm.bin")
    _run(["run_csrmm", "pl", 64, "gespmm", 0], tmp_path, env={"SPMM_DRIVER_DUMP": one})
    out = _run(["run_csrmm", "pl", 64, "gespmm", 0, "--gpus", 1, "--chunks", chunks], tmp_path,
               env={"SPMM_DRIVER_DUMP": multi})
    assert f"multi-GPU: ngpu=1 chunks={chunks}" in out and "compute + all-gather" in out
    assert out.rstrip().endswith("end")
    prep.rng_seed(1234)
    B = prep.random_dense_matrix(20000, 64)
    got = _check_dump(multi, rp, ci, B, f"run_csrmm --gpus 1 --chunks {chunks}")
    if chunks == 1:
        ref = np.fromfile(one, dtype=np.float32).reshape(got.shape)
        assert np.array_equal(got, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("impl", ["rocsparse", "cusparse"])
def test_run_bsrmm_cli(tmp_path, impl):
    from spmm_hip import prep
    rp, ci = prep.community_csr(8000, 40.0, 64, 256, 0.9, 3)
    os.makedirs(tmp_path / "tmp", exist_ok=True)
    prep.dump_csr(str(tmp_path / "tmp" / "cm"), rp, ci)
    dump = str(tmp_path / "C.bin")
    out = _run(["run_bsrmm", "cm", 32, 64, impl], tmp_path, env={"SPMM_DRIVER_DUMP": dump})
    assert f"nnz={ci.size}" in out and "bsrmm cost time" in out
    assert out.rstrip().endswith("end")
    # y = randomDenseMatrix(nb*bs, dim) read column-major with ldb = nb*bs
    n, bs, dim = rp.size - 1, 32, 64
    nbs = (n + bs - 1) // bs * bs
    prep.rng_seed(1234)
    y = prep.random_dense_matrix(nbs, dim).reshape(-1)
    B = y.reshape(dim, nbs).T  # column-major nbs x dim
    _check_dump(dump, rp, ci, B, f"run_bsrmm {impl}")


@pytest.mark.gpu
def test_test_bsrmm_cli(tmp_path):
    out = _run(["test_bsrmm", 0.002, 32, 64, "rocsparse", 0], tmp_path)
    assert "GFLOPs" in out and out.rstrip().endswith("end")
