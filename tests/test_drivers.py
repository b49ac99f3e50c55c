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
@pytest.mark.parametrize("impl,tb", [("gespmm", 0), ("gespmm_hot", 0), ("cusparseScsrmm", 0),
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
    if impl == "gespmm_hot":
        assert "hot-column analysis time" in out
    prep.rng_seed(1234)
    B = prep.random_dense_matrix(20000, 64)
    _check_dump(dump, rp, ci, B, f"run_csrmm {impl}")


@pytest.mark.gpu
@pytest.mark.parametrize("chunks", [1, 3])
def test_run_csrmm_multi_gpu_cli(tmp_path, chunks):
    """--gpus 1 (single-process RCCL, ncclCommInitAll over this box's one
    GPU), one and three chunks, against the oracle and the single-GPU run.
    (The gespmm entry sizes its grid without nnz, the multi entry with it, so
    rows split by a merge-path wave boundary may associate differently; the
    bit-identity of the multi entry with spmm_csrmm_ex_f32 is asserted in
    test_gpu_configs.py.)"""
    from spmm_hip import prep
    rp, ci = prep.powerlaw_csr(20000, 200000, 500, 2.3, 5)
    os.makedirs(tmp_path / "tmp", exist_ok=True)
    prep.dump_csr(str(tmp_path / "tmp" / "pl"), rp, ci)
    one, multi = str(tmp_path / "C1.bin"), str(tmp_path / "Cm.bin")
    _run(["run_csrmm", "pl", 64, "gespmm", 0], tmp_path, env={"SPMM_DRIVER_DUMP": one})
    out = _run(["run_csrmm", "pl", 64, "gespmm", 0, "--gpus", 1, "--chunks", chunks], tmp_path,
               env={"SPMM_DRIVER_DUMP": multi})
    assert f"multi-GPU: ngpu=1 chunks={chunks}" in out and "compute + exchange" in out
    assert out.rstrip().endswith("end")
    prep.rng_seed(1234)
    B = prep.random_dense_matrix(20000, 64)
    got = _check_dump(multi, rp, ci, B, f"run_csrmm --gpus 1 --chunks {chunks}")
    ref = np.fromfile(one, dtype=np.float32).reshape(got.shape)
    assert np.mean(got == ref) > 0.9  # unsplit rows: the same FMA chain


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


@pytest.mark.gpu
@pytest.mark.parametrize("p", [0.01, 0.1])
def test_csr2bsr_differential_program(tmp_path, p):
    """csr2bsr.cu (:87-311) reproduced: randomCSRMatrix(1000, 1200, p) and
    randomDenseMatrix(1200, 100) from the seeded generator, device csr2bsr
    (bs = 2), csrmm vs bsrmm with the reference's |delta| <= 0.01 verdict;
    the bsrmm result also against the f64 oracle."""
    from helpers import TOL_F32, assert_normwise, load_oracle, oracle_csrmm_f64
    from spmm_hip import prep
    dump = str(tmp_path / "z2.bin")
    out = _run(["csr2bsr_check", p], tmp_path, env={"SPMM_DRIVER_DUMP": dump})
    assert "\nsame result" in out and out.rstrip().endswith("end")
    prep.rng_seed(1234)
    rp, ci, v = prep.random_csr(1000, 1200, p)
    y = prep.random_dense_matrix(1200, 100).reshape(-1)
    B = np.ascontiguousarray(y.reshape(100, 1200).T)  # column-major, ldb = n
    got = np.fromfile(dump, dtype=np.float32).reshape(1000, 100)
    ref, absd = oracle_csrmm_f64(load_oracle(), 1000, 100, rp, ci, v, B, 100, 0)
    assert_normwise(got, ref, absd, TOL_F32, f"csr2bsr.cu p={p}")


@pytest.mark.gpu
@pytest.mark.parametrize("p,bs", [(0.01, 4), (0.05, 16), (0.02, 32)])
def test_bsr2csr_differential_program(tmp_path, p, bs):
    """bsr2csr.cu (:90-311) reproduced: randomBSRMatrix(4096/bs, 4096/bs, bs,
    p) (the reference's generator) and randomDenseMatrix(4096, 100), device
    bsr2csr, bsrmm vs csrmm with its |delta| <= 0.05 verdict; bsrmm against
    the f64 oracle."""
    from helpers import TOL_F32, assert_normwise, load_oracle, oracle_bsrmm_f64
    from spmm_hip import prep
    dump = str(tmp_path / "z2.bin")
    out = _run(["bsr2csr_check", p, bs], tmp_path, env={"SPMM_DRIVER_DUMP": dump})
    assert "\nsame result" in out and out.rstrip().endswith("end")
    mb = 4096 // bs
    prep.rng_seed(1234)
    brp, bci, bval = prep.random_bsr(mb, mb, bs, p)
    y = prep.random_dense_matrix(4096, 100).reshape(-1)
    B = np.ascontiguousarray(y.reshape(100, 4096).T)
    got = np.fromfile(dump, dtype=np.float32).reshape(4096, 100)
    ref, absd = oracle_bsrmm_f64(load_oracle(), 0, mb, 100, bs, brp, bci, bval, B, 100, 0)
    assert_normwise(got, ref, absd, TOL_F32, f"bsr2csr.cu p={p} bs={bs}")


def _kat_problems(kats) -> tuple[str, list]:
    """The known-answer programs as compat_kat input, with expected outputs."""
    lines, want = [], []

    def j(xs):
        return " ".join(str(x) for x in xs)
    for name in ("csrmm_cu", "try_cublas_cu"):
        k = kats[name]
        m, kk, n = k["m"], k["k"], k["n"]
        B = np.array(k["B_colmajor"], float).reshape(n, kk).T  # -> row-major k x n
        lines.append(f"csr {m} {kk} {n} {len(k['colind'])} {j(k['rowptr'])} {j(k['colind'])} "
                     f"{j(k['val'])} {j(B.reshape(-1).tolist())}")
        want.append(np.array(k["C_colmajor"], float).reshape(n, m).T.reshape(-1))
    k = kats["bsrmm_cu"]
    lines.append(f"bsr {k['dir']} 0 {k['mb']} {k['kb']} {k['n']} {k['bs']} {len(k['colind'])} "
                 f"{k['ldb']} {k['ldc']} 0 {j(k['rowptr'])} {j(k['colind'])} {j(k['val'])} "
                 f"{j(k['B_colmajor'])}")
    want.append(np.array(k["C_colmajor"], float))
    k = kats["block_cublas_cu"]
    lines.append(f"bsr {k['dir']} 1 {k['mb']} {k['kb']} {k['n']} {k['bs']} {len(k['colind'])} "
                 f"{k['ldb']} {k['ldc']} {k['beta']} {j(k['rowptr'])} {j(k['colind'])} "
                 f"{j(k['val'])} {j(k['B_rowmajor'])}")
    want.append(np.array(k["C_colmajor"], float))
    return "\n".join(lines) + "\n", want


@pytest.mark.gpu
@pytest.mark.parametrize("T", ["float", "double"])
def test_compat_header_drivers_on_the_kats(golden, T):
    """Driver code written against the reference's call shapes
    (gespmm_csrmm<T>, rocsparse_bsrmm_template<T>, through spmm_compat.hpp)
    reproduces the known-answer programs exactly."""
    text, want = _kat_problems(golden["kats"])
    exe = os.path.join(BIN, "compat_kat")
    r = subprocess.run([exe, T], input=text, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    got = [np.array([float(x) for x in l.split()[1:]]) for l in r.stdout.splitlines()
           if l.startswith("C")]
    assert len(got) == len(want)
    for g, w in zip(got, want):
        assert np.array_equal(g, w), (g, w)
    assert r.stdout.count("status SPMM_STATUS_SUCCESS") == 2


@pytest.mark.gpu
@pytest.mark.parametrize("impl,tb,n", [("rocsparse", 0, 8000), ("cusparse", 1, 8000),
                                       ("hybrid", 0, 8000), ("hybrid", 1, 7990),
                                       ("rocsparse", 0, 7990)])
def test_divide_cli(tmp_path, impl, tb, n):
    """divide.cu:195-378 reproduced: divide_matrix at density 0.05, then
    csrmm2 + bsrmm (or the library's hybrid call) accumulating into the
    column-major z with alpha = beta = 1, transB N (y column-major) or T (y
    row-major); its lines, and z against the f64 oracle of the whole
    unit-valued product. n = 7990 is not a multiple of bs = 32 (the driver
    then reads y with ldb = n1, printed)."""
    from spmm_hip import prep
    rp, ci = prep.community_csr(n, 40.0, 64, 256, 0.9, 3)
    os.makedirs(tmp_path / "tmp", exist_ok=True)
    prep.dump_csr(str(tmp_path / "tmp" / "cm"), rp, ci)
    dump = str(tmp_path / "C.bin")
    dim, bs = 64, 32
    out = _run(["divide", "cm", bs, dim, impl, tb, 0.05], tmp_path,
               env={"SPMM_DRIVER_DUMP": dump})
    assert "csr nnz = " in out and "bsr nnzb = " in out and out.rstrip().endswith("end")
    assert ("hybrid cost time" in out) if impl == "hybrid" else (
        "csrmm cost time" in out and "bsrmm cost time" in out and "total cost time" in out)
    nb = (n + bs - 1) // bs
    n1 = nb * bs
    # the split itself: divide_matrix's counts (host restatement, bit-exact with divide.cu)
    _, _, _, brp, _, _ = prep.divide(n, rp, ci, np.ones(ci.size, np.float32), bs, 0.05)
    csr_nnz = int(out.split("csr nnz = ")[1].split()[0])
    assert int(out.split("bsr nnzb = ")[1].split()[0]) == int(brp[-1]) and csr_nnz < ci.size
    prep.rng_seed(1234)
    y = prep.random_dense_matrix(n1, dim).reshape(-1)
    if tb == 1:
        B = y.reshape(n1, dim)  # row-major, ldb = dim
    else:
        ldb = n1 if n1 != n else n
        assert ("note: ldb = n1" in out) == (n1 != n)
        B = np.ascontiguousarray(y[:ldb * dim].reshape(dim, ldb).T)  # column-major
    _check_dump(dump, rp, ci, B, f"divide {impl} transB={tb} n={n}")
