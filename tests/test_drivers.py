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


def _run(args, cwd, timeout=300):
    exe = os.path.join(BIN, args[0])
    if not os.path.exists(exe):
        pytest.fail(f"{exe} not built (make -C spmm-denseblock_amd all)")
    r = subprocess.run([exe] + [str(a) for a in args[1:]], cwd=cwd, capture_output=True,
                       text=True, timeout=timeout)
    assert r.returncode == 0, r.stdout + r.stderr
    return r.stdout


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
    from spmm_hip import prep
    rp, ci = prep.powerlaw_csr(20000, 200000, 500, 2.3, 5)
    os.makedirs(tmp_path / "tmp", exist_ok=True)
    prep.dump_csr(str(tmp_path / "tmp" / "pl"), rp, ci)
    out = _run(["run_csrmm", "pl", 64, impl, tb], tmp_path)
    assert "n=20000 nnz=200000" in out and "average csrmm cost time" in out
    assert out.rstrip().endswith("end")


@pytest.mark.gpu
@pytest.mark.parametrize("impl", ["rocsparse", "cusparse"])
def test_run_bsrmm_cli(tmp_path, impl):
    from spmm_hip import prep
    rp, ci = prep.community_csr(8000, 40.0, 64, 256, 0.9, 3)
    os.makedirs(tmp_path / "tmp", exist_ok=True)
    prep.dump_csr(str(tmp_path / "tmp" / "cm"), rp, ci)
    out = _run(["run_bsrmm", "cm", 32, 64, impl], tmp_path)
    assert f"nnz={ci.size}" in out and "bsrmm cost time" in out
    assert out.rstrip().endswith("end")


@pytest.mark.gpu
def test_test_bsrmm_cli(tmp_path):
    out = _run(["test_bsrmm", 0.002, 32, 64, "rocsparse", 0], tmp_path)
    assert "GFLOPs" in out and out.rstrip().endswith("end")
