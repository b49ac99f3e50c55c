"""bench.py helpers that need no GPU: the --gpus N launch path, the BSR workloads' PMC traffic lookup
(profiles/r03_pmc_bytes/bytes.jsonl), the CSR roofline rule,
the CPU-baseline timing helpers and the reorder-in-the-loop graph builder
 on a small community graph."""
from __future__ import annotations

import importlib.util
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    saved = sys.argv
    sys.argv = ["bench.py"]
    try:
        spec.loader.exec_module(mod)
    finally:
        sys.argv = saved
    return mod


KEY = {"workload": "products_bsr16_f16", "kernel": "bsr16_f16_cs_kernel", "K": 512,
       "dtype": "fp16", "nnzb": 5040000, "layout_BC": "row", "variant": "default",
       "kernel_src": "0123456789abcdef"}


def test_bsr_traffic_lookup_needs_every_key(tmp_path, monkeypatch):
    """Counter bytes are used only for the exact workload, kernel, K, dtype,
    nnzb, variant and kernel build they were measured on (a
    --K 256 run must not divide K = 512 bytes by its own time)."""
    b = _bench()
    f = tmp_path / "bytes.jsonl"
    recs = [dict(KEY, counter_bytes_per_launch=111), dict(KEY, K=256, counter_bytes_per_launch=222),
            dict(KEY, counter_bytes_per_launch=333)]  # the last matching record wins
    f.write_text("".join(json.dumps(r) + "\n" for r in recs))
    monkeypatch.setattr(b, "BSR_TRAFFIC", str(f))
    assert b.bsr_traffic(KEY) == 333
    assert b.bsr_traffic(dict(KEY, K=256)) == 222
    for k, v in (("K", 128), ("dtype", "fp32"), ("nnzb", 1), ("variant", "6104"),
                 ("kernel_src", "fedcba9876543210"), ("layout_BC", "col"),
                 ("workload", "products_rcm_bsr16_f16")):
        assert b.bsr_traffic(dict(KEY, **{k: v})) is None, k
    monkeypatch.setattr(b, "BSR_TRAFFIC", str(tmp_path / "missing.jsonl"))
    assert b.bsr_traffic(KEY) is None


def test_committed_traffic_records_are_consistent():
    """Every committed record carries the full lookup key and its counter
    bytes are FETCH_SIZE x calibration + WRITE_SIZE (MI355X_MICROARCH.md HBM
    recipe)."""
    b = _bench()
    if not os.path.exists(b.BSR_TRAFFIC):
        return
    for line in open(b.BSR_TRAFFIC):
        r = json.loads(line)
        assert {"workload", "kernel", "K", "dtype", "nnzb", "variant", "kernel_src"} <= set(r)
        got = r["counter_bytes_per_launch"]
        assert got > 0
        assert abs(r["fetch_size_bytes_raw"] * r["fetch_correction"] +
                   r["write_size_bytes"] - got) < 1e-3 * got


def test_csr_roofline_never_above_the_peak():
    b = _bench()
    ci = np.random.default_rng(0).integers(0, 1000, 50000).astype(np.int32)
    # a slow launch: the gather model
    r = b.csr_roofline(1000, ci, 128, 10.0)
    assert r["bytes_model"].startswith("SURVEY") and r["frac"] <= 1
    assert r["algorithmic_bytes_per_launch"] == b.csr_bytes(1000, ci.size, 128)
    # a launch faster than the gather model allows (B cache-resident): compulsory bytes
    r = b.csr_roofline(1000, ci, 128, 1e-4)
    assert r["bytes_model"].startswith("compulsory")
    assert r["algorithmic_bytes_per_launch"] == 4 * 1001 + 8 * ci.size + 4 * 128 * 1000 * 2
    assert r["gather_model_GBps"] > b.HBM_PEAK_GBPS


def test_batched_samples_and_spread():
    b = _bench()
    calls = []
    reps, ts = b._batched_samples(lambda: calls.append(1), min_sample_s=0.001, nsamples=5)
    # warm-up, a calibration loop of >= min_sample_s, then 1 + nsamples samples of reps calls
    calib = len(calls) - 1 - 6 * reps
    assert len(ts) == 5 and reps >= 1 and calib >= 1
    sp = b._spread([1.0, 2.0, 3.0])
    assert sp["median_s"] == 2.0 and sp["spread"] == 1.0


def test_community_graph_reorder_record():
    b = _bench()
    W = dict(n=6000, avg_deg=40.0, cmin=64, cmax=256, p_in=0.97, reorder="rcm")
    rp, ci, rec, data = b.community_graph(W, 32)
    assert rp.size == 6001 and ci.size == rp[-1]
    assert rec["method"] == "rcm" and "scrambled" in data
    # scrambling destroys the blocking; RCM recovers part of it, never more than the
    # generator's community order (the upper bound the record keeps beside it)
    assert rec["nnzb_scrambled"] > rec["nnzb_reordered"] >= rec["community_order_upper_bound"]["nnzb"]
    W2 = dict(W)
    W2.pop("reorder")
    rp2, ci2, rec2, data2 = b.community_graph(W2, 32)
    assert rec2 is None and "community-ordered" in data2
    # the reordered graph is a relabelling of the same graph: same degree multiset
    assert np.array_equal(np.sort(np.diff(rp)), np.sort(np.diff(rp2)))


def test_gpus_n_without_launcher_starts_ranks_or_fails():
    """`bench.py --gpus N` (N > 1) with no torch.distributed launcher starts N
    ranks as a child torch.distributed.run of the same command line (the
    driver's form, rendezvous on 127.0.0.1); with fewer than N GPUs visible
    (this container has none) it exits 2 with no JSON line, so no line ever
    reports n_gpus != --gpus."""
    import subprocess
    b = _bench()
    argv = b.launch_argv(["--gpus", "8", "--steps", "3"], 8, 29577)
    assert argv[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in argv and "--nnodes=1" in argv
    assert argv[argv.index("--master-addr") + 1] == "127.0.0.1"
    assert argv[argv.index("--master-port") + 1] == "29577"
    assert argv[-4:] == ["--gpus", "8", "--steps", "3"]
    assert argv[-5] == os.path.join(ROOT, "bench.py")
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 2, r.stderr[-2000:]
    assert "--gpus 2 but 0 GPU(s) visible" in r.stderr
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    # under a launcher, --gpus must equal WORLD_SIZE (before any GPU call)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1"],
                       env=dict(env, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0"),
                       capture_output=True, text=True, timeout=300)
    assert r.returncode != 0 and "--gpus 1 but WORLD_SIZE=2" in r.stderr
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
