"""bench.py helpers that need no GPU: the BSR workloads' PMC traffic lookup
(profiles/r02_pmc_bytes/bytes.jsonl) and the reorder-in-the-loop
graph builder on a small community graph."""
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


def test_bsr_traffic_lookup_matches_the_committed_records():
    b = _bench()
    recs = [json.loads(line) for line in open(b.BSR_TRAFFIC)]
    assert recs, "committed PMC byte records"
    for wl, kern in {(r["workload"], r["kernel"]) for r in recs}:
        want = [r for r in recs if r["workload"] == wl and r["kernel"] == kern][-1]
        got = b.bsr_traffic(wl, kern)
        assert got == want["counter_bytes_per_launch"] and got > 0
        # FETCH_SIZE x calibration + WRITE_SIZE (MI355X_MICROARCH.md HBM recipe)
        assert abs(want["fetch_size_bytes_raw"] * want["fetch_correction"] +
                   want["write_size_bytes"] - got) < 1e-3 * got
    assert b.bsr_traffic("no_such_workload", "bsr32_f32_cs2_kernel") is None


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
