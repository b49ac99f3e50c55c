"""Run the case round 3's sc1 store form failed (test_reference_generator_bsr_on_mfma
[32-0.05-128], profiles/r03_sc1_store_tests.log) on a given libspmm_hip.so,
with C pre-filled two ways, and print what the wrong elements hold.

  python tools/sc1_run.py <libspmm_hip.so> [reps]

A store that never happened leaves the pre-fill (NaN, or the 0x00000D80
sentinel = 4.8e-42, the value round 3 saw); a store whose data registers were
overwritten before it read them writes some other value. One JSON line per
pre-fill. (A tool: tests/ and the product load the in-tree library only.)
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "spmm-denseblock_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main() -> None:
    from spmm_hip import _lib
    _lib.LIB_PATH = os.path.abspath(sys.argv[1])
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    import torch
    from helpers import load_oracle, oracle_bsrmm_f64
    from spmm_hip import ops, prep
    oracle = load_oracle()
    bs, p, n = 32, 0.05, 128
    mb = 4096 // bs
    prep.rng_seed(1234)
    rp, ci, v = prep.random_bsr(mb, mb, bs, p)
    B = prep.random_dense_matrix(mb * bs, n)
    dev = torch.device("cuda", 0)
    drp, dci, dv, dB = (torch.from_numpy(np.ascontiguousarray(a)).to(dev) for a in (rp, ci, v, B))
    ref, absd = oracle_bsrmm_f64(oracle, 0, mb, n, bs, rp, ci, v, B, n, 0)
    for name, fill in (("nan", float("nan")), ("sentinel_0xD80", None)):
        bad_total, kinds = 0, {}
        for _ in range(reps):
            C = torch.empty((mb * bs, n), dtype=torch.float32, device=dev)
            if fill is None:
                C.view(torch.int32).fill_(0xD80)
            else:
                C.fill_(fill)
            ops.bsrmm(drp, dci, dv, dB, mb=mb, kb=mb, n=n, bs=bs, ldb=n, C=C, ldc=n)
            torch.cuda.synchronize()
            got = C.cpu().numpy().astype(np.float64)
            bad = ~(np.abs(got - ref) <= 1e-5 * absd + 1e-30)
            bad_total += int(bad.sum())
            for x in C.cpu().numpy()[bad][:64]:
                k = "prefill" if (np.isnan(x) if fill is not None else x.view(np.int32) == 0xD80) \
                    else "other"
                kinds[k] = kinds.get(k, 0) + 1
            rows = np.unique(np.nonzero(bad)[0] % bs)
        print(json.dumps({"lib": sys.argv[1], "prefill": name, "reps": reps,
                          "wrong_elements": bad_total, "wrong_kinds_sampled": kinds,
                          "rows_in_block_of_wrong": rows.tolist()[:32]}), flush=True)


if __name__ == "__main__":
    main()
