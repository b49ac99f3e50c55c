#!/bin/bash
# Hybrid timings with and without SPMM_HYBRID_SPLIT_BF16 (HOPTS), two workloads,
# one JSON line per run into gpurun_out/hsplit.jsonl.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; : > gpurun_out/hsplit.jsonl
for wl in products_hybrid32 reddit_hybrid32; do for o in ${HOPTS:-0 4 2 6 0 4}; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --workload $wl --hybrid-options $o --steps 20 --warmup 5 > gpurun_out/hs_last.log 2>&1 || { echo "rc=$? $wl $o"; tail -5 gpurun_out/hs_last.log; exit 1; }
  grep '^{' gpurun_out/hs_last.log >> gpurun_out/hsplit.jsonl; echo "$wl $o $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/hs_last.log)"
done; done
