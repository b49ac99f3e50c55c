#!/bin/bash
# Bench sweep on one GPU box: every BASELINE workload plus K / waves-per-CU
# variants of the headline. One JSON line per run into gpurun_out/sweep.jsonl.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out/sweep.jsonl
: > $OUT
run() { echo "== $*"; timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/sweep_last.log 2>&1; rc=$?; grep '^{' gpurun_out/sweep_last.log >> $OUT; tail -1 gpurun_out/sweep_last.log | cut -c1-300; if [ $rc -ne 0 ]; then echo "rc=$rc stop"; cat gpurun_out/sweep_last.log | tail -20; exit $rc; fi; }
for args in ${SWEEP:-"--workload arxiv_csr" "--workload products_csr_k256" "--workload reddit_bsr32" "--workload products_bsr16_f16" "--K 32" "--K 64" "--K 512" "--waves-per-cu 8" "--waves-per-cu 24" "--waves-per-cu 32"}; do
  run $args --steps 10 --warmup 3
done
