#!/bin/bash
# Ad-hoc GPU pass: gpu tests, bs16 variant sweeps, hybrid bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
WL=products_bsr16_f16 VARS="41 33 9 10 34 66" bash tools/bsr_variants.sh || exit 1
WL=products_bsr16_f16 EXTRA="--dtype fp32" VARS="41 33 9 10 34 66" bash tools/bsr_variants.sh || exit 1
timeout -k 10 300 python bench.py --workload reddit_hybrid32 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/hyb.log 2>&1 || { tail -20 gpurun_out/hyb.log; exit 1; }
grep '^{' gpurun_out/hyb.log
