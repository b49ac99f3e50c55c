#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python bench.py --workload reddit_rcm_hybrid32 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r.log 2>&1 || { tail -20 gpurun_out/r.log; exit 1; }
grep '^{' gpurun_out/r.log
