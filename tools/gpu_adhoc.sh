#!/bin/bash
# Ad-hoc GPU pass: products bs32 variants + hybrid, BSR/hybrid profiles.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
WL=products_bsr32 VARS="40 44 42" bash tools/bsr_variants.sh || exit 1
WL=products_bsr16_f16 VARS="-1" bash tools/bsr_variants.sh || exit 1
timeout -k 10 300 python bench.py --workload products_hybrid32 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/hyb.log 2>&1 || { tail -20 gpurun_out/hyb.log; exit 1; }
grep '^{' gpurun_out/hyb.log
WL=reddit_bsr32 bash tools/profile_bsr.sh || exit 1
WL=reddit_hybrid32 bash tools/profile_bsr.sh || exit 1
