#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash tools/gpu_round.sh || exit 1
: > gpurun_out/sweep.jsonl
for a in "--workload arxiv_csr" "--workload products_csr_k256" "--workload reddit_bsr32" "--workload products_bsr32" "--workload products_bsr16_f16" "--workload reddit_hybrid32" "--workload products_hybrid32" "--workload reddit_rcm_hybrid32" "--K 64" "--K 512"; do
  timeout -k 10 300 python bench.py --no-cpu-baseline $a --steps 10 --warmup 3 > gpurun_out/sweep_last.log 2>&1 || { tail -20 gpurun_out/sweep_last.log; exit 1; }
  grep '^{' gpurun_out/sweep_last.log >> gpurun_out/sweep.jsonl
done
echo sweep done
WLS="products_bsr16_f16" bash tools/profile_kt.sh || exit 1
