#!/bin/bash
# Round-2 closing pass on one GPU box: pytest -m gpu, smoke, the default
# bench, its rocprofv3 kernel trace, every BSR / hybrid workload line, and the
# counter bytes of the shipped BSR kernels. Each GPU step has its own limit;
# a failure stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); export TMPDIR=/tmp
mkdir -p gpurun_out
PYTEST_ARGS="--timeout 300 --timeout-method thread" bash tools/gpu_round.sh || exit 1
O=$R/gpurun_out/kt_headline; mkdir -p $O
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O -o kt --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline) > $O/run.log 2>&1 || { tail -5 $O/run.log; exit 1; }
grep '^{' $O/run.log | cut -c1-200
: > gpurun_out/workloads.jsonl
for w in reddit_bsr32 products_bsr32 products_bsr16_f16 reddit_rcm_bsr32 products_rcm_bsr32 products_rcm_bsr16_f16 reddit_hybrid32 products_hybrid32 reddit_rcm_hybrid32 arxiv_csr products_csr_k256; do
  timeout -k 10 300 python bench.py --workload $w --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bw.log 2>&1 || { tail -5 gpurun_out/bw.log; exit 1; }
  grep '^{' gpurun_out/bw.log >> gpurun_out/workloads.jsonl
  grep '^{' gpurun_out/bw.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print('$w', r['ms_per_step'], r['roofline'].get('kernel_ms'), r.get('csr_same_matrix_ms'))"
done
timeout -k 10 900 python tools/determinism.py 3 > gpurun_out/determinism.log 2>&1 || { tail -5 gpurun_out/determinism.log; exit 1; }
tail -12 gpurun_out/determinism.log
WLS="${PMC_WLS:-reddit_bsr32 products_bsr32 products_bsr16_f16}" bash tools/pmc_bytes.sh
