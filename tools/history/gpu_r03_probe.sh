#!/bin/bash
# Round-3 opening probe: this box's times for the two BSR kernels the round
# works on (config 5 bs 16 fp16, products bs 32), then the world-1 RCCL paths.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/probe.jsonl
for w in products_bsr16_f16 products_bsr32 reddit_bsr32; do
  timeout -k 10 300 python bench.py --workload $w --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bw.log 2>&1 || { tail -5 gpurun_out/bw.log; exit 1; }
  grep '^{' gpurun_out/bw.log >> gpurun_out/probe.jsonl
  grep '^{' gpurun_out/bw.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print('$w', r['ms_per_step'], r['roofline'].get('kernel_ms'), r.get('csr_same_matrix_ms'))"
done
