#!/bin/bash
# Diagnostic builds of the bs 16 fp16 column stream (970D, wrong results,
# timing only): which part of the work bounds products_bsr16_f16.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/cs16_diag.jsonl
for v in 5021 9701 9702 9704 9706 9708 9715 5021; do
  SPMM_BSR_VARIANT=$v timeout -k 10 300 python bench.py --workload products_bsr16_f16 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bw.log 2>&1 || { tail -5 gpurun_out/bw.log; exit 1; }
  grep '^{' gpurun_out/bw.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); r['variant']=$v; print(json.dumps(r))" >> gpurun_out/cs16_diag.jsonl
  grep '^{' gpurun_out/bw.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print($v, r['ms_per_step'], r['roofline'].get('kernel_ms'))"
done
