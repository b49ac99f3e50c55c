#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for K in 64 48; do
  for opt in 1 3; do
    timeout -k 10 300 python bench.py --K $K --csr-options $opt --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/k.log 2>&1 || { tail -5 gpurun_out/k.log; exit 1; }
    grep '^{' gpurun_out/k.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print('K=$K opt=$opt', r['roofline']['kernel_ms'], r['roofline']['frac'], r['ms_per_step'])"
  done
done
