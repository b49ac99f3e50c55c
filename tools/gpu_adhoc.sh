#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
# 1-rank rehearsal of the N > 1 chunked exchange path (RCCL, world 1)
for c in 1 4; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 10 --warmup 3 --no-cpu-baseline --chunks $c > gpurun_out/d.log 2>&1 || { tail -20 gpurun_out/d.log; exit 1; }
  grep '^{' gpurun_out/d.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print('chunks=$c', r['ms_per_step'], r['roofline']['kernel_ms'], r['config'].get('exchange_chunks'))"
done
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/d.log 2>&1 || { tail -20 gpurun_out/d.log; exit 1; }
grep '^{' gpurun_out/d.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print('plain', r['ms_per_step'], r['roofline']['kernel_ms'], r['config'].get('exchange_chunks'))"
