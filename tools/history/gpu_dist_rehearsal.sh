#!/bin/bash
# One-GPU rehearsal of bench.py's N > 1 code paths through torch.distributed.run
# (world 1, RCCL): weak scaling and strong scaling (config 4 as stated) with 4
# exchange chunks, so every step runs the chunked in-place all-gathers through RCCL.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for mode in weak strong; do
  echo "== torchrun world 1 --scaling $mode"
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
      --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 10 --warmup 3 \
      --scaling $mode --chunks 4 > gpurun_out/dist_$mode.log 2>&1
  rc=$?
  grep '^{' gpurun_out/dist_$mode.log | cut -c1-1200 || tail -20 gpurun_out/dist_$mode.log
  [ $rc -eq 0 ] || { tail -20 gpurun_out/dist_$mode.log; exit $rc; }
done
