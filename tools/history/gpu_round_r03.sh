#!/bin/bash
# Round-3 pass on one GPU box: pytest -m gpu, smoke, the default bench line
# (with the CPU baseline legs), the parity subset under every accepted
# SPMM_BSR_VARIANT, the BSR / hybrid workload lines, config 2's reference
# mode and the world-1 torch.distributed rehearsal. A GPU fault, abort or
# time limit (rc >= 124) stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
stop_on_fault() { rc=$1; if [ "$rc" -ge 124 ]; then echo "GPU step fault rc=$rc, stopping"; exit "$rc"; fi; }
PYTEST_ARGS="--timeout 300 --timeout-method thread" bash tools/gpu_round.sh; stop_on_fault $?
grep '^{' gpurun_out/bench.log | cut -c1-400
TESTV="${TESTV:-4516 4496 4126 6104 4725}" RUNS="${RUNS:-reddit_bsr32:d products_bsr32:d products_bsr16_f16:d}" REPS=1 bash tools/gpu_var.sh; stop_on_fault $?
if [ -n "${WLS:-}" ]; then
  : > gpurun_out/workloads.jsonl
  for w in $WLS; do
    timeout -k 10 300 python bench.py --workload $w --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bw.log 2>&1; rc=$?; stop_on_fault $rc
    [ $rc -eq 0 ] || { tail -5 gpurun_out/bw.log; continue; }
    grep '^{' gpurun_out/bw.log >> gpurun_out/workloads.jsonl
    grep '^{' gpurun_out/bw.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); f=r['roofline']; print('$w', r['ms_per_step'], f.get('kernel_ms'), 'frac', f.get('frac'), 'csr', r.get('csr_same_matrix_ms'))"
  done
fi
[ -n "${CONFIG2:-}" ] && { bash tools/gpu_config2_refmode.sh; stop_on_fault $?; }
[ -n "${DIST:-}" ] && { bash tools/gpu_dist_rehearsal.sh; stop_on_fault $?; }
exit 0
