#!/bin/bash
# Variant A/B on one GPU box: the BSR parity tests under each variant of
# TESTV (space-separated; "-" skips), then REPS interleaved timing passes over
# the workload:variant pairs of RUNS (variant "d" = library default).
# Lines go to gpurun_out/var_sweep.jsonl.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in ${TESTV:--}; do
  [ "$v" = "-" ] && continue
  SPMM_BSR_VARIANT=$v timeout -k 10 600 python -u -m pytest tests/test_gpu_bsr.py -x -q --timeout 120 --timeout-method thread -k "${PYTEST_EXPR:-not hybrid}" > gpurun_out/var_tests_$v.log 2>&1; rc=$?
  echo "tests variant $v: $(tail -1 gpurun_out/var_tests_$v.log)"
  [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/var_tests_$v.log | head -20; exit 1; }
done
: > gpurun_out/var_sweep.jsonl
for rep in $(seq ${REPS:-2}); do
  for wv in ${RUNS}; do
    w=${wv%%:*}; v=${wv##*:}
    if [ "$v" = "d" ]; then unset SPMM_BSR_VARIANT; else export SPMM_BSR_VARIANT=$v; fi
    timeout -k 10 300 python bench.py --workload $w --steps 20 --warmup 5 --no-cpu-baseline ${BENCH_EXTRA:-} > gpurun_out/bw.log 2>&1 || { tail -5 gpurun_out/bw.log; exit 1; }
    grep '^{' gpurun_out/bw.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); r['variant']='$v'; r['rep']=$rep; print(json.dumps(r))" >> gpurun_out/var_sweep.jsonl
    grep '^{' gpurun_out/bw.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print('$w', '$v', r['ms_per_step'], r['roofline'].get('kernel_ms'))"
  done
done
unset SPMM_BSR_VARIANT
