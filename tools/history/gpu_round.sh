#!/bin/bash
# One GPU-box pass: parity tests, smoke, bench. Each GPU step has its own time
# limit; a fault/abort/timeout (rc >= 124 or signal) stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
stop_on_fault() { rc=$1; if [ "$rc" -ge 124 ] || [ "$rc" -ge 128 ]; then echo "GPU step fault rc=$rc, stopping"; exit "$rc"; fi; }
echo "== pytest -m gpu"; timeout -k 10 ${T_TEST:-900} python -m pytest tests -m gpu -x -q ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -5 gpurun_out/pytest_gpu.log; stop_on_fault $rc
echo "== smoke"; timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1; rc=$?; tail -3 gpurun_out/smoke.log; stop_on_fault $rc
echo "== bench"; timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1; rc=$?; tail -3 gpurun_out/bench.log; stop_on_fault $rc
