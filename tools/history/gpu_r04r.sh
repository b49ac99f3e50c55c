#!/bin/bash
# Round 4, last pass: the whole GPU suite, smoke and the default bench on the release library,
# then the tiles-together A/B of the bs 16 column streams (tools/gpu_r04q.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04r; mkdir -p $O
stop() { rc=$1; if [ "$rc" -ge 124 ]; then echo "GPU step fault rc=$rc, stopping"; exit "$rc"; fi; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; tail -1 $O/pytest_gpu.log; stop $rc
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; tail -1 $O/smoke.log; stop $rc
timeout -k 10 600 python bench.py > $O/bench.log 2>&1; rc=$?; grep '^{' $O/bench.log | cut -c1-250; stop $rc
bash tools/gpu_r04q.sh
