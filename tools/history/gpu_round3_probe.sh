#!/bin/bash
# Round-2 check after the bs 16 fp16 column-stream default: pytest -m gpu,
# smoke, default bench, run-to-run determinism of every shipped path, then
# the counter bytes of the config-5 kernel.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
PYTEST_ARGS="--timeout 300 --timeout-method thread" bash tools/gpu_round.sh || exit 1
timeout -k 10 600 python tools/determinism.py 4 > gpurun_out/determinism.log 2>&1 || { tail -5 gpurun_out/determinism.log; exit 1; }
tail -12 gpurun_out/determinism.log
WLS="products_bsr16_f16" bash tools/pmc_bytes.sh
