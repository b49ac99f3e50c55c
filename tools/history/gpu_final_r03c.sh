#!/bin/bash
# Last pass of round 3 on the single-resource hot kernel: hot-path GPU tests, smoke,
# the default bench line, the hot workload line, counter bytes of plain and hot CSR,
# the hot kernel's trace. Output in gpurun_out/final_c/ (+ gpurun_out/pmcb/).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); export TMPDIR=/tmp
O=$R/gpurun_out/final_c; mkdir -p $O
stop() { rc=$1; if [ "$rc" -ge 124 ]; then echo "GPU step fault rc=$rc, stopping"; exit "$rc"; fi; }
echo "== hot tests"; timeout -k 10 400 python -u -m pytest tests/test_gpu_csr_hot.py tests/test_drivers.py -x -q --timeout 200 --timeout-method thread > $O/pytest_hot.log 2>&1; rc=$?; tail -1 $O/pytest_hot.log; stop $rc
[ $rc -ne 0 ] && { tail -30 $O/pytest_hot.log; exit $rc; }
echo "== smoke"; timeout -k 10 300 python __graft_entry__.py smoke > $O/smoke.log 2>&1; rc=$?; tail -1 $O/smoke.log; stop $rc
echo "== bench"; timeout -k 10 600 python bench.py > $O/bench.log 2>&1; rc=$?; grep '^{' $O/bench.log | cut -c1-200; stop $rc
echo "== counter bytes"; WLS="products_csr products_csr_hot" BENCH_EXTRA="--no-hot-side" bash tools/pmc_bytes.sh; stop $?
echo "== hot line"; timeout -k 10 300 python bench.py --workload products_csr_hot --steps 20 --warmup 5 --no-cpu-baseline > $O/bw_hot.log 2>&1; rc=$?; stop $rc
grep '^{' $O/bw_hot.log | cut -c1-200
exit 0
