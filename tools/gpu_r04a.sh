#!/bin/bash
# Round 4, first pass: the sc1 store-form repro (the round-3 form and the same
# with s_nop 1), the new full-size analysed / non-finite tests, the rest of the
# GPU suite, the bench lines with their new side fields, and the reference's
# column-major call shapes at full size. Output in gpurun_out/r04a/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); export TMPDIR=/tmp
O=$R/gpurun_out/r04a; mkdir -p $O
stop() { rc=$1; if [ "$rc" -ge 124 ]; then echo "GPU step fault rc=$rc, stopping"; exit "$rc"; fi; }
echo "== sc1 repro"
timeout -k 10 120 python tools/sc1_run.py tools/_sc1/libspmm_hip.so 1 > $O/sc1_form.log 2>&1; rc=$?; cat $O/sc1_form.log | grep '^{'; stop $rc
timeout -k 10 120 python tools/sc1_run.py tools/_sc1nop/libspmm_hip.so 1 > $O/sc1_nop.log 2>&1; rc=$?; cat $O/sc1_nop.log | grep '^{'; stop $rc
echo "== new tests"
timeout -k 10 900 python -u -m pytest tests/test_gpu_csr.py tests/test_gpu_scale.py tests/test_gpu_bsr.py tests/test_gpu_configs.py -x -v --timeout 200 --timeout-method thread -k "analysed_bs or nonfinite or dense_block or default_stream or native_multi or split_rows" > $O/pytest_new.log 2>&1; rc=$?; tail -3 $O/pytest_new.log; stop $rc
[ $rc -ne 0 ] && { grep -E "Error|assert" $O/pytest_new.log | head -20; exit $rc; }
echo "== full gpu suite"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; tail -2 $O/pytest_gpu.log; stop $rc
[ $rc -ne 0 ] && { grep -E "FAILED|Error" $O/pytest_gpu.log | head -20; exit $rc; }
echo "== bench lines"
for w in products_csr reddit_bsr32 products_bsr16_f16 products_bsr32; do
  timeout -k 10 400 python bench.py --workload $w --steps 20 --warmup 5 --no-cpu-baseline > $O/bw_$w.log 2>&1; rc=$?; stop $rc
  grep '^{' $O/bw_$w.log | cut -c1-300
done
echo "== reference call shapes (column-major B and C)"
timeout -k 10 400 python bench.py --workload reddit_bsr32 --bsr-layout col --steps 20 --warmup 5 --no-cpu-baseline > $O/bw_reddit_bsr32_col.log 2>&1; rc=$?; stop $rc
grep '^{' $O/bw_reddit_bsr32_col.log | cut -c1-300
timeout -k 10 400 python bench.py --workload products_csr --csr-layout col --steps 20 --warmup 5 --no-cpu-baseline > $O/bw_products_csr_col.log 2>&1; rc=$?; stop $rc
grep '^{' $O/bw_products_csr_col.log | cut -c1-300
exit 0
