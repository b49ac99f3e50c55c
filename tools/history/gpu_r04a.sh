#!/bin/bash
# Round 4 pass: the new GPU tests (full-size analysed entries, non-finite contracts,
# split-row tickets, bs 2/4/8/64 kernels, the grouped bs 16 stream), bench lines, the
# whole GPU suite, the reference's column-major call shapes. Output in gpurun_out/r04a/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); export TMPDIR=/tmp
O=$R/gpurun_out/r04a; mkdir -p $O
stop() { rc=$1; if [ "$rc" -ge 124 ]; then echo "GPU step fault rc=$rc, stopping"; exit "$rc"; fi; }
echo "== new tests"
timeout -k 10 900 python -u -m pytest tests/test_gpu_csr.py tests/test_gpu_scale.py tests/test_gpu_bsr.py tests/test_gpu_configs.py -v --timeout 200 --timeout-method thread -k "analysed_bs or nonfinite or dense_block or default_stream or native_multi or split_rows or small_bs or bsr64 or grouped" > $O/pytest_new.log 2>&1; rc=$?; tail -3 $O/pytest_new.log; stop $rc
grep -E "FAILED|Error" $O/pytest_new.log | head -20
echo "== bench lines"
for w in products_csr arxiv_csr products_bsr16_f16 products_bsr16_f16_grp reddit_bsr32 products_bsr32 reddit_bsr8 reddit_bsr64; do
  timeout -k 10 400 python bench.py --workload $w --steps 20 --warmup 5 --no-cpu-baseline > $O/bw_$w.log 2>&1; rc=$?; stop $rc
  grep '^{' $O/bw_$w.log | cut -c1-400
done
echo "== full gpu suite"
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; tail -2 $O/pytest_gpu.log; stop $rc
grep -E "FAILED|Error" $O/pytest_gpu.log | head -20
echo "== reference call shapes (column-major B and C)"
timeout -k 10 400 python bench.py --workload reddit_bsr32 --bsr-layout col --steps 20 --warmup 5 --no-cpu-baseline --no-analysed-side > $O/bw_reddit_bsr32_col.log 2>&1; rc=$?; stop $rc
grep '^{' $O/bw_reddit_bsr32_col.log | cut -c1-300
timeout -k 10 400 python bench.py --workload products_csr --csr-layout col --steps 20 --warmup 5 --no-cpu-baseline > $O/bw_products_csr_col.log 2>&1; rc=$?; stop $rc
grep '^{' $O/bw_products_csr_col.log | cut -c1-300
exit 0
