#!/bin/bash
# Round-4 closing pass on one GPU box (release library): the whole GPU suite, smoke, the
# default bench line (CPU baseline legs and side lines included) and its rocprofv3 kernel
# trace, every workload line, counter bytes of the plain and hot CSR kernels (the bench's
# traffic and hot-line counter bytes), determinism. Output in gpurun_out/final_r04/ (+
# gpurun_out/pmcb/). PHASE selects a (suite, smoke, bench, trace), b (workload lines),
# k (kernel traces of workload lines), c (counter bytes, determinism). A GPU fault, abort or
# time limit (rc >= 124) stops it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); export TMPDIR=/tmp
O=$R/gpurun_out/final_r04; mkdir -p $O
stop() { rc=$1; if [ "$rc" -ge 124 ]; then echo "GPU step fault rc=$rc, stopping"; exit "$rc"; fi; }
PH=${PHASE:-abc}
if [[ $PH == *a* ]]; then
echo "== gpu suite"
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; tail -2 $O/pytest_gpu.log; stop $rc
grep -E "FAILED|Error" $O/pytest_gpu.log | head -20
echo "== smoke"; timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; tail -1 $O/smoke.log; stop $rc
echo "== bench"; timeout -k 10 600 python bench.py > $O/bench.log 2>&1; rc=$?; grep '^{' $O/bench.log | cut -c1-300; stop $rc
echo "== kernel trace"
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline) > $O/bench_under_rocprof.log 2>&1; rc=$?; grep '^{' $O/bench_under_rocprof.log | cut -c1-200; stop $rc
fi
if [[ $PH == *b* ]]; then
: > $O/workloads.jsonl
for w in ${WLS:-arxiv_csr products_csr_k256 products_csr_hot reddit_bsr32 products_bsr32 reddit_bsr32_grp products_bsr32_grp products_bsr16_f16 products_bsr16_f16_grp products_rcm_bsr16_f16_grp reddit_bsr8 reddit_bsr64 reddit_hybrid32 products_hybrid32}; do
  timeout -k 10 300 python bench.py --workload $w --steps 20 --warmup 5 --no-cpu-baseline > $O/bw.log 2>&1; rc=$?; stop $rc
  [ $rc -eq 0 ] || { tail -5 $O/bw.log; continue; }
  grep '^{' $O/bw.log >> $O/workloads.jsonl
  grep '^{' $O/bw.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); f=r['roofline']; print('$w', r['ms_per_step'], f.get('kernel_ms'), 'frac', f.get('frac'), 'mfma', f.get('mfma_frac'))"
done
fi
if [[ $PH == *k* ]]; then
echo "== kernel traces of the workload lines"
WLS="arxiv_csr reddit_bsr32_grp products_bsr16_f16_grp reddit_bsr8 reddit_bsr64" KT_TAG=_r04 bash tools/profile_kt.sh; stop $?
fi
if [[ $PH == *c* ]]; then
echo "== counter bytes, plain and hot CSR"
WLS="products_csr products_csr_hot" BENCH_EXTRA="--no-hot-side" bash tools/pmc_bytes.sh; stop $?
cp gpurun_out/pmcb/bytes.jsonl $O/csr_bytes.jsonl
echo "== determinism"; timeout -k 10 900 python tools/determinism.py 3 > $O/determinism.log 2>&1; rc=$?; tail -3 $O/determinism.log; stop $rc
fi
exit 0
