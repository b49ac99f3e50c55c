#!/bin/bash
# Round-3 closing pass on one GPU box: pytest -m gpu, smoke, the default bench
# line (CPU baseline legs included), its rocprofv3 kernel trace, every BSR /
# hybrid / CSR workload line, and the determinism reruns (PHASE=a: the first four, b: the
# rest). Output in gpurun_out/final/. A GPU fault, abort or time limit (rc >= 124) stops it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); export TMPDIR=/tmp
O=$R/gpurun_out/final; mkdir -p $O
stop() { rc=$1; if [ "$rc" -ge 124 ]; then echo "GPU step fault rc=$rc, stopping"; exit "$rc"; fi; }
PH=${PHASE:-ab}
if [[ $PH == *a* ]]; then
echo "== pytest -m gpu"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; tail -3 $O/pytest_gpu.log; stop $rc
echo "== smoke"; timeout -k 10 300 python __graft_entry__.py smoke > $O/smoke.log 2>&1; rc=$?; tail -1 $O/smoke.log; stop $rc
echo "== bench"; timeout -k 10 600 python bench.py > $O/bench.log 2>&1; rc=$?; grep '^{' $O/bench.log | cut -c1-300; stop $rc
echo "== kernel trace"
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline) > $O/bench_under_rocprof.log 2>&1; rc=$?; grep '^{' $O/bench_under_rocprof.log | cut -c1-200; stop $rc
fi
if [[ $PH == *b* ]]; then
: > $O/workloads.jsonl
for w in ${WLS:-reddit_bsr32 products_bsr32 products_bsr32_an reddit_bsr32_an products_bsr16_f16 products_bsr16_f16_an products_rcm_bsr32_an reddit_rcm_bsr32_an products_rcm_bsr16_f16_an reddit_rcm_bsr32 products_rcm_bsr32 products_rcm_bsr16_f16 reddit_hybrid32 products_hybrid32 reddit_rcm_hybrid32 arxiv_csr products_csr_k256}; do
  timeout -k 10 300 python bench.py --workload $w --steps 20 --warmup 5 --no-cpu-baseline > $O/bw.log 2>&1; rc=$?; stop $rc
  [ $rc -eq 0 ] || { tail -5 $O/bw.log; continue; }
  grep '^{' $O/bw.log >> $O/workloads.jsonl
  grep '^{' $O/bw.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); f=r['roofline']; print('$w', r['ms_per_step'], f.get('kernel_ms'), 'frac', f.get('frac'), 'mfma', f.get('mfma_frac'), 'csr', r.get('csr_same_matrix_ms'))"
done
echo "== determinism"; timeout -k 10 900 python tools/determinism.py 3 > $O/determinism.log 2>&1; rc=$?; tail -8 $O/determinism.log; stop $rc
fi
exit 0
