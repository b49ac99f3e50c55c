#!/bin/bash
# Round-3 closing pass (second session) on one GPU box: the default bench line
# (CPU baseline legs and the hot-column side line included), its rocprofv3
# kernel trace, every workload line (hot-column CSR included), counter bytes of
# the plain and hot CSR kernels, determinism. Output in gpurun_out/final_b/.
# A GPU fault, abort or time limit (rc >= 124) stops it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); export TMPDIR=/tmp
O=$R/gpurun_out/final_b; mkdir -p $O
stop() { rc=$1; if [ "$rc" -ge 124 ]; then echo "GPU step fault rc=$rc, stopping"; exit "$rc"; fi; }
PH=${PHASE:-abc}
if [[ $PH == *a* ]]; then
echo "== bench"; timeout -k 10 600 python bench.py > $O/bench.log 2>&1; rc=$?; grep '^{' $O/bench.log | cut -c1-300; stop $rc
echo "== kernel trace"
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline) > $O/bench_under_rocprof.log 2>&1; rc=$?; grep '^{' $O/bench_under_rocprof.log | cut -c1-200; stop $rc
fi
if [[ $PH == *b* ]]; then
: > $O/workloads.jsonl
for w in ${WLS:-products_csr_hot reddit_bsr32 products_bsr32 products_bsr32_an reddit_bsr32_an products_bsr16_f16 products_bsr16_f16_an products_rcm_bsr32_an reddit_rcm_bsr32_an products_rcm_bsr16_f16_an reddit_rcm_bsr32 products_rcm_bsr32 products_rcm_bsr16_f16 reddit_hybrid32 products_hybrid32 reddit_rcm_hybrid32 arxiv_csr products_csr_k256}; do
  timeout -k 10 300 python bench.py --workload $w --steps 20 --warmup 5 --no-cpu-baseline > $O/bw.log 2>&1; rc=$?; stop $rc
  [ $rc -eq 0 ] || { tail -5 $O/bw.log; continue; }
  grep '^{' $O/bw.log >> $O/workloads.jsonl
  grep '^{' $O/bw.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); f=r['roofline']; print('$w', r['ms_per_step'], f.get('kernel_ms'), 'frac', f.get('frac'), 'mfma', f.get('mfma_frac'), 'csr', r.get('csr_same_matrix_ms'))"
done
fi
if [[ $PH == *c* ]]; then
echo "== counter bytes, plain and hot CSR"
WLS="products_csr products_csr_hot" BENCH_EXTRA="--no-hot-side" bash tools/pmc_bytes.sh; stop $?
echo "== determinism"; timeout -k 10 900 python tools/determinism.py 3 > $O/determinism.log 2>&1; rc=$?; tail -8 $O/determinism.log; stop $rc
fi
exit 0
