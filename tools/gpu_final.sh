#!/bin/bash
# Closing pass on one GPU box (release library), round ${ROUND:-r06}: the whole GPU suite, smoke,
# the default bench line (CPU baseline legs and side lines included) and its rocprofv3 kernel
# trace, bench.py's N > 1 path rehearsed at world 1 through torch.distributed.run, every workload
# line, counter bytes of every BSR / hybrid workload's kernel and of the plain and hot CSR
# kernels, determinism, the reference's sweep. Output in gpurun_out/final_$ROUND/ (+
# gpurun_out/pmcb/). PHASE selects a (suite, smoke, bench, trace, rehearsal), b (workload
# lines), p (BSR counter bytes), c (CSR counter bytes, determinism), s (sweep). A GPU fault,
# abort or time limit (rc >= 124) stops it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); export TMPDIR=/tmp
RD=${ROUND:-r06}
O=$R/gpurun_out/final_$RD; mkdir -p $O
stop() { rc=$1; if [ "$rc" -ge 124 ]; then echo "GPU step fault rc=$rc, stopping"; exit "$rc"; fi; }
BSR_WLS="reddit_bsr32 products_bsr32 products_rcm_bsr16_f16 products_rcm_bsr32 reddit_bsr32_an products_bsr32_an reddit_bsr32_grp products_bsr32_grp products_bsr16_f16 products_bsr16_f16_an products_bsr16_f16_grp products_rcm_bsr16_f16_grp reddit_rcm_bsr32 reddit_rcm_bsr32_an products_rcm_bsr32_an reddit_bsr8 reddit_bsr4 reddit_bsr2 reddit_bsr64 reddit_bsr8_rb32 reddit_hybrid32 products_hybrid32"
PH=${PHASE:-abpcs}
if [[ $PH == *a* ]]; then
echo "== gpu suite"
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; tail -2 $O/pytest_gpu.log; stop $rc
grep -E "FAILED|Error" $O/pytest_gpu.log | head -20
echo "== smoke"; timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; tail -1 $O/smoke.log; stop $rc
echo "== bench"; timeout -k 10 600 python bench.py > $O/bench.log 2>&1; rc=$?; grep '^{' $O/bench.log | cut -c1-300; stop $rc
echo "== kernel trace"
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline) > $O/bench_under_rocprof.log 2>&1; rc=$?; grep '^{' $O/bench_under_rocprof.log | cut -c1-200; stop $rc
echo "== N > 1 path at world 1 (torch.distributed.run, 4 chunks, RCCL)"
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29613 bench.py --gpus 1 --workload products_csr_k256 --chunks 4 --steps 10 --warmup 3 > $O/dist_world1.log 2>&1; rc=$?; grep '^{' $O/dist_world1.log | cut -c1-300; stop $rc
echo "== --gpus 2 on one GPU (must exit 2, no line)"
timeout -k 10 120 python bench.py --gpus 2 > $O/gpus2.log 2>&1; echo "rc=$?" >> $O/gpus2.log; tail -2 $O/gpus2.log
fi
if [[ $PH == *b* ]]; then
: > $O/workloads.jsonl
for w in ${WLS:-arxiv_csr products_csr_k256 products_csr_hot $BSR_WLS reddit_bsr4_rb32 reddit_bsr2_rb32}; do
  timeout -k 10 300 python bench.py --workload $w --steps 20 --warmup 5 --no-cpu-baseline > $O/bw.log 2>&1; rc=$?; stop $rc
  [ $rc -eq 0 ] || { tail -5 $O/bw.log; continue; }
  grep '^{' $O/bw.log >> $O/workloads.jsonl
  grep '^{' $O/bw.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); f=r['roofline']; print('$w', r['ms_per_step'], f.get('kernel_ms'), 'frac', f.get('frac'), 'mfma', f.get('mfma_frac'), 'traffic', f.get('traffic'))"
done
fi
if [[ $PH == *p* ]]; then
echo "== counter bytes of every BSR / hybrid workload"
WLS="${PWLS:-$BSR_WLS}" BENCH_EXTRA="--no-analysed-side" T_STEP=300 bash tools/pmc_bytes.sh; stop $?
cp gpurun_out/pmcb/bytes.jsonl $O/bsr_bytes.jsonl
fi
if [[ $PH == *c* ]]; then
echo "== counter bytes, plain and hot CSR"
rm -rf gpurun_out/pmcb/kt_products_csr* gpurun_out/pmcb/fetch_products_csr* gpurun_out/pmcb/write_products_csr*
WLS="products_csr products_csr_hot" BENCH_EXTRA="--no-hot-side --no-bsr-sides" bash tools/pmc_bytes.sh; stop $?
cp gpurun_out/pmcb/bytes.jsonl $O/csr_bytes.jsonl
echo "== determinism"; timeout -k 10 900 python tools/determinism.py 3 > $O/determinism.log 2>&1; rc=$?; tail -3 $O/determinism.log; stop $rc
fi
if [[ $PH == *s* ]]; then
echo "== the reference's sweep"
timeout -k 10 900 python -u tools/ref_sweep.py > $O/sweep.jsonl 2> $O/sweep.log; rc=$?; tail -1 $O/sweep.log; stop $rc
fi
exit 0
