#!/bin/bash
# The bs 32 panel stream on one box: its bitwise tests, then the bs 32 GPU tests, the reference
# sweep's bs 32 / 64 cells (with a kernel trace of the p = 2e-2 ones), and the drop-in bs 32
# workloads. A GPU fault, abort or time limit stops it. Output in gpurun_out/panel/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); export TMPDIR=/tmp; O=$R/gpurun_out/panel; mkdir -p $O
stop() { rc=$1; if [ "$rc" -ne 0 ]; then echo "stopping rc=$rc"; exit "$rc"; fi; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_bsr.py -x -q --timeout 120 --timeout-method thread -k "panel_stream" > $O/pytest_panel.log 2>&1; rc=$?; tail -2 $O/pytest_panel.log; stop $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_bsr.py tests/test_gpu_scale.py -x -q --timeout 200 --timeout-method thread > $O/pytest_bsr.log 2>&1; rc=$?; tail -2 $O/pytest_bsr.log; stop $rc
timeout -k 10 300 python -u tools/ref_sweep.py --densities 0.02,0.002 --bs 32,64 --dims 64,128,256,512 --transB 0,1 --skip-csr --reps 10 > $O/sweep.jsonl 2> $O/sweep.log; rc=$?; stop $rc
python3 -c "
import json
for l in open('$O/sweep.jsonl'):
    r=json.loads(l); print(r['p'], r['bs'], r['dim'], r['transB'], r['ms'], r['fp32_frac'])"
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 $R/tools/ref_sweep.py --densities 0.02 --bs 32,64 --dims 64,128 --transB 1 --skip-csr --reps 3) > $O/kt.log 2>&1; rc=$?; stop $rc
for w in reddit_bsr32 products_bsr32 reddit_bsr64; do
  timeout -k 10 200 python bench.py --workload $w --steps 20 --warmup 5 --no-cpu-baseline --no-analysed-side > $O/bw_$w.log 2>&1; rc=$?; stop $rc
  grep "^{" $O/bw_$w.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); f=r['roofline']; print('$w', r['ms_per_step'], f.get('kernel_ms'), f.get('mfma_frac'))"
done
