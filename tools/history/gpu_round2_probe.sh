set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_scale.py -x -v --timeout 300 --timeout-method thread -k reordered > gpurun_out/scale_ro.log 2>&1 || { tail -20 gpurun_out/scale_ro.log; exit 1; }
tail -4 gpurun_out/scale_ro.log
: > gpurun_out/ro_bench.jsonl
for w in reddit_rcm_bsr32 products_rcm_bsr32 products_rcm_bsr16_f16; do
  timeout -k 10 400 python bench.py --workload $w --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/ro_$w.log 2>&1 || { tail -5 gpurun_out/ro_$w.log; exit 1; }
  grep '^{' gpurun_out/ro_$w.log >> gpurun_out/ro_bench.jsonl
  grep '^{' gpurun_out/ro_$w.log | cut -c1-300
done
bash tools/pmc_bytes.sh
