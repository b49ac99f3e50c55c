set -u
mkdir -p gpurun_out
: > gpurun_out/hybcs.jsonl
for w in reddit_hybrid32 products_hybrid32; do
  for v in -1 4516 4126; do
    if [ $v -lt 0 ]; then unset SPMM_BSR_VARIANT; else export SPMM_BSR_VARIANT=$v; fi
    timeout -k 10 300 python bench.py --workload $w --steps 20 --warmup 5 --no-cpu-baseline --hybrid-options 2 > gpurun_out/bw.log 2>&1 || { tail -5 gpurun_out/bw.log; exit 1; }
    grep '^{' gpurun_out/bw.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); r['variant']=$v; print(json.dumps(r))" >> gpurun_out/hybcs.jsonl
    grep '^{' gpurun_out/bw.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print('$w', $v, r['ms_per_step'], r.get('part_kernel_ms'))"
  done
done
