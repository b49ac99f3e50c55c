#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
cp spmm-denseblock_amd/lib/libspmm_hip.so /tmp/lib_512.so
for v in 512 256 128; do
  cp tools/tmp_libs/lib_$v.so spmm-denseblock_amd/lib/libspmm_hip.so 2>/dev/null || cp /tmp/lib_512.so spmm-denseblock_amd/lib/libspmm_hip.so
  for wl in arxiv_csr products_csr; do
    timeout -k 10 300 python bench.py --workload $wl --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/g.log 2>&1 || { tail -20 gpurun_out/g.log; exit 1; }
    grep '^{' gpurun_out/g.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print('$v $wl', r['ms_per_step'], r['roofline']['kernel_ms'])"
  done
done
cp /tmp/lib_512.so spmm-denseblock_amd/lib/libspmm_hip.so
