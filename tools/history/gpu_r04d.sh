#!/bin/bash
# Round 4: merge-path grid size on the arxiv stand-in (K = 128) and products: waves per CU x
# minimum items per wave (SPMM_CSR_MIN_ITEMS, TUNING build lib_tuning/ copied over lib/ on
# the box only), release build first as the control. Output gpurun_out/r04d/csr_grid.jsonl.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); export TMPDIR=/tmp
O=$R/gpurun_out/r04d; mkdir -p $O
: > $O/csr_grid.jsonl
row() {  # tag workload
  python3 - "$1" "$2" >> $O/csr_grid.jsonl <<'PY'
import json, sys
d = json.loads([l for l in open("gpurun_out/r04d/b.log") if l.startswith("{")][-1])
print(json.dumps({"tag": sys.argv[1], "workload": sys.argv[2], "ms": d["ms_per_step"],
                  "kernel_ms": d["roofline"]["kernel_ms"], "graph": d["config"].get("hip_graph")}))
PY
  tail -1 $O/csr_grid.jsonl
}
run() {  # tag workload args...
  local tag=$1 wl=$2; shift 2
  timeout -k 10 240 python bench.py --workload $wl --steps ${STEPS:-50} --warmup 10 --no-cpu-baseline --no-hot-side "$@" > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
  row "$tag" "$wl"
}
run release arxiv_csr
run release_graph arxiv_csr --graph
cp spmm-denseblock_amd/lib_tuning/libspmm_hip.so spmm-denseblock_amd/lib/libspmm_hip.so
for wpc in 16 24 32; do
  for mi in 512 256 128; do
    SPMM_CSR_MIN_ITEMS=$mi run "w${wpc}_m${mi}" arxiv_csr --waves-per-cu $wpc
  done
done
for wpc in 16 24 32; do
  run "w${wpc}" products_csr --waves-per-cu $wpc
done
