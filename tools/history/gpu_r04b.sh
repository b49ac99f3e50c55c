#!/bin/bash
# Round 4: A/B of the grouped bs 16 fp16 stream on the TUNING build (lib_tuning/, copied
# over lib/ on the box only): block rows per group W x (stages, occupancy hint)
# (SPMM_GRP_VARIANT = 10 P + OCC). Output gpurun_out/r04b/grp_sweep.jsonl.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); export TMPDIR=/tmp
O=$R/gpurun_out/r04b; mkdir -p $O
cp spmm-denseblock_amd/lib_tuning/libspmm_hip.so spmm-denseblock_amd/lib/libspmm_hip.so
: > $O/grp_sweep.jsonl
for W in ${WS:-4 8 2}; do
  for v in ${GVS:-30 33 50 54}; do
    SPMM_GRP_VARIANT=$v timeout -k 10 300 python bench.py --workload products_bsr16_f16_grp --group-rows $W --steps 10 --warmup 3 --no-cpu-baseline > $O/b.log 2>&1; rc=$?
    if [ $rc -ne 0 ]; then tail -5 $O/b.log; exit $rc; fi
    python3 - $W $v >> $O/grp_sweep.jsonl <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[0] if False else "gpurun_out/r04b/b.log") if l.startswith("{")][-1])
print(json.dumps({"W": int(sys.argv[1]), "variant": int(sys.argv[2]), "ms": d["ms_per_step"],
                  "kernel_ms": d["roofline"]["kernel_ms"], "analysis_ms": d.get("analysis_ms")}))
PY
    tail -1 $O/grp_sweep.jsonl
  done
done
