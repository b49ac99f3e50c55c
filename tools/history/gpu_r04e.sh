#!/bin/bash
# Round 4: second A/B of the grouped bs 16 fp16 stream (TUNING build lib_tuning/, copied
# over lib/ on the box only): block rows per group W x (stages, occupancy hint) x XCD chunk
# (SPMM_GRP_VARIANT = 10 P + OCC, + 100 for the vector row-index loads; SPMM_GRP_XM = groups
# per XCD chunk, 0 = as dispatched).
# Output gpurun_out/r04e/grp_sweep.jsonl.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); export TMPDIR=/tmp
O=$R/gpurun_out/r04e; mkdir -p $O
cp spmm-denseblock_amd/lib_tuning/libspmm_hip.so spmm-denseblock_amd/lib/libspmm_hip.so
: > $O/grp_sweep.jsonl
one() {  # W variant xm [workload]
  SPMM_GRP_VARIANT=$2 SPMM_GRP_XM=$3 timeout -k 10 300 python bench.py --workload ${4:-products_bsr16_f16_grp} --group-rows $1 --steps 10 --warmup 3 --no-cpu-baseline > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
  python3 - "$@" >> $O/grp_sweep.jsonl <<'PY'
import json, sys
d = json.loads([l for l in open("gpurun_out/r04e/b.log") if l.startswith("{")][-1])
a = sys.argv[1:]
print(json.dumps({"W": int(a[0]), "variant": int(a[1]), "xm": int(a[2]),
                  "workload": a[3] if len(a) > 3 else "products_bsr16_f16_grp",
                  "ms": d["ms_per_step"], "kernel_ms": d["roofline"]["kernel_ms"]}))
PY
  tail -1 $O/grp_sweep.jsonl
}
for xm in 0 8; do for v in 33 133 43 53 32 42; do one 4 $v $xm; done; done
for xm in 0 4; do for v in 33 24 43; do one 8 $v $xm; done; done
for xm in 0 16; do for v in 33 43 53; do one 2 $v $xm; done; done
