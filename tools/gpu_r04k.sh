#!/bin/bash
# Round 4: the grouped bs 32 stream with k = 2 MFMAs on column pairs (four output blocks,
# SPMM_GRP32_VARIANT 1033 / 1034, TUNING build) against the shipped k = 1 form: a numerics
# check, then reddit and products lines interleaved. Output gpurun_out/r04k/lines.jsonl.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04k; mkdir -p $O
cp spmm-denseblock_amd/lib_tuning/libspmm_hip.so spmm-denseblock_amd/lib/libspmm_hip.so
SPMM_GRP32_VARIANT=1033 timeout -k 10 120 python tools/k2_check.py > $O/k2_check.log 2>&1 || { cat $O/k2_check.log; exit 1; }
cat $O/k2_check.log
: > $O/lines.jsonl
for wl in reddit_bsr32_grp products_bsr32_grp; do
  for W in 2 4; do
  for v in 33 1033 1034 33 1033; do
    SPMM_GRP32_VARIANT=$v timeout -k 10 300 python bench.py --workload $wl --group-rows $W --steps 20 --warmup 5 --no-cpu-baseline > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
    python3 - $wl $v $W >> $O/lines.jsonl <<'PY'
import json, sys
d = json.loads([l for l in open("gpurun_out/r04k/b.log") if l.startswith("{")][-1])
print(json.dumps({"workload": sys.argv[1], "variant": int(sys.argv[2]), "W": int(sys.argv[3]),
                  "ms": d["ms_per_step"], "kernel_ms": d["roofline"]["kernel_ms"]}))
PY
    tail -1 $O/lines.jsonl
  done
  done
done
