#!/bin/bash
# Round 4: what bounds the grouped bs 32 stream: the same runs with and without its MFMAs
# (SPMM_GRP32_VARIANT 933, a TUNING-only diagnostic that returns wrong results) on reddit and
# products. Output gpurun_out/r04j/lines.jsonl.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04j; mkdir -p $O
cp spmm-denseblock_amd/lib_tuning/libspmm_hip.so spmm-denseblock_amd/lib/libspmm_hip.so
: > $O/lines.jsonl
for wl in reddit_bsr32_grp products_bsr32_grp; do
  for v in 33 933 33 933; do
    SPMM_GRP32_VARIANT=$v timeout -k 10 300 python bench.py --workload $wl --steps 20 --warmup 5 --no-cpu-baseline > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
    python3 - $wl $v >> $O/lines.jsonl <<'PY'
import json, sys
d = json.loads([l for l in open("gpurun_out/r04j/b.log") if l.startswith("{")][-1])
print(json.dumps({"workload": sys.argv[1], "variant": int(sys.argv[2]), "ms": d["ms_per_step"],
                  "kernel_ms": d["roofline"]["kernel_ms"]}))
PY
    tail -1 $O/lines.jsonl
  done
done
