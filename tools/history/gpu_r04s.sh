#!/bin/bash
# Round 4: the grouped bs 16 stream with its A fragments through LDS (SPMM_GRP_VARIANT 1033 /
# 1043: W / 2 copies of 1 KB per item instead of W 8-B loads; TUNING build) against the
# release form (33): the grouped tests under 1033, then interleaved lines. Output gpurun_out/r04s/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04s; mkdir -p $O
cp spmm-denseblock_amd/lib_tuning/libspmm_hip.so spmm-denseblock_amd/lib/libspmm_hip.so
SPMM_GRP_VARIANT=1033 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_bsr.py tests/test_gpu_scale.py -k "grouped_f16 or grouped_bs16 or random_shapes or empty_matrix" > $O/pytest_al.log 2>&1 || { tail -30 $O/pytest_al.log; exit 1; }
tail -1 $O/pytest_al.log
: > $O/lines.jsonl
for wl in products_bsr16_f16_grp products_rcm_bsr16_f16_grp; do
  for v in 33 1033 1043 33 1033; do
    SPMM_GRP_VARIANT=$v timeout -k 10 300 python bench.py --workload $wl --steps 20 --warmup 5 --no-cpu-baseline > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
    python3 - $wl $v >> $O/lines.jsonl <<'PY'
import json, sys
d = json.loads([l for l in open("gpurun_out/r04s/b.log") if l.startswith("{")][-1])
print(json.dumps({"workload": sys.argv[1], "variant": int(sys.argv[2]), "ms": d["ms_per_step"], "kernel_ms": d["roofline"]["kernel_ms"]}))
PY
    tail -1 $O/lines.jsonl
  done
done
