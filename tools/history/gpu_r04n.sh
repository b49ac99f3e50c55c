#!/bin/bash
# Round 4: the grouped bs 16 stream with a group's column tiles consecutive on one XCD
# (SPMM_GRP_TT=1, TUNING build: the later tile reads the A fragments from L2) against the
# release mapping: the grouped GPU tests under TT = 1, then interleaved lines on products and
# RCM products. Output gpurun_out/r04n/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04n; mkdir -p $O
cp spmm-denseblock_amd/lib_tuning/libspmm_hip.so spmm-denseblock_amd/lib/libspmm_hip.so
SPMM_GRP_TT=1 timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_bsr.py tests/test_gpu_scale.py -k "grouped_f16 or grouped_bs16 or random_shapes" > $O/pytest_tt.log 2>&1 || { tail -30 $O/pytest_tt.log; exit 1; }
tail -1 $O/pytest_tt.log
: > $O/lines.jsonl
for wl in products_bsr16_f16_grp products_rcm_bsr16_f16_grp; do
  for tt in 0 1 0 1; do
    SPMM_GRP_TT=$tt timeout -k 10 300 python bench.py --workload $wl --steps 20 --warmup 5 --no-cpu-baseline > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
    python3 - $wl $tt >> $O/lines.jsonl <<'PY'
import json, sys
d = json.loads([l for l in open("gpurun_out/r04n/b.log") if l.startswith("{")][-1])
print(json.dumps({"workload": sys.argv[1], "tt": int(sys.argv[2]), "ms": d["ms_per_step"], "kernel_ms": d["roofline"]["kernel_ms"]}))
PY
    tail -1 $O/lines.jsonl
  done
done
