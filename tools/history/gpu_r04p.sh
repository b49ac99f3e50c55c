#!/bin/bash
# Round 4: grouped streams' empty-matrix test, then the grouped bs 16 stream with tiles
# together at W = 2 / 4 / 8 and XCD chunks around the default (TUNING build), interleaved.
# Output gpurun_out/r04p/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04p; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_bsr.py -k "empty_matrix" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
cp spmm-denseblock_amd/lib_tuning/libspmm_hip.so spmm-denseblock_amd/lib/libspmm_hip.so
: > $O/lines.jsonl
for cfg in "4 8" "8 4" "2 16" "4 4" "4 16" "8 2" "4 8"; do
  set -- $cfg
  SPMM_GRP_XM=$2 timeout -k 10 300 python bench.py --workload products_bsr16_f16_grp --group-rows $1 --steps 20 --warmup 5 --no-cpu-baseline > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
  python3 - $1 $2 >> $O/lines.jsonl <<'PY'
import json, sys
d = json.loads([l for l in open("gpurun_out/r04p/b.log") if l.startswith("{")][-1])
print(json.dumps({"W": int(sys.argv[1]), "xm": int(sys.argv[2]), "ms": d["ms_per_step"], "kernel_ms": d["roofline"]["kernel_ms"]}))
PY
  tail -1 $O/lines.jsonl
done
