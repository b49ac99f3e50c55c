#!/bin/bash
# Round 4: the grouped bs 16 stream with two items per barrier (SPMM_GRP_VARIANT 243 / 262 /
# 263: P stages, occupancy hint, IPB = 2) against the release form (33), interleaved, after
# the grouped GPU tests on the release build. Output gpurun_out/r04m/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04m; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_bsr.py -k "grouped" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
cp spmm-denseblock_amd/lib_tuning/libspmm_hip.so spmm-denseblock_amd/lib/libspmm_hip.so
: > $O/lines.jsonl
for v in 33 243 262 263 33 243 263; do
  SPMM_GRP_VARIANT=$v timeout -k 10 300 python bench.py --workload products_bsr16_f16_grp --steps 20 --warmup 5 --no-cpu-baseline > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
  python3 - $v >> $O/lines.jsonl <<'PY'
import json, sys
d = json.loads([l for l in open("gpurun_out/r04m/b.log") if l.startswith("{")][-1])
print(json.dumps({"variant": int(sys.argv[1]), "ms": d["ms_per_step"], "kernel_ms": d["roofline"]["kernel_ms"]}))
PY
  tail -1 $O/lines.jsonl
done
