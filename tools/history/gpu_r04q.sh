#!/bin/bash
# Round 4: tiles together for the drop-in and analysed bs 16 column streams (SPMM_CS16_TT=1,
# TUNING build), with the A copies nt (default, 6404) or plain (SPMM_BSR_VARIANT=6104): the
# bs 16 fp16 GPU tests under TT = 1, then interleaved lines. Output gpurun_out/r04q/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04q; mkdir -p $O
cp spmm-denseblock_amd/lib_tuning/libspmm_hip.so spmm-denseblock_amd/lib/libspmm_hip.so
SPMM_CS16_TT=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_bsr.py tests/test_gpu_scale.py -k "f16 and not grouped" > $O/pytest_tt.log 2>&1 || { tail -30 $O/pytest_tt.log; exit 1; }
tail -1 $O/pytest_tt.log
: > $O/lines.jsonl
line() {  # tag workload env...
  local tag=$1 wl=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --workload $wl --steps 20 --warmup 5 --no-cpu-baseline --no-analysed-side > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
  python3 - "$tag" "$wl" >> $O/lines.jsonl <<'PY'
import json, sys
d = json.loads([l for l in open("gpurun_out/r04q/b.log") if l.startswith("{")][-1])
print(json.dumps({"tag": sys.argv[1], "workload": sys.argv[2], "ms": d["ms_per_step"], "kernel_ms": d["roofline"]["kernel_ms"]}))
PY
  tail -1 $O/lines.jsonl
}
for r in 1 2; do
  line nt_tt0 products_bsr16_f16 SPMM_CS16_TT=0
  line nt_tt1 products_bsr16_f16 SPMM_CS16_TT=1
  line plain_tt0 products_bsr16_f16 SPMM_CS16_TT=0 SPMM_BSR_VARIANT=6104
  line plain_tt1 products_bsr16_f16 SPMM_CS16_TT=1 SPMM_BSR_VARIANT=6104
  line an_tt0 products_bsr16_f16_an SPMM_CS16_TT=0
  line an_tt1 products_bsr16_f16_an SPMM_CS16_TT=1
done
