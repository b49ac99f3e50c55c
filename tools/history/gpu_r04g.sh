#!/bin/bash
# Round 4: the grouped bs 32 fp32 stream. Its GPU tests, the release lines (reddit and
# products, grouped against the drop-in and analysed entries on the same box), then a
# TUNING sweep of W x (stages, occupancy hint) x XCD chunk (SPMM_GRP32_VARIANT = 10 P + OCC,
# SPMM_GRP_XM). Output gpurun_out/r04g/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); export TMPDIR=/tmp
O=$R/gpurun_out/r04g; mkdir -p $O
stop() { rc=$1; if [ "$rc" -ge 124 ]; then echo "GPU step fault rc=$rc, stopping"; exit "$rc"; fi; }
echo "== tests"
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_bsr.py -k "grouped_f32" > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; stop $rc
[ $rc -eq 0 ] || { grep -E "Error|assert" $O/pytest.log | head -20; exit $rc; }
: > $O/lines.jsonl
line() {  # tag workload args...
  local tag=$1 wl=$2; shift 2
  timeout -k 10 300 python bench.py --workload $wl --steps 20 --warmup 5 --no-cpu-baseline "$@" > $O/b.log 2>&1; rc=$?
  if [ $rc -ne 0 ]; then tail -5 $O/b.log; exit $rc; fi
  python3 - "$tag" "$wl" >> $O/lines.jsonl <<'PY'
import json, sys
d = json.loads([l for l in open("gpurun_out/r04g/b.log") if l.startswith("{")][-1])
r = d["roofline"]
print(json.dumps({"tag": sys.argv[1], "workload": sys.argv[2], "ms": d["ms_per_step"],
                  "kernel_ms": r.get("kernel_ms"), "mfma_frac": r.get("mfma_frac"),
                  "kernel": r.get("kernel"), "analysis_ms": d.get("analysis_ms"),
                  "grouped_entry": d.get("grouped_entry"), "analysed_entry": d.get("analysed_entry")}))
PY
  tail -1 $O/lines.jsonl | cut -c1-400
}
echo "== release"
line release reddit_bsr32
line release reddit_bsr32_grp
line release products_bsr32
line release products_bsr32_grp
echo "== sweep (TUNING)"
cp spmm-denseblock_amd/lib_tuning/libspmm_hip.so spmm-denseblock_amd/lib/libspmm_hip.so
for wl in reddit_bsr32_grp products_bsr32_grp; do
  for W in 2 4; do
    for v in 33 34 43 44 32; do
      SPMM_GRP32_VARIANT=$v line "W${W}_v${v}" $wl --group-rows $W --no-analysed-side
    done
  done
done
for xm in 1 8 32; do SPMM_GRP_XM=$xm line "W2_v33_xm$xm" reddit_bsr32_grp --group-rows 2; done
