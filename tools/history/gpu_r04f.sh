#!/bin/bash
# Round 4: the grouped bs 16 stream after the scalar row loads: XCD chunk size around the
# release default (32 / W groups; TUNING build, SPMM_GRP_XM), then the release build's
# grouped and drop-in lines on products and RCM products, then PMC of both on products
# (tools/profile_bsr.sh). Output gpurun_out/r04f/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); export TMPDIR=/tmp
O=$R/gpurun_out/r04f; mkdir -p $O
stop() { rc=$1; if [ "$rc" -ge 124 ]; then echo "GPU step fault rc=$rc, stopping"; exit "$rc"; fi; }
: > $O/lines.jsonl
line() {  # tag workload args...
  local tag=$1 wl=$2; shift 2
  timeout -k 10 300 python bench.py --workload $wl --steps 10 --warmup 3 --no-cpu-baseline "$@" > $O/b.log 2>&1; rc=$?
  if [ $rc -ne 0 ]; then tail -5 $O/b.log; exit $rc; fi
  python3 - "$tag" "$wl" >> $O/lines.jsonl <<'PY'
import json, sys
d = json.loads([l for l in open("gpurun_out/r04f/b.log") if l.startswith("{")][-1])
r = d["roofline"]
print(json.dumps({"tag": sys.argv[1], "workload": sys.argv[2], "ms": d["ms_per_step"],
                  "kernel_ms": r.get("kernel_ms"), "kernel": r.get("kernel"),
                  "grouped_entry": d.get("grouped_entry"), "analysed_entry": d.get("analysed_entry")}))
PY
  tail -1 $O/lines.jsonl | cut -c1-300
}
echo "== release lines"
line release products_bsr16_f16_grp
line release products_bsr16_f16
line release products_rcm_bsr16_f16_grp
echo "== PMC (release)"
WLS="products_bsr16_f16_grp products_bsr16_f16" bash tools/gpu_r04c.sh; stop $?
cp -r gpurun_out/r04c $O/pmc
echo "== XCD chunk sweep (TUNING)"
cp spmm-denseblock_amd/lib_tuning/libspmm_hip.so spmm-denseblock_amd/lib/libspmm_hip.so
for xm in 1 4 8 16 32; do SPMM_GRP_XM=$xm line "w4_xm$xm" products_bsr16_f16_grp --group-rows 4; done
for xm in 2 8; do SPMM_GRP_XM=$xm line "w8_xm$xm" products_bsr16_f16_grp --group-rows 8; done
