#!/bin/bash
# The panel probe's threshold: tools/panel_fill.py with the library built to force the column
# stream (lib_var/pmin33.so: kPanelMin 33) and the panel stream (lib_var/pmin0.so: kPanelMin 0),
# twice, interleaved. Release library restored. Output in gpurun_out/ab_panel_fill/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
L=spmm-denseblock_amd/lib; O=gpurun_out/ab_panel_fill; mkdir -p $O
cp $L/libspmm_hip.so $O/release.so
for rep in 1 2; do
for v in pmin33 pmin0; do
  cp spmm-denseblock_amd/lib_var/$v.so $L/libspmm_hip.so
  TAG=$v timeout -k 10 300 python -u tools/panel_fill.py > $O/${v}_$rep.jsonl 2> $O/${v}_$rep.log; rc=$?
  [ $rc -ne 0 ] && { cp $O/release.so $L/libspmm_hip.so; tail -3 $O/${v}_$rep.log; exit $rc; }
done
done
cp $O/release.so $L/libspmm_hip.so
python3 - <<'PY'
import json, glob
rows = {}
for f in sorted(glob.glob("gpurun_out/ab_panel_fill/*.jsonl")):
    for l in open(f):
        r = json.loads(l); rows.setdefault((r["F"], r["dim"], r["lib"]), []).append(r["ms"])
for (F, d, lib), v in sorted(rows.items()):
    print(F, d, lib, v)
PY
