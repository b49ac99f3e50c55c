#!/bin/bash
# Round-3 PMC of the shipped column streams (tools/profile_bsr.sh per workload),
# summarised per dispatch of the dominant kernel into gpurun_out/r03_pmc.jsonl.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
: > gpurun_out/r03_pmc.jsonl
for wl in ${WLS:-products_bsr16_f16 products_bsr32}; do
  WL=$wl TAG=_r03 bash tools/profile_bsr.sh || exit 1
  python3 - "$R/gpurun_out/prof_${wl}_r03" "$wl" >> gpurun_out/r03_pmc.jsonl <<'PY'
import csv, glob, json, sys, collections
o, wl = sys.argv[1], sys.argv[2]
kern = "bsr16_f16_cs_kernel" if "bsr16" in wl else "bsr32_f32_cs2_kernel"
acc = collections.defaultdict(list)
for f in glob.glob(o + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if kern in r.get("Kernel_Name", ""):
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
dur = []
for f in glob.glob(o + "/kt/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if kern in r.get("Kernel_Name", ""):
            dur.append(float(r["End_Timestamp"]) - float(r["Start_Timestamp"]))
out = {"workload": wl, "kernel": kern, "trace_ms": round(sum(dur) / len(dur) / 1e6, 4) if dur else None}
out.update({k: round(sum(x) / len(x)) for k, x in sorted(acc.items())})
print(json.dumps(out))
PY
  tail -1 gpurun_out/r03_pmc.jsonl
done
