#!/bin/bash
# Round 4: PMC of the grouped bs 16 stream against the drop-in column stream on the
# products stand-in (K = 512): kernel trace + SQ / TCC / TCP / TA counter passes
# (tools/profile_bsr.sh), summarised per dispatch into gpurun_out/r04c/pmc.jsonl.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); export TMPDIR=/tmp
mkdir -p gpurun_out/r04c
: > gpurun_out/r04c/pmc.jsonl
for wl in ${WLS:-products_bsr16_f16_grp products_bsr16_f16}; do
  WL=$wl TAG=_r04 EXTRA="--no-analysed-side ${GEXTRA:-}" bash tools/profile_bsr.sh || exit 1
  python3 - "$R/gpurun_out/prof_${wl}_r04" "$wl" >> gpurun_out/r04c/pmc.jsonl <<'PY'
import csv, glob, json, sys, collections
o, wl = sys.argv[1], sys.argv[2]
kern = "bsr16_f16_grp_kernel" if "grp" in wl else "bsr16_f16_cs_kernel"
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
  tail -1 gpurun_out/r04c/pmc.jsonl | cut -c1-600
done
