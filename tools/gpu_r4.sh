#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
echo "== nt experiment"; SWEEP_OUT=1 
for a in "--csr-options 0" "--csr-options 1" "--csr-options 0" "--csr-options 1"; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 --warmup 5 $a > gpurun_out/nt.log 2>&1 || { tail gpurun_out/nt.log; exit 1; }
  grep '^{' gpurun_out/nt.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print('$a', r['ms_per_step'], r['roofline']['kernel_ms'])"
done
bash tools/profile_bsr.sh
