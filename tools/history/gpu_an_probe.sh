#!/bin/bash
# Analysed column streams on the box: their GPU tests, then each analysed
# workload beside its shipped form (ms per step, kernel ms, rooflines).
timeout -k 10 400 python -u -m pytest tests/test_gpu_bsr.py -x -q --timeout 120 --timeout-method thread -k "${PYK:-analys}" > gpurun_out/an_tests.log 2>&1; rc=$?; tail -5 gpurun_out/an_tests.log; [ $rc -eq 0 ] || exit $rc
for w in ${WLS:-products_bsr16_f16_an products_bsr16_f16 products_rcm_bsr16_f16_an products_bsr32_an}; do timeout -k 10 300 python bench.py --workload $w --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/an_$w.log 2>&1 || exit 1; grep '^{' gpurun_out/an_$w.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); f=r['roofline']; print('$w', r['ms_per_step'], f['kernel_ms'], 'frac', f['frac'], 'mfma', f['mfma_frac'], 'an', r.get('analysis_ms'), 'csr', r.get('csr_same_matrix_ms'))"; done
