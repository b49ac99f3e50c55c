set -o pipefail
mkdir -p gpurun_out/v1
timeout -k 10 700 python -u -m pytest tests/test_gpu_csr.py tests/test_gpu_configs.py tests/test_gpu_bsr.py -k "csr or config or group" -x -q --timeout 200 --timeout-method thread > gpurun_out/v1/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/v1/pytest.log; [ $rc -eq 0 ] || exit $rc
for w in arxiv_csr products_csr reddit_bsr32_grp products_bsr32_grp; do
  timeout -k 10 300 python bench.py --workload $w --steps 20 --warmup 5 --no-cpu-baseline --no-bsr-sides --no-hot-side > gpurun_out/v1/bw_$w.log 2>&1 || exit $?
  grep '^{' gpurun_out/v1/bw_$w.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); f=r['roofline']; print('$w', r['ms_per_step'], f.get('kernel_ms'), r.get('analysis_ms'))"
done
