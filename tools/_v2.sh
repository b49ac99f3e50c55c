set -o pipefail
export TMPDIR=/tmp
R=$(pwd); mkdir -p gpurun_out/v2
for w in reddit_bsr32_grp products_bsr32_grp; do
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/v2/$w -o kt --output-format csv -- python3 $R/bench.py --workload $w --steps 5 --warmup 2 --no-cpu-baseline) > gpurun_out/v2/$w.log 2>&1 || exit $?
done
