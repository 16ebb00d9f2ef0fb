# A/B of the few-frame gather block size (FVP_FEW_MULT x one pass of columns) on the B=1 step
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
for wl in ${WORKLOADS:-c2}; do for m in ${MULTS:-1 2}; do
  FVP_FEW_MULT=$m timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/few_${wl}_$m -o run -- python3 tools/latency_b1.py --workload $wl > gpurun_out/few_${wl}_$m.log 2>&1 || exit 1
  echo "$wl mult $m: $(grep '^{' gpurun_out/few_${wl}_$m.log)"
done; done
