# Default bench line (traffic PMC + CPU baseline) and its rocprofv3 kernel-trace summary, for profiles/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; mkdir -p gpurun_out
T0=$(date +%s)
timeout -k 10 600 python bench.py > gpurun_out/final_bench.json 2> gpurun_out/final_bench.err; rc=$?
echo "bench rc=$rc in $(( $(date +%s) - T0 )) s"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/final_prof -o run -- python3 bench.py --traffic off --cpu-baseline off > gpurun_out/final_prof.log 2>&1
echo "prof rc=$?"
