# round 3 GPU batch 3: L2 hit of the camera-outer replay vs the shipped gather (PMC), C5 combined knobs
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 120 python3 tools/gather_probe.py --modes FULL,TAPS,TAPS_L1,TAPS_L2,CAM_OUTER --lds-tiles "" > gpurun_out/r3b3_probe.log 2>&1 || exit 1
for m in FULL CAM_OUTER TAPS TAPS_L2; do
  for grp in "TCC_HIT_sum TCC_MISS_sum" "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum" "TD_TD_BUSY_sum TD_TC_STALL_sum"; do
    tag=$(echo $grp | cut -d' ' -f1)
    timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/r3pmc_${m}_$tag -o run -- python3 tools/gather_probe.py --modes $m --iters 5 --lds-tiles "" > gpurun_out/r3pmc_${m}_$tag.log 2>&1 || exit 1
  done
done
echo pmc ok
WL=c5
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 150 python3 bench.py --workload $WL --steps 10 --warmup 2 --traffic off --cpu-baseline off > gpurun_out/ab_${tag}.log 2>&1 || return 1
  echo "$tag $(grep '^{' gpurun_out/ab_${tag}.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], r["kernel_ms"], r["frac"], r["tap_rate"]["frac"])')"
}
run c5_base || exit 1
run c5_v256b8 FVP_EXP_VOXELS=256 FVP_EXP_BAND=8 || exit 1
run c5_v192 FVP_EXP_VOXELS=192 || exit 1
run c5_v256 FVP_EXP_VOXELS=256 || exit 1
run c5_v256b4 FVP_EXP_VOXELS=256 FVP_EXP_BAND=4 || exit 1
timeout -k 10 300 python -u -m pytest tests/test_cnn_1d_weight.py tests/test_integration.py tests/test_gpu_fullsize.py -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r3b3_tests.log 2>&1; echo "tests rc=$?"
