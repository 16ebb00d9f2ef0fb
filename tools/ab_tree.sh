# A/B of two source trees on C1-C3 (kernel stats under rocprofv3): build the
# baseline tree into ab_old/ first (git archive <rev> | tar -x -C ab_old; link
# ab_old/tests/golden to ../../tests/golden; make -C ab_old/faster-voxelpose_amd/csrc).
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
for wl in ${WLS:-c1 c2 c3}; do
 for side in old new; do
  if [ $side = old ]; then d=ab_old; else d=.; fi
  (cd $d && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/ab_${wl}_$side -o run -- python3 bench.py --workload $wl --steps 10 --warmup 2 --traffic off --cpu-baseline off --batch ${B:-256} > $GRAFT_REPO_ROOT/gpurun_out/ab_${wl}_$side.json 2>/dev/null) || exit 1
  echo "$wl $side done"
 done
done
