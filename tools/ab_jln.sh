# bench_jln.py under env settings "NAME=VAL,NAME=VAL ..." (one run each).
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
i=0
for cfg in $CONFIGS; do
  i=$((i+1))
  env $(echo $cfg | tr ',' ' ') timeout -k 10 200 python tools/bench_jln.py --frames 32 > gpurun_out/jln_$i.log 2>&1
  rc=$?; echo "$cfg rc=$rc $(tail -1 gpurun_out/jln_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["us_per_proposal"], d["per_frame_calls_us_per_proposal"])' 2>/dev/null)"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
