#!/bin/bash
# Round 4 GPU call Q: C2 / C4 with the coordinates projected in the gather (div_pair makes the
# projection cheaper) against the cached packed grid.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; O=gpurun_out/r4q; mkdir -p $O
for r in 1 2; do
  for wl in c2 c4; do
    for otf in off on; do
      timeout -k 10 300 python bench.py --workload $wl --on-the-fly $otf --steps 10 --warmup 2 --traffic off --cpu-baseline off > $O/${wl}_${otf}_${r}.json 2> $O/${wl}_${otf}_$r.err || { tail -20 $O/${wl}_${otf}_$r.err; exit 1; }
      tail -1 $O/${wl}_${otf}_${r}.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$wl otf=$otf rep$r', d['value'], d['ms_per_step'], r['frac'], r['kernel_ms'])"
    done
  done
done
echo callQ done
